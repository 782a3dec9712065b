// abstract_server_table_logic.hpp — the server-table logic plugin seam
// (src/petuum_ps_common/include/abstract_server_table_logic.hpp:13-32 of the reference).
// Apps register a logic class under an id and select it per table with
// TableInfo.server_table_logic:
//
//   petuum::ClassRegistry<petuum::AbstractServerTableLogic>::GetRegistry().AddCreator(
//       1, petuum::CreateObj<petuum::AbstractServerTableLogic, petuum::AdaRevisionServerTableLogic>);
//
// (apps/matrixfact/src/matrixfact_adarevision.cpp:633-635).  The interface is the
// reference's.  On MI355X the server rows live in HBM and every record is applied by device
// kernels (libpsx), so a host object is never called per record: the runtime creates the
// registered logic, calls Init, and asks it which built-in device logic it stands for
// (GetDeviceLogic, the one addition to the interface).  A logic without a device
// implementation makes CreateTable fail loudly instead of running on the host.  The
// device logics built into libpsx: AdaRevision (psx_table_set_adarevision).
#pragma once

#include <cstddef>
#include <cstdint>

#include <petuum_ps_common/include/configs.hpp>

namespace petuum {

// The server row a logic receives in the reference (petuum_ps/server/server_row.hpp); on
// MI355X it is a slot of a device table and host code never dereferences it.
class ServerRow;

typedef void (*ApplyRowBatchIncFunc)(const int32_t *column_ids, const void *updates, int32_t num_updates,
                                     ServerRow *server_row);

// The built-in device logic a registered logic selects, with its parameters.
enum class DeviceTableLogicKind : int32_t { kNone = 0, kAdaRevision = 1 };

struct DeviceTableLogic {
  DeviceTableLogicKind kind = DeviceTableLogicKind::kNone;
  // AdaRevision (adarevision_server_table_logic.cpp:8-10): FLAGS_init_step_size,
  // FLAGS_random_init == "guassian", FLAGS_old_grad_upper_bound
  float init_step_size = 0.1f;
  bool gaussian_init = true;
  uint64_t old_grad_upper_bound = 10000;
  // HBM snapshot slots per row (1..8; 0 = 4); the reference's map is unbounded
  int32_t max_snapshots_per_row = 0;
};

class AbstractServerTableLogic {
 public:
  AbstractServerTableLogic() {}
  virtual ~AbstractServerTableLogic() {}

  virtual void Init(const TableInfo &table_info, ApplyRowBatchIncFunc RowBatchInc) = 0;

  virtual void ServerRowCreated(int32_t row_id, ServerRow *server_row) = 0;
  virtual void ApplyRowOpLog(int32_t row_id, const int32_t *col_ids, const void *updates, int32_t num_updates,
                             ServerRow *server_row, uint64_t row_version, bool end_of_version) = 0;

  virtual void ServerRowSent(int32_t row_id, uint64_t version, size_t num_clients) = 0;
  virtual bool AllowSend() = 0;

  // MI355X: the device logic this object stands for (called once, after Init).
  virtual DeviceTableLogic GetDeviceLogic() const { return DeviceTableLogic(); }
};

}  // namespace petuum
