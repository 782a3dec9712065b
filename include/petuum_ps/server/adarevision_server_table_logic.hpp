// adarevision_server_table_logic.hpp — AdaRevisionServerTableLogic
// (src/petuum_ps/server/adarevision_server_table_logic.hpp:38-76 and .cpp of the reference),
// the server-table logic apps/matrixfact's matrixfact_adarevision registers.  The logic runs
// on the device (psx_ada.hip: per record and element the adaptive-revision step on accum /
// z / z_max state beside every row, snapshots of accum per (row, version) for the clients a
// row was sent to); this class selects it and carries its flags.
//
// The reference defines the logic's flags with gflags in the .cpp (:8-10) and apps declare
// them (DECLARE_double(init_step_size), matrixfact_adarevision.cpp:26).  gflags is not part
// of this build: the flags are plain globals with the same names and
// defaults, set before PSTableGroup::CreateTable.
#pragma once

#include <cstdint>
#include <string>

#include <petuum_ps_common/include/abstract_server_table_logic.hpp>

inline double FLAGS_init_step_size = 0.1;             // "init step size"
inline uint64_t FLAGS_old_grad_upper_bound = 10000;   // "gradient upper bound"
inline std::string FLAGS_random_init = "guassian";    // "initialize server row" (the reference's spelling)

namespace petuum {

class AdaRevisionServerTableLogic : public AbstractServerTableLogic {
 public:
  AdaRevisionServerTableLogic() {}
  ~AdaRevisionServerTableLogic() override {}

  void Init(const TableInfo &table_info, ApplyRowBatchIncFunc RowBatchInc) override {
    table_info_ = table_info;
    RowBatchInc_ = RowBatchInc;
    init_step_size_ = (float)FLAGS_init_step_size;
  }
  // Per-row work happens on the device (psx_ada.hip); these are never called by the runtime.
  void ServerRowCreated(int32_t, ServerRow *) override {}
  void ApplyRowOpLog(int32_t, const int32_t *, const void *, int32_t, ServerRow *, uint64_t, bool) override {}
  void ServerRowSent(int32_t, uint64_t, size_t) override {}
  // The device logic applies AllowSend (live snapshots < old_grad_upper_bound) to the
  // partial push itself.
  bool AllowSend() override { return true; }

  DeviceTableLogic GetDeviceLogic() const override {
    DeviceTableLogic d;
    d.kind = DeviceTableLogicKind::kAdaRevision;
    d.init_step_size = init_step_size_;
    d.gaussian_init = FLAGS_random_init == "guassian";
    d.old_grad_upper_bound = FLAGS_old_grad_upper_bound;
    return d;
  }

 private:
  TableInfo table_info_;
  ApplyRowBatchIncFunc RowBatchInc_ = nullptr;
  float init_step_size_ = 0.1f;
};

}  // namespace petuum
