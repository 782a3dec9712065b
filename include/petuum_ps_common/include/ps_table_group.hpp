// ps_table_group.hpp — PSTableGroup, the process-wide entry point of the App API
// (src/petuum_ps_common/include/ps_table_group.hpp:30-140).  Backed by the MI355X client
// runtime (libpetuum_ps.so): tables live on the GPU (one psx context per comm channel =
// server shard) and the process caches rows on the host.
#pragma once

#include <cstdint>

#include <petuum_ps_common/include/abstract_row.hpp>
#include <petuum_ps_common/include/configs.hpp>
#include <petuum_ps_common/include/table.hpp>
#include <petuum_ps_common/util/class_register.hpp>

namespace petuum {

namespace runtime {
// libpetuum_ps.so
int32_t Init(const TableGroupConfig &config, bool table_access);
void ShutDown();
bool CreateTable(int32_t table_id, const ClientTableConfig &config);
void CreateTableDone();
void WaitThreadRegister();
AbstractClientTable *GetTableOrDie(int32_t table_id);
int32_t RegisterThread();
void DeregisterThread();
void Clock();
void GlobalBarrier();
}  // namespace runtime

class PSTableGroup {
 public:
  // Once per process, after RegisterRow and before anything else; returns the init thread id.
  static int Init(const TableGroupConfig &table_group_config, bool table_access) {
    return runtime::Init(table_group_config, table_access);
  }
  static void ShutDown() { runtime::ShutDown(); }

  template <typename ROW>
  static void RegisterRow(int32_t row_type) {
    ClassRegistry<AbstractRow>::GetRegistry().AddCreator(row_type, CreateObj<AbstractRow, ROW>);
  }

  static bool CreateTable(int32_t table_id, const ClientTableConfig &table_config) {
    return runtime::CreateTable(table_id, table_config);
  }
  static void CreateTableDone() { runtime::CreateTableDone(); }
  static void WaitThreadRegister() { runtime::WaitThreadRegister(); }

  template <typename UPDATE>
  static Table<UPDATE> GetTableOrDie(int32_t table_id) {
    return Table<UPDATE>(runtime::GetTableOrDie(table_id));
  }

  static int32_t RegisterThread() { return runtime::RegisterThread(); }
  static void DeregisterThread() { runtime::DeregisterThread(); }
  // Advance the calling app thread's clock (one vector clock per process).
  static void Clock() { runtime::Clock(); }
  // Clock staleness + 1 times: every table thread then sees every other's updates.
  static void GlobalBarrier() { runtime::GlobalBarrier(); }
  static void TurnOnEarlyComm() {}
  static void TurnOffEarlyComm() {}
};

}  // namespace petuum
