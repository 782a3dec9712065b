// init_table_config.hpp — InitTableConfig / InitTableGroupConfig
// (src/petuum_ps_common/include/init_table_config.cpp:13-42, init_table_group_config.cpp:5-55).
// The reference fills them from gflags; without gflags this fills the same defaults
// (table_gflags.cpp:8-24, system_gflags.cpp:6-45) and apps set fields directly.
#pragma once

#include <petuum_ps_common/include/configs.hpp>

namespace petuum {

inline void InitTableConfig(ClientTableConfig *c) {
  c->table_info.table_staleness = 0;
  c->table_info.row_type = 0;
  c->table_info.row_oplog_type = RowOpLogType::kDenseRowOpLog;   // --row_oplog_type 0 (table_gflags.cpp)
  c->table_info.oplog_dense_serialized = true;                   // --oplog_dense_serialized
  c->table_info.server_push_row_upper_bound = 100;
  c->table_info.server_table_logic = -1;
  c->table_info.version_maintain = false;
  c->oplog_type = Dense;
  c->process_storage_type = BoundedDense;
  c->no_oplog_replay = false;
}

inline void InitTableGroupConfig(TableGroupConfig *c, int32_t num_tables) {
  c->num_tables = num_tables;
  c->consistency_model = SSPPush;                                // --consistency_model SSPPush
  c->num_comm_channels_per_client = 1;
  c->num_total_clients = 1;
  c->client_id = 0;
}

}  // namespace petuum
