// configs.hpp — the petuum_ps configuration structs apps fill before PSTableGroup::Init
// and CreateTable (same names, fields and defaults as
// src/petuum_ps_common/include/configs.hpp:14-252 of the reference).  Fields the MI355X
// runtime does not use (NUMA, bandwidth management, out-of-core paths, ...) are kept so
// app code compiles unchanged; see README/INTEGRATION for what is honoured.
#pragma once

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include <petuum_ps_common/include/constants.hpp>
#include <petuum_ps_common/include/host_info.hpp>

namespace petuum {

enum ConsistencyModel { SSP = 0, SSPPush = 1, SSPAggr = 2, LocalOOC = 6 };

enum UpdateSortPolicy { FIFO = 0, Random = 1, RelativeMagnitude = 2, FIFO_N_ReMag = 3, FixedOrder = 4 };

struct RowOpLogType {
  static const int32_t kDenseRowOpLog = 0;
  static const int32_t kSparseRowOpLog = 1;
  static const int32_t kSparseVectorRowOpLog = 2;
  static const int32_t kDenseRowOpLogFloat16 = 3;
};

enum OpLogType { Sparse = 0, AppendOnly = 1, Dense = 2 };

enum AppendOnlyOpLogType { Inc = 0, BatchInc = 1, DenseBatchInc = 2 };

enum ProcessStorageType { BoundedDense = 0, BoundedSparse = 1 };

enum NumaPolicy { Even = 0, Center = 1 };

struct TableGroupConfig {
  std::string stats_path;
  int32_t num_comm_channels_per_client = 1;   // server shards (one psx context each)
  int32_t num_tables = 1;
  int32_t num_total_clients = 1;
  int32_t num_local_app_threads = 2;          // threads that call RegisterThread + the init thread
  std::map<int32_t, HostInfo> host_map;
  int32_t client_id = 0;
  bool aggressive_clock = false;
  ConsistencyModel consistency_model = SSPPush;
  int32_t aggressive_cpu = 0;
  int32_t server_ring_size = 0;
  int32_t snapshot_clock = -1;
  int32_t resume_clock = -1;
  std::string snapshot_dir;
  std::string resume_dir;
  std::string ooc_path_prefix;
  UpdateSortPolicy update_sort_policy = Random;
  long bg_idle_milli = 2;
  double client_bandwidth_mbps = 40;
  double server_bandwidth_mbps = 40;
  size_t thread_oplog_batch_size = 100 * 1000 * 1000;
  long server_idle_milli = 0;
  long row_candidate_factor = 5;
  bool numa_opt = false;
  int32_t numa_index = 0;
  NumaPolicy numa_policy = Even;
  bool naive_table_oplog_meta = true;
  bool suppression_on = false;
  bool use_approx_sort = false;
  size_t num_zmq_threads = 1;
};

struct TableInfo {
  int32_t table_staleness = 0;
  int32_t row_type = -1;                      // id given to PSTableGroup::RegisterRow<ROW>
  size_t row_capacity = 0;
  bool oplog_dense_serialized = false;
  int32_t row_oplog_type = 1;
  size_t dense_row_oplog_capacity = 0;
  size_t server_push_row_upper_bound = 100;
  int32_t server_table_logic = -1;
  bool version_maintain = false;
};

struct ClientTableConfig {
  TableInfo table_info;
  size_t process_cache_capacity = 0;          // also the row-id range of the table: rows [0, capacity)
  size_t thread_cache_capacity = 1;
  size_t oplog_capacity = 0;
  OpLogType oplog_type = Dense;
  AppendOnlyOpLogType append_only_oplog_type = Inc;
  size_t append_only_buff_capacity = 10 * k1_Mi;
  size_t per_thread_append_only_buff_pool_size = 3;
  int32_t bg_apply_append_oplog_freq = 1;
  ProcessStorageType process_storage_type = BoundedDense;
  bool no_oplog_replay = false;
  size_t client_send_oplog_upper_bound = 100;
};

}  // namespace petuum
