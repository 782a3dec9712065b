// petuum_flags.cpp — the petuum_ps flags and the two config initialisers apps call
// (part of libpetuum_ps.so, as the reference's libpetuum-ps.a carries table_gflags.cpp,
// system_gflags.cpp, init_table_config.cpp and init_table_group_config.cpp).
//
// Built where gflags is installed, the flags are gflags flags with the reference's names,
// defaults and help strings (table_gflags.cpp:8-24, system_gflags.cpp:6-45), so an app's
// `--table_staleness 2 --consistency_model SSP` reaches its tables.  Built without it (this
// image), the declare headers supply each flag as a constant at that same default, and the
// initialisers below read the same names either way.
#include <petuum_ps_common/include/table_gflags_declare.hpp>
#include <petuum_ps_common/include/system_gflags_declare.hpp>
#include <petuum_ps_common/include/init_table_config.hpp>
#include <petuum_ps_common/include/init_table_group_config.hpp>

#include <cstdio>
#include <cstdlib>

#if PETUUM_PS_HAVE_GFLAGS
DEFINE_int32(table_staleness, 0, "table staleness");
DEFINE_int32(row_type, 0, "table row type");
DEFINE_int32(row_oplog_type, petuum::RowOpLogType::kDenseRowOpLog, "row oplog type");
DEFINE_bool(oplog_dense_serialized, true, "dense serialized oplog");
DEFINE_string(oplog_type, "Sparse", "use append only oplog?");
DEFINE_string(append_only_oplog_type, "Inc", "append only oplog type?");
DEFINE_uint64(append_only_buffer_capacity, 1024 * 1024, "buffer capacity in bytes");
DEFINE_uint64(append_only_buffer_pool_size, 3, "append_ only buffer pool size");
DEFINE_int32(bg_apply_append_oplog_freq, 4, "bg apply append oplog freq");
DEFINE_string(process_storage_type, "BoundedSparse", "proess storage type");
DEFINE_bool(no_oplog_replay, false, "oplog replay?");
DEFINE_uint64(server_push_row_upper_bound, 100, "Server push row threshold");
DEFINE_uint64(client_send_oplog_upper_bound, 100, "client send oplog upper bound");
DEFINE_int32(server_table_logic, -1, "server table logic");
DEFINE_bool(version_maintain, false, "version maintain");

DEFINE_string(stats_path, "", "stats file path prefix");
DEFINE_int32(num_clients, 1, "total number of clients");
DEFINE_int32(num_comm_channels_per_client, 1, "no. of comm channels per client");
DEFINE_bool(init_thread_access_table, false, "whether init thread accesses table");
DEFINE_int32(num_table_threads, 1, "no. of worker threads per client");
DEFINE_int32(client_id, 0, "This client's ID");
DEFINE_string(hostfile, "", "path to Petuum PS server configuration file");
DEFINE_string(consistency_model, "SSPPush", "SSPAggr/SSPPush/SSP");
DEFINE_uint64(client_bandwidth_mbps, 40, "per-thread bandwidth limit, in mbps");
DEFINE_uint64(server_bandwidth_mbps, 40, "per-thread bandwidth limit, in mbps");
DEFINE_uint64(bg_idle_milli, 10, "Bg idle millisecond");
DEFINE_uint64(thread_oplog_batch_size, 100 * 1000 * 1000, "thread oplog batch size");
DEFINE_uint64(row_candidate_factor, 5, "server row candidate factor");
DEFINE_int32(server_idle_milli, 10, "server idle time out in millisec");
DEFINE_string(update_sort_policy, "Random", "Update sort policy");
DEFINE_int32(snapshot_clock, -1, "snapshot clock");
DEFINE_int32(resume_clock, -1, "resume clock");
DEFINE_string(snapshot_dir, "", "snap shot directory");
DEFINE_string(resume_dir, "", "resume directory");
DEFINE_bool(numa_opt, false, "numa opt on?");
DEFINE_int32(numa_index, 0, "numa node index");
DEFINE_string(numa_policy, "Even", "numa policy");
DEFINE_bool(naive_table_oplog_meta, true, "naive table oplog meta");
DEFINE_bool(suppression_on, false, "suppression on");
DEFINE_bool(use_approx_sort, true, "use_approx_sort");
DEFINE_uint64(num_zmq_threads, 1, "number of zmq threads");
#endif

namespace petuum {

// init_table_config.cpp:13-42
void InitTableConfig(ClientTableConfig *config) {
  config->table_info.table_staleness = FLAGS_table_staleness;
  config->table_info.row_type = FLAGS_row_type;
  config->table_info.oplog_dense_serialized = FLAGS_oplog_dense_serialized;
  config->table_info.row_oplog_type = FLAGS_row_oplog_type;
  config->oplog_type = GetOpLogType(FLAGS_oplog_type);
  if (config->oplog_type == AppendOnly)
    config->append_only_oplog_type = GetAppendOnlyOpLogType(FLAGS_append_only_oplog_type);
  config->append_only_buff_capacity = FLAGS_append_only_buffer_capacity;
  config->per_thread_append_only_buff_pool_size = FLAGS_append_only_buffer_pool_size;
  config->bg_apply_append_oplog_freq = FLAGS_bg_apply_append_oplog_freq;
  config->process_storage_type = GetProcessStroageType(FLAGS_process_storage_type);
  config->no_oplog_replay = FLAGS_no_oplog_replay;
  config->table_info.server_push_row_upper_bound = FLAGS_server_push_row_upper_bound;
  config->client_send_oplog_upper_bound = FLAGS_client_send_oplog_upper_bound;
  config->table_info.server_table_logic = FLAGS_server_table_logic;
  config->table_info.version_maintain = FLAGS_version_maintain;
}

// init_table_group_config.cpp:5-55
void InitTableGroupConfig(TableGroupConfig *config, int32_t num_tables) {
  config->stats_path = FLAGS_stats_path;
  config->num_comm_channels_per_client = FLAGS_num_comm_channels_per_client;
  config->num_tables = num_tables;
  config->num_total_clients = FLAGS_num_clients;
  config->num_local_app_threads = FLAGS_init_thread_access_table ? FLAGS_num_table_threads : FLAGS_num_table_threads + 1;
  GetHostInfos(FLAGS_hostfile, &config->host_map);
  config->client_id = FLAGS_client_id;
  config->consistency_model = GetConsistencyModel(FLAGS_consistency_model);
  config->aggressive_clock = false;
  config->aggressive_cpu = false;
  config->server_ring_size = 0;
  config->snapshot_clock = FLAGS_snapshot_clock;
  config->resume_clock = FLAGS_resume_clock;
  config->snapshot_dir = FLAGS_snapshot_dir;
  config->resume_dir = FLAGS_resume_dir;
  config->update_sort_policy = GetUpdateSortPolicy(FLAGS_update_sort_policy);
  config->bg_idle_milli = FLAGS_bg_idle_milli;
  config->client_bandwidth_mbps = FLAGS_client_bandwidth_mbps;
  config->server_bandwidth_mbps = FLAGS_server_bandwidth_mbps;
  config->thread_oplog_batch_size = FLAGS_thread_oplog_batch_size;
  config->row_candidate_factor = FLAGS_row_candidate_factor;
  config->server_idle_milli = FLAGS_server_idle_milli;
  config->numa_opt = FLAGS_numa_opt;
  config->numa_index = FLAGS_numa_index;
  if (FLAGS_numa_opt) {
    if (FLAGS_numa_policy == "Even") {
      config->numa_policy = Even;
    } else if (FLAGS_numa_policy == "Center") {
      config->numa_policy = Center;
    } else {
      std::fprintf(stderr, "petuum: unknown NUMA policy = %s\n", std::string(FLAGS_numa_policy).c_str());
      std::abort();   // LOG(FATAL), init_table_group_config.cpp:43
    }
  }
  config->naive_table_oplog_meta = FLAGS_naive_table_oplog_meta;
  config->suppression_on = FLAGS_suppression_on;
  config->use_approx_sort = FLAGS_use_approx_sort;
  config->num_zmq_threads = FLAGS_num_zmq_threads;
}

}  // namespace petuum
