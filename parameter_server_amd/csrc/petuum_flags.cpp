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
DEFINE_int32(table_staleness, 0, "SSP staleness bound of a table, in clocks");
DEFINE_int32(row_type, 0, "registered row type id of a table");
DEFINE_int32(row_oplog_type, petuum::RowOpLogType::kDenseRowOpLog, "client row-oplog kind (0 dense, 1 sparse, 2 sparse vector, 3 dense binary16)");
DEFINE_bool(oplog_dense_serialized, true, "send dense row oplogs as full-width records");
DEFINE_string(oplog_type, "Sparse", "client oplog store: Sparse, AppendOnly or Dense");
DEFINE_string(append_only_oplog_type, "Inc", "append-only oplog mode: Inc, BatchInc or DenseBatchInc");
DEFINE_uint64(append_only_buffer_capacity, 1024 * 1024, "bytes per append-only oplog buffer");
DEFINE_uint64(append_only_buffer_pool_size, 3, "append-only buffers per worker thread");
DEFINE_int32(bg_apply_append_oplog_freq, 4, "append-only buffers a bg thread merges per apply");
DEFINE_string(process_storage_type, "BoundedSparse", "client row cache: BoundedDense or BoundedSparse");
DEFINE_bool(no_oplog_replay, false, "skip replaying oplogs onto rows the server sends back");
DEFINE_uint64(server_push_row_upper_bound, 100, "most rows a server pushes per table per clock (SSPAggr)");
DEFINE_uint64(client_send_oplog_upper_bound, 100, "most row oplogs a client sends per table per clock (SSPAggr)");
DEFINE_int32(server_table_logic, -1, "registered server table logic id, -1 for the plain apply");
DEFINE_bool(version_maintain, false, "keep a version counter in each server row");

DEFINE_string(stats_path, "", "prefix of the stats output file");
DEFINE_int32(num_clients, 1, "client processes in the job");
DEFINE_int32(num_comm_channels_per_client, 1, "server/bg thread pairs per client");
DEFINE_bool(init_thread_access_table, false, "the init thread also reads and writes tables");
DEFINE_int32(num_table_threads, 1, "worker threads per client that access tables");
DEFINE_int32(client_id, 0, "id of this client process");
DEFINE_string(hostfile, "", "file listing id, ip and port of every server");
DEFINE_string(consistency_model, "SSPPush", "consistency model: SSP, SSPPush or SSPAggr");
DEFINE_uint64(client_bandwidth_mbps, 40, "bg thread send budget in Mbit/s (SSPAggr)");
DEFINE_uint64(server_bandwidth_mbps, 40, "server thread send budget in Mbit/s (SSPAggr)");
DEFINE_uint64(bg_idle_milli, 10, "bg thread idle period in ms before it sends");
DEFINE_uint64(thread_oplog_batch_size, 100 * 1000 * 1000, "worker thread oplog bytes buffered before a flush");
DEFINE_uint64(row_candidate_factor, 5, "candidate rows per pushed row when sorting by importance");
DEFINE_int32(server_idle_milli, 10, "server thread idle period in ms before it pushes");
DEFINE_string(update_sort_policy, "Random", "order of partial sends: Random, FIFO, RelativeMagnitude or FIFO_N_ReMag");
DEFINE_int32(snapshot_clock, -1, "clock interval between table snapshots, -1 for none");
DEFINE_int32(resume_clock, -1, "clock to resume from, -1 for a fresh start");
DEFINE_string(snapshot_dir, "", "directory table snapshots are written to");
DEFINE_string(resume_dir, "", "directory table snapshots are read from");
DEFINE_bool(numa_opt, false, "pin threads to NUMA nodes");
DEFINE_int32(numa_index, 0, "NUMA node this client uses");
DEFINE_string(numa_policy, "Even", "NUMA placement: Even or Center");
DEFINE_bool(naive_table_oplog_meta, true, "use the simple per-table oplog metadata");
DEFINE_bool(suppression_on, false, "suppress small updates (SSPAggr)");
DEFINE_bool(use_approx_sort, true, "sort partial sends approximately");
DEFINE_uint64(num_zmq_threads, 1, "ZeroMQ I/O threads per context");
#endif

namespace petuum {

// The flags-mode marker the declare headers reference (see table_gflags_declare.hpp).
namespace flags_mode {
#if PETUUM_PS_HAVE_GFLAGS
extern const int libpetuum_ps_built_with_gflags = 1;
#else
extern const int libpetuum_ps_built_without_gflags = 1;
#endif
}  // namespace flags_mode

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
