// system_gflags_declare.hpp — the system flags every petuum_ps app includes
// (src/petuum_ps_common/include/system_gflags_declare.hpp:1-52 of the reference; defined,
// with the reference's defaults, in libpetuum_ps.so: parameter_server_amd/csrc/petuum_flags.cpp
// restating system_gflags.cpp:6-45).  With gflags on the include path these are gflags
// flags and InitTableGroupConfig reads them; without it each is a constant at the
// reference's default (see table_gflags_declare.hpp).
#pragma once

#include <cstdint>
#include <string>

#include <petuum_ps_common/include/configs.hpp>
#include <petuum_ps_common/util/utils.hpp>

#if __has_include(<gflags/gflags.h>)
#include <gflags/gflags.h>
#if __has_include(<glog/logging.h>)
#include <glog/logging.h>
#endif
#ifndef PETUUM_PS_HAVE_GFLAGS
#define PETUUM_PS_HAVE_GFLAGS 1
#endif

DECLARE_string(stats_path);
// Topology Configs
DECLARE_int32(num_clients);
DECLARE_int32(num_comm_channels_per_client);
DECLARE_bool(init_thread_access_table);
DECLARE_int32(num_table_threads);
DECLARE_int32(client_id);
DECLARE_string(hostfile);

// Execution Configs
DECLARE_string(consistency_model);

// SSPAggr Configs -- client side
DECLARE_uint64(client_bandwidth_mbps);
DECLARE_uint64(server_bandwidth_mbps);
DECLARE_uint64(bg_idle_milli);

DECLARE_uint64(thread_oplog_batch_size);

// SSPAggr Configs -- server side
DECLARE_uint64(row_candidate_factor);
DECLARE_int32(server_idle_milli);
DECLARE_string(update_sort_policy);

// Snapshot Configs
DECLARE_int32(snapshot_clock);
DECLARE_int32(resume_clock);
DECLARE_string(snapshot_dir);
DECLARE_string(resume_dir);

// numa flags
DECLARE_bool(numa_opt);
DECLARE_int32(numa_index);
DECLARE_string(numa_policy);
DECLARE_bool(naive_table_oplog_meta);
DECLARE_bool(suppression_on);
DECLARE_bool(use_approx_sort);

DECLARE_uint64(num_zmq_threads);

#else  // no gflags: the reference's defaults (system_gflags.cpp:6-45) as constants

#ifndef PETUUM_PS_HAVE_GFLAGS
#define PETUUM_PS_HAVE_GFLAGS 0
#endif
static const std::string FLAGS_stats_path = "";
static const int32_t FLAGS_num_clients = 1;
static const int32_t FLAGS_num_comm_channels_per_client = 1;
static const bool FLAGS_init_thread_access_table = false;
static const int32_t FLAGS_num_table_threads = 1;
static const int32_t FLAGS_client_id = 0;
static const std::string FLAGS_hostfile = "";
static const std::string FLAGS_consistency_model = "SSPPush";
static const uint64_t FLAGS_client_bandwidth_mbps = 40;
static const uint64_t FLAGS_server_bandwidth_mbps = 40;
static const uint64_t FLAGS_bg_idle_milli = 10;
static const uint64_t FLAGS_thread_oplog_batch_size = 100 * 1000 * 1000;
static const uint64_t FLAGS_row_candidate_factor = 5;
static const int32_t FLAGS_server_idle_milli = 10;
static const std::string FLAGS_update_sort_policy = "Random";
static const int32_t FLAGS_snapshot_clock = -1;
static const int32_t FLAGS_resume_clock = -1;
static const std::string FLAGS_snapshot_dir = "";
static const std::string FLAGS_resume_dir = "";
static const bool FLAGS_numa_opt = false;
static const int32_t FLAGS_numa_index = 0;
static const std::string FLAGS_numa_policy = "Even";
static const bool FLAGS_naive_table_oplog_meta = true;
static const bool FLAGS_suppression_on = false;
static const bool FLAGS_use_approx_sort = true;
static const uint64_t FLAGS_num_zmq_threads = 1;

#endif

namespace petuum {
void InitTableGroupConfig(TableGroupConfig *config, int32_t num_tables);
}

// Link-time mode check: the app's headers and libpetuum_ps.so must agree on
// whether the flags are gflags flags.  Each TU that includes a declare header references
// the marker of the mode IT was compiled in; the library defines only the marker of its
// own mode, so a mismatch is an undefined-symbol error at link time naming the mode,
// instead of an app silently reading constant defaults (or missing FLAGS_* definitions).
#ifndef PETUUM_PS_FLAGS_MODE_CHECK
#define PETUUM_PS_FLAGS_MODE_CHECK
namespace petuum {
namespace flags_mode {
#if PETUUM_PS_HAVE_GFLAGS
extern const int libpetuum_ps_built_with_gflags;
__attribute__((used)) static const int *const app_mode_marker = &libpetuum_ps_built_with_gflags;
#else
extern const int libpetuum_ps_built_without_gflags;
__attribute__((used)) static const int *const app_mode_marker = &libpetuum_ps_built_without_gflags;
#endif
}  // namespace flags_mode
}  // namespace petuum
#endif
