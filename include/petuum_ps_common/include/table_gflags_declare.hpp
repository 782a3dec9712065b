// table_gflags_declare.hpp — the table flags every petuum_ps app includes
// (src/petuum_ps_common/include/table_gflags_declare.hpp:1-22 of the reference; defined,
// with the reference's defaults, in libpetuum_ps.so: parameter_server_amd/csrc/petuum_flags.cpp
// restating table_gflags.cpp:8-24).
//
// With gflags on the include path (as on any box that builds the reference's apps) these
// are gflags flags and InitTableConfig reads them, so `--table_staleness 2` reaches the
// table.  Without gflags (this repo's own examples) each flag is a constant at the
// reference's default value, and InitTableConfig reads the same names.
#pragma once

#include <cstdint>
#include <string>

#if __has_include(<gflags/gflags.h>)
#include <gflags/gflags.h>
#if __has_include(<glog/logging.h>)
#include <glog/logging.h>
#endif
#ifndef PETUUM_PS_HAVE_GFLAGS
#define PETUUM_PS_HAVE_GFLAGS 1
#endif

DECLARE_int32(table_staleness);
DECLARE_int32(row_type);
DECLARE_int32(row_oplog_type);
DECLARE_bool(oplog_dense_serialized);
DECLARE_string(oplog_type);
DECLARE_string(append_only_oplog_type);
DECLARE_uint64(append_only_buffer_capacity);
DECLARE_uint64(append_only_buffer_pool_size);
DECLARE_int32(bg_apply_append_oplog_freq);
DECLARE_string(process_storage_type);
DECLARE_bool(no_oplog_replay);

DECLARE_uint64(server_push_row_upper_bound);
DECLARE_uint64(client_send_oplog_upper_bound);
DECLARE_int32(server_table_logic);
DECLARE_bool(version_maintain);

#else  // no gflags: the reference's defaults (table_gflags.cpp:10-24) as constants

#ifndef PETUUM_PS_HAVE_GFLAGS
#define PETUUM_PS_HAVE_GFLAGS 0
#endif
static const int32_t FLAGS_table_staleness = 0;
static const int32_t FLAGS_row_type = 0;
static const int32_t FLAGS_row_oplog_type = 0;   // RowOpLogType::kDenseRowOpLog
static const bool FLAGS_oplog_dense_serialized = true;
static const std::string FLAGS_oplog_type = "Sparse";
static const std::string FLAGS_append_only_oplog_type = "Inc";
static const uint64_t FLAGS_append_only_buffer_capacity = 1024 * 1024;
static const uint64_t FLAGS_append_only_buffer_pool_size = 3;
static const int32_t FLAGS_bg_apply_append_oplog_freq = 4;
static const std::string FLAGS_process_storage_type = "BoundedSparse";
static const bool FLAGS_no_oplog_replay = false;
static const uint64_t FLAGS_server_push_row_upper_bound = 100;
static const uint64_t FLAGS_client_send_oplog_upper_bound = 100;
static const int32_t FLAGS_server_table_logic = -1;
static const bool FLAGS_version_maintain = false;

#endif

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
