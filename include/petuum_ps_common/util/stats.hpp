// stats.hpp — the STATS_* instrumentation macros apps call (src/petuum_ps_common/util/stats.hpp).
//
// The reference compiles two forms: with PETUUM_STATS a thread-registered Stats class, without it
// every macro expands to ((void) 0) (stats.hpp:317-436).  Apps (matrixfact, lda, mlr) call the
// STATS_APP_* macros unconditionally, so both forms must exist for them to build unchanged.
//
// Here, without PETUUM_STATS (the reference's default build): every macro is a no-op, with the
// same names and argument lists.  With PETUUM_STATS: the app-side timers and app-defined values
// are kept per process (a small header-only accumulator), the client-bg and server-thread
// macros stay no-ops — the server is the MI355X shard context, whose apply counters
// (STATS_SERVER_ACCUM_APPLY_OPLOG_BEGIN/END -> server_accum_apply_oplog_sec,
// server_accum_oplog_recv_mb, server_thread.cpp:240-244) come from psx_ctx_stats (include/psx.h)
// through petuum::runtime::ServerApplyStats() — and STATS_PRINT() writes both to stderr.
#pragma once

#include <cstdint>
#include <string>

namespace petuum {
class TableGroupConfig;
namespace runtime {
// The psx_ctx_stats counters summed over this process's server shard contexts
// (libpetuum_ps.so); zeros before PSTableGroup::Init.
struct ServerApplyStatsSum {
  uint64_t calls = 0, messages = 0, oplog_bytes = 0, settled_calls = 0;
  double apply_sec = 0.0;
};
ServerApplyStatsSum ServerApplyStats();
}  // namespace runtime
}  // namespace petuum

#ifdef PETUUM_STATS
#include <chrono>
#include <cstdio>
#include <map>
#include <mutex>
#include <vector>

namespace petuum {
// Per-process accumulators of the app-side macros (the reference keeps them per thread and
// merges them at DeregisterThread, stats.cpp; the totals printed are the same).
class Stats {
 public:
  enum Timer { kLoadData, kInit, kBootstrap, kComp, kObjComp, kTgClock, kAppDefined, kNumTimers };
  static Stats &Get() {
    static Stats s;
    return s;
  }
  void Begin(Timer t) { start_()[t] = Clock::now(); }
  void End(Timer t) {
    const double s = std::chrono::duration<double>(Clock::now() - start_()[t]).count();
    std::lock_guard<std::mutex> g(mtx_);
    sec_[t] += s;
  }
  void SetName(int which, const std::string &n) {
    std::lock_guard<std::mutex> g(mtx_);
    names_[which] = n;
  }
  void AccumVal(double d) {
    std::lock_guard<std::mutex> g(mtx_);
    val_ += d;
  }
  void AppendVec(double v) {
    std::lock_guard<std::mutex> g(mtx_);
    vec_.push_back(v);
  }
  void Print() {
    static const char *kName[kNumTimers] = {"app_load_data_sec", "app_init_sec", "app_bootstrap_sec",
                                            "app_accum_comp_sec", "app_accum_obj_comp_sec",
                                            "app_accum_tg_clock_sec", "app_defined_accum_sec"};
    std::lock_guard<std::mutex> g(mtx_);
    for (int t = 0; t < kNumTimers; ++t)
      std::fprintf(stderr, "%s: %.6f\n", t == kAppDefined && names_.count(0) ? names_[0].c_str() : kName[t], sec_[t]);
    std::fprintf(stderr, "%s: %.6f\n", names_.count(1) ? names_[1].c_str() : "app_defined_accum_val", val_);
    std::fprintf(stderr, "%s:", names_.count(2) ? names_[2].c_str() : "app_defined_vec");
    for (double v : vec_) std::fprintf(stderr, " %g", v);
    std::fprintf(stderr, "\n");
    const runtime::ServerApplyStatsSum s = runtime::ServerApplyStats();
    std::fprintf(stderr, "server_accum_apply_oplog_sec: %.6f\nserver_accum_oplog_recv_mb: %.6f\n"
                         "server_oplog_msg_recv: %llu\n", s.apply_sec, s.oplog_bytes / double(1 << 20),
                 (unsigned long long)s.messages);
  }

 private:
  using Clock = std::chrono::steady_clock;
  static Clock::time_point *start_() {
    thread_local Clock::time_point t[kNumTimers];
    return t;
  }
  std::mutex mtx_;
  double sec_[kNumTimers] = {};
  double val_ = 0.0;
  std::vector<double> vec_;
  std::map<int, std::string> names_;
};
}  // namespace petuum

#define STATS_APP_LOAD_DATA_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kLoadData)
#define STATS_APP_LOAD_DATA_END() petuum::Stats::Get().End(petuum::Stats::kLoadData)
#define STATS_APP_INIT_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kInit)
#define STATS_APP_INIT_END() petuum::Stats::Get().End(petuum::Stats::kInit)
#define STATS_APP_BOOTSTRAP_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kBootstrap)
#define STATS_APP_BOOTSTRAP_END() petuum::Stats::Get().End(petuum::Stats::kBootstrap)
#define STATS_APP_ACCUM_COMP_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kComp)
#define STATS_APP_ACCUM_COMP_END() petuum::Stats::Get().End(petuum::Stats::kComp)
#define STATS_APP_ACCUM_OBJ_COMP_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kObjComp)
#define STATS_APP_ACCUM_OBJ_COMP_END() petuum::Stats::Get().End(petuum::Stats::kObjComp)
#define STATS_APP_ACCUM_TG_CLOCK_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kTgClock)
#define STATS_APP_ACCUM_TG_CLOCK_END() petuum::Stats::Get().End(petuum::Stats::kTgClock)
#define STATS_SET_APP_DEFINED_ACCUM_SEC_NAME(name) petuum::Stats::Get().SetName(0, name)
#define STATS_APP_DEFINED_ACCUM_SEC_BEGIN() petuum::Stats::Get().Begin(petuum::Stats::kAppDefined)
#define STATS_APP_DEFINED_ACCUM_SEC_END() petuum::Stats::Get().End(petuum::Stats::kAppDefined)
#define STATS_SET_APP_DEFINED_ACCUM_VAL_NAME(name) petuum::Stats::Get().SetName(1, name)
#define STATS_APP_DEFINED_ACCUM_VAL_INC(delta) petuum::Stats::Get().AccumVal(delta)
#define STATS_SET_APP_DEFINED_VEC_NAME(name) petuum::Stats::Get().SetName(2, name)
#define STATS_APPEND_APP_DEFINED_VEC(val) petuum::Stats::Get().AppendVec(val)
#define STATS_PRINT() petuum::Stats::Get().Print()
#endif  // PETUUM_STATS

// Every other macro (and, without PETUUM_STATS, all of them): no-ops with the reference's
// names and argument lists.
#ifndef STATS_INIT
#define STATS_INIT(table_group_config) ((void)0)
#endif
#ifndef STATS_REGISTER_THREAD
#define STATS_REGISTER_THREAD(thread_type) ((void)0)
#endif
#ifndef STATS_DEREGISTER_THREAD
#define STATS_DEREGISTER_THREAD() ((void)0)
#endif
#ifndef STATS_APP_LOAD_DATA_BEGIN
#define STATS_APP_LOAD_DATA_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_LOAD_DATA_END
#define STATS_APP_LOAD_DATA_END() ((void)0)
#endif
#ifndef STATS_APP_INIT_BEGIN
#define STATS_APP_INIT_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_INIT_END
#define STATS_APP_INIT_END() ((void)0)
#endif
#ifndef STATS_APP_BOOTSTRAP_BEGIN
#define STATS_APP_BOOTSTRAP_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_BOOTSTRAP_END
#define STATS_APP_BOOTSTRAP_END() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_COMP_BEGIN
#define STATS_APP_ACCUM_COMP_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_COMP_END
#define STATS_APP_ACCUM_COMP_END() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_OBJ_COMP_BEGIN
#define STATS_APP_ACCUM_OBJ_COMP_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_OBJ_COMP_END
#define STATS_APP_ACCUM_OBJ_COMP_END() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_TG_CLOCK_BEGIN
#define STATS_APP_ACCUM_TG_CLOCK_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_TG_CLOCK_END
#define STATS_APP_ACCUM_TG_CLOCK_END() ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_SSP_GET_BEGIN
#define STATS_APP_SAMPLE_SSP_GET_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_SSP_GET_END
#define STATS_APP_SAMPLE_SSP_GET_END(table_id, hit) ((void)0)
#endif
#ifndef STATS_APP_ACCUM_SSPPUSH_GET_COMM_BLOCK_BEGIN
#define STATS_APP_ACCUM_SSPPUSH_GET_COMM_BLOCK_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_ACCUM_SSPPUSH_GET_COMM_BLOCK_END
#define STATS_APP_ACCUM_SSPPUSH_GET_COMM_BLOCK_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_ACCUM_SSP_GET_SERVER_FETCH_BEGIN
#define STATS_APP_ACCUM_SSP_GET_SERVER_FETCH_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_ACCUM_SSP_GET_SERVER_FETCH_END
#define STATS_APP_ACCUM_SSP_GET_SERVER_FETCH_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_INC_BEGIN
#define STATS_APP_SAMPLE_INC_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_INC_END
#define STATS_APP_SAMPLE_INC_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_BATCH_INC_BEGIN
#define STATS_APP_SAMPLE_BATCH_INC_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_BATCH_INC_END
#define STATS_APP_SAMPLE_BATCH_INC_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_BATCH_INC_OPLOG_BEGIN
#define STATS_APP_SAMPLE_BATCH_INC_OPLOG_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_BATCH_INC_OPLOG_END
#define STATS_APP_SAMPLE_BATCH_INC_OPLOG_END() ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_BATCH_INC_PROCESS_STORAGE_BEGIN
#define STATS_APP_SAMPLE_BATCH_INC_PROCESS_STORAGE_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_BATCH_INC_PROCESS_STORAGE_END
#define STATS_APP_SAMPLE_BATCH_INC_PROCESS_STORAGE_END() ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_THREAD_GET_BEGIN
#define STATS_APP_SAMPLE_THREAD_GET_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_THREAD_GET_END
#define STATS_APP_SAMPLE_THREAD_GET_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_THREAD_INC_BEGIN
#define STATS_APP_SAMPLE_THREAD_INC_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_THREAD_INC_END
#define STATS_APP_SAMPLE_THREAD_INC_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_THREAD_BATCH_INC_BEGIN
#define STATS_APP_SAMPLE_THREAD_BATCH_INC_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_THREAD_BATCH_INC_END
#define STATS_APP_SAMPLE_THREAD_BATCH_INC_END(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_CLOCK_BEGIN
#define STATS_APP_SAMPLE_CLOCK_BEGIN(table_id) ((void)0)
#endif
#ifndef STATS_APP_SAMPLE_CLOCK_END
#define STATS_APP_SAMPLE_CLOCK_END(table_id) ((void)0)
#endif
#ifndef STATS_SET_APP_DEFINED_ACCUM_SEC_NAME
#define STATS_SET_APP_DEFINED_ACCUM_SEC_NAME(name) ((void)0)
#endif
#ifndef STATS_APP_DEFINED_ACCUM_SEC_BEGIN
#define STATS_APP_DEFINED_ACCUM_SEC_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_DEFINED_ACCUM_SEC_END
#define STATS_APP_DEFINED_ACCUM_SEC_END() ((void)0)
#endif
#ifndef STATS_SET_APP_DEFINED_ACCUM_VAL_NAME
#define STATS_SET_APP_DEFINED_ACCUM_VAL_NAME(name) ((void)0)
#endif
#ifndef STATS_APP_DEFINED_ACCUM_VAL_INC
#define STATS_APP_DEFINED_ACCUM_VAL_INC(delta) ((void)0)
#endif
#ifndef STATS_APP_ACCUM_APPEND_ONLY_FLUSH_OPLOG_BEGIN
#define STATS_APP_ACCUM_APPEND_ONLY_FLUSH_OPLOG_BEGIN() ((void)0)
#endif
#ifndef STATS_APP_ACCUM_APPEND_ONLY_FLUSH_OPLOG_END
#define STATS_APP_ACCUM_APPEND_ONLY_FLUSH_OPLOG_END() ((void)0)
#endif
#ifndef STATS_SET_APP_DEFINED_VEC_NAME
#define STATS_SET_APP_DEFINED_VEC_NAME(name) ((void)0)
#endif
#ifndef STATS_APPEND_APP_DEFINED_VEC
#define STATS_APPEND_APP_DEFINED_VEC(val) ((void)0)
#endif
#ifndef STATS_BG_ACCUM_OPLOG_SERIALIZE_BEGIN
#define STATS_BG_ACCUM_OPLOG_SERIALIZE_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_OPLOG_SERIALIZE_END
#define STATS_BG_ACCUM_OPLOG_SERIALIZE_END() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_CLOCK_END_OPLOG_SERIALIZE_BEGIN
#define STATS_BG_ACCUM_CLOCK_END_OPLOG_SERIALIZE_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_CLOCK_END_OPLOG_SERIALIZE_END
#define STATS_BG_ACCUM_CLOCK_END_OPLOG_SERIALIZE_END() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_SERVER_PUSH_ROW_APPLY_BEGIN
#define STATS_BG_ACCUM_SERVER_PUSH_ROW_APPLY_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_SERVER_PUSH_ROW_APPLY_END
#define STATS_BG_ACCUM_SERVER_PUSH_ROW_APPLY_END() ((void)0)
#endif
#ifndef STATS_BG_CLOCK
#define STATS_BG_CLOCK() ((void)0)
#endif
#ifndef STATS_BG_ADD_PER_CLOCK_OPLOG_SIZE
#define STATS_BG_ADD_PER_CLOCK_OPLOG_SIZE(oplog_size) ((void)0)
#endif
#ifndef STATS_BG_ADD_PER_CLOCK_SERVER_PUSH_ROW_SIZE
#define STATS_BG_ADD_PER_CLOCK_SERVER_PUSH_ROW_SIZE(server_push_row_size) ((void)0)
#endif
#ifndef STATS_BG_ACCUM_SERVER_PUSH_OPLOG_ROW_APPLIED_ADD_ONE
#define STATS_BG_ACCUM_SERVER_PUSH_OPLOG_ROW_APPLIED_ADD_ONE() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_SERVER_PUSH_UPDATE_APPLIED_ADD_ONE
#define STATS_BG_ACCUM_SERVER_PUSH_UPDATE_APPLIED_ADD_ONE() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_SERVER_PUSH_VERSION_DIFF_ADD
#define STATS_BG_ACCUM_SERVER_PUSH_VERSION_DIFF_ADD(diff) ((void)0)
#endif
#ifndef STATS_BG_SAMPLE_PROCESS_CACHE_INSERT_BEGIN
#define STATS_BG_SAMPLE_PROCESS_CACHE_INSERT_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_SAMPLE_PROCESS_CACHE_INSERT_END
#define STATS_BG_SAMPLE_PROCESS_CACHE_INSERT_END() ((void)0)
#endif
#ifndef STATS_BG_SAMPLE_SERVER_PUSH_DESERIALIZE_BEGIN
#define STATS_BG_SAMPLE_SERVER_PUSH_DESERIALIZE_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_SAMPLE_SERVER_PUSH_DESERIALIZE_END
#define STATS_BG_SAMPLE_SERVER_PUSH_DESERIALIZE_END() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_NUM_OPLOG_METAS_READ
#define STATS_BG_ACCUM_NUM_OPLOG_METAS_READ() ((void)0)
#endif
#ifndef STATS_BG_IDLE_INVOKE_INC_ONE
#define STATS_BG_IDLE_INVOKE_INC_ONE() ((void)0)
#endif
#ifndef STATS_BG_IDLE_SEND_INC_ONE
#define STATS_BG_IDLE_SEND_INC_ONE() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_PUSH_ROW_MSG_RECEIVED_INC_ONE
#define STATS_BG_ACCUM_PUSH_ROW_MSG_RECEIVED_INC_ONE() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_IDLE_SEND_BEGIN
#define STATS_BG_ACCUM_IDLE_SEND_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_IDLE_SEND_END
#define STATS_BG_ACCUM_IDLE_SEND_END() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_IDLE_OPLOG_SENT_BYTES
#define STATS_BG_ACCUM_IDLE_OPLOG_SENT_BYTES(num_bytes) ((void)0)
#endif
#ifndef STATS_BG_ACCUM_HANDLE_APPEND_OPLOG_BEGIN
#define STATS_BG_ACCUM_HANDLE_APPEND_OPLOG_BEGIN() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_HANDLE_APPEND_OPLOG_END
#define STATS_BG_ACCUM_HANDLE_APPEND_OPLOG_END() ((void)0)
#endif
#ifndef STATS_BG_APPEND_ONLY_CREATE_ROW_OPLOG_INC
#define STATS_BG_APPEND_ONLY_CREATE_ROW_OPLOG_INC() ((void)0)
#endif
#ifndef STATS_BG_APPEND_ONLY_RECYCLE_ROW_OPLOG_INC
#define STATS_BG_APPEND_ONLY_RECYCLE_ROW_OPLOG_INC() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_IMPORTANCE
#define STATS_BG_ACCUM_IMPORTANCE(table_id, meta_row_oplog, row_sent) ((void)0)
#endif
#ifndef STATS_BG_ACCUM_IMPORTANCE_VALUE
#define STATS_BG_ACCUM_IMPORTANCE_VALUE(table_id, importance, row_sent) ((void)0)
#endif
#ifndef STATS_BG_ACCUM_WAITS_ON_ACK_IDLE
#define STATS_BG_ACCUM_WAITS_ON_ACK_IDLE() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_WAITS_ON_ACK_CLOCK
#define STATS_BG_ACCUM_WAITS_ON_ACK_CLOCK() ((void)0)
#endif
#ifndef STATS_BG_ACCUM_TABLE_OPLOG_SENT
#define STATS_BG_ACCUM_TABLE_OPLOG_SENT(table_id, row_id, count) ((void)0)
#endif
#ifndef STATS_BG_ACCUM_TABLE_ROW_RECVED
#define STATS_BG_ACCUM_TABLE_ROW_RECVED(table_id, row_id, count) ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_PUSH_ROW_BEGIN
#define STATS_SERVER_ACCUM_PUSH_ROW_BEGIN() ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_PUSH_ROW_END
#define STATS_SERVER_ACCUM_PUSH_ROW_END() ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_APPLY_OPLOG_BEGIN
#define STATS_SERVER_ACCUM_APPLY_OPLOG_BEGIN() ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_APPLY_OPLOG_END
#define STATS_SERVER_ACCUM_APPLY_OPLOG_END() ((void)0)
#endif
#ifndef STATS_SERVER_CLOCK
#define STATS_SERVER_CLOCK() ((void)0)
#endif
#ifndef STATS_SERVER_ADD_PER_CLOCK_OPLOG_SIZE
#define STATS_SERVER_ADD_PER_CLOCK_OPLOG_SIZE(oplog_size) ((void)0)
#endif
#ifndef STATS_SERVER_ADD_PER_CLOCK_PUSH_ROW_SIZE
#define STATS_SERVER_ADD_PER_CLOCK_PUSH_ROW_SIZE(push_row_size) ((void)0)
#endif
#ifndef STATS_SERVER_ADD_PER_CLOCK_ACCUM_DUP_ROWS_SENT
#define STATS_SERVER_ADD_PER_CLOCK_ACCUM_DUP_ROWS_SENT(rows_sent) ((void)0)
#endif
#ifndef STATS_SERVER_OPLOG_MSG_RECV_INC_ONE
#define STATS_SERVER_OPLOG_MSG_RECV_INC_ONE() ((void)0)
#endif
#ifndef STATS_SERVER_PUSH_ROW_MSG_SEND_INC_ONE
#define STATS_SERVER_PUSH_ROW_MSG_SEND_INC_ONE() ((void)0)
#endif
#ifndef STATS_SERVER_IDLE_INVOKE_INC_ONE
#define STATS_SERVER_IDLE_INVOKE_INC_ONE() ((void)0)
#endif
#ifndef STATS_SERVER_IDLE_SEND_INC_ONE
#define STATS_SERVER_IDLE_SEND_INC_ONE() ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_IDLE_ROW_SENT_BYTES
#define STATS_SERVER_ACCUM_IDLE_ROW_SENT_BYTES(num_bytes) ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_IMPORTANCE
#define STATS_SERVER_ACCUM_IMPORTANCE(table_id, importance, row_sent) ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_WAITS_ON_ACK_IDLE
#define STATS_SERVER_ACCUM_WAITS_ON_ACK_IDLE() ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_WAITS_ON_ACK_CLOCK
#define STATS_SERVER_ACCUM_WAITS_ON_ACK_CLOCK() ((void)0)
#endif
#ifndef STATS_SERVER_ACCUM_CHECK
#define STATS_SERVER_ACCUM_CHECK(table_id, permitted, logic_info_size) ((void)0)
#endif
#ifndef STATS_PRINT
#define STATS_PRINT() ((void)0)
#endif
#ifndef STATS_Server_ACCUM_IDLE_SEND_BEGIN
#define STATS_Server_ACCUM_IDLE_SEND_BEGIN() ((void)0)
#endif
#ifndef STATS_Server_ACCUM_IDLE_SEND_END
#define STATS_Server_ACCUM_IDLE_SEND_END() ((void)0)
#endif
