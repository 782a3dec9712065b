// psx_runtime.cpp — host runtime behind include/psx.h.
//
// One psx_ctx == one reference ServerThread's Server (server_thread.hpp:90): it owns
// the shard's tables in HBM, the per-sender version map (server.cpp:21-24,124-126) and
// a HIP stream.  Every apply call enqueues the kernel pipeline of psx_kernels.hip and
// returns; device-detected errors surface at psx_sync().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "../../include/psx.h"
#include "psx_device.hpp"

namespace psx {
hipError_t launch_decode(StreamSet ss, const TableDir &dir, Seg *segs, uint64_t *recoff,
                         uint32_t *call_status, uint32_t *counters, uint32_t *ntouched, const IdxSet &ix,
                         uint32_t *idxw, const WalkCount *wc, hipStream_t st);
bool dense_apply_checks_rows(const DenseArgs &a, bool rec_f16);
hipError_t launch_split_count(const SplitArgs &a, hipStream_t st);
hipError_t launch_split_scatter(const SplitArgs &a, const int64_t *pos, const uint32_t *val, int32_t nwords,
                                hipStream_t st);
hipError_t launch_walk(StreamSet ss, const TableDir &dir, Seg *segs, uint64_t *recoff, uint32_t *call_status,
                       uint32_t *counters, uint32_t *ntouched, void *ws, uint32_t spec_wpr, unsigned blocks,
                       uint32_t epoch, uint64_t trace_items, const WalkCount *wc, uint64_t items, int levels,
                       int shape, hipStream_t st);
size_t walk_trace_offset(uint64_t items);
size_t walk_ws_bytes(uint64_t items, int levels);
uint64_t walk_window_bytes(int shape);
// PSX_VARIANT_DECODE: 1 (default) walked messages with sparse tables decode window-parallel
// where eligible, 0 one workgroup per message.
int g_decode_walk = 1;
int g_walk_calls = 0;    // PSX_STAT_WALK_CALLS
int g_walk_trace = 0;    // PSX_DEBUG_WALK_TRACE: walked calls write per-window timestamps
int g_walk_count = 1;   // PSX_VARIANT_WALK_COUNT: 1 = split tables counted by the walk (unpipelined walked calls)
int g_fold_finish = 1;  // PSX_VARIANT_FOLD_FINISH: 1 = a call ending in an ordered apply finishes in it
int g_ord_probe = 0;    // PSX_DEBUG_ORD_PROBE: timing probes of the register apply (results wrong)
int g_ord_lite = 0;     // PSX_VARIANT_ORD_LITE: 1 = split tables take light rows four to a wave (C3 apply
                        // 0.054 ms against 0.048 with it off, profiles/r05/s9: a variant, not the default)
int g_walk_skew = 0;    // PSX_DEBUG_WALK_SKEW: skew early-published walk states (tests the cross-check)
int g_walk_levels = 4;  // PSX_VARIANT_WALK_LEVELS: composed exit-map levels of the walk (0 = window by window)
int g_walk_all_cus = 1;  // PSX_VARIANT_WALK_CUS: the walk's persistent grid: 0 half the CUs, 1 every CU, n >= 2 n blocks per CU
int g_walk_rank = 1;     // PSX_VARIANT_WALK_RANK: split tables' counts also give each record's list place (wfill)
int g_call_events = 0;   // PSX_VARIANT_CALL_EVENTS: bit 0 an event pair per call for psx_ctx_stats (else one per
                         // sync interval), bit 1 the slot-free event on every call (else only when pipelining)
int g_walk_shape = 4;    // PSX_VARIANT_WALK_SHAPE: the walk's threads per block x window words (psx_walk.hip kWalkShapes)
int g_dense_store_nt = 1;   // PSX_VARIANT_DENSE_STORE
int g_prep_halves = 1;   // PSX_VARIANT_PREP_HALVES: a pipelined call's split tables prep in two halves
int g_walk_cus_pipelined = 0;   // PSX_VARIANT_WALK_CUS_PIPELINED: PSX_VARIANT_WALK_CUS for pipelined calls
int g_stream_priority = 0;      // PSX_VARIANT_STREAM_PRIORITY (read when a context is created)
int g_ord_bucket = 1;           // PSX_VARIANT_ORD_BUCKET: split tables' record lists in buckets
int g_pipe_slots = 0;           // PSX_VARIANT_PIPE_SLOTS: pipelined bucket calls classify slots in the dry run
int g_side_cu_mask = 0;        // PSX_VARIANT_SIDE_CU_MASK (read when a context is created)
int g_event_scope = 2;         // PSX_VARIANT_EVENT_SCOPE (read when a context is created)
// Granule tags of the window-parallel decode: unique per call across every context of the
// process, so a granule left in a recycled allocation by another context (or an earlier
// call of this slot) can never carry the tag a walk waits for.  (Round 2's fault: epochs
// restarted at 1 per context and the workspace was zeroed by a null-stream hipMemset that
// the context's non-blocking streams do not wait for, so a new context's walk could take a
// freed context's granule as its predecessor's state, or have its own published granule
// zeroed under it: an out-of-range recoff write, or a lost hand-off.)
std::atomic<uint32_t> g_walk_epoch{0};
uint32_t next_walk_epoch() {
  uint32_t e;
  do e = g_walk_epoch.fetch_add(1, std::memory_order_relaxed) + 1; while (e == 0);
  return e;
}
hipError_t launch_dense_index(StreamSet ss, const IdxSet &ix, uint32_t rows_mask, const Seg *segs, int t, int B,
                              int64_t stride,
                              int64_t row_offset, int64_t row_stride, int64_t max_rows, int32_t *inv,
                              InvLayout L, uint32_t *call_status, hipStream_t st);
hipError_t launch_dense_verify(const int32_t *inv, InvLayout L, int t, int B, int64_t max_rows,
                               uint32_t *counters, hipStream_t st);
hipError_t launch_finish(uint32_t *sticky, uint32_t *call_status, uint32_t *log, hipStream_t st);
hipError_t launch_flags_or(uint8_t *flags, int64_t first, int64_t num, uint8_t bits, hipStream_t st);
hipError_t launch_flags_and(uint8_t *flags, int64_t num, uint8_t bits, hipStream_t st);
hipError_t launch_gather_rows(int dtype, const void *table, const int64_t *slots, int32_t n,
                              int64_t row_cap, void *out, hipStream_t st);
hipError_t launch_gather_flags(const uint8_t *flags, const int64_t *slots, int32_t n, uint8_t *out,
                               hipStream_t st);

hipError_t launch_dense_apply(int dtype, const DenseArgs &a, hipStream_t st, bool rec_f16);
hipError_t launch_fill_u64(uint64_t *p, int64_t n, uint64_t v, hipStream_t st);
hipError_t launch_fill_f32(float *p, int64_t n, float v, hipStream_t st);
hipError_t launch_ada_new_rows(const AdaArgs &a, hipStream_t st);
hipError_t launch_ada_sort(void *tmp, size_t *bytes, const uint64_t *kin, uint64_t *kout, const int32_t *vin,
                           int32_t *vout, int n, hipStream_t st);
hipError_t launch_ada_init_rows(const AdaArgs &a, const int32_t *slots, const float *deltas, int32_t n,
                                hipStream_t st);
hipError_t launch_ada_apply(const AdaArgs &a, hipStream_t st);
hipError_t launch_ada_sent(const AdaArgs &a, const int32_t *list, const int64_t *sizes, int64_t n,
                           uint64_t clients, const uint64_t *subs, int check_only, hipStream_t st);
hipError_t launch_gather_u64(const uint64_t *src, const int64_t *slots, int32_t n, uint64_t *out, hipStream_t st);
hipError_t launch_ordered_prep(int dtype, const OrdArgs &a, int2 *wfill, hipStream_t st);
hipError_t launch_ordered_prep_records(const OrdArgs &a, int2 *wfill, int4 *plist, hipStream_t st);
hipError_t launch_ordered_prep_rows(int dtype, const OrdArgs &a, const int4 *plist, hipStream_t st);
bool ordered_prep_in_dry_run(const OrdArgs &a);
hipError_t launch_ordered_count(const OrdArgs &a, int2 *wfill, hipStream_t st);
hipError_t launch_ordered_prep_slots(int dtype, const OrdArgs &a, int2 *wfill, bool with_count, hipStream_t st);
hipError_t launch_ordered_apply(int dtype, const OrdArgs &a, hipStream_t st, const Fork &fk);
extern int g_ord_split;
hipError_t launch_ada_check(const AdaArgs &a, hipStream_t st);
hipError_t launch_gate(const Seg *segs, const uint32_t *counters, const TableMask &m, int B,
                       uint32_t *call_status, hipStream_t st);
hipError_t launch_serve_sizes(const ServeArgs &a, hipStream_t st);
hipError_t launch_serve_emit(const ServeArgs &a, hipStream_t st);
hipError_t launch_put_words(uint8_t *out, const Words &w, hipStream_t st);
hipError_t launch_serve_clear(uint8_t *flags, double *imp, const uint64_t *subs, int64_t n, hipStream_t st);
hipError_t launch_subscribe(uint8_t *flags, uint64_t *subs, const int64_t *slots, int32_t n, uint64_t bit,
                            hipStream_t st);
hipError_t launch_push_walk(const uint8_t *body, uint64_t size, PushEntry *ent, uint32_t *nent, uint32_t max_ent,
                            uint32_t *status, hipStream_t st);
hipError_t launch_push_apply(const uint8_t *body, const PushEntry *ent, const uint32_t *nent, uint32_t max_ent,
                             const ClientTable *ct, int nt, int insert, uint32_t *status, hipStream_t st);
hipError_t launch_serve_list_sizes(const ServeArgs &a, hipStream_t st);
hipError_t launch_serve_emit_list(const ServeArgs &a, hipStream_t st);
hipError_t launch_pack_count(int dtype, PackTab t, hipStream_t st);
hipError_t launch_pack_emit(int dtype, PackTab t, uint8_t *out, uint64_t *recoff, hipStream_t st);
hipError_t launch_pack_header(uint8_t *out, const PackHdr &h, hipStream_t st);
hipError_t launch_sort_desc(void *temp, size_t *temp_bytes, const double *keys_in, double *keys_out,
                            const int32_t *vals_in, int32_t *vals_out, int64_t n, hipStream_t st);
hipError_t launch_gather_entries(int dtype, const int32_t *nent, const uint8_t *entries, int64_t max_entries,
                                 const int64_t *slots, int32_t n, int32_t *out_n, uint8_t *out,
                                 hipStream_t st);
}  // namespace psx

namespace {

constexpr int kRing = psx::kCallRing;   // per-call status slots
// Bucket record lists of split tables (OrdArgs::bucket_m): kBucketM places per slot per call
// — a well-formed call has at most one record of a row per message and at most 16 messages
// (PSX_MAX_FUSED_STREAMS); a call with more records for one row (a row repeated inside a
// message) sets kStDuplicateRow and is replayed with prefix lists.
constexpr int kBucketM = psx::kMaxFused;
constexpr int64_t kBucketMaxRows = 2 << 20;

int vsize_of(int32_t dt) { return (dt == PSX_F32 || dt == PSX_I32) ? 4 : 8; }

struct TableState {
  psx_table_config cfg{};
  int vsize = 4;
  int es = 8;                      // sizeof(Entry<V>) for sorted/map rows
  int64_t max_entries = 0;
  void *d_data = nullptr;          // dense rows
  int32_t *d_nent = nullptr;       // sorted/map: entries per slot
  uint8_t *d_entries = nullptr;    // sorted/map: [max_rows][max_entries] Entry<V>
  uint8_t *d_flags = nullptr;
  int32_t *d_inv[2] = {nullptr, nullptr};   // fast dense path inverse index, one per call slot
  int32_t *d_cnt = nullptr;        // ordered path: per-slot counts (zero between calls), [2][R] by call slot
  int32_t *d_off = nullptr;        // ordered path: exclusive prefix (max_rows + 1)
  int32_t *d_tsum = nullptr;       // ordered path: scan tile sums, [2][tsum_slot] by call slot
  int64_t tsum_slot = 0;
  int32_t *d_touched = nullptr;    // ordered path: touched slots (max_rows)
  uint32_t *d_keyflag = nullptr;   // sorted/map: a key outside [0, max_entries) was seen
  int32_t *d_grow = nullptr;       // split sorted/map tables: per-slot entry growth of a call
  int32_t *d_split = nullptr;      // split sorted/map tables: [3][max_rows] row descriptor lists
  uint32_t *d_nsplit = nullptr;    // their lengths
  int32_t *d_plist = nullptr;      // split tables, pipelined calls: [2][max_rows] int4 touched-row
                                   // entries by call slot (ordered_place -> ordered_classify)
  uint64_t *d_bucket[2] = {nullptr, nullptr};   // split tables: bucket record lists by call slot,
                                                // [max_rows][kBucketM] (OrdArgs::bucket_m)
  uint64_t *d_subs = nullptr;      // CallBackSubs::subscriptions_ per slot (bit c = client c), lazily
  int64_t *d_srv_sizes = nullptr;  // serve-back: record bytes per slot
  int64_t *d_srv_offs = nullptr;   // serve-back: exclusive prefix + scan tile sums
  double *d_imp = nullptr;         // accum_importance: ServerRow::importance_ per slot
  uint64_t *d_ver = nullptr;       // version_maintain: VersionServerRow::version_ per slot (1 at creation)
  // AdaRevision server-table logic (psx_table_set_adarevision)
  bool ada = false;
  psx_adarevision_config ada_cfg{};
  float *d_acc = nullptr, *d_z = nullptr, *d_zmax = nullptr;   // AdaRevisionRow [max_rows][row_capacity]
  uint64_t *d_snap_ver = nullptr, *d_snap_cnt = nullptr;       // old_accum_gradients_ slots [max_rows][S]
  float *d_snap_acc = nullptr;                                 // [max_rows][S][row_capacity]
  uint32_t *d_ada_words = nullptr;                             // [0] live snapshots [1] new rows [2] errors
  uint64_t *d_new_keys = nullptr;                              // [2][max_rows]: unsorted, sorted
  int32_t *d_new_slots = nullptr;                              // [2][max_rows]
  void *d_new_tmp = nullptr;
  size_t new_tmp_bytes = 0;
  float *d_init = nullptr;                                     // initial deltas of new rows
  size_t init_cap = 0;
  std::shared_ptr<std::mt19937> ada_gen;                       // gen_ (adarevision_server_table_logic.cpp:32)
  std::shared_ptr<std::normal_distribution<float>> ada_dist;   // dist_ (:33)
  // partial push scratch (allocated on first psx_serialize_partial)
  double *d_pkeys[2] = {nullptr, nullptr};
  int32_t *d_pvals[2] = {nullptr, nullptr};
  int64_t *d_lsizes = nullptr;
  int64_t *d_loffs = nullptr;
  void *d_sort_tmp = nullptr;
  size_t sort_tmp_bytes = 0;
  bool fast() const { return cfg.row_kind == PSX_ROW_DENSE && cfg.oplog_dense_serialized; }
  // sorted/map rows that need the 1,024-entry register image: applied by two concurrent
  // launches (rows that stay within 256 entries, the rest)
  bool split() const { return cfg.row_kind != PSX_ROW_DENSE && max_entries > 256 && max_entries <= 1024; }
  bool rec_f16() const { return cfg.row_oplog_type == 3; }
  // Bytes of a dense record after its row id: V[cap] (dense_row_oplog.hpp:138-144), plus
  // {uint64 version; bool end_of_version} for version tables (version_dense_row_oplog.hpp:173-180),
  // or uint16[cap] for kDenseRowOpLogFloat16 (dense_row_oplog_float16.hpp:144-157).
  int64_t dense_body() const {
    if (rec_f16()) return cfg.dense_row_oplog_capacity * 2;
    return cfg.dense_row_oplog_capacity * vsize + (cfg.version_maintain ? 9 : 0);
  }
  int64_t dense_stride() const { return 4 + dense_body(); }
};

void free_table(TableState &t) {
  void *ptrs[] = {t.d_data, t.d_nent, t.d_entries, t.d_flags, t.d_inv[0], t.d_inv[1],
                  t.d_cnt, t.d_off, t.d_tsum, t.d_touched, t.d_keyflag, t.d_grow, t.d_split, t.d_nsplit, t.d_plist, t.d_bucket[0], t.d_bucket[1], t.d_subs, t.d_srv_sizes, t.d_srv_offs,
                  t.d_imp, t.d_ver, t.d_acc, t.d_z, t.d_zmax, t.d_snap_ver, t.d_snap_cnt, t.d_snap_acc,
                  t.d_ada_words, t.d_new_keys, t.d_new_slots, t.d_new_tmp, t.d_init, t.d_pkeys[0], t.d_pkeys[1], t.d_pvals[0], t.d_pvals[1],
                  t.d_lsizes, t.d_loffs, t.d_sort_tmp};
  for (void *p : ptrs)
    if (p) hipFree(p);
}

struct PendingCall {
  std::vector<psx_stream> streams;
  int ring;
  hipEvent_t ev_a = nullptr, ev_b = nullptr;   // the call's first stage / its finish (psx_ctx_stats)
};

struct EventPair {
  std::string name;
  hipEvent_t a, b;
};

}  // namespace

struct psx_ctx {
  int device = 0;
  int32_t server_id = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  std::map<int32_t, int64_t> versions;   // bg_version_map_
  std::map<int32_t, int32_t> clocks;     // bg_clock_ (VectorClock::vec_clock_)
  int32_t min_clock = -1;                // VectorClock::min_clock_
  int32_t num_clients = 1;               // GlobalContext::get_num_clients (per-client push)
  int32_t compat = 0;                    // psx_ctx_set_compat flags
  std::vector<TableState> tables;
  bool has_ada = false;                  // some table runs the AdaRevision logic
  // Per-call state lives in two slots (call k uses slot k & 1) so that the decode/index
  // stage of call k+1 can run on the side stream while call k applies on the main stream.
  psx::Seg *d_segs[2] = {nullptr, nullptr};
  uint32_t *d_counters[2] = {nullptr, nullptr};
  uint32_t *d_ntouched[2] = {nullptr, nullptr};   // ordered path: touched-row count per table
  uint64_t *d_recoff[2] = {nullptr, nullptr};
  int2 *d_wfill[2] = {nullptr, nullptr};          // walk-ranked calls: per record {slot, list place}
  size_t recoff_cap[2] = {0, 0};                  // entries
  void *d_walk[2] = {nullptr, nullptr};           // window-parallel decode workspace (psx_walk.hip)
  int walk_last_slot = 0;                         // the last walked call (psx_debug_walk_trace)
  uint64_t walk_last_items = 0;
  size_t walk_cap[2] = {0, 0};                    // bytes
  uint32_t walk_epoch[2] = {0, 0};                // granule tag of the slot's last call
  psx::WalkCount *d_wcount[2] = {nullptr, nullptr};   // walk-counted split tables per call slot (kMaxTables entries)
  std::vector<psx::WalkCount> h_wcount[2];             // what d_wcount[slot] holds
  bool wcount_dirty[2] = {false, false};   // a walk counted into the slot and the call's ordered
                                           // prep (whose ordered_fill zeroes the counts) was never
                                           // enqueued: the next call on the slot clears them first
  hipStream_t side = nullptr;                     // decode/index/verify stage
  hipStream_t aux = nullptr;                      // launches beside the context stream
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipEvent_t ev_push[2] = {nullptr, nullptr};     // psx_serialize_push: a body emitted (main -> copy stream)
  hipEvent_t ev_ready[2] = {nullptr, nullptr};    // slot's index stage done (side -> main)
  hipEvent_t ev_free[2] = {nullptr, nullptr};     // slot's apply stage done (main -> side)
  int pipeline = 0;     // psx_ctx_set_pipeline: 0 off, PSX_PIPELINE_LISTED (calls whose dense
                       // tables all place records from record-row lists), PSX_PIPELINE_ALL.
                       // Walked calls lose (their index stage reads 1 GB of DRAM lines on
                       // C2), listed calls gain (profiles/r02/s17_bench_*.log)
  uint32_t *d_ndirty = nullptr;          // partial push: dirty-row count
  uint8_t *d_push_body = nullptr;        // psx_apply_push_body: host body staged in HBM
  size_t push_body_cap = 0;
  psx::PushEntry *d_push_ent = nullptr;  // the body's records
  size_t push_ent_cap = 0;
  uint32_t *d_push_words = nullptr;      // [0] records, [1] status
  psx::ClientTable *d_client_tabs = nullptr;
  int64_t *d_pack = nullptr;             // psx_pack_stream: sparse record sizes + offsets
  size_t pack_cap = 0;                   // entries
  uint32_t *d_status = nullptr;          // [0] sticky, [1 + k] call ring, [1 + kRing + k] call log,
                                         // [1 + 2 kRing] the folded finish's block counter (zero)
  uint8_t *d_zero = nullptr;
  uint8_t *d_staging = nullptr;
  size_t staging_cap = 0;
  // psx_apply_stream (PSX_SEAM_ASYNC): two HBM staging slots filled on the copy stream; a
  // slot is reused once the call that read it has applied (ev_seam_free)
  int seam_mode = PSX_SEAM_ASYNC;
  hipStream_t h2d = nullptr;
  uint8_t *d_seam[2] = {nullptr, nullptr};
  size_t seam_cap[2] = {0, 0};
  hipEvent_t ev_seam_copied[2] = {nullptr, nullptr};
  hipEvent_t ev_seam_free[2] = {nullptr, nullptr};
  bool seam_used[2] = {false, false};
  int64_t seam_k = 0;
  void *d_split_fixed = nullptr, *d_split_recoff = nullptr, *d_split_scratch = nullptr;   // psx_split_stream
  size_t split_fixed_cap = 0, split_recoff_cap = 0, split_scratch_cap = 0;
  uint64_t *d_list = nullptr;            // ordered path: record lists ((message << 56) | offset),
                                         // list_cap entries, then as many of sort scratch
  size_t list_cap = 0;
  std::vector<PendingCall> pending;      // calls since the last psx_sync (duplicate-row replay)
  int64_t call_seq = 0;
  int64_t pending_calls = 0;
  psx_status deferred = PSX_OK;
  std::string err;
  int timing = 0;                        // 0 off, 1 every kernel, 2 the apply kernels only
  std::vector<EventPair> pending_ev;
  std::vector<hipEvent_t> ev_pool;
  std::map<std::string, std::pair<double, int64_t>> times;
  psx_apply_stats stats{};               // psx_ctx_stats (STATS_SERVER_ACCUM_APPLY_OPLOG_*)
  hipEvent_t stats_open = nullptr;       // the open sync interval's first-call event (psx_ctx_stats)
  uint64_t stats_open_calls = 0;         // calls accepted since it
};

namespace {

psx_status fail(psx_ctx *c, psx_status s, const std::string &msg) {
  if (c) c->err = msg;
  return s;
}

psx_status hip_fail(psx_ctx *c, hipError_t e, const char *what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  return fail(c, e == hipErrorOutOfMemory ? PSX_ERR_OOM : PSX_ERR_DEVICE, m);
}

#define HIP_TRY(c, expr)                                   \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return hip_fail((c), _e, #expr); \
  } while (0)

hipEvent_t get_event(psx_ctx *c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// The kernels timing mode 2 brackets: the applies, whose launch durations the roofline
// divides by (one event pair per launch instead of one per pipeline kernel).
static bool is_apply_kernel(const char *name) {
  return !strcmp(name, "dense_apply") || !strcmp(name, "ada_apply") || !strcmp(name, "ordered_apply");
}

// Run `launch` (which enqueues on `st`), bracketed by HIP events on `st` when timing is on.
template <typename F>
psx_status timed(psx_ctx *c, const char *name, F launch, hipStream_t st) {
  hipEvent_t a = nullptr, b = nullptr;
  const bool on = c->timing == 1 || (c->timing == 2 && is_apply_kernel(name));
  if (on) {
    a = get_event(c);
    b = get_event(c);
    if (a) hipEventRecord(a, st);
  }
  hipError_t e = launch();
  if (e != hipSuccess) return hip_fail(c, e, name);
  if (on && a && b) {
    hipEventRecord(b, st);
    c->pending_ev.push_back({name, a, b});
  }
  return PSX_OK;
}
template <typename F>
psx_status timed(psx_ctx *c, const char *name, F launch) {
  return timed(c, name, launch, c->stream);
}

void collect_timing(psx_ctx *c) {
  for (auto &p : c->pending_ev) {
    float ms = 0.f;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      auto &acc = c->times[p.name];
      acc.first += ms;
      acc.second += 1;
    }
    c->ev_pool.push_back(p.a);
    c->ev_pool.push_back(p.b);
  }
  c->pending_ev.clear();
}

TableState *find_table(psx_ctx *c, int32_t table_id, int *index = nullptr) {
  for (size_t i = 0; i < c->tables.size(); ++i)
    if (c->tables[i].cfg.table_id == table_id) {
      if (index) *index = (int)i;
      return &c->tables[i];
    }
  return nullptr;
}

// Slot of row r in table t, or -1 (context.hpp:291-304 geometry, see psx.h).
int64_t slot_of(const TableState &t, int64_t r) {
  int64_t d = r - t.cfg.row_offset;
  if (d < 0 || d % t.cfg.row_stride) return -1;
  d /= t.cfg.row_stride;
  return d < t.cfg.max_rows ? d : -1;
}

uint32_t rd32h(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
uint64_t rd64h(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}

// Float16Compressor::compress on the host (psx_serialize_rows; psx_device.hpp f32_to_half_fc
// is the device twin; tests check both against the CPU restatement).
uint16_t f32_to_half_fc(float value) {
  const int32_t infN = 0x7F800000, maxN = 0x477FE000, minN = 0x38800000;
  const int32_t infC = infN >> 13, nanN = (infC + 1) << 13, maxC = maxN >> 13, minC = minN >> 13;
  const int32_t subC = 0x003FF, maxD = infC - maxC - 1, minD = minC - subC - 1;
  uint32_t u;
  memcpy(&u, &value, 4);
  uint32_t sign = u & 0x80000000u;
  int32_t v = (int32_t)(u ^ sign);
  sign >>= 16;
  float mag, mul;
  memcpy(&mag, &v, 4);
  const int32_t mulN = 0x52000000;
  memcpy(&mul, &mulN, 4);
  const int32_t sub = minN > v ? (int32_t)(mul * mag) : 0;
  v ^= (sub ^ v) & -(int32_t)(minN > v);
  v ^= (infN ^ v) & -(int32_t)((infN > v) & (v > maxN));
  v ^= (nanN ^ v) & -(int32_t)((nanN > v) & (v > infN));
  v = (int32_t)((uint32_t)v >> 13);
  v ^= ((v - maxD) ^ v) & -(int32_t)(v > maxC);
  v ^= ((v - minD) ^ v) & -(int32_t)(v > subC);
  return (uint16_t)(((uint32_t)v | sign) & 0xffffu);
}


// Kernel arguments of the AdaRevision kernels for table t (index ti).
psx::AdaArgs ada_args(TableState &t, int ti) {
  psx::AdaArgs a{};
  a.t = ti;
  a.stride = t.dense_stride();
  a.cap = t.cfg.row_capacity;
  a.max_rows = t.cfg.max_rows;
  a.table = (float *)t.d_data;
  a.flags = t.d_flags;
  a.imp = t.d_imp;
  a.ver = t.d_ver;
  a.acc = t.d_acc;
  a.z = t.d_z;
  a.zmax = t.d_zmax;
  a.version_records = t.cfg.version_maintain;
  a.step = t.ada_cfg.init_step_size;
  a.S = t.ada_cfg.max_snapshots_per_row;
  a.snap_ver = t.d_snap_ver;
  a.snap_cnt = t.d_snap_cnt;
  a.snap_acc = t.d_snap_acc;
  a.words = t.d_ada_words;
  a.new_keys = t.d_new_keys;
  a.new_slots = t.d_new_slots;
  return a;
}

psx_status enqueue_ada(psx_ctx *c, TableState &t, const psx::AdaArgs &a);

bool has_sparse_serialized(const psx_ctx *c) {
  for (auto &t : c->tables)
    if (!t.cfg.oplog_dense_serialized) return true;
  return false;
}

// Window-parallel decode (psx_walk.hip): by default 48 KiB windows on 512-thread blocks
// (77 KB of LDS) over every CU; a call runs it when its messages have at most kWalkMaxItems
// (message, window) items (B x the largest message's windows).  A window's speculative work
// is LDS-bound inside its CU (~12 us at 48 KiB), the chain between windows hops 16 windows
// at a time on the composed exit maps, so spreading the windows over the whole chip is what
// shortens the walk (the 96 KiB x 1,024-thread shape on half the CUs, round
// 3's default, is PSX_VARIANT_WALK_SHAPE 0 with PSX_VARIANT_WALK_CUS 0).
constexpr uint64_t kWalkMaxItems = 1u << 17;

unsigned walk_blocks(psx_ctx *c, bool pipelined) {
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device) != hipSuccess || cus <= 0)
    cus = 256;
  // a pipelined walk shares the chip with the previous call's apply: on half the CUs it
  // leaves the apply more of them (C3 pipelined 15,430 -> 15,660 M updates/s; unpipelined,
  // alone on the chip, it needs them all: 13,800 -> 11,600, profiles/r06/s4)
  const int v = pipelined ? psx::g_walk_cus_pipelined : psx::g_walk_all_cus;
  if (pipelined && std::abs(psx::g_side_cu_mask) >= 2)   // max(v, 1) blocks per CU of the prep stream's mask
    return (unsigned)std::max(1, cus / std::abs(psx::g_side_cu_mask) * std::max(v, 1));
  return (unsigned)std::max(1, v <= 0 ? cus / 2 : v == 1 ? cus : cus * std::min(v, 8));
}

// Smallest record of any table in the context: bounds the records a message can hold
// (ordered-path record lists are sized by it).  Sparse records are >= 8 bytes
// ({int32 row_id; int32 n}); dense ones 4 + dense_body.
size_t min_record_bytes(const psx_ctx *c) {
  int64_t m = 8;
  for (auto &t : c->tables)
    if (t.cfg.oplog_dense_serialized && 4 + t.dense_body() < m) m = 4 + t.dense_body();
  return (size_t)m;
}

// Bucket record lists for split table t on this call: selected, allocated, not a replay
// (a replay takes prefix lists: it may be the replay of a bucket overflow), and no
// AdaRevision table in the context (an overflow is replayed, and that logic has no replay).
bool bucket_ok(const psx_ctx *c, const TableState &t, bool force_ordered) {
  return psx::g_ord_bucket && t.d_bucket[0] && !force_ordered && !c->has_ada;
}

// Enqueue the device pipeline for n messages already resident in HBM (versions checked).
// force_ordered: every table goes through the ordered path (duplicate-row replay).
//
// Error contract: every check runs before any table is touched — decode (framing,
// unknown tables), the dense index (row range), the ordered prep (row range, columns,
// the sorted/map capacity dry run), the AdaRevision state check, and the duplicate-row
// gate — so a call that fails applies nothing.
psx_status enqueue_apply(psx_ctx *c, const psx_stream *s, int32_t n, bool force_ordered,
                         const uint64_t *const *record_offsets = nullptr,
                         const int32_t *const *record_rows = nullptr) {
  const int slot = (int)(c->call_seq & 1);
  psx::StreamSet ss{};
  ss.n = n;
  size_t rec_need = 0, list_need = 0;
  const bool sparse = has_sparse_serialized(c);
  bool any_ordered = sparse || force_ordered;
  const size_t min_rec = min_record_bytes(c);
  for (int i = 0; i < n; ++i) {
    ss.data[i] = (const uint8_t *)s[i].data;
    ss.size[i] = s[i].size;
    ss.recoff_base[i] = rec_need;
    if (sparse) rec_need += s[i].size / 8 + 1;
    list_need += s[i].size / min_rec + 1;
  }
  // every ordered table keeps its record lists from its stage 1 to its apply: one
  // list_need-sized region each
  size_t n_ord = 0;
  for (auto &t : c->tables)
    if (!t.fast() || force_ordered) ++n_ord;
  const size_t list_region = list_need;
  list_need *= n_ord ? n_ord : 1;
  if (rec_need > c->recoff_cap[slot] || (any_ordered && list_need > c->list_cap)) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->side));
    if (rec_need > c->recoff_cap[slot]) {
      if (c->d_recoff[slot]) hipFree(c->d_recoff[slot]);
      if (c->d_wfill[slot]) hipFree(c->d_wfill[slot]);
      c->d_recoff[slot] = nullptr;
      c->d_wfill[slot] = nullptr;
      c->recoff_cap[slot] = 0;
      HIP_TRY(c, hipMalloc(&c->d_recoff[slot], rec_need * sizeof(uint64_t)));
      HIP_TRY(c, hipMalloc(&c->d_wfill[slot], rec_need * sizeof(int2)));
      c->recoff_cap[slot] = rec_need;
    }
    if (any_ordered && list_need > c->list_cap) {
      if (c->d_list) hipFree(c->d_list);
      c->d_list = nullptr;
      c->list_cap = 0;
      // the lists of call slot 0, of call slot 1 (a pipelined call fills its lists on the
      // prep stream while the previous call's apply reads its own), then the long-list
      // sort's scratch (psx_ordered.hip wave_sort_long, rows with > 64 records in one call;
      // the apply's only, on the context stream)
      HIP_TRY(c, hipMalloc(&c->d_list, 3 * list_need * sizeof(uint64_t)));
      c->list_cap = list_need;
    }
  }
  psx::IdxSet ix{};
  uint32_t rows_given = 0;
  for (int i = 0; i < n; ++i) {
    if (record_offsets) ix.p[i] = record_offsets[i];
    if (record_rows && record_rows[i] && !force_ordered) {
      ix.rows[i] = record_rows[i];
      rows_given |= 1u << i;
    }
  }
  // Producer record rows replace the stream's row ids for fast tables whose apply kernel
  // checks them (rows_mask[ti]); the others index from the stream.
  std::vector<uint32_t> rows_mask(c->tables.size(), 0);
  const uint32_t all_msgs = n >= 32 ? ~0u : ((1u << n) - 1);
  bool light = rows_given == all_msgs;   // no fast table reads row ids from the stream
  for (size_t ti = 0; ti < c->tables.size(); ++ti) {
    TableState &t = c->tables[ti];
    if (!t.fast() || force_ordered) continue;
    if (rows_given && !t.ada) {
      psx::DenseArgs probe{};
      probe.ss = ss;
      probe.B = n;
      probe.stride = t.dense_stride();
      probe.max_rows = t.cfg.max_rows;
      probe.imp = t.d_imp;
      if (psx::dense_apply_checks_rows(probe, t.rec_f16())) rows_mask[ti] = rows_given;
    }
    if (rows_mask[ti] != all_msgs) light = false;
  }
  // Stage 1 (decode, index, verify) runs on the side stream once the slot's previous
  // user (call k-2) has finished applying, overlapping call k-1's apply; stage 2 runs on
  // the main stream after it.
  const bool pipelined = c->pipeline == PSX_PIPELINE_ALL || (c->pipeline == PSX_PIPELINE_LISTED && light);
  hipStream_t prep = pipelined ? c->side : c->stream;
  // psx_ctx_stats: the call's device time, from its first stage to its finish (replays of a
  // counted call are not counted again); the event goes back to the pool on an early return
  struct EventGuard {
    psx_ctx *c;
    hipEvent_t e;
    ~EventGuard() {
      if (e) c->ev_pool.push_back(e);
    }
  } call_ev{c, force_ordered || !(psx::g_call_events & 1) ? nullptr : get_event(c)};
  psx::TableDir dir{};
  dir.n = (int32_t)c->tables.size();
  for (size_t i = 0; i < c->tables.size(); ++i) {
    dir.table_id[i] = c->tables[i].cfg.table_id;
    dir.vsize[i] = c->tables[i].vsize;
    dir.dense_serialized[i] = c->tables[i].cfg.oplog_dense_serialized;
    dir.dense_body[i] = c->tables[i].dense_body();
  }
  const int ring = (int)(c->call_seq % kRing);
  uint32_t *sticky = c->d_status;
  uint32_t *call_st = c->d_status + 1 + ring;
  uint32_t *call_log = c->d_status + 1 + kRing + ring;
  psx::Seg *segs = c->d_segs[slot];
  uint32_t *counters = c->d_counters[slot];
  if (pipelined) HIP_TRY(c, hipStreamWaitEvent(prep, c->ev_free[slot], 0));
  if (call_ev.e) HIP_TRY(c, hipEventRecord(call_ev.e, prep));
  if (!force_ordered && !(psx::g_call_events & 1) && !c->stats_open) {
    // psx_ctx_stats: the interval's device time starts at its first call's first stage
    c->stats_open = get_event(c);
    if (c->stats_open) HIP_TRY(c, hipEventRecord(c->stats_open, prep));
    c->stats_open_calls = 0;
  }
  if (c->wcount_dirty[slot]) {
    // the slot's last call failed between its counting walk and its ordered prep
    for (auto &t : c->tables) {
      if (!t.d_cnt || !t.split()) continue;
      const size_t R = (size_t)t.cfg.max_rows;
      HIP_TRY(c, hipMemsetAsync(t.d_cnt + slot * R, 0, R * sizeof(int32_t), prep));
      if (t.d_grow) HIP_TRY(c, hipMemsetAsync(t.d_grow + slot * R, 0, R * sizeof(int32_t), prep));
      if (t.d_nsplit) HIP_TRY(c, hipMemsetAsync(t.d_nsplit + 5 * psx::kNsStride * slot, 0, 5 * psx::kNsStride * sizeof(uint32_t), prep));
      if (t.d_tsum) HIP_TRY(c, hipMemsetAsync(t.d_tsum + slot * (size_t)t.tsum_slot, 0,
                                              (size_t)t.tsum_slot * sizeof(int32_t), prep));
    }
    c->wcount_dirty[slot] = false;
  }
  // Walked messages with sparse tables: the window-parallel decode (psx_walk.hip) when every
  // sparse table of the context has one record pair size and the window items are bounded;
  // otherwise (and for producer record offsets) one workgroup per message.
  uint32_t spec_wpr = 0;
  bool walk = psx::g_decode_walk && sparse;
  for (int i = 0; i < n; ++i)
    if (ix.p[i]) walk = false;
  for (auto &t : c->tables) {
    if (t.cfg.oplog_dense_serialized) continue;
    const uint32_t w = 1 + (uint32_t)t.vsize / 4;
    if (spec_wpr && spec_wpr != w) walk = false;
    spec_wpr = w;
  }
  if (spec_wpr > 3) walk = false;   // psx_walk.hip next_of's 32-bit link: values of at most 8 bytes
  uint64_t maxw = 0;
  const int walk_shape = psx::g_walk_shape;
  const uint64_t wbytes = psx::walk_window_bytes(walk_shape);
  for (int i = 0; i < n; ++i) maxw = std::max<uint64_t>(maxw, (s[i].size + wbytes - 1) / wbytes);
  const uint64_t items = (uint64_t)n * maxw;
  if (items == 0 || items > kWalkMaxItems) walk = false;
  // composed exit maps cost kCand x 8 B per (item, level) of workspace: up to 4,096 items
  const int walk_levels = items <= 4096 ? std::max(0, std::min(psx::g_walk_levels, 8)) : 0;
  if (walk) {
    const size_t need = psx::walk_ws_bytes(items, walk_levels);
    if (need > c->walk_cap[slot]) {
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->side));
      if (c->d_walk[slot]) hipFree(c->d_walk[slot]);
      c->d_walk[slot] = nullptr;
      c->walk_cap[slot] = 0;
      HIP_TRY(c, hipMalloc(&c->d_walk[slot], need));
      // ordered before the walk on the stream that runs it (the context's streams are
      // non-blocking: the null stream does not order against them)
      HIP_TRY(c, hipMemsetAsync(c->d_walk[slot], 0, need, prep));
      c->walk_cap[slot] = need;
    }
    c->walk_epoch[slot] = psx::next_walk_epoch();
    ++psx::g_walk_calls;
    c->walk_last_slot = slot;
    c->walk_last_items = items;
  }
  // Split sorted/map tables on a walked call: the walk does ordered_count's work as it
  // writes the record offsets (WalkCount), into this call slot's count state (a pipelined
  // walk runs beside the previous call's ordered work, which uses the other slot's), and
  // the ordered prep skips that launch.
  // An indexed call (every message with the producer's record offsets) counts the same way,
  // in idx_verify (psx_walk.hip), which checks the offsets over a grid.
  bool idx_all = !walk && n > 0;
  for (int i = 0; i < n; ++i) idx_all = idx_all && ix.p[i];
  bool wcount = false;
  if ((walk || idx_all) && psx::g_walk_count) {
    std::vector<psx::WalkCount> w(c->tables.size());
    for (size_t ti = 0; ti < c->tables.size(); ++ti) {
      TableState &t = c->tables[ti];
      psx::WalkCount &x = w[ti];
      std::memset(&x, 0, sizeof x);
      if ((t.fast() && !force_ordered) || !t.split() || !psx::g_ord_split) continue;
      x.row_offset = t.cfg.row_offset;
      x.row_stride = t.cfg.row_stride;
      x.max_rows = t.cfg.max_rows;
      x.cnt = t.d_cnt + (int64_t)slot * t.cfg.max_rows;
      x.grow = t.d_grow + (int64_t)slot * t.cfg.max_rows;
      x.nsplit = t.d_nsplit + 5 * psx::kNsStride * slot;
      x.tsum = t.d_tsum + (int64_t)slot * t.tsum_slot;
      x.wfill = psx::g_walk_rank ? c->d_wfill[slot] : nullptr;
      if (x.wfill && bucket_ok(c, t, force_ordered)) {
        x.bucket = t.d_bucket[slot];
        x.bucket_m = kBucketM;
      }
      x.on = 1;
#ifdef PSX_DEBUG_BUILD
      x.pad2 = (psx::g_ord_probe >> 8) & 3;   // walk timing probes (results unchanged)
#endif
      wcount = true;
    }
    if (wcount) {
      std::vector<psx::WalkCount> &hw = c->h_wcount[slot];
      if (!c->d_wcount[slot]) HIP_TRY(c, hipMalloc(&c->d_wcount[slot], sizeof(psx::WalkCount) * psx::kMaxTables));
      if (w.size() != hw.size() || std::memcmp(w.data(), hw.data(), sizeof(psx::WalkCount) * w.size())) {
        // a slot's contents change only with the tables (rarely): wait for every copy still
        // reading the context's persistent vector before it changes — the source is pageable,
        // so stream order alone does not say when HIP has read it
        HIP_TRY(c, hipStreamSynchronize(prep));
        hw = w;
        HIP_TRY(c, hipMemcpyAsync(c->d_wcount[slot], hw.data(), sizeof(psx::WalkCount) * w.size(),
                                  hipMemcpyHostToDevice, prep));
      }
    }
  }
  if (wcount) c->wcount_dirty[slot] = true;
  psx_status st = timed(
      c, "decode_streams",
      [&] {
        if (walk)
          return psx::launch_walk(ss, dir, segs, c->d_recoff[slot], call_st, counters, c->d_ntouched[slot],
                                  c->d_walk[slot], spec_wpr, (unsigned)std::min<uint64_t>(items, walk_blocks(c, pipelined)),
                                  c->walk_epoch[slot], psx::g_walk_trace ? c->walk_cap[slot] ? items : 0 : 0,
                                  wcount ? c->d_wcount[slot] : nullptr, items,
                                  walk_levels | (psx::g_walk_skew && walk_levels > 0 ? 0x100 : 0), walk_shape, prep);
        return psx::launch_decode(ss, dir, segs, c->d_recoff[slot], call_st, counters, c->d_ntouched[slot], ix,
                                  c->d_ntouched[slot] + psx::kMaxTables, wcount ? c->d_wcount[slot] : nullptr, prep);
      },
      prep);
  if (st) return st;

  // 1) fast dense tables: inverse index (batch-major [b][slot]) + per-message claim counts
  psx::TableMask fast{};
  const psx::InvLayout L0{1, 0};
  for (size_t ti = 0; ti < c->tables.size(); ++ti) {
    TableState &t = c->tables[ti];
    if (!t.fast() || force_ordered) continue;
    fast.t[fast.n++] = (int32_t)ti;
    const int64_t stride = t.dense_stride();
    const psx::InvLayout L{L0.ss, t.cfg.max_rows};
    st = timed(
        c, "dense_index",
        [&] {
          return psx::launch_dense_index(ss, ix, rows_mask[ti], segs, (int)ti, n, stride, t.cfg.row_offset,
                                         t.cfg.row_stride, t.cfg.max_rows, t.d_inv[slot], L, call_st, prep);
        },
        prep);
    if (st) return st;
    st = timed(
        c, "dense_verify",
        [&] { return psx::launch_dense_verify(t.d_inv[slot], L, (int)ti, n, t.cfg.max_rows, counters, prep); },
        prep);
    if (st) return st;
  }
  // 2) ordered tables, stage 1: record lists, validation, capacity dry run.  A split table
  //    of a pipelined call does the half of it that depends only on the call's records
  //    (counts, list ranges, record lists: ordered_place + ordered_fill) on the prep stream,
  //    beside the previous call's apply; the half that depends on the rows' images after
  //    that apply (ordered_classify, the dry run) on the context stream.  Its record lists
  //    live in the call slot's own region for that reason.
  std::vector<psx::OrdArgs> ord(c->tables.size());
  std::vector<char> halves(c->tables.size(), 0);
  size_t ord_k = 0;
  for (size_t ti = 0; ti < c->tables.size(); ++ti) {
    TableState &t = c->tables[ti];
    if (t.fast() && !force_ordered) continue;
    psx::OrdArgs &a = ord[ti];
    a = psx::OrdArgs{};
    a.fin_ring = -1;
    a.ss = ss;
    a.segs = segs;
    a.t = (int)ti;
    a.B = n;
    a.kind = t.cfg.row_kind;
    a.dense_records = t.cfg.oplog_dense_serialized;
    a.stride = t.dense_stride();
    a.ver = t.d_ver;
    a.rec_f16 = t.rec_f16() ? 1 : 0;
    a.cap = t.cfg.dense_row_oplog_capacity;
    a.row_cap = t.cfg.row_capacity;
    a.row_offset = t.cfg.row_offset;
    a.row_stride = t.cfg.row_stride;
    a.max_rows = t.cfg.max_rows;
    a.recoff = c->d_recoff[slot];
    a.cnt = t.d_cnt + (int64_t)slot * t.cfg.max_rows;
    a.off = t.d_off;
    a.tsum = t.d_tsum + (int64_t)slot * t.tsum_slot;
    // slot regions at multiples of the allocated capacity, not of this call's need: the
    // previous call (the other slot) may have sized its lists larger and still be reading them
    a.list = c->d_list + (size_t)slot * c->list_cap + list_region * ord_k;
    a.list_tmp = c->d_list + 2 * c->list_cap + list_region * ord_k;
    ++ord_k;
    a.touched = t.d_touched;
    a.ntouched = c->d_ntouched[slot] + ti;
    a.dense = t.d_data;
    a.nent = t.d_nent;
    a.entries = t.d_entries;
    a.max_entries = t.max_entries;
    a.flags = t.d_flags;
    a.call_status = call_st;
    a.sticky = sticky;
    a.force = force_ordered ? 1 : 0;
    a.imp = t.d_imp;
    a.keyflag = t.d_keyflag;
    if (t.split() && psx::g_ord_split) {
      a.grow = t.d_grow + (int64_t)slot * t.cfg.max_rows;
      a.split = t.d_split;
      a.nsplit = t.d_nsplit + 5 * psx::kNsStride * slot;
      a.spill = psx::g_ord_split == 2 ? 1 : psx::g_ord_split == 3 ? 3 : 0;
      // light rows four to a wave (psx_ordered.hip lite_quad): spill mode, sorted/map rows
      // without importance (the light path does not sum it)
      a.lite = psx::g_ord_lite && a.spill && !t.d_imp ? psx::g_ord_lite : 0;
#ifdef PSX_DEBUG_BUILD
      a.probe = psx::g_ord_probe;
#endif
      a.counted = wcount && c->h_wcount[slot][ti].on ? (c->h_wcount[slot][ti].wfill ? 2 : 1)
                  : (psx::g_walk_rank && !t.cfg.oplog_dense_serialized && c->d_wfill[slot] ? 3 : 0);
      // bucket lists: the walk (counted 2, WalkCount.bucket set above) or ordered_count
      // (counted 3) writes each record's list entry at [slot][place]
      if ((a.counted == 2 && c->h_wcount[slot][ti].bucket) || (a.counted == 3 && bucket_ok(c, t, force_ordered))) {
        a.bucket_m = kBucketM;
        a.list = t.d_bucket[slot];
      }
      if (pipelined && psx::g_prep_halves) {
        int2 *wfill = a.counted >= 2 ? c->d_wfill[slot] : nullptr;
        if (psx::g_pipe_slots && psx::ordered_prep_in_dry_run(a)) {
          // bucket lists: the records' half is the count alone (if the walk did not do it);
          // the rows' half classifies the slots inside the dry run (halves = 2)
          halves[ti] = 2;
          if (a.counted == 3) {
            st = timed(c, "ordered_count", [&] { return psx::launch_ordered_count(a, wfill, prep); }, prep);
            if (st) return st;
          }
        } else {
          halves[ti] = 1;
          int4 *plist = reinterpret_cast<int4 *>(t.d_plist) + (size_t)slot * t.cfg.max_rows;
          st = timed(c, "ordered_place", [&] { return psx::launch_ordered_prep_records(a, wfill, plist, prep); },
                     prep);
          if (st) return st;
        }
      }
    }
  }
  if (pipelined) {
    HIP_TRY(c, hipEventRecord(c->ev_ready[slot], prep));
    HIP_TRY(c, hipStreamWaitEvent(c->stream, c->ev_ready[slot], 0));
  }
  for (size_t ti = 0; ti < c->tables.size(); ++ti) {
    TableState &t = c->tables[ti];
    if (t.fast() && !force_ordered) continue;
    const psx::OrdArgs &a = ord[ti];
    if (halves[ti] == 2) {
      st = timed(c, "ordered_classify", [&] { return psx::launch_ordered_prep_slots(t.cfg.dtype, a, nullptr, false, c->stream); });
      if (st) return st;
      continue;
    }
    if (halves[ti]) {
      const int4 *plist = reinterpret_cast<const int4 *>(t.d_plist) + (size_t)slot * t.cfg.max_rows;
      st = timed(c, "ordered_classify", [&] { return psx::launch_ordered_prep_rows(t.cfg.dtype, a, plist, c->stream); });
      if (st) return st;
      continue;
    }
    int2 *wfill = a.counted >= 2 ? c->d_wfill[slot] : nullptr;
    if (psx::ordered_prep_in_dry_run(a)) {   // bucket lists: the prep is the dry run's prologue
      st = timed(c, "ordered_prep", [&] { return psx::launch_ordered_prep_slots(t.cfg.dtype, a, wfill, true, c->stream); });
      if (st) return st;
      continue;
    }
    st = timed(c, "ordered_prep", [&] { return psx::launch_ordered_prep(t.cfg.dtype, a, wfill, c->stream); });
    if (st) return st;
  }
  c->wcount_dirty[slot] = false;   // every walk-counted table's ordered_fill is enqueued
  // 3) AdaRevision tables with version records: every record's snapshot must exist
  std::vector<psx::AdaArgs> ada(c->tables.size());
  for (int i = 0; i < fast.n; ++i) {
    const int ti = fast.t[i];
    TableState &t = c->tables[ti];
    if (!t.ada) continue;
    psx::AdaArgs &aa = ada[ti];
    aa = ada_args(t, ti);
    aa.ss = ss;
    aa.segs = segs;
    aa.B = n;
    aa.inv = t.d_inv[slot];
    aa.inv_ss = L0.ss;
    aa.inv_sb = t.cfg.max_rows;
    aa.counters = counters;
    aa.sticky = sticky;
    aa.call_status = call_st;
    if (t.cfg.version_maintain) {
      st = timed(c, "ada_check", [&] { return psx::launch_ada_check(aa, c->stream); });
      if (st) return st;
    }
  }
  // 4) a duplicate row in any fast table turns the whole call into a replay (or, with an
  //    AdaRevision table in the context, into an error: that logic has no ordered replay).
  //    A single fast table with nothing else in the call checks its own counts.
  if (fast.n > 1 || (fast.n && (any_ordered || c->has_ada))) {
    st = timed(c, "dup_gate", [&] {
      return psx::launch_gate(segs, counters, fast, n, call_st, c->stream);
    });
    if (st) return st;
  }
  // 5) applies: ordered tables, then fast dense tables.  When the call's last launch is an
  //    ordered apply on the context stream, it also does finish_call's work (its last block,
  //    psx_ordered.hip finish_tail) and no finish launch follows.
  int last_ord = -1;
  for (size_t ti = 0; ti < c->tables.size(); ++ti)
    if (!c->tables[ti].fast() || force_ordered) last_ord = (int)ti;
  const bool fold_finish = psx::g_fold_finish && fast.n == 0 && last_ord >= 0 &&
                           !(ord[last_ord].grow && !ord[last_ord].spill);   // concurrent launches: join first
  for (size_t ti = 0; ti < c->tables.size(); ++ti) {
    TableState &t = c->tables[ti];
    if (t.fast() && !force_ordered) continue;
    const psx::Fork fk{c->aux, c->ev_fork, c->ev_join};
    psx::OrdArgs oa = ord[ti];
    oa.fin_ring = fold_finish && (int)ti == last_ord ? ring : -1;
    st = timed(c, "ordered_apply", [&] { return psx::launch_ordered_apply(t.cfg.dtype, oa, c->stream, fk); });
    if (st) return st;
  }
  for (int i = 0; i < fast.n; ++i) {
    const int ti = fast.t[i];
    TableState &t = c->tables[ti];
    if (t.ada) {
      st = enqueue_ada(c, t, ada[ti]);
      if (st) return st;
      continue;
    }
    psx::DenseArgs a{};
    a.ss = ss;
    a.segs = segs;
    a.t = ti;
    a.B = n;
    a.stride = t.dense_stride();
    a.cap = t.cfg.dense_row_oplog_capacity;
    a.row_cap = t.cfg.row_capacity;
    a.max_rows = t.cfg.max_rows;
    a.table = t.d_data;
    a.ver = t.d_ver;
    a.flags = t.d_flags;
    a.inv = t.d_inv[slot];
    a.inv_ss = L0.ss;
    a.inv_sb = t.cfg.max_rows;
    a.counters = counters;
    a.sticky = sticky;
    a.call_status = call_st;
    a.zero_chunk = c->d_zero;
    a.imp = t.d_imp;
    a.rows_mask = rows_mask[ti];
    a.row_offset = t.cfg.row_offset;
    a.row_stride = t.cfg.row_stride;
    a.store_nt = psx::g_dense_store_nt;
    st = timed(c, "dense_apply", [&] { return psx::launch_dense_apply(t.cfg.dtype, a, c->stream, t.rec_f16()); });
    if (st) return st;
  }
  if (!fold_finish) {
    st = timed(c, "finish_call", [&] { return psx::launch_finish(sticky, call_st, call_log, c->stream); });
    if (st) return st;
  }
  // a pipelined context's call marks its slot free (a later call's stage 1 waits on it;
  // psx_ctx_set_pipeline drains the streams when the mode changes, so a stale event is never
  // waited for with the slot still in use)
  if (c->pipeline || (psx::g_call_events & 2)) HIP_TRY(c, hipEventRecord(c->ev_free[slot], c->stream));
  PendingCall pc;
  pc.streams.assign(s, s + n);
  pc.ring = ring;
  if (call_ev.e) {
    hipEvent_t b = get_event(c);
    if (b && hipEventRecord(b, c->stream) == hipSuccess) {
      pc.ev_a = call_ev.e;
      pc.ev_b = b;
      call_ev.e = nullptr;
    } else if (b) {
      c->ev_pool.push_back(b);
    }
  }
  if (!force_ordered) {
    if (c->stats_open) c->stats_open_calls++;
    c->stats.calls++;
    c->stats.messages += (uint64_t)n;
    for (int i = 0; i < n; ++i) c->stats.oplog_bytes += s[i].size;
  }
  c->pending.push_back(pc);
  c->call_seq++;
  c->pending_calls++;
  return PSX_OK;
}

// AdaRevision stage of one call for table t: rows the call creates get their
// ServerRowCreated initial deltas (drawn on the host from the table's generator, in
// creation order), then every record goes through the logic.  Synchronous when the
// table draws Gaussian initial rows.
psx_status enqueue_ada(psx_ctx *c, TableState &t, const psx::AdaArgs &a) {
  if (t.ada_cfg.gaussian_init) {
    HIP_TRY(c, hipMemsetAsync(t.d_ada_words + 1, 0, sizeof(uint32_t), c->stream));
    psx_status st = timed(c, "ada_new_rows", [&] { return psx::launch_ada_new_rows(a, c->stream); });
    if (st) return st;
    uint32_t nn = 0;
    HIP_TRY(c, hipMemcpyAsync(&nn, t.d_ada_words + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (nn) {
      // CreateRow order = first touch (message, position); each new row takes row_capacity
      // draws of the one generator (ServerRowCreated, adarevision_server_table_logic.cpp:43-46)
      const int64_t R = t.cfg.max_rows;
      size_t tb = t.new_tmp_bytes;
      HIP_TRY(c, psx::launch_ada_sort(t.d_new_tmp, &tb, t.d_new_keys, t.d_new_keys + R, t.d_new_slots,
                                      t.d_new_slots + R, (int)nn, c->stream));
      const size_t need = (size_t)nn * (size_t)t.cfg.row_capacity;
      std::vector<float> d(need);
      for (float &x : d) x = (*t.ada_dist)(*t.ada_gen);
      if (need > t.init_cap) {
        if (t.d_init) hipFree(t.d_init);
        t.d_init = nullptr;
        t.init_cap = 0;
        HIP_TRY(c, hipMalloc(&t.d_init, need * sizeof(float)));
        t.init_cap = need;
      }
      HIP_TRY(c, hipMemcpyAsync(t.d_init, d.data(), need * sizeof(float), hipMemcpyHostToDevice, c->stream));
      st = timed(c, "ada_init_rows", [&] {
        return psx::launch_ada_init_rows(a, t.d_new_slots + R, t.d_init, (int32_t)nn, c->stream);
      });
      if (st) return st;
      HIP_TRY(c, hipStreamSynchronize(c->stream));   // `d` is pageable host memory
    }
  }
  return timed(c, "ada_apply", [&] { return psx::launch_ada_apply(a, c->stream); });
}

// ServerRowSent for the rows a push emits (sizes != 0) or for a list of slots; num_clients
// is `clients`, or each row's subscriber count when subs is given.  check_only: verify
// that every such row can take its snapshot (a free slot or a live one for its version),
// writing nothing — pushes run it before they clear any dirty bit.
psx_status ada_rows_sent(psx_ctx *c, TableState &t, int ti, const int32_t *list, const int64_t *sizes, int64_t n,
                         uint64_t clients, const uint64_t *subs, bool check_only) {
  psx::AdaArgs a = ada_args(t, ti);
  HIP_TRY(c, hipMemsetAsync(t.d_ada_words + 2, 0, sizeof(uint32_t), c->stream));
  HIP_TRY(c, psx::launch_ada_sent(a, list, sizes, n, clients, subs, check_only ? 1 : 0, c->stream));
  uint32_t err = 0;
  HIP_TRY(c, hipMemcpyAsync(&err, t.d_ada_words + 2, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (err)
    return fail(c, PSX_ERR_CAPACITY,
                "AdaRevision: a sent row already holds max_snapshots_per_row live snapshots (nothing was sent)");
  return PSX_OK;
}

psx_status sticky_error(psx_ctx *c, uint32_t sticky) {
  if (sticky & psx::kStUnknownTable) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table id in a device stream");
  if (sticky & psx::kStMalformed) return fail(c, PSX_ERR_MALFORMED, "malformed device stream");
  if (sticky & psx::kStRowsMismatch)
    return fail(c, PSX_ERR_MALFORMED,
                "producer record rows disagree with the stream's row ids: the rows whose records disagree were "
                "left unchanged, every other row of the call was applied");
  if (sticky & psx::kStRowRange) return fail(c, PSX_ERR_ROW_RANGE, "row id outside this shard's range");
  if (sticky & psx::kStState)
    return fail(c, PSX_ERR_STATE, "AdaRevision: a record names a (row, version) without a snapshot");
  if (sticky & psx::kStCapacity) return fail(c, PSX_ERR_CAPACITY, "row capacity exceeded (column >= row_capacity or sorted/map row over max_entries)");
  if (sticky & psx::kStWalkBound)
    return fail(c, PSX_ERR_DEVICE, "window-parallel decode: a walker state outside its message, or an exit state "
                                   "published early that the window's resolve disagrees with (internal error; "
                                   "nothing applied)");
  if (sticky & psx::kStWalkLost) {
    char m[256];
    uint32_t d[2][8] = {};
    for (int k = 0; k < 2; ++k)
      if (c->d_walk[k]) (void)hipMemcpy(d[k], c->d_walk[k], sizeof(d[k]), hipMemcpyDeviceToHost);
    const int k = d[0][1] ? 0 : 1;
    snprintf(m, sizeof m,
             "window-parallel decode: a window's predecessor state never arrived (nothing applied; ticket %u "
             "message %u window %u epoch %u tag seen %u lanes tagged 0x%x)",
             d[k][2], d[k][3], d[k][4], d[k][5], d[k][6], d[k][7]);
    return fail(c, PSX_ERR_DEVICE, m);
  }
  if (sticky & psx::kStUnsupported)
    return fail(c, PSX_ERR_UNSUPPORTED, "table repeated within one message (or a sparse table at an unaligned offset)");
  return PSX_OK;
}

psx_status sync_impl(psx_ctx *c) {
  HIP_TRY(c, hipSetDevice(c->device));
  struct CloseGuard {   // the interval's closing event goes back to the pool on every path
    psx_ctx *c;
    hipEvent_t e;
    ~CloseGuard() {
      if (e) c->ev_pool.push_back(e);
    }
  } stats_close{c, nullptr};
  if (c->stats_open) {
    stats_close.e = get_event(c);
    if (stats_close.e && hipEventRecord(stats_close.e, c->stream) != hipSuccess) {
      c->ev_pool.push_back(stats_close.e);
      stats_close.e = nullptr;
    }
  }
  HIP_TRY(c, hipStreamSynchronize(c->side));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  collect_timing(c);
  if (c->stats_open) {
    // the interval's device time: its first call's first stage to the last call's finish
    float ms = 0.f;
    if (stats_close.e && hipEventElapsedTime(&ms, c->stats_open, stats_close.e) == hipSuccess) {
      c->stats.apply_sec += ms * 1e-3;
      c->stats.settled_calls += c->stats_open_calls;
    }
    c->ev_pool.push_back(c->stats_open);
    c->stats_open = nullptr;
    c->stats_open_calls = 0;
  }
  uint32_t sticky = 0;
  HIP_TRY(c, hipMemcpy(&sticky, c->d_status, sizeof(uint32_t), hipMemcpyDeviceToHost));
  std::vector<PendingCall> pending;
  pending.swap(c->pending);
  c->pending_calls = 0;
  for (PendingCall &p : pending) {
    if (!p.ev_a) continue;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, p.ev_a, p.ev_b) == hipSuccess) {
      c->stats.apply_sec += ms * 1e-3;
      c->stats.settled_calls++;
    }
    c->ev_pool.push_back(p.ev_a);
    c->ev_pool.push_back(p.ev_b);
    p.ev_a = p.ev_b = nullptr;
  }
  if (sticky) {
    uint32_t zero = 0;
    HIP_TRY(c, hipMemcpy(c->d_status, &zero, sizeof(uint32_t), hipMemcpyHostToDevice));
  }
  // A call the device rejected applied nothing (kStFatal: framing, table, row range,
  // capacity, ...).  Its senders' versions are given back where no later call from the same
  // sender has been accepted since, so the corrected message can be sent again with the same
  // version (the reference has no such case: it aborts, server.cpp:124 / reader :112).
  // Otherwise the version stays consumed; the error names the call either way.
  std::string rejected;
  if (sticky & psx::kStFatal) {
    std::vector<uint32_t> log(kRing);
    HIP_TRY(c, hipMemcpy(log.data(), c->d_status + 1 + kRing, sizeof(uint32_t) * kRing, hipMemcpyDeviceToHost));
    // newest call first, so that consecutive rejected calls of one sender all come back
    for (auto pi = pending.rbegin(); pi != pending.rend(); ++pi) {
      const PendingCall &p = *pi;
      if (!(log[p.ring] & psx::kStFatal)) continue;
      // last message first: a call may carry several messages of one sender (consecutive
      // versions), which come back newest to oldest
      for (auto mi = p.streams.rbegin(); mi != p.streams.rend(); ++mi) {
        const psx_stream &m = *mi;
        auto it = c->versions.find(m.bg_id);
        const bool back = it != c->versions.end() && it->second == (int64_t)m.version;
        if (back) it->second = (int64_t)m.version - 1;
        if (rejected.size() < 512)
          rejected += " [bg_id " + std::to_string(m.bg_id) + " version " + std::to_string(m.version) +
                      (back ? ": version given back]" : ": version stays consumed, a later call from the sender "
                                                        "was accepted]");
      }
    }
  }
  // An error stored by an earlier automatic sync is reported after this sync has done
  // its own work (the replay below), so no accepted call is ever dropped.
  const psx_status deferred = c->deferred;
  const std::string deferred_msg = c->err;
  c->deferred = PSX_OK;
  auto finish = [&](psx_status s) {
    if (deferred != PSX_OK) {
      c->err = deferred_msg;
      return deferred;
    }
    return s;
  };
  uint32_t replay_sticky = 0;
  if ((sticky & psx::kStDuplicateRow) && c->has_ada) {
    // the call with the duplicate and every later one applied nothing, and the AdaRevision
    // logic has no ordered replay
    psx_status e = sticky_error(c, sticky & ~psx::kStDuplicateRow);
    if (e) return finish(e);
    return finish(fail(c, PSX_ERR_UNSUPPORTED,
                       "a row occurs twice in one message: contexts with an AdaRevision table have no ordered replay"));
  }
  if (sticky & psx::kStDuplicateRow) {
    // A message held a row twice: that call and every later one were skipped.  Replay
    // them, in order, on the ordered path (per-row record order preserved).
    std::vector<uint32_t> log(kRing);
    HIP_TRY(c, hipMemcpy(log.data(), c->d_status + 1 + kRing, sizeof(uint32_t) * kRing, hipMemcpyDeviceToHost));
    size_t first = pending.size();
    for (size_t i = 0; i < pending.size(); ++i)
      if (log[pending[i].ring] & psx::kStDuplicateRow) { first = i; break; }
    for (size_t i = first; i < pending.size(); ++i) {
      psx_status st = enqueue_apply(c, pending[i].streams.data(), (int32_t)pending[i].streams.size(), true);
      if (st) return finish(st);
    }
    c->pending.clear();
    c->pending_calls = 0;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    collect_timing(c);
    HIP_TRY(c, hipMemcpy(&replay_sticky, c->d_status, sizeof(uint32_t), hipMemcpyDeviceToHost));
    if (replay_sticky) {
      uint32_t zero = 0;
      HIP_TRY(c, hipMemcpy(c->d_status, &zero, sizeof(uint32_t), hipMemcpyHostToDevice));
    }
  }
  psx_status e = sticky_error(c, sticky & ~psx::kStDuplicateRow);
  if (e) {
    if (!rejected.empty()) c->err += "; rejected (nothing applied):" + rejected;
    return finish(e);
  }
  return finish(sticky_error(c, replay_sticky));
}

// Serve-back kernel arguments for table t (allocates its size/offset scratch once).
psx_status serve_args(psx_ctx *c, TableState &t, psx::ServeArgs *out) {
  const int64_t R = t.cfg.max_rows;
  if (!t.d_srv_sizes) {
    HIP_TRY(c, hipMalloc(&t.d_srv_sizes, sizeof(int64_t) * R));
    HIP_TRY(c, hipMalloc(&t.d_srv_offs, sizeof(int64_t) * (R + 1 + (R + 1023) / 1024)));
  }
  psx::ServeArgs a{};
  a.flags = t.d_flags;
  a.nent = t.d_nent;
  a.dense = (const uint8_t *)t.d_data;
  a.entries = t.d_entries;
  a.kind = t.cfg.row_kind;
  a.vsize = t.vsize;
  a.row_cap = t.cfg.row_capacity;
  a.max_entries = t.max_entries;
  a.row_offset = t.cfg.row_offset;
  a.row_stride = t.cfg.row_stride;
  a.max_rows = R;
  a.sizes = t.d_srv_sizes;
  a.offs = t.d_srv_offs;
  a.ver = t.d_ver;
  a.f16 = t.cfg.row_bytes_f16;
  *out = a;
  return PSX_OK;
}

}  // namespace

extern "C" {

int32_t psx_abi_version(void) { return PSX_ABI_VERSION; }

const char *psx_status_string(psx_status s) {
  switch (s) {
    case PSX_OK: return "ok";
    case PSX_ERR_INVALID_ARG: return "invalid argument";
    case PSX_ERR_VERSION: return "version gap";
    case PSX_ERR_UNKNOWN_TABLE: return "unknown table";
    case PSX_ERR_MALFORMED: return "malformed stream";
    case PSX_ERR_ROW_RANGE: return "row outside shard";
    case PSX_ERR_CAPACITY: return "capacity exceeded";
    case PSX_ERR_DEVICE: return "device error";
    case PSX_ERR_OOM: return "out of device memory";
    case PSX_ERR_BUFFER_TOO_SMALL: return "buffer too small";
    case PSX_ERR_UNSUPPORTED: return "unsupported";
    case PSX_ERR_SENDER: return "unknown sender";
    case PSX_ERR_NO_DEVICE: return "no HIP device";
    case PSX_ERR_STATE: return "server logic state missing";
  }
  return "?";
}

psx_status psx_device_count(int32_t *n) {
  if (!n) return PSX_ERR_INVALID_ARG;
  int d = 0;
  if (hipGetDeviceCount(&d) != hipSuccess || d <= 0) {
    *n = 0;
    return PSX_ERR_NO_DEVICE;
  }
  *n = d;
  return PSX_OK;
}

psx_status psx_ctx_create(int32_t device, int32_t server_id, psx_ctx **out) {
  if (!out) return PSX_ERR_INVALID_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return PSX_ERR_NO_DEVICE;
  if (device < 0 || device >= ndev) return PSX_ERR_INVALID_ARG;
  psx_ctx *c = new psx_ctx();
  c->device = device;
  c->server_id = server_id;
  auto cleanup = [&](psx_status s) {
    psx_ctx_destroy(c);
    return s;
  };
  if (hipSetDevice(device) != hipSuccess) return cleanup(PSX_ERR_DEVICE);
  // Stream priorities (PSX_VARIANT_STREAM_PRIORITY): 1 the prep stream (a pipelined call's
  // decode, index and records' half of the ordered prep, all beside the previous call's
  // apply) at the lowest priority, so the dispatcher hands CUs to the apply first; 2 also
  // the context's own stream at the highest.
  int prio_lo = 0, prio_hi = 0;
  if (hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi) != hipSuccess) prio_lo = prio_hi = 0;
  const int sp = psx::g_stream_priority;
  // CU masks (PSX_VARIANT_SIDE_CU_MASK k >= 2): the prep stream on one 32-bit word of the
  // queue's CU mask in k; -k also confines the context's own stream to the other words
  const int km = std::abs(psx::g_side_cu_mask);
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) ncu = 0;
  const uint32_t words = (uint32_t)(ncu + 31) / 32;
  std::vector<uint32_t> side_mask(words), own_mask(words);
  for (uint32_t w = 0; w < words; ++w) {
    const uint32_t all = (int)(32 * w + 32) <= ncu ? ~0u : (1u << (ncu - 32 * w)) - 1;
    side_mask[w] = w % (uint32_t)std::max(km, 1) == 0 ? all : 0;
    own_mask[w] = all & ~side_mask[w];
  }
  hipError_t own_e = km >= 2 && psx::g_side_cu_mask < 0 && words > 0
                         ? hipExtStreamCreateWithCUMask(&c->own, words, own_mask.data())
                         : hipStreamCreateWithPriority(&c->own, hipStreamNonBlocking, sp >= 2 ? prio_hi : 0);
  if (own_e != hipSuccess) return cleanup(PSX_ERR_DEVICE);
  c->stream = c->own;
  hipError_t side_e = km >= 2 && words > 0
                          ? hipExtStreamCreateWithCUMask(&c->side, words, side_mask.data())
                          : hipStreamCreateWithPriority(&c->side, hipStreamNonBlocking, sp >= 1 ? prio_lo : 0);
  // Events that only order one of the context's streams after another on this device (the
  // pipelined call slots' ev_ready / ev_free, the concurrent apply launches' fork / join):
  // PSX_VARIANT_EVENT_SCOPE 2 (the default) records them with no system-scope fence (the
  // kernels' own device-scope fences order them on this device; hipEventDisableSystemFence
  // gives up visibility to the host and other devices only), 1 with a device-scope release,
  // 0 HIP's default (system scope).  The system-scope acquire at each wait cost a pipelined C3
  // call ~3 us (16,400-16,550 -> 16,880-17,120 M updates/s, indexed 19,190-19,260 ->
  // 20,090-20,170; a device-scope release alone changes nothing, profiles/r06/s21).  Events
  // the host waits on, or that order a copy to the host, keep HIP's default.
  const unsigned dev_ev = hipEventDisableTiming | (psx::g_event_scope == 1   ? hipEventReleaseToDevice
                                                   : psx::g_event_scope == 2 ? hipEventDisableSystemFence
                                                                             : 0u);
  if (side_e != hipSuccess ||
      hipStreamCreateWithFlags(&c->aux, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fork, dev_ev) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, dev_ev) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_push[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_push[1], hipEventDisableTiming) != hipSuccess)
    return cleanup(PSX_ERR_DEVICE);
  for (int k = 0; k < 2; ++k) {
    if (hipEventCreateWithFlags(&c->ev_ready[k], dev_ev) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_free[k], dev_ev) != hipSuccess)
      return cleanup(PSX_ERR_DEVICE);
    if (hipMalloc(&c->d_segs[k], sizeof(psx::Seg) * psx::kMaxFused * psx::kMaxTables) != hipSuccess ||
        hipMalloc(&c->d_counters[k], sizeof(uint32_t) * psx::kMaxFused * psx::kMaxTables) != hipSuccess ||
        // (then idx_verify's 4 words per message: psx_kernels.hip decode_streams)
        hipMalloc(&c->d_ntouched[k], sizeof(uint32_t) * (psx::kMaxTables + 4 * psx::kMaxFused)) != hipSuccess)
      return cleanup(PSX_ERR_OOM);
    if (hipMemset(c->d_counters[k], 0, sizeof(uint32_t) * psx::kMaxFused * psx::kMaxTables) != hipSuccess)
      return cleanup(PSX_ERR_DEVICE);
  }
#ifdef PSX_DEBUG_BUILD
  if (const char *pv = getenv("PSX_PIPELINE")) c->pipeline = atoi(pv);   // A/B runs (debug build only)
#endif
  if (hipMalloc(&c->d_status, sizeof(uint32_t) * (2 + 2 * kRing)) != hipSuccess ||
      hipMalloc(&c->d_zero, 4096) != hipSuccess)
    return cleanup(PSX_ERR_OOM);
  if (hipMemset(c->d_status, 0, sizeof(uint32_t) * (2 + 2 * kRing)) != hipSuccess ||
      hipMemset(c->d_zero, 0, 4096) != hipSuccess)
    return cleanup(PSX_ERR_DEVICE);
  *out = c;
  return PSX_OK;
}

psx_status psx_ctx_destroy(psx_ctx *c) {
  if (!c) return PSX_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  if (c->side) hipStreamSynchronize(c->side);
  if (c->aux) hipStreamSynchronize(c->aux);
  if (c->stream) hipStreamSynchronize(c->stream);
  if (c->h2d) hipStreamSynchronize(c->h2d);
  for (auto &t : c->tables) free_table(t);
  if (c->d_list) hipFree(c->d_list);
  if (c->d_split_fixed) hipFree(c->d_split_fixed);
  if (c->d_split_recoff) hipFree(c->d_split_recoff);
  if (c->d_split_scratch) hipFree(c->d_split_scratch);
  for (auto &p : c->pending_ev) {
    hipEventDestroy(p.a);
    hipEventDestroy(p.b);
  }
  for (auto e : c->ev_pool) hipEventDestroy(e);
  for (auto &p : c->pending) {
    if (p.ev_a) hipEventDestroy(p.ev_a);
    if (p.ev_b) hipEventDestroy(p.ev_b);
  }
  if (c->stats_open) hipEventDestroy(c->stats_open);
  for (int k = 0; k < 2; ++k) {
    if (c->d_segs[k]) hipFree(c->d_segs[k]);
    if (c->d_counters[k]) hipFree(c->d_counters[k]);
    if (c->d_ntouched[k]) hipFree(c->d_ntouched[k]);
    if (c->d_recoff[k]) hipFree(c->d_recoff[k]);
    if (c->d_wfill[k]) hipFree(c->d_wfill[k]);
    if (c->d_walk[k]) hipFree(c->d_walk[k]);
    if (c->ev_ready[k]) hipEventDestroy(c->ev_ready[k]);
    if (c->ev_free[k]) hipEventDestroy(c->ev_free[k]);
  }
  if (c->side) hipStreamDestroy(c->side);
  if (c->aux) hipStreamDestroy(c->aux);
  if (c->ev_fork) hipEventDestroy(c->ev_fork);
  if (c->ev_join) hipEventDestroy(c->ev_join);
  for (hipEvent_t e : c->ev_push)
    if (e) hipEventDestroy(e);
  if (c->d_status) hipFree(c->d_status);
  if (c->d_zero) hipFree(c->d_zero);
  if (c->d_ndirty) hipFree(c->d_ndirty);
  if (c->d_push_body) hipFree(c->d_push_body);
  if (c->d_push_ent) hipFree(c->d_push_ent);
  if (c->d_push_words) hipFree(c->d_push_words);
  if (c->d_client_tabs) hipFree(c->d_client_tabs);
  if (c->d_pack) hipFree(c->d_pack);
  if (c->d_staging) hipFree(c->d_staging);
  for (int k = 0; k < 2; ++k) {
    if (c->d_seam[k]) hipFree(c->d_seam[k]);
    if (c->ev_seam_copied[k]) hipEventDestroy(c->ev_seam_copied[k]);
    if (c->ev_seam_free[k]) hipEventDestroy(c->ev_seam_free[k]);
  }
  if (c->h2d) hipStreamDestroy(c->h2d);
  for (int k = 0; k < 2; ++k)
    if (c->d_wcount[k]) hipFree(c->d_wcount[k]);
  if (c->own) hipStreamDestroy(c->own);
  delete c;
  return PSX_OK;
}

psx_status psx_ctx_set_stream(psx_ctx *c, void *hip_stream) {
  if (!c) return PSX_ERR_INVALID_ARG;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->side));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  c->stream = hip_stream ? (hipStream_t)hip_stream : c->own;
  return PSX_OK;
}

void *psx_ctx_get_stream(psx_ctx *c) { return c ? (void *)c->stream : nullptr; }

psx_status psx_register_sender(psx_ctx *c, int32_t bg_id) {
  if (!c) return PSX_ERR_INVALID_ARG;
  if (!c->versions.count(bg_id)) {
    c->versions[bg_id] = -1;
    // bg_clock_.AddClock(bg, 0) (server.cpp:21-24, vector_clock.cpp:19-26)
    c->clocks[bg_id] = 0;
    if (c->min_clock == -1 || 0 < c->min_clock) c->min_clock = 0;
  }
  return PSX_OK;
}

psx_status psx_clock_until(psx_ctx *c, int32_t bg_id, int32_t clock, int32_t *new_min_clock) {
  if (!c || !new_min_clock) return PSX_ERR_INVALID_ARG;
  *new_min_clock = 0;
  auto it = c->clocks.find(bg_id);
  if (it == c->clocks.end()) return fail(c, PSX_ERR_SENDER, "bg_id " + std::to_string(bg_id) + " not registered");
  // VectorClock::TickUntil (vector_clock.cpp:38-51): one Tick (:28-36) per clock; a tick by
  // the unique slowest sender advances the min clock (IsUniqueMin, :66-79)
  for (int32_t k = clock - it->second; k > 0; --k) {
    bool unique_min = it->second == c->min_clock;
    if (unique_min) {
      int num_min = 0;
      for (auto &kv : c->clocks)
        if (kv.second == c->min_clock && ++num_min > 1) { unique_min = false; break; }
    }
    ++it->second;
    if (unique_min) *new_min_clock = ++c->min_clock;
  }
  return PSX_OK;
}

psx_status psx_min_clock(psx_ctx *c, int32_t *min_clock) {
  if (!c || !min_clock) return PSX_ERR_INVALID_ARG;
  *min_clock = c->min_clock;
  return PSX_OK;
}

psx_status psx_sender_clock(psx_ctx *c, int32_t bg_id, int32_t *clock) {
  if (!c || !clock) return PSX_ERR_INVALID_ARG;
  auto it = c->clocks.find(bg_id);
  if (it == c->clocks.end()) return fail(c, PSX_ERR_SENDER, "unknown sender");
  *clock = it->second;
  return PSX_OK;
}

psx_status psx_set_num_clients(psx_ctx *c, int32_t num_clients) {
  if (!c || num_clients < 1 || num_clients > PSX_MAX_CLIENTS) return PSX_ERR_INVALID_ARG;
  c->num_clients = num_clients;
  return PSX_OK;
}

psx_status psx_sender_version(psx_ctx *c, int32_t bg_id, int64_t *version) {
  if (!c || !version) return PSX_ERR_INVALID_ARG;
  auto it = c->versions.find(bg_id);
  if (it == c->versions.end()) return fail(c, PSX_ERR_SENDER, "unknown sender");
  *version = it->second;
  return PSX_OK;
}

// The record-format half of a table config — dtype, row kind, record variant, widths —
// checked and copied into t (nothing allocated).  psx_table_create adds the shard geometry
// and the storage; psx_split_stream_formats needs only this.
static psx_status table_format(psx_ctx *c, const psx_table_config *cfg, TableState &t) {
  if (cfg->dtype < PSX_F32 || cfg->dtype > PSX_I64) return fail(c, PSX_ERR_INVALID_ARG, "bad dtype");
  if (cfg->row_kind < PSX_ROW_DENSE || cfg->row_kind > PSX_ROW_MAP) return fail(c, PSX_ERR_INVALID_ARG, "bad row kind");
  if ((cfg->row_bytes_f16 != 0 && cfg->row_bytes_f16 != 1) || cfg->server_push_row_upper_bound < 0 ||
      (cfg->accum_importance != 0 && cfg->accum_importance != 1) ||
      (cfg->version_maintain != 0 && cfg->version_maintain != 1) || cfg->row_oplog_type < 0 ||
      cfg->row_oplog_type > 3)
    return fail(c, PSX_ERR_INVALID_ARG,
                "bad accum_importance / version_maintain / row_oplog_type / row_bytes_f16 / server_push_row_upper_bound");
  if (cfg->row_bytes_f16 && (cfg->row_kind != PSX_ROW_DENSE || cfg->dtype != PSX_F32))
    return fail(c, PSX_ERR_UNSUPPORTED, "binary16 row bytes (DenseRowFloat16) need dense f32 rows (vector_store_float16.hpp:12)");
  const bool f16 = cfg->row_oplog_type == 3 && cfg->oplog_dense_serialized;
  if (cfg->version_maintain && (cfg->row_kind != PSX_ROW_DENSE || !cfg->oplog_dense_serialized || f16))
    // the reference's sparse version records are inconsistent between writer and reader
    // (version_dense_row_oplog.hpp:133-159 vs abstract_row_oplog.hpp:64-78), and the version
    // sample oplog exists only for kDenseRowOpLog (server_table.cpp:56-67)
    return fail(c, PSX_ERR_UNSUPPORTED, "version_maintain needs dense rows with dense-serialized kDenseRowOpLog records");
  if (f16 && cfg->dtype != PSX_F32)
    return fail(c, PSX_ERR_UNSUPPORTED, "float16 records need f32 rows (dense_row_oplog_float16.hpp:28)");
  t.cfg = *cfg;
  if (!f16) t.cfg.row_oplog_type = 0;   // kSparse*RowOpLog: no server-side difference for sparse records
  if (t.cfg.server_push_row_upper_bound == 0) t.cfg.server_push_row_upper_bound = 100;   // table_gflags.cpp:21
  t.vsize = vsize_of(cfg->dtype);
  t.es = t.vsize == 4 ? 8 : 16;
  if (cfg->row_kind == PSX_ROW_DENSE) {
    if (cfg->row_capacity <= 0) return fail(c, PSX_ERR_INVALID_ARG, "row_capacity must be > 0");
    if (cfg->oplog_dense_serialized &&
        (cfg->dense_row_oplog_capacity <= 0 || cfg->dense_row_oplog_capacity > cfg->row_capacity))
      return fail(c, PSX_ERR_INVALID_ARG, "dense_row_oplog_capacity must be in [1, row_capacity]");
  } else {
    // A dense record needs NumericStoreRow::ApplyDenseBatchIncUnsafe -> store GetPtr,
    // which only VectorStore has (vector_store.hpp:104-108).
    if (cfg->oplog_dense_serialized)
      return fail(c, PSX_ERR_UNSUPPORTED, "sorted/map rows take sparse-serialized oplogs only");
    t.max_entries = cfg->max_entries > 0 ? cfg->max_entries : cfg->row_capacity;
    if (t.max_entries <= 0) return fail(c, PSX_ERR_INVALID_ARG, "sorted/map rows need max_entries (or row_capacity) > 0");
    if (t.max_entries * t.es > 150 * 1024)
      return fail(c, PSX_ERR_UNSUPPORTED, "max_entries * sizeof(Entry) must fit one wave's LDS image (150 KiB)");
  }
  return PSX_OK;
}

psx_status psx_table_create(psx_ctx *c, const psx_table_config *cfg) {
  if (!c || !cfg) return PSX_ERR_INVALID_ARG;
  if (c->tables.size() >= (size_t)psx::kMaxTables) return fail(c, PSX_ERR_INVALID_ARG, "too many tables");
  if (find_table(c, cfg->table_id)) return fail(c, PSX_ERR_INVALID_ARG, "table exists");
  if (cfg->dtype < PSX_F32 || cfg->dtype > PSX_I64) return fail(c, PSX_ERR_INVALID_ARG, "bad dtype");
  if (cfg->row_kind < PSX_ROW_DENSE || cfg->row_kind > PSX_ROW_MAP) return fail(c, PSX_ERR_INVALID_ARG, "bad row kind");
  if (cfg->max_rows <= 0 || cfg->row_stride <= 0) return fail(c, PSX_ERR_INVALID_ARG, "bad shard geometry");
  if (cfg->max_rows > ((int64_t)1 << 31) - 2) return fail(c, PSX_ERR_INVALID_ARG, "max_rows exceeds int32 row ids");
  if (c->has_ada && !cfg->oplog_dense_serialized)
    return fail(c, PSX_ERR_UNSUPPORTED, "contexts with an AdaRevision table take dense-serialized tables only");
  TableState t;
  psx_status fe = table_format(c, cfg, t);
  if (fe) return fe;
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t R = (size_t)cfg->max_rows;
  const size_t ntiles = (R + 1023) / 1024;
  hipError_t e = hipSuccess;
  if (cfg->row_kind == PSX_ROW_DENSE) {
    const size_t data_bytes = R * (size_t)cfg->row_capacity * t.vsize;
    e = hipMalloc(&t.d_data, data_bytes);
    if (e == hipSuccess) e = hipMemsetAsync(t.d_data, 0, data_bytes, c->stream);   // VectorStore::Init zeroes
  } else {
    e = hipMalloc(&t.d_nent, R * sizeof(int32_t));
    if (e == hipSuccess) e = hipMalloc(&t.d_entries, R * (size_t)t.max_entries * t.es);
    if (e == hipSuccess) e = hipMemsetAsync(t.d_nent, 0, R * sizeof(int32_t), c->stream);
  }
  if (e == hipSuccess && cfg->accum_importance) {
    e = hipMalloc(&t.d_imp, R * sizeof(double));
    if (e == hipSuccess) e = hipMemsetAsync(t.d_imp, 0, R * sizeof(double), c->stream);
  }
  if (e == hipSuccess && cfg->version_maintain) {
    e = hipMalloc(&t.d_ver, R * sizeof(uint64_t));
    if (e == hipSuccess) e = psx::launch_fill_u64(t.d_ver, (int64_t)R, 1, c->stream);
  }
  if (e == hipSuccess) e = hipMalloc(&t.d_flags, R);
  if (e == hipSuccess) e = hipMemsetAsync(t.d_flags, 0, R, c->stream);
  if (e == hipSuccess && t.fast()) {
    const size_t inv_bytes = R * psx::kMaxFused * sizeof(int32_t);
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
      e = hipMalloc(&t.d_inv[k], inv_bytes);
      if (e == hipSuccess) e = hipMemsetAsync(t.d_inv[k], 0xff, inv_bytes, c->stream);
    }
  }
  // the per-call count state twice, one per call slot: a pipelined walk counts the next
  // call's records while this call's ordered work still uses its own (WalkCount)
  if (e == hipSuccess) e = hipMalloc(&t.d_cnt, 2 * R * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemsetAsync(t.d_cnt, 0, 2 * R * sizeof(int32_t), c->stream);
  if (e == hipSuccess) e = hipMalloc(&t.d_off, (R + 1) * sizeof(int32_t));
  if (e == hipSuccess) e = hipMalloc(&t.d_tsum, 2 * ntiles * sizeof(int32_t));
  t.tsum_slot = (int64_t)ntiles;
  if (e == hipSuccess) e = hipMalloc(&t.d_touched, R * sizeof(int32_t));
  if (e == hipSuccess && cfg->row_kind != PSX_ROW_DENSE) {
    e = hipMalloc(&t.d_keyflag, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemsetAsync(t.d_keyflag, 0, sizeof(uint32_t), c->stream);
  }
  if (e == hipSuccess && t.split()) {
    e = hipMalloc(&t.d_grow, 2 * R * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemsetAsync(t.d_grow, 0, 2 * R * sizeof(int32_t), c->stream);
    if (e == hipSuccess) e = hipMalloc(&t.d_split, 4 * R * 4 * sizeof(int32_t));   // int4 descriptors x 4 lists
    if (e == hipSuccess) e = hipMalloc(&t.d_nsplit, 2 * 5 * psx::kNsStride * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&t.d_plist, 2 * R * 4 * sizeof(int32_t));
    // bucket lists, up to 2M rows (2 x 256 MiB): a slot's records at [slot][place]
    if (e == hipSuccess && R <= (int64_t)kBucketMaxRows)
      // each slot: the list entries, then each entry's pair count (int32, o_grow)
      for (int k = 0; k < 2 && e == hipSuccess; ++k)
        e = hipMalloc(&t.d_bucket[k], R * kBucketM * (sizeof(uint64_t) + sizeof(int32_t)));
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    free_table(t);
    return hip_fail(c, e, "table allocation");
  }
  c->tables.push_back(t);
  return PSX_OK;
}

// Row-range addressing of the row accessors.  Every accessor first settles the calls
// still in flight (their replays included), so it observes every accepted message —
// and reports a device-detected error of those calls, as psx_sync would.
static psx_status row_range(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows,
                            TableState **out, int64_t *first_slot) {
  TableState *t = find_table(c, table_id);
  if (!t) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table");
  if (num_rows < 0) return fail(c, PSX_ERR_INVALID_ARG, "num_rows < 0");
  int64_t s = slot_of(*t, first_row);
  if (s < 0 || s + num_rows > t->cfg.max_rows) return fail(c, PSX_ERR_ROW_RANGE, "row range outside shard");
  psx_status st = sync_impl(c);
  if (st) return st;
  *out = t;
  *first_slot = s;
  return PSX_OK;
}

psx_status psx_table_load_rows(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows,
                               const void *src, int32_t src_on_device) {
  if (!c || (!src && num_rows)) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  if (t->cfg.row_kind != PSX_ROW_DENSE) return fail(c, PSX_ERR_UNSUPPORTED, "load_rows: dense tables only");
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t rb = (size_t)t->cfg.row_capacity * t->vsize;
  HIP_TRY(c, hipMemcpyAsync((uint8_t *)t->d_data + (size_t)s * rb, src, (size_t)num_rows * rb,
                            src_on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, psx::launch_flags_or(t->d_flags, s, num_rows, 1, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_table_read_rows(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows,
                               void *dst, int32_t dst_on_device) {
  if (!c || (!dst && num_rows)) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  if (t->cfg.row_kind != PSX_ROW_DENSE)
    return fail(c, PSX_ERR_UNSUPPORTED, "read_rows: dense tables only (use psx_serialize_rows)");
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t rb = (size_t)t->cfg.row_capacity * t->vsize;
  HIP_TRY(c, hipMemcpyAsync(dst, (const uint8_t *)t->d_data + (size_t)s * rb, (size_t)num_rows * rb,
                            dst_on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_row_flags(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows, uint8_t *dst) {
  if (!c || (!dst && num_rows)) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipMemcpyAsync(dst, t->d_flags + s, (size_t)num_rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_clear_dirty(psx_ctx *c, int32_t table_id) {
  if (!c) return PSX_ERR_INVALID_ARG;
  TableState *t = find_table(c, table_id);
  if (!t) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table");
  psx_status sst = sync_impl(c);
  if (sst) return sst;
  HIP_TRY(c, psx::launch_flags_and(t->d_flags, t->cfg.max_rows, (uint8_t)~2u, c->stream));
  return PSX_OK;
}

psx_status psx_row_importance(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows, double *dst) {
  if (!c || (!dst && num_rows)) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  if (!t->d_imp) {
    for (int64_t i = 0; i < num_rows; ++i) dst[i] = 0.0;
    return PSX_OK;
  }
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipMemcpyAsync(dst, t->d_imp + s, sizeof(double) * (size_t)num_rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_row_versions(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows, uint64_t *dst) {
  if (!c || (!dst && num_rows)) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  for (int64_t i = 0; i < num_rows; ++i) dst[i] = 0;
  if (!t->d_ver || num_rows == 0) return PSX_OK;
  std::vector<uint8_t> flags((size_t)num_rows);
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipMemcpyAsync(dst, t->d_ver + s, sizeof(uint64_t) * (size_t)num_rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipMemcpyAsync(flags.data(), t->d_flags + s, (size_t)num_rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < num_rows; ++i)
    if (!(flags[i] & 1)) dst[i] = 0;   // no ServerRow: nothing to report
  return PSX_OK;
}

static psx_status apply_device_impl(psx_ctx *c, const psx_stream *s, int32_t n,
                                    const uint64_t *const *record_offsets,
                                    const int32_t *const *record_rows = nullptr);

psx_status psx_apply_indexed(psx_ctx *c, const psx_stream *s, const uint64_t *const *record_offsets, int32_t n) {
  if (!c || !s || !record_offsets || n <= 0 || n > PSX_MAX_FUSED_STREAMS) return PSX_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i)
    if (record_offsets[i] && ((uintptr_t)record_offsets[i] & 7))
      return fail(c, PSX_ERR_INVALID_ARG, "record_offsets must be 8-byte aligned device arrays");
  return apply_device_impl(c, s, n, record_offsets);
}

psx_status psx_apply_indexed_rows(psx_ctx *c, const psx_stream *s, const uint64_t *const *record_offsets,
                                  const int32_t *const *record_rows, int32_t n) {
  if (!c || !s || (!record_offsets && !record_rows) || n <= 0 || n > PSX_MAX_FUSED_STREAMS)
    return PSX_ERR_INVALID_ARG;
  for (int i = 0; i < n; ++i) {
    if (record_offsets && record_offsets[i] && ((uintptr_t)record_offsets[i] & 7))
      return fail(c, PSX_ERR_INVALID_ARG, "record_offsets must be 8-byte aligned device arrays");
    if (record_rows && record_rows[i] && ((uintptr_t)record_rows[i] & 3))
      return fail(c, PSX_ERR_INVALID_ARG, "record_rows must be 4-byte aligned device arrays");
  }
  return apply_device_impl(c, s, n, record_offsets, record_rows);
}

psx_status psx_apply_streams_device(psx_ctx *c, const psx_stream *s, int32_t n) {
  if (!c || !s || n <= 0 || n > PSX_MAX_FUSED_STREAMS) return PSX_ERR_INVALID_ARG;
  return apply_device_impl(c, s, n, nullptr);
}

static psx_status apply_device_impl(psx_ctx *c, const psx_stream *s, int32_t n,
                                    const uint64_t *const *record_offsets, const int32_t *const *record_rows) {
  // A full call ring is settled first: the settle may give a rejected call's version back,
  // which the version check below must see.
  if (c->pending_calls >= kRing - 1) {
    psx_status d = sync_impl(c);
    if (d != PSX_OK) c->deferred = d;
  }
  // Version rule of Server::ApplyOpLogUpdateVersion (server.cpp:124-126), checked for
  // the whole batch before anything is enqueued.
  std::map<int32_t, int64_t> v = c->versions;
  for (int i = 0; i < n; ++i) {
    if ((c->compat & PSX_COMPAT_INT32_STREAM_OFFSETS) && s[i].size > (size_t)INT32_MAX)
      return fail(c, PSX_ERR_UNSUPPORTED, "stream of " + std::to_string(s[i].size) +
                                              " bytes: the reference reader's int32 offset_ caps messages below 2 GiB");
    if (s[i].size && (!s[i].data || ((uintptr_t)s[i].data & 3)))
      return fail(c, PSX_ERR_INVALID_ARG, "device stream must be non-null and 4-byte aligned");
    auto it = v.find(s[i].bg_id);
    if (it == v.end()) return fail(c, PSX_ERR_SENDER, "bg_id " + std::to_string(s[i].bg_id) + " not registered");
    if (it->second + 1 != (int64_t)s[i].version)
      return fail(c, PSX_ERR_VERSION, "bg_thread_id = " + std::to_string(s[i].bg_id) + ": expected version " +
                                          std::to_string(it->second + 1) + ", got " + std::to_string(s[i].version));
    it->second = s[i].version;
  }
  HIP_TRY(c, hipSetDevice(c->device));
  psx_status st = enqueue_apply(c, s, n, false, record_offsets, record_rows);
  if (st) return st;
  c->versions = v;
  return PSX_OK;
}

psx_status psx_apply_stream(psx_ctx *c, const void *oplog, size_t oplog_size, int32_t bg_id,
                            uint32_t version) {
  if (!c || (oplog_size && !oplog)) return PSX_ERR_INVALID_ARG;
  if ((c->compat & PSX_COMPAT_INT32_STREAM_OFFSETS) && oplog_size > (size_t)INT32_MAX)
    return fail(c, PSX_ERR_UNSUPPORTED, "stream of " + std::to_string(oplog_size) +
                                            " bytes: the reference reader's int32 offset_ caps messages below 2 GiB");
  const uint8_t *p = (const uint8_t *)oplog;
  const bool empty = oplog_size == 0 || (oplog_size >= 4 && rd32h(p) == 0);   // server.cpp:128, Restart() false
  const int s = (int)(c->seam_k & 1);   // the staging slot an async call takes
  if (!empty) {
    // Settles this call may need happen before its version is checked: a settle may give a
    // rejected call's version back (sync_impl).
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->pending_calls >= kRing - 1) {
      psx_status d = sync_impl(c);
      if (d != PSX_OK) c->deferred = d;
    }
    if (c->seam_mode == PSX_SEAM_ASYNC && c->seam_used[s]) {   // slot s last held call seam_k - 2's message
      HIP_TRY(c, hipEventSynchronize(c->ev_seam_free[s]));
      // A duplicate-row replay re-reads its calls' messages when it settles: settle it
      // while slot s still holds the bytes of every pending call
      uint32_t sticky = 0;
      HIP_TRY(c, hipMemcpy(&sticky, c->d_status, sizeof(uint32_t), hipMemcpyDeviceToHost));
      if (sticky & psx::kStDuplicateRow) {
        psx_status d = sync_impl(c);
        if (d != PSX_OK) c->deferred = d;
      }
    }
  }
  auto it = c->versions.find(bg_id);
  if (it == c->versions.end()) return fail(c, PSX_ERR_SENDER, "bg_id " + std::to_string(bg_id) + " not registered");
  if (it->second + 1 != (int64_t)version)
    return fail(c, PSX_ERR_VERSION, "bg_thread_id = " + std::to_string(bg_id) + ": expected version " +
                                        std::to_string(it->second + 1) + ", got " + std::to_string(version));
  if (empty) {
    it->second = version;
    return PSX_OK;
  }
  psx_status st;
  if (c->seam_mode == PSX_SEAM_ASYNC) {
    // The device validates everything before it touches a row (decode, index, ordered
    // prep); the host only copies.  Slot s last held call seam_k - 2's message.
    if (!c->h2d) {
      HIP_TRY(c, hipStreamCreateWithFlags(&c->h2d, hipStreamNonBlocking));
      for (int k = 0; k < 2; ++k) {
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_seam_copied[k], hipEventDisableTiming));
        HIP_TRY(c, hipEventCreateWithFlags(&c->ev_seam_free[k], hipEventDisableTiming));
      }
    }
    if (oplog_size > c->seam_cap[s]) {
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->side));
      if (c->d_seam[s]) hipFree(c->d_seam[s]);
      c->d_seam[s] = nullptr;
      c->seam_cap[s] = 0;
      HIP_TRY(c, hipMalloc(&c->d_seam[s], oplog_size));
      c->seam_cap[s] = oplog_size;
    }
    HIP_TRY(c, hipMemcpyAsync(c->d_seam[s], oplog, oplog_size, hipMemcpyHostToDevice, c->h2d));
    HIP_TRY(c, hipEventRecord(c->ev_seam_copied[s], c->h2d));
    // the caller's bytes have been read once the copy is done: they may be freed on return
    HIP_TRY(c, hipEventSynchronize(c->ev_seam_copied[s]));
    psx_stream one{c->d_seam[s], oplog_size, bg_id, version};
    st = enqueue_apply(c, &one, 1, false);
    if (st) return st;
    it->second = version;
    HIP_TRY(c, hipEventRecord(c->ev_seam_free[s], c->stream));
    c->seam_used[s] = true;
    ++c->seam_k;
    return PSX_OK;
  }
  // PSX_SEAM_SYNC.  The staging buffer may still feed an earlier call's kernels.
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (oplog_size > c->staging_cap) {
    if (c->d_staging) hipFree(c->d_staging);
    c->d_staging = nullptr;
    c->staging_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_staging, oplog_size));
    c->staging_cap = oplog_size;
  }
  HIP_TRY(c, hipMemcpyAsync(c->d_staging, oplog, oplog_size, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));   // the caller frees `oplog` after we return
  psx_stream one{c->d_staging, oplog_size, bg_id, version};
  st = enqueue_apply(c, &one, 1, false);
  if (st) return st;
  it->second = version;
  // Host messages are applied synchronously, like the reference server thread; this
  // also lets a duplicate-row replay read the staging buffer before it is reused.  A
  // message the device rejects gives its version back here (sync_impl), so the caller can
  // correct it and send it again with the same version.
  return sync_impl(c);
}

psx_status psx_sync(psx_ctx *c) {
  if (!c) return PSX_ERR_INVALID_ARG;
  return sync_impl(c);
}

psx_status psx_serialize_rows(psx_ctx *c, int32_t table_id, const int32_t *row_ids, int32_t n, void *out,
                              size_t cap, size_t *used) {
  if (!c || !used || n < 0 || (n && !row_ids)) return PSX_ERR_INVALID_ARG;
  *used = 0;
  TableState *t = find_table(c, table_id);
  if (!t) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table");
  if (n == 0) return PSX_OK;
  psx_status sst = sync_impl(c);
  if (sst) return sst;
  std::vector<int64_t> slots(n);
  for (int32_t i = 0; i < n; ++i) slots[i] = slot_of(*t, row_ids[i]);
  const bool dense = t->cfg.row_kind == PSX_ROW_DENSE;
  const size_t rb = dense ? (size_t)t->cfg.row_capacity * t->vsize : (size_t)t->max_entries * t->es;
  int64_t *d_slots = nullptr;
  uint8_t *d_out = nullptr;
  int32_t *d_cnt = nullptr;
  uint8_t *d_flags = nullptr;
  uint64_t *d_vers = nullptr;
  std::vector<uint8_t> rows(rb * n);
  std::vector<int32_t> counts(n, 0);
  std::vector<uint8_t> flags(n, 0);
  std::vector<uint64_t> vers(n, 0);
  hipError_t e = hipMalloc(&d_slots, sizeof(int64_t) * n);
  if (e == hipSuccess && t->d_ver) e = hipMalloc(&d_vers, sizeof(uint64_t) * n);
  if (e == hipSuccess) e = hipMalloc(&d_out, rb * n);
  if (e == hipSuccess) e = hipMalloc(&d_cnt, sizeof(int32_t) * n);
  if (e == hipSuccess) e = hipMalloc(&d_flags, n);
  if (e == hipSuccess) e = hipMemcpyAsync(d_slots, slots.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess)
    e = dense ? psx::launch_gather_rows(t->cfg.dtype, t->d_data, d_slots, n, t->cfg.row_capacity, d_out, c->stream)
              : psx::launch_gather_entries(t->cfg.dtype, t->d_nent, t->d_entries, t->max_entries, d_slots, n, d_cnt,
                                           d_out, c->stream);
  if (e == hipSuccess) e = psx::launch_gather_flags(t->d_flags, d_slots, n, d_flags, c->stream);
  if (e == hipSuccess && d_vers) e = psx::launch_gather_u64(t->d_ver, d_slots, n, d_vers, c->stream);
  if (e == hipSuccess && d_vers)
    e = hipMemcpyAsync(vers.data(), d_vers, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(rows.data(), d_out, rb * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess && !dense) e = hipMemcpyAsync(counts.data(), d_cnt, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(flags.data(), d_flags, n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (d_slots) hipFree(d_slots);
  if (d_out) hipFree(d_out);
  if (d_cnt) hipFree(d_cnt);
  if (d_flags) hipFree(d_flags);
  if (d_vers) hipFree(d_vers);
  if (e != hipSuccess) return hip_fail(c, e, "serialize gather");
  // RecordBuff::Append framing {int32 row_id; size_t size; bytes} (record_buff.hpp:41-53);
  // rows absent from the shard's storage are skipped, as ServerTable only holds created rows.
  size_t off = 0;
  uint8_t *o = (uint8_t *)out;
  for (int32_t i = 0; i < n; ++i) {
    if (slots[i] < 0 || !(flags[i] & 1)) continue;
    const uint8_t *src = rows.data() + (size_t)i * rb;
    size_t body;
    if (dense && t->cfg.row_bytes_f16) {
      body = (size_t)t->cfg.row_capacity * 2;             // VectorStoreFloat16::Serialize
    } else if (dense) {
      body = rb;                                          // VectorStore::Serialize
    } else if (t->cfg.row_kind == PSX_ROW_SORTED_MAP) {
      body = (size_t)counts[i] * t->es;                   // Entry<V>[n] as stored
    } else {
      body = (size_t)counts[i] * (4 + t->vsize);          // MapStore::Serialize packs {int32, V}
    }
    const size_t trailer = t->d_ver ? 8 : 0;   // VersionServerRow::Serialize (version_server_row.hpp:59-64)
    if (off + 12 + body + trailer > cap) return fail(c, PSX_ERR_BUFFER_TOO_SMALL, "serialize: output buffer too small");
    uint64_t sz = body + trailer;
    memcpy(o + off, &row_ids[i], 4);
    memcpy(o + off + 4, &sz, 8);
    if (dense && t->cfg.row_bytes_f16) {
      for (int64_t k = 0; k < t->cfg.row_capacity; ++k) {
        float x;
        memcpy(&x, src + (size_t)k * 4, 4);
        const uint16_t h = f32_to_half_fc(x);
        memcpy(o + off + 12 + (size_t)k * 2, &h, 2);
      }
    } else if (t->cfg.row_kind == PSX_ROW_MAP) {
      uint8_t *d = o + off + 12;
      for (int32_t k = 0; k < counts[i]; ++k) {
        memcpy(d, src + (size_t)k * t->es, 4);
        memcpy(d + 4, src + (size_t)k * t->es + (t->vsize == 4 ? 4 : 8), t->vsize);
        d += 4 + t->vsize;
      }
    } else {
      memcpy(o + off + 12, src, body);
    }
    if (trailer) memcpy(o + off + 12 + body, &vers[i], 8);
    off += 12 + body + trailer;
  }
  *used = off;
  return PSX_OK;
}

psx_status psx_serialize_dirty(psx_ctx *c, void *out, size_t cap, size_t *used, int32_t out_on_device,
                               int32_t clear_dirty) {
  if (!c || !used) return PSX_ERR_INVALID_ARG;
  *used = 0;
  if (out_on_device && ((uintptr_t)out & 3)) return fail(c, PSX_ERR_INVALID_ARG, "device output must be 4-byte aligned");
  // every accepted message is applied before the push is built (server_thread.cpp:241-288)
  psx_status sst = sync_impl(c);
  if (sst) return sst;
  const size_t T = c->tables.size();
  std::vector<psx::ServeArgs> args(T);
  for (size_t i = 0; i < T; ++i) {
    TableState &t = c->tables[i];
    psx_status st = serve_args(c, t, &args[i]);
    if (st) return st;
    HIP_TRY(c, psx::launch_serve_sizes(args[i], c->stream));
  }
  // lay out {table_id, records..., -1 | -2} per table (server.cpp:189-309)
  psx::Words w{};
  std::vector<int64_t> base(T);
  int64_t pos = 0;
  for (size_t i = 0; i < T; ++i) {
    int64_t total = 0;
    HIP_TRY(c, hipMemcpyAsync(&total, args[i].offs + args[i].max_rows, sizeof(int64_t), hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    w.pos[w.n] = pos;
    w.val[w.n++] = c->tables[i].cfg.table_id;
    pos += 4;
    base[i] = pos;
    pos += total;
    w.pos[w.n] = pos;
    w.val[w.n++] = i + 1 < T ? -1 : -2;
    pos += 4;
  }
  *used = (size_t)pos;
  if ((size_t)pos > cap) return fail(c, PSX_ERR_BUFFER_TOO_SMALL, "serialize_dirty: *used bytes needed");
  if (pos == 0) return PSX_OK;
  for (size_t i = 0; i < T && clear_dirty; ++i) {   // ServerRowSent must not fail after the clear
    TableState &t = c->tables[i];
    if (!t.ada) continue;
    psx_status st = ada_rows_sent(c, t, (int)i, nullptr, args[i].sizes, args[i].max_rows,
                                  (uint64_t)t.ada_cfg.push_clients, nullptr, true);
    if (st) {
      *used = 0;
      return st;
    }
  }
  uint8_t *dst = (uint8_t *)out;
  if (!out_on_device) {
    if ((size_t)pos > c->staging_cap) {
      if (c->d_staging) hipFree(c->d_staging);
      c->d_staging = nullptr;
      c->staging_cap = 0;
      HIP_TRY(c, hipMalloc(&c->d_staging, (size_t)pos));
      c->staging_cap = (size_t)pos;
    }
    dst = c->d_staging;
  }
  for (size_t i = 0; i < T; ++i) {
    args[i].out = dst + base[i];
    args[i].flags_rw = clear_dirty ? c->tables[i].d_flags : nullptr;
    args[i].imp_rw = clear_dirty ? c->tables[i].d_imp : nullptr;
    HIP_TRY(c, psx::launch_serve_emit(args[i], c->stream));
  }
  HIP_TRY(c, psx::launch_put_words(dst, w, c->stream));
  for (size_t i = 0; i < T && clear_dirty; ++i) {   // ServerRowSent (server_table.cpp:252-255)
    TableState &t = c->tables[i];
    if (!t.ada) continue;
    psx_status st = ada_rows_sent(c, t, (int)i, nullptr, args[i].sizes, args[i].max_rows,
                                  (uint64_t)t.ada_cfg.push_clients, nullptr, false);
    if (st) return st;
  }
  if (!out_on_device) HIP_TRY(c, hipMemcpyAsync(out, dst, (size_t)pos, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_serialize_partial(psx_ctx *c, void *out, size_t cap, size_t *used, int32_t out_on_device,
                                 int32_t clear_dirty) {
  if (!c || !used) return PSX_ERR_INVALID_ARG;
  *used = 0;
  if (out_on_device && ((uintptr_t)out & 3)) return fail(c, PSX_ERR_INVALID_ARG, "device output must be 4-byte aligned");
  psx_status sst = sync_impl(c);
  if (sst) return sst;
  if (!c->d_ndirty) HIP_TRY(c, hipMalloc(&c->d_ndirty, sizeof(uint32_t)));
  const size_t T = c->tables.size();
  std::vector<psx::ServeArgs> args(T);
  std::vector<int64_t> bytes(T, 0);
  bool any = false;
  for (size_t i = 0; i < T; ++i) {
    TableState &t = c->tables[i];
    const int64_t R = t.cfg.max_rows;
    psx_status st = serve_args(c, t, &args[i]);
    if (st) return st;
    if (!t.d_pkeys[0]) {
      for (int k = 0; k < 2; ++k) {
        HIP_TRY(c, hipMalloc(&t.d_pkeys[k], sizeof(double) * R));
        HIP_TRY(c, hipMalloc(&t.d_pvals[k], sizeof(int32_t) * R));
      }
      HIP_TRY(c, hipMalloc(&t.d_lsizes, sizeof(int64_t) * R));
      HIP_TRY(c, hipMalloc(&t.d_loffs, sizeof(int64_t) * (R + 1 + (R + 1023) / 1024)));
      size_t tb = 0;
      HIP_TRY(c, psx::launch_sort_desc(nullptr, &tb, t.d_pkeys[0], t.d_pkeys[1], t.d_pvals[0], t.d_pvals[1], R,
                                       c->stream));
      HIP_TRY(c, hipMalloc(&t.d_sort_tmp, tb ? tb : 1));
      t.sort_tmp_bytes = tb;
    }
    psx::ServeArgs &a = args[i];
    a.imp = t.d_imp;
    a.keys = t.d_pkeys[0];
    a.vals = t.d_pvals[0];
    a.ndirty = c->d_ndirty;
    HIP_TRY(c, hipMemsetAsync(c->d_ndirty, 0, sizeof(uint32_t), c->stream));
    HIP_TRY(c, psx::launch_serve_sizes(a, c->stream));
    size_t tb = t.sort_tmp_bytes;
    HIP_TRY(c, psx::launch_sort_desc(t.d_sort_tmp, &tb, t.d_pkeys[0], t.d_pkeys[1], t.d_pvals[0], t.d_pvals[1], R,
                                     c->stream));
    uint32_t nd = 0;
    HIP_TRY(c, hipMemcpyAsync(&nd, c->d_ndirty, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    a.keys = nullptr;
    a.sel = t.d_pvals[1];
    a.nsel = std::min<int64_t>((int64_t)nd, t.cfg.server_push_row_upper_bound);
    if (t.ada) {   // !AllowSend(): too many live snapshots (adarevision_server_table_logic.cpp:192-197)
      uint32_t live = 0;
      HIP_TRY(c, hipMemcpy(&live, t.d_ada_words, sizeof(uint32_t), hipMemcpyDeviceToHost));
      if ((uint64_t)live >= t.ada_cfg.old_grad_upper_bound) a.nsel = 0;
    }
    a.lsizes = t.d_lsizes;
    a.loffs = t.d_loffs;
    if (a.nsel > 0) {
      any = true;
      HIP_TRY(c, psx::launch_serve_list_sizes(a, c->stream));
      HIP_TRY(c, hipMemcpyAsync(&bytes[i], a.loffs + a.nsel, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
  }
  if (!any) return PSX_OK;   // nothing to send (server.cpp:348)
  psx::Words w{};
  std::vector<int64_t> base(T);
  int64_t pos = 0;
  for (size_t i = 0; i < T; ++i) {
    w.pos[w.n] = pos;
    w.val[w.n++] = c->tables[i].cfg.table_id;
    pos += 4;
    base[i] = pos;
    pos += bytes[i];
    w.pos[w.n] = pos;
    w.val[w.n++] = i + 1 < T ? -1 : -2;
    pos += 4;
  }
  *used = (size_t)pos;
  if ((size_t)pos > cap) return fail(c, PSX_ERR_BUFFER_TOO_SMALL, "serialize_partial: *used bytes needed");
  for (size_t i = 0; i < T && clear_dirty; ++i) {
    TableState &t = c->tables[i];
    if (!t.ada || args[i].nsel <= 0) continue;
    psx_status st = ada_rows_sent(c, t, (int)i, args[i].sel, nullptr, args[i].nsel,
                                  (uint64_t)t.ada_cfg.push_clients, nullptr, true);
    if (st) {
      *used = 0;
      return st;
    }
  }
  uint8_t *dst = (uint8_t *)out;
  if (!out_on_device) {
    if ((size_t)pos > c->staging_cap) {
      if (c->d_staging) hipFree(c->d_staging);
      c->d_staging = nullptr;
      c->staging_cap = 0;
      HIP_TRY(c, hipMalloc(&c->d_staging, (size_t)pos));
      c->staging_cap = (size_t)pos;
    }
    dst = c->d_staging;
  }
  for (size_t i = 0; i < T; ++i) {
    args[i].out = dst + base[i];
    args[i].flags_rw = clear_dirty ? c->tables[i].d_flags : nullptr;
    args[i].imp_rw = clear_dirty ? c->tables[i].d_imp : nullptr;
    HIP_TRY(c, psx::launch_serve_emit_list(args[i], c->stream));
  }
  HIP_TRY(c, psx::launch_put_words(dst, w, c->stream));
  for (size_t i = 0; i < T && clear_dirty; ++i) {   // ServerRowSent (server_table.cpp:412-415)
    TableState &t = c->tables[i];
    if (!t.ada || args[i].nsel <= 0) continue;
    psx_status st = ada_rows_sent(c, t, (int)i, args[i].sel, nullptr, args[i].nsel,
                                  (uint64_t)t.ada_cfg.push_clients, nullptr, false);
    if (st) return st;
  }
  if (!out_on_device) HIP_TRY(c, hipMemcpyAsync(out, dst, (size_t)pos, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_table_set_adarevision(psx_ctx *c, int32_t table_id, const psx_adarevision_config *cfg) {
  if (!c || !cfg) return PSX_ERR_INVALID_ARG;
  TableState *t = find_table(c, table_id);
  if (!t) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table");
  if (t->ada) return fail(c, PSX_ERR_INVALID_ARG, "AdaRevision already attached");
  if (cfg->push_clients < 0 || cfg->max_snapshots_per_row < 0 || cfg->max_snapshots_per_row > psx::kAdaMaxS)
    return fail(c, PSX_ERR_INVALID_ARG, "bad push_clients / max_snapshots_per_row (1..8, 0 -> 4)");
  if (t->cfg.row_kind != PSX_ROW_DENSE || t->cfg.dtype != PSX_F32 || !t->cfg.oplog_dense_serialized ||
      t->rec_f16() || t->cfg.dense_row_oplog_capacity != t->cfg.row_capacity)
    return fail(c, PSX_ERR_UNSUPPORTED,
                "AdaRevision needs f32 dense rows with row-wide dense records (adarevision_server_table_logic.cpp:65-68)");
  for (auto &o : c->tables)
    if (!o.cfg.oplog_dense_serialized)
      return fail(c, PSX_ERR_UNSUPPORTED, "contexts with an AdaRevision table take dense-serialized tables only");
  psx_adarevision_config k = *cfg;
  if (k.push_clients == 0) k.push_clients = 1;
  if (k.max_snapshots_per_row == 0) k.max_snapshots_per_row = 4;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->side));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  const size_t R = (size_t)t->cfg.max_rows, cap = (size_t)t->cfg.row_capacity, S = (size_t)k.max_snapshots_per_row;
  TableState &x = *t;
  hipError_t e = hipMalloc(&x.d_acc, R * cap * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&x.d_z, R * cap * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&x.d_zmax, R * cap * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&x.d_snap_ver, R * S * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&x.d_snap_cnt, R * S * sizeof(uint64_t));
  if (e == hipSuccess) e = hipMalloc(&x.d_snap_acc, R * S * cap * sizeof(float));
  if (e == hipSuccess) e = hipMalloc(&x.d_ada_words, 4 * sizeof(uint32_t));
  // AdaRevisionRow(row_size): accum 0, z 1, z_max 1 (adarevision_server_table_logic.hpp:12-16)
  if (e == hipSuccess) e = hipMemsetAsync(x.d_acc, 0, R * cap * sizeof(float), c->stream);
  if (e == hipSuccess) e = psx::launch_fill_f32(x.d_z, (int64_t)(R * cap), 1.0f, c->stream);
  if (e == hipSuccess) e = psx::launch_fill_f32(x.d_zmax, (int64_t)(R * cap), 1.0f, c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(x.d_snap_cnt, 0, R * S * sizeof(uint64_t), c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(x.d_ada_words, 0, 4 * sizeof(uint32_t), c->stream);
  if (e == hipSuccess && k.gaussian_init) {
    e = hipMalloc(&x.d_new_keys, 2 * R * sizeof(uint64_t));
    if (e == hipSuccess) e = hipMalloc(&x.d_new_slots, 2 * R * sizeof(int32_t));
    size_t tb = 0;
    if (e == hipSuccess)
      e = psx::launch_ada_sort(nullptr, &tb, x.d_new_keys, x.d_new_keys + R, x.d_new_slots, x.d_new_slots + R,
                               (int)R, c->stream);
    if (e == hipSuccess) e = hipMalloc(&x.d_new_tmp, tb ? tb : 1);
    x.new_tmp_bytes = tb;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return hip_fail(c, e, "AdaRevision state allocation");
  x.ada_gen = std::make_shared<std::mt19937>(12345);                          // :32
  x.ada_dist = std::make_shared<std::normal_distribution<float>>(0.0f, 0.1f);  // :33
  x.ada_cfg = k;
  x.ada = true;
  c->has_ada = true;
  return PSX_OK;
}

psx_status psx_row_sent(psx_ctx *c, int32_t table_id, const int32_t *row_ids, int32_t n, int32_t num_clients) {
  if (!c || n < 0 || (n && !row_ids) || num_clients <= 0) return PSX_ERR_INVALID_ARG;
  int ti = 0;
  TableState *t = find_table(c, table_id, &ti);
  if (!t) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table");
  if (n == 0) return PSX_OK;
  std::vector<int32_t> slots(n);
  std::vector<int64_t> slots64(n);
  for (int32_t i = 0; i < n; ++i) {
    const int64_t s = slot_of(*t, row_ids[i]);
    if (s < 0) return fail(c, PSX_ERR_ROW_RANGE, "row " + std::to_string(row_ids[i]) + " not owned by this shard");
    slots[i] = (int32_t)s;
    slots64[i] = s;
  }
  psx_status sst = sync_impl(c);
  if (sst) return sst;
  // the replied rows exist (the request path creates them, server.cpp:107-118)
  std::vector<uint8_t> flags(n);
  for (int32_t i = 0; i < n; ++i)
    HIP_TRY(c, hipMemcpyAsync(&flags[i], t->d_flags + slots64[i], 1, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  for (int32_t i = 0; i < n; ++i)
    if (!(flags[i] & 1)) return fail(c, PSX_ERR_INVALID_ARG, "row " + std::to_string(row_ids[i]) + " does not exist");
  if (!t->ada) return PSX_OK;   // ServerTable::RowSent: only a logic reacts (server_table.cpp:191-195)
  int32_t *d = nullptr;
  HIP_TRY(c, hipMalloc(&d, sizeof(int32_t) * n));
  hipError_t e = hipMemcpyAsync(d, slots.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, c->stream);
  psx_status st = e == hipSuccess ? ada_rows_sent(c, *t, ti, d, nullptr, n, (uint64_t)num_clients, nullptr, false)
                                  : hip_fail(c, e, "row_sent upload");
  hipStreamSynchronize(c->stream);
  hipFree(d);
  return st;
}

psx_status psx_adarevision_state(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows, float *accum,
                                 float *z, float *z_max, uint64_t *live_snapshots) {
  if (!c) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  if (!t->ada) return fail(c, PSX_ERR_INVALID_ARG, "table has no AdaRevision logic");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->side));
  const size_t cap = (size_t)t->cfg.row_capacity, nb = (size_t)num_rows * cap * sizeof(float);
  const size_t off = (size_t)s * cap;
  if (accum && nb) HIP_TRY(c, hipMemcpyAsync(accum, t->d_acc + off, nb, hipMemcpyDeviceToHost, c->stream));
  if (z && nb) HIP_TRY(c, hipMemcpyAsync(z, t->d_z + off, nb, hipMemcpyDeviceToHost, c->stream));
  if (z_max && nb) HIP_TRY(c, hipMemcpyAsync(z_max, t->d_zmax + off, nb, hipMemcpyDeviceToHost, c->stream));
  uint32_t live = 0;
  HIP_TRY(c, hipMemcpyAsync(&live, t->d_ada_words, sizeof(uint32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (live_snapshots) *live_snapshots = live;
  return PSX_OK;
}

// psx_split_stream (psx_split.hip): the client's per-server split of one packed message.
// fmts: the record formats of the tables a message may carry (the context's own tables for
// psx_split_stream, the caller's configs for psx_split_stream_formats).
static psx_status split_impl(psx_ctx *c, const std::vector<TableState> &fmts, const void *stream, size_t size,
                             const uint64_t *record_offsets, int32_t nowners, const int64_t *row_begin, void *out,
                             size_t out_cap, uint64_t *out_sizes) {
  if (!c || !out_sizes || !row_begin || nowners < 1 || nowners > PSX_MAX_SPLIT_OWNERS || (size && !stream))
    return PSX_ERR_INVALID_ARG;
  for (int32_t o = 0; o < nowners; ++o) {
    out_sizes[o] = 0;
    if (row_begin[o + 1] < row_begin[o]) return fail(c, PSX_ERR_INVALID_ARG, "row_begin must be non-decreasing");
  }
  if (((uintptr_t)stream & 3) || (size & 3) || (out && ((uintptr_t)out & 3)))
    return fail(c, PSX_ERR_INVALID_ARG, "split streams are 4-byte aligned");
  if (size == 0) return PSX_OK;   // an empty message splits into empty messages
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t st = c->stream;
  // sparse record offsets: at most one per 8 bytes of message; none when every table is
  // dense-serialized (fixed stride: the decode writes no offsets), so a dense message of
  // any size costs no offset buffer
  bool any_sparse = false;
  for (const TableState &t : fmts) any_sparse |= !t.cfg.oplog_dense_serialized;
  const size_t nrecoff = any_sparse ? size / 8 + 1 : 1;
  auto grow = [&](void *&p, size_t &cap, size_t need) -> psx_status {
    if (need <= cap) return PSX_OK;
    HIP_TRY(c, hipStreamSynchronize(st));
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    HIP_TRY(c, hipMalloc(&p, need));
    cap = need;
    return PSX_OK;
  };
  // 1) decode the message (tables, sparse record offsets) into the split's own buffers
  psx_status e = grow(c->d_split_fixed, c->split_fixed_cap,
                      sizeof(psx::Seg) * psx::kMaxFused * psx::kMaxTables + 8192);
  if (e) return e;
  if ((e = grow(c->d_split_recoff, c->split_recoff_cap, nrecoff * sizeof(uint64_t)))) return e;
  psx::Seg *segs = reinterpret_cast<psx::Seg *>(c->d_split_fixed);
  uint32_t *words = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(c->d_split_fixed) +
                                                 sizeof(psx::Seg) * psx::kMaxFused * psx::kMaxTables);
  uint32_t *status = words, *counters = words + 16, *ntouched = words + 16 + psx::kMaxFused * psx::kMaxTables;
  HIP_TRY(c, hipMemsetAsync(status, 0, sizeof(uint32_t), st));
  psx::StreamSet ss{};
  ss.n = 1;
  ss.data[0] = (const uint8_t *)stream;
  ss.size[0] = size;
  psx::TableDir dir{};
  dir.n = (int32_t)fmts.size();
  for (size_t i = 0; i < fmts.size(); ++i) {
    dir.table_id[i] = fmts[i].cfg.table_id;
    dir.vsize[i] = fmts[i].vsize;
    dir.dense_serialized[i] = fmts[i].cfg.oplog_dense_serialized;
    dir.dense_body[i] = fmts[i].dense_body();
  }
  psx::IdxSet ix{};
  ix.p[0] = record_offsets;
  uint64_t *recoff = reinterpret_cast<uint64_t *>(c->d_split_recoff);
  HIP_TRY(c, psx::launch_decode(ss, dir, segs, recoff, status, counters, ntouched, ix, ntouched + psx::kMaxTables,
                                nullptr, st));
  std::vector<psx::Seg> hs(psx::kMaxTables);
  uint32_t hst = 0;
  HIP_TRY(c, hipMemcpyAsync(hs.data(), segs, sizeof(psx::Seg) * psx::kMaxTables, hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(&hst, status, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  if (hst & psx::kStFatal) return sticky_error(c, hst);
  // 2) the message's tables with records, in stream order
  struct T { int ti; uint64_t first; };
  std::vector<T> order;
  for (int ti = 0; ti < dir.n; ++ti) {
    const psx::Seg &g = hs[ti];
    if (g.rec0 < 0 || g.num_rows <= 0) continue;
    uint64_t first = (uint64_t)g.rec0;
    if (g.sparse) HIP_TRY(c, hipMemcpy(&first, recoff + g.rec0, sizeof(uint64_t), hipMemcpyDeviceToHost));
    order.push_back({ti, first});
  }
  std::sort(order.begin(), order.end(), [](const T &a, const T &b) { return a.first < b.first; });
  const int ntab = (int)order.size();
  if (ntab == 0) return PSX_OK;
  std::vector<psx::SplitTab> tabs(ntab);
  int64_t nrec = 0;
  for (int j = 0; j < ntab; ++j) {
    const TableState &t = fmts[order[j].ti];
    const psx::Seg &g = hs[order[j].ti];
    tabs[j].k0 = nrec;
    tabs[j].rec0 = g.rec0;
    tabs[j].sparse = g.sparse;
    tabs[j].stride = t.dense_stride();
    tabs[j].vsize = t.vsize;
    nrec += g.num_rows;
  }
  const int64_t ntiles = (nrec + 63) / 64;
  const int64_t nb = (int64_t)nowners * ntiles;
  // scratch: tabs | src_off[nrec] meta[nrec] | tile_bytes[nb] tile_pre[nb+1] scan_tmp | ot_count ot_bytes |
  //          owner_base hdr_shift | words pos/val
  const size_t nscan = (size_t)((nb + 1023) / 1024) + 1;
  const size_t nwmax = (size_t)nowners * (1 + 4 * ntab);
  size_t off = 0;
  auto take = [&](size_t bytes) { const size_t at = off; off += (bytes + 255) / 256 * 256; return at; };
  const size_t o_tabs = take(sizeof(psx::SplitTab) * ntab), o_src = take(8 * nrec), o_meta = take(8 * nrec),
               o_tb = take(8 * nb), o_tp = take(8 * (nb + 1)), o_st = take(8 * nscan),
               o_oc = take(8 * (size_t)nowners * ntab), o_ob = take(8 * (size_t)nowners * ntab),
               o_base = take(8 * (size_t)nowners), o_hs = take(8 * (size_t)nowners * ntab), o_wp = take(8 * nwmax),
               o_wv = take(4 * nwmax);
  if ((e = grow(c->d_split_scratch, c->split_scratch_cap, off))) return e;
  uint8_t *sc = reinterpret_cast<uint8_t *>(c->d_split_scratch);
  psx::SplitArgs a{};
  a.msg = (const uint8_t *)stream;
  a.recoff = recoff;
  a.tabs = reinterpret_cast<const psx::SplitTab *>(sc + o_tabs);
  a.ntab = ntab;
  a.nowners = nowners;
  a.nrec = nrec;
  a.ntiles = ntiles;
  for (int o = 0; o <= nowners; ++o) a.row_begin[o] = row_begin[o];
  a.src_off = reinterpret_cast<uint64_t *>(sc + o_src);
  a.meta = reinterpret_cast<uint64_t *>(sc + o_meta);
  a.tile_bytes = reinterpret_cast<int64_t *>(sc + o_tb);
  a.tile_pre = reinterpret_cast<int64_t *>(sc + o_tp);
  a.scan_tmp = reinterpret_cast<int64_t *>(sc + o_st);
  a.ot_count = reinterpret_cast<int64_t *>(sc + o_oc);
  a.ot_bytes = reinterpret_cast<int64_t *>(sc + o_ob);
  a.owner_base = reinterpret_cast<const int64_t *>(sc + o_base);
  a.hdr_shift = reinterpret_cast<const int64_t *>(sc + o_hs);
  a.out = (uint8_t *)out;
  a.status = status;
  HIP_TRY(c, hipMemcpyAsync(sc + o_tabs, tabs.data(), sizeof(psx::SplitTab) * ntab, hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemsetAsync(a.tile_bytes, 0, 8 * nb, st));
  HIP_TRY(c, hipMemsetAsync(a.ot_count, 0, 8 * (size_t)nowners * ntab, st));
  HIP_TRY(c, hipMemsetAsync(a.ot_bytes, 0, 8 * (size_t)nowners * ntab, st));
  // 3) owners and sizes; per owner the tile bytes scanned
  HIP_TRY(c, psx::launch_split_count(a, st));
  std::vector<int64_t> cnt((size_t)nowners * ntab), byt((size_t)nowners * ntab);
  HIP_TRY(c, hipMemcpyAsync(cnt.data(), a.ot_count, 8 * cnt.size(), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(byt.data(), a.ot_bytes, 8 * byt.size(), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipMemcpyAsync(&hst, status, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  HIP_TRY(c, hipStreamSynchronize(st));
  if (hst & psx::kStFatal) return sticky_error(c, hst);
  // 4) every owner's message: int32 num_tables; per table {id, size_t update_size, num_rows}, records
  std::vector<int64_t> base(nowners), shift((size_t)nowners * ntab, 0);
  std::vector<int64_t> wpos;
  std::vector<uint32_t> wval;
  uint64_t total = 0;
  for (int o = 0; o < nowners; ++o) {
    int nt_o = 0;
    uint64_t rb = 0;
    for (int j = 0; j < ntab; ++j)
      if (cnt[(size_t)o * ntab + j]) ++nt_o, rb += (uint64_t)byt[(size_t)o * ntab + j];
    out_sizes[o] = nt_o ? 4 + 16 * (uint64_t)nt_o + rb : 0;
    base[o] = (int64_t)total;
    if (nt_o) {
      wpos.push_back(base[o]);
      wval.push_back((uint32_t)nt_o);
      int r = 0;
      uint64_t before = 0;
      for (int j = 0; j < ntab; ++j) {
        const int64_t n_oj = cnt[(size_t)o * ntab + j];
        if (!n_oj) continue;
        const int64_t hpos = base[o] + 4 + 16 * r + (int64_t)before;
        const TableState &t = fmts[order[j].ti];
        const uint64_t usz = (uint64_t)t.vsize;
        wpos.insert(wpos.end(), {hpos, hpos + 4, hpos + 8, hpos + 12});
        wval.insert(wval.end(), {(uint32_t)t.cfg.table_id, (uint32_t)usz, (uint32_t)(usz >> 32), (uint32_t)n_oj});
        ++r;
        shift[(size_t)o * ntab + j] = 4 + 16 * (int64_t)r;
        before += (uint64_t)byt[(size_t)o * ntab + j];
      }
    }
    total += out_sizes[o];
  }
  if (!out || out_cap < total)
    return fail(c, PSX_ERR_BUFFER_TOO_SMALL, "split output needs " + std::to_string(total) + " bytes");
  HIP_TRY(c, hipMemcpyAsync(sc + o_base, base.data(), 8 * base.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(sc + o_hs, shift.data(), 8 * shift.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(sc + o_wp, wpos.data(), 8 * wpos.size(), hipMemcpyHostToDevice, st));
  HIP_TRY(c, hipMemcpyAsync(sc + o_wv, wval.data(), 4 * wval.size(), hipMemcpyHostToDevice, st));
  // 5) records to their owners' messages, then the headers
  HIP_TRY(c, psx::launch_split_scatter(a, reinterpret_cast<const int64_t *>(sc + o_wp),
                                       reinterpret_cast<const uint32_t *>(sc + o_wv), (int32_t)wpos.size(), st));
  HIP_TRY(c, hipStreamSynchronize(st));   // the host vectors above are pageable
  return PSX_OK;
}

psx_status psx_split_stream(psx_ctx *c, const void *stream, size_t size, const uint64_t *record_offsets,
                            int32_t nowners, const int64_t *row_begin, void *out, size_t out_cap,
                            uint64_t *out_sizes) {
  if (!c) return PSX_ERR_INVALID_ARG;
  return split_impl(c, c->tables, stream, size, record_offsets, nowners, row_begin, out, out_cap, out_sizes);
}

psx_status psx_split_stream_formats(psx_ctx *c, const psx_table_config *formats, int32_t nformats,
                                    const void *stream, size_t size, const uint64_t *record_offsets,
                                    int32_t nowners, const int64_t *row_begin, void *out, size_t out_cap,
                                    uint64_t *out_sizes) {
  if (!c || nformats < 0 || nformats > psx::kMaxTables || (nformats && !formats)) return PSX_ERR_INVALID_ARG;
  std::vector<TableState> fmts((size_t)nformats);
  for (int32_t i = 0; i < nformats; ++i) {
    for (int32_t j = 0; j < i; ++j)
      if (formats[j].table_id == formats[i].table_id) return fail(c, PSX_ERR_INVALID_ARG, "table id twice in formats");
    psx_status e = table_format(c, &formats[i], fmts[(size_t)i]);
    if (e) return e;
  }
  return split_impl(c, fmts, stream, size, record_offsets, nowners, row_begin, out, out_cap, out_sizes);
}

psx_status psx_pack_stream(psx_ctx *c, const psx_pack_table *tables, int32_t n, void *out, size_t cap,
                           size_t *used, uint64_t *record_offsets) {
  return psx_pack_stream_indexed(c, tables, n, out, cap, used, record_offsets, nullptr);
}

psx_status psx_pack_stream_indexed(psx_ctx *c, const psx_pack_table *tables, int32_t n, void *out, size_t cap,
                                   size_t *used, uint64_t *record_offsets, int32_t *record_rows) {
  if (!c || !used || n < 0 || n > PSX_MAX_TABLES || (n && !tables)) return PSX_ERR_INVALID_ARG;
  *used = 0;
  if (out && ((uintptr_t)out & 3)) return fail(c, PSX_ERR_INVALID_ARG, "pack output must be 4-byte aligned");
  std::vector<const psx_pack_table *> live;
  for (int32_t i = 0; i < n; ++i) {
    const psx_pack_table &t = tables[i];
    if (t.dtype < PSX_F32 || t.dtype > PSX_I64 || t.capacity <= 0 || t.num_rows < 0 || t.reserved0 ||
        t.num_rows > INT32_MAX || (t.num_rows && (!t.row_ids || !t.oplogs)))
      return fail(c, PSX_ERR_INVALID_ARG, "bad psx_pack_table " + std::to_string(i));
    for (int32_t j = 0; j < i; ++j)
      if (tables[j].table_id == t.table_id) return fail(c, PSX_ERR_INVALID_ARG, "table listed twice");
    if (t.num_rows) live.push_back(&t);
  }
  // OpLogSerializer keeps tables in a std::map: ascending table id (oplog_serializer.hpp:12-37)
  std::sort(live.begin(), live.end(),
            [](const psx_pack_table *a, const psx_pack_table *b) { return a->table_id < b->table_id; });
  if (live.empty()) return PSX_OK;   // empty message (abstract_bg_worker.cpp:670-682)
  HIP_TRY(c, hipSetDevice(c->device));
  // scratch: per sparse table sizes[n] + offs[n + 1 + tiles]
  size_t need = 0;
  for (auto *t : live)
    if (!t->dense_serialized) need += 2 * (size_t)t->num_rows + 1 + ((size_t)t->num_rows + 1023) / 1024;
  if (need > c->pack_cap) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->d_pack) hipFree(c->d_pack);
    c->d_pack = nullptr;
    c->pack_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_pack, need * sizeof(int64_t)));
    c->pack_cap = need;
  }
  std::vector<psx::PackTab> pt(live.size());
  size_t sc = 0;
  std::vector<int64_t> bytes(live.size(), 0);
  for (size_t k = 0; k < live.size(); ++k) {
    const psx_pack_table &t = *live[k];
    psx::PackTab &p = pt[k];
    p = psx::PackTab{};
    p.row_ids = t.row_ids;
    p.oplogs = (const uint8_t *)t.oplogs;
    p.nrows = t.num_rows;
    p.cap = t.capacity;
    p.vsize = vsize_of(t.dtype);
    p.sparse = t.dense_serialized ? 0 : 1;
    p.src16 = ((uintptr_t)t.oplogs % 16 == 0 && (t.capacity * p.vsize) % 16 == 0) ? 1 : 0;
    if (p.sparse) {
      p.sizes = c->d_pack + sc;
      p.offs = p.sizes + t.num_rows;
      sc += 2 * (size_t)t.num_rows + 1 + ((size_t)t.num_rows + 1023) / 1024;
      HIP_TRY(c, psx::launch_pack_count(t.dtype, p, c->stream));
      HIP_TRY(c, hipMemcpyAsync(&bytes[k], p.offs + t.num_rows, sizeof(int64_t), hipMemcpyDeviceToHost, c->stream));
    } else {
      bytes[k] = t.num_rows * (4 + t.capacity * p.vsize);
    }
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  // layout: int32 num_tables; per table {int32 id; size_t update_size; int32 num_rows} + records
  psx::PackHdr h{};
  h.pos[0] = 0;
  h.len[0] = 1;
  h.w[0][0] = (uint32_t)live.size();
  h.n = 1;
  int64_t pos = 4, rec_base = 0;
  for (size_t k = 0; k < live.size(); ++k) {
    const psx_pack_table &t = *live[k];
    h.pos[h.n] = pos;
    h.len[h.n] = 4;
    h.w[h.n][0] = (uint32_t)t.table_id;
    h.w[h.n][1] = (uint32_t)pt[k].vsize;   // size_t update_size, little endian
    h.w[h.n][2] = 0;
    h.w[h.n][3] = (uint32_t)t.num_rows;
    h.n++;
    pos += 16;
    pt[k].rec0 = pos;
    pt[k].rec_base = rec_base;
    rec_base += t.num_rows;
    pos += bytes[k];
  }
  *used = (size_t)pos;
  if (!out || (size_t)pos > cap) return fail(c, PSX_ERR_BUFFER_TOO_SMALL, "pack: *used bytes needed");
  for (size_t k = 0; k < live.size(); ++k) {
    HIP_TRY(c, psx::launch_pack_emit(live[k]->dtype, pt[k], (uint8_t *)out, record_offsets, c->stream));
    // the record-row list: the rows packed, in record order (what the producer already holds)
    if (record_rows)
      HIP_TRY(c, hipMemcpyAsync(record_rows + pt[k].rec_base, live[k]->row_ids, sizeof(int32_t) * live[k]->num_rows,
                                hipMemcpyDeviceToDevice, c->stream));
  }
  HIP_TRY(c, psx::launch_pack_header((uint8_t *)out, h, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

// ---- subscriptions and the per-client push (SSPPush) ---------------------------------

static psx_status ensure_subs(psx_ctx *c, TableState &t) {
  if (t.d_subs) return PSX_OK;
  const size_t R = (size_t)t.cfg.max_rows;
  HIP_TRY(c, hipMalloc(&t.d_subs, R * sizeof(uint64_t)));
  HIP_TRY(c, hipMemsetAsync(t.d_subs, 0, R * sizeof(uint64_t), c->stream));
  return PSX_OK;
}

psx_status psx_row_subscribe(psx_ctx *c, int32_t table_id, const int32_t *row_ids, int32_t n, int32_t client_id) {
  if (!c || n < 0 || (n && !row_ids) || client_id < 0 || client_id >= PSX_MAX_CLIENTS) return PSX_ERR_INVALID_ARG;
  int ti = 0;
  TableState *t = find_table(c, table_id, &ti);
  if (!t) return fail(c, PSX_ERR_UNKNOWN_TABLE, "unknown table");
  if (n == 0) return PSX_OK;
  std::vector<int64_t> slots(n);
  for (int32_t i = 0; i < n; ++i) {
    slots[i] = slot_of(*t, row_ids[i]);
    if (slots[i] < 0) return fail(c, PSX_ERR_ROW_RANGE, "row " + std::to_string(row_ids[i]) + " not owned by this shard");
  }
  psx_status st = sync_impl(c);
  if (st) return st;
  st = ensure_subs(c, *t);
  if (st) return st;
  int64_t *d_slots = nullptr;
  HIP_TRY(c, hipMalloc(&d_slots, sizeof(int64_t) * n));
  std::unique_ptr<int64_t, decltype(&hipFree)> hold(d_slots, &hipFree);
  HIP_TRY(c, hipMemcpyAsync(d_slots, slots.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, c->stream));
  if (t->ada && t->ada_cfg.gaussian_init) {
    // ServerTable::CreateRow -> ServerRowCreated for the rows that do not exist yet, in
    // request order (adarevision_server_table_logic.cpp:38-50): N(0, 0.1) draws of the
    // table's generator added to the zero row
    std::vector<uint8_t> flags(n);
    uint8_t *d_flags = nullptr;
    HIP_TRY(c, hipMalloc(&d_flags, n));
    std::unique_ptr<uint8_t, decltype(&hipFree)> hold_f(d_flags, &hipFree);
    HIP_TRY(c, psx::launch_gather_flags(t->d_flags, d_slots, n, d_flags, c->stream));
    HIP_TRY(c, hipMemcpyAsync(flags.data(), d_flags, n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    std::vector<int32_t> fresh;
    for (int32_t i = 0; i < n; ++i)
      if (!(flags[i] & 1) && std::find(fresh.begin(), fresh.end(), (int32_t)slots[i]) == fresh.end())
        fresh.push_back((int32_t)slots[i]);
    if (!fresh.empty()) {
      const size_t cap = (size_t)t->cfg.row_capacity;
      std::vector<float> d(fresh.size() * cap);
      for (float &x : d) x = (*t->ada_dist)(*t->ada_gen);
      int32_t *d_fresh = nullptr;
      float *d_vals = nullptr;
      HIP_TRY(c, hipMalloc(&d_fresh, sizeof(int32_t) * fresh.size()));
      std::unique_ptr<int32_t, decltype(&hipFree)> hold_s(d_fresh, &hipFree);
      HIP_TRY(c, hipMalloc(&d_vals, sizeof(float) * d.size()));
      std::unique_ptr<float, decltype(&hipFree)> hold_v(d_vals, &hipFree);
      HIP_TRY(c, hipMemcpyAsync(d_fresh, fresh.data(), sizeof(int32_t) * fresh.size(), hipMemcpyHostToDevice,
                                c->stream));
      HIP_TRY(c, hipMemcpyAsync(d_vals, d.data(), sizeof(float) * d.size(), hipMemcpyHostToDevice, c->stream));
      HIP_TRY(c, psx::launch_ada_init_rows(ada_args(*t, ti), d_fresh, d_vals, (int32_t)fresh.size(), c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
  }
  HIP_TRY(c, psx::launch_subscribe(t->d_flags, t->d_subs, d_slots, n, (uint64_t)1 << client_id, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_row_subscriptions(psx_ctx *c, int32_t table_id, int64_t first_row, int64_t num_rows, uint64_t *dst) {
  if (!c || (!dst && num_rows)) return PSX_ERR_INVALID_ARG;
  TableState *t;
  int64_t s;
  psx_status st = row_range(c, table_id, first_row, num_rows, &t, &s);
  if (st) return st;
  if (!t->d_subs) {
    for (int64_t i = 0; i < num_rows; ++i) dst[i] = 0;
    return PSX_OK;
  }
  HIP_TRY(c, hipMemcpyAsync(dst, t->d_subs + s, sizeof(uint64_t) * (size_t)num_rows, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  return PSX_OK;
}

psx_status psx_serialize_push(psx_ctx *c, void *const *out, const size_t *cap, size_t *used, int32_t out_on_device,
                              int32_t clear_dirty) {
  if (!c || !used || !cap) return PSX_ERR_INVALID_ARG;
  const int C = c->num_clients;
  for (int k = 0; k < C; ++k) {
    used[k] = 0;
    if (out && out[k] && out_on_device && ((uintptr_t)out[k] & 3))
      return fail(c, PSX_ERR_INVALID_ARG, "device outputs must be 4-byte aligned");
  }
  psx_status st = sync_impl(c);
  if (st) return st;
  const size_t T = c->tables.size();
  std::vector<psx::ServeArgs> args(T);
  for (size_t i = 0; i < T; ++i) {
    st = serve_args(c, c->tables[i], &args[i]);
    if (st) return st;
    st = ensure_subs(c, c->tables[i]);
    if (st) return st;
    args[i].subs = c->tables[i].d_subs;
  }
  // sizes: per client, per table {table_id, records, -1 | -2}
  std::vector<std::vector<int64_t>> tot(C, std::vector<int64_t>(T, 0));
  bool small = false;
  for (int k = 0; k < C; ++k) {
    int64_t pos = 0;
    for (size_t i = 0; i < T; ++i) {
      args[i].cmask = (uint64_t)1 << k;
      HIP_TRY(c, psx::launch_serve_sizes(args[i], c->stream));
      HIP_TRY(c, hipMemcpyAsync(&tot[k][i], args[i].offs + args[i].max_rows, sizeof(int64_t), hipMemcpyDeviceToHost,
                                c->stream));
      HIP_TRY(c, hipStreamSynchronize(c->stream));
      pos += 8 + tot[k][i];
    }
    used[k] = (size_t)pos;
    if (used[k] > cap[k] || !out || !out[k]) small = true;
  }
  if (small) return fail(c, PSX_ERR_BUFFER_TOO_SMALL, "serialize_push: used[] bytes needed");
  // ServerRowSent must not fail after a row was cleared: check every AdaRevision table first
  for (size_t i = 0; i < T && clear_dirty; ++i) {
    TableState &t = c->tables[i];
    if (!t.ada) continue;
    args[i].cmask = ~(uint64_t)0;
    HIP_TRY(c, psx::launch_serve_sizes(args[i], c->stream));
    st = ada_rows_sent(c, t, (int)i, nullptr, args[i].sizes, args[i].max_rows, 0, t.d_subs, true);
    if (st) {
      for (int k = 0; k < C; ++k) used[k] = 0;
      return st;
    }
  }
  // host outputs: every client's body staged in its own part of one device buffer, so
  // that each body's copy to host starts as soon as it is emitted and the copies run back
  // to back on two streams (the emits are ~1% of the copy time; PCIe is the limit)
  size_t stage = 0;
  for (int k = 0; k < C; ++k) stage += (used[k] + 3) & ~(size_t)3;
  if (!out_on_device && stage > c->staging_cap) {
    if (c->d_staging) hipFree(c->d_staging);
    c->d_staging = nullptr;
    c->staging_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_staging, stage));
    c->staging_cap = stage;
  }
  hipStream_t copy_st[2] = {c->side, c->aux};
  size_t soff = 0;
  for (int k = 0; k < C; ++k) {
    uint8_t *dst = out_on_device ? (uint8_t *)out[k] : c->d_staging + soff;
    soff += (used[k] + 3) & ~(size_t)3;
    psx::Words w{};
    int64_t pos = 0;
    for (size_t i = 0; i < T; ++i) {
      w.pos[w.n] = pos;
      w.val[w.n++] = c->tables[i].cfg.table_id;
      pos += 4;
      args[i].cmask = (uint64_t)1 << k;
      args[i].out = dst + pos;
      args[i].flags_rw = nullptr;   // cleared once, after every client's body
      args[i].imp_rw = nullptr;
      if (tot[k][i]) {
        HIP_TRY(c, psx::launch_serve_sizes(args[i], c->stream));
        HIP_TRY(c, psx::launch_serve_emit(args[i], c->stream));
      }
      pos += tot[k][i];
      w.pos[w.n] = pos;
      w.val[w.n++] = i + 1 < T ? -1 : -2;
      pos += 4;
    }
    HIP_TRY(c, psx::launch_put_words(dst, w, c->stream));
    if (!out_on_device) {
      hipStream_t cs = copy_st[k & 1];
      HIP_TRY(c, hipEventRecord(c->ev_push[k & 1], c->stream));
      HIP_TRY(c, hipStreamWaitEvent(cs, c->ev_push[k & 1], 0));
      HIP_TRY(c, hipMemcpyAsync(out[k], dst, used[k], hipMemcpyDeviceToHost, cs));
    }
  }
  if (clear_dirty) {
    for (size_t i = 0; i < T; ++i) {
      TableState &t = c->tables[i];
      if (t.ada) {   // ServerRowSent(row, version, subscriber count) (server_table.cpp:250-255)
        args[i].cmask = ~(uint64_t)0;
        HIP_TRY(c, psx::launch_serve_sizes(args[i], c->stream));
        st = ada_rows_sent(c, t, (int)i, nullptr, args[i].sizes, args[i].max_rows, 0, t.d_subs, false);
        if (st) return st;
      }
      HIP_TRY(c, psx::launch_serve_clear(t.d_flags, t.d_imp, t.d_subs, t.cfg.max_rows, c->stream));
    }
  }
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (!out_on_device) {
    HIP_TRY(c, hipStreamSynchronize(copy_st[0]));
    HIP_TRY(c, hipStreamSynchronize(copy_st[1]));
  }
  return PSX_OK;
}

// ---- client side of serve-back ----------------------------------------------------------

psx_status psx_apply_push_body(psx_ctx *c, const void *body, size_t size, int32_t body_on_device,
                               int32_t insert_missing) {
  if (!c || (size && !body)) return PSX_ERR_INVALID_ARG;
  if (body_on_device && ((uintptr_t)body & 3)) return fail(c, PSX_ERR_INVALID_ARG, "device body must be 4-byte aligned");
  if (size == 0) return PSX_OK;
  psx_status st = sync_impl(c);
  if (st) return st;
  for (auto &t : c->tables)
    if (t.cfg.row_bytes_f16 && (t.cfg.row_capacity & 1))
      return fail(c, PSX_ERR_UNSUPPORTED, "push bodies of binary16 rows of odd width (2-byte records) are not walked on "
                                          "the device");
  const size_t max_ent = size / 12 + 1;
  if (!body_on_device && size > c->push_body_cap) {
    if (c->d_push_body) hipFree(c->d_push_body);
    c->d_push_body = nullptr;
    c->push_body_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_push_body, size));
    c->push_body_cap = size;
  }
  if (max_ent > c->push_ent_cap) {
    if (c->d_push_ent) hipFree(c->d_push_ent);
    c->d_push_ent = nullptr;
    c->push_ent_cap = 0;
    HIP_TRY(c, hipMalloc(&c->d_push_ent, max_ent * sizeof(psx::PushEntry)));
    c->push_ent_cap = max_ent;
  }
  if (!c->d_push_words) HIP_TRY(c, hipMalloc(&c->d_push_words, 2 * sizeof(uint32_t)));
  if (!c->d_client_tabs) HIP_TRY(c, hipMalloc(&c->d_client_tabs, psx::kMaxTables * sizeof(psx::ClientTable)));
  std::vector<psx::ClientTable> ct(c->tables.size());
  for (size_t i = 0; i < c->tables.size(); ++i) {
    TableState &t = c->tables[i];
    psx::ClientTable &x = ct[i];
    x = psx::ClientTable{};
    x.table_id = t.cfg.table_id;
    x.kind = t.cfg.row_kind;
    x.vsize = t.vsize;
    x.es = t.es;
    x.row_cap = t.cfg.row_capacity;
    x.max_entries = t.max_entries;
    x.row_offset = t.cfg.row_offset;
    x.row_stride = t.cfg.row_stride;
    x.max_rows = t.cfg.max_rows;
    x.flags = t.d_flags;
    x.dense = (uint8_t *)t.d_data;
    x.entries = t.d_entries;
    x.nent = t.d_nent;
    x.ver = t.d_ver;
    x.claim = t.d_cnt;   // the ordered path's per-slot counts: zero between calls
    x.f16 = t.cfg.row_bytes_f16;
  }
  const uint8_t *dbody = (const uint8_t *)body;
  if (!body_on_device) {
    HIP_TRY(c, hipMemcpyAsync(c->d_push_body, body, size, hipMemcpyHostToDevice, c->stream));
    dbody = c->d_push_body;
  }
  HIP_TRY(c, hipMemcpyAsync(c->d_client_tabs, ct.data(), ct.size() * sizeof(psx::ClientTable), hipMemcpyHostToDevice,
                            c->stream));
  HIP_TRY(c, hipMemsetAsync(c->d_push_words, 0, 2 * sizeof(uint32_t), c->stream));
  uint32_t *nent = c->d_push_words, *status = c->d_push_words + 1;
  st = timed(c, "push_walk", [&] {
    return psx::launch_push_walk(dbody, size, c->d_push_ent, nent, (uint32_t)max_ent, status, c->stream);
  });
  if (st) return st;
  st = timed(c, "push_apply", [&] {
    return psx::launch_push_apply(dbody, c->d_push_ent, nent, (uint32_t)max_ent, c->d_client_tabs, (int)ct.size(),
                                  insert_missing ? 1 : 0, status, c->stream);
  });
  if (st) return st;
  uint32_t words[2] = {0, 0};
  HIP_TRY(c, hipMemcpyAsync(words, c->d_push_words, sizeof(words), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  if (words[1] & psx::kStUnknownTable) return fail(c, PSX_ERR_UNKNOWN_TABLE, "push body names a table this context lacks");
  if (words[1] & psx::kStMalformed) return fail(c, PSX_ERR_MALFORMED, "malformed push body");
  if (words[1] & psx::kStCapacity) return fail(c, PSX_ERR_CAPACITY, "pushed row exceeds max_entries");
  return PSX_OK;
}

// ---- message headers (ps_msgs.hpp / msg_base.hpp) ---------------------------------------

namespace {
void put32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
void put64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
}  // namespace

// ArbitrarySizedMsg prefix: MsgType(4) seq(8) ack(8) avai_size(8) (msg_base.hpp:81-188)
psx_status psx_encode_oplog_header(const psx_oplog_msg_header *h, void *out) {
  if (!h || !out) return PSX_ERR_INVALID_ARG;
  uint8_t *p = (uint8_t *)out;
  put32(p + 0, (uint32_t)PSX_MSG_CLIENT_SEND_OPLOG);
  put64(p + 4, h->seq_num);
  put64(p + 12, h->ack_num);
  put64(p + 20, h->avai_size);
  p[28] = h->is_clock ? 1 : 0;                 // bool is_clock (ps_msgs.hpp:1018-1021)
  put32(p + 29, (uint32_t)h->client_id);       // :1023-1026
  put32(p + 33, h->version);                   // :1028-1032
  put32(p + 37, (uint32_t)h->bg_clock);        // :1034-1038
  return PSX_OK;
}

psx_status psx_decode_oplog_header(const void *msg, size_t msg_size, psx_oplog_msg_header *h) {
  if (!msg || !h) return PSX_ERR_INVALID_ARG;
  if (msg_size < PSX_OPLOG_MSG_HEADER_BYTES) return PSX_ERR_MALFORMED;
  const uint8_t *p = (const uint8_t *)msg;
  if ((int32_t)rd32h(p) != PSX_MSG_CLIENT_SEND_OPLOG) return PSX_ERR_MALFORMED;
  h->seq_num = rd64h(p + 4);
  h->ack_num = rd64h(p + 12);
  h->avai_size = rd64h(p + 20);
  h->is_clock = p[28] ? 1 : 0;
  h->client_id = (int32_t)rd32h(p + 29);
  h->version = rd32h(p + 33);
  h->bg_clock = (int32_t)rd32h(p + 37);
  // get_size() = header + avai_size (:1045-1048): the payload must be all there
  if (h->avai_size > msg_size - PSX_OPLOG_MSG_HEADER_BYTES) return PSX_ERR_MALFORMED;
  return PSX_OK;
}

psx_status psx_encode_push_header(const psx_push_msg_header *h, void *out) {
  if (!h || !out) return PSX_ERR_INVALID_ARG;
  uint8_t *p = (uint8_t *)out;
  put32(p + 0, (uint32_t)PSX_MSG_SERVER_PUSH_ROW);
  put64(p + 4, h->seq_num);
  put64(p + 12, h->ack_num);
  put64(p + 20, h->avai_size);
  put32(p + 28, (uint32_t)h->clock);           // ServerPushRowMsg::get_clock (ps_msgs.hpp:1072-1075)
  put32(p + 32, h->version);                   // :1077-1080
  p[36] = h->is_clock ? 1 : 0;                 // :1082-1086
  return PSX_OK;
}

psx_status psx_decode_push_header(const void *msg, size_t msg_size, psx_push_msg_header *h) {
  if (!msg || !h) return PSX_ERR_INVALID_ARG;
  if (msg_size < PSX_PUSH_MSG_HEADER_BYTES) return PSX_ERR_MALFORMED;
  const uint8_t *p = (const uint8_t *)msg;
  if ((int32_t)rd32h(p) != PSX_MSG_SERVER_PUSH_ROW) return PSX_ERR_MALFORMED;
  h->seq_num = rd64h(p + 4);
  h->ack_num = rd64h(p + 12);
  h->avai_size = rd64h(p + 20);
  h->clock = (int32_t)rd32h(p + 28);
  h->version = rd32h(p + 32);
  h->is_clock = p[36] ? 1 : 0;
  if (h->avai_size > msg_size - PSX_PUSH_MSG_HEADER_BYTES) return PSX_ERR_MALFORMED;
  return PSX_OK;
}

psx_status psx_ctx_set_pipeline(psx_ctx *c, int32_t mode) {
  if (!c || mode < 0 || mode > PSX_PIPELINE_ALL) return PSX_ERR_INVALID_ARG;
  if (mode != c->pipeline) {
    // no call in flight across the change: the slot-free events are recorded only while
    // pipelining, so the first pipelined call must not find a slot still in use
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->side));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
  }
  c->pipeline = mode;
  return PSX_OK;
}

psx_status psx_ctx_set_seam(psx_ctx *c, int32_t mode) {
  if (!c || (mode != PSX_SEAM_ASYNC && mode != PSX_SEAM_SYNC)) return PSX_ERR_INVALID_ARG;
  c->seam_mode = mode;
  return PSX_OK;
}

psx_status psx_ctx_set_compat(psx_ctx *c, int32_t flags) {
  if (!c || (flags & ~PSX_COMPAT_INT32_STREAM_OFFSETS)) return PSX_ERR_INVALID_ARG;
  c->compat = flags;
  return PSX_OK;
}

psx_status psx_handle_oplog_msg(psx_ctx *c, const void *msg, size_t msg_size, int32_t sender,
                                int32_t *clock_changed) {
  if (!c || !msg || !clock_changed) return PSX_ERR_INVALID_ARG;
  *clock_changed = 0;
  psx_oplog_msg_header h;
  psx_status st = psx_decode_oplog_header(msg, msg_size, &h);
  if (st) return fail(c, st, "not a ClientSendOpLogMsg (41-byte header + avai_size payload bytes)");
  st = psx_apply_stream(c, (const uint8_t *)msg + PSX_OPLOG_MSG_HEADER_BYTES, (size_t)h.avai_size, sender, h.version);
  if (st) return st;
  if (h.is_clock) {
    int32_t changed = 0;
    st = psx_clock_until(c, sender, h.bg_clock, &changed);
    if (st) return st;
    *clock_changed = changed;
  }
  return PSX_OK;
}

const char *psx_last_error(psx_ctx *c) { return c ? c->err.c_str() : "null context"; }

psx_status psx_timing_enable(psx_ctx *c, int32_t on) {
  if (!c) return PSX_ERR_INVALID_ARG;
  if (on < 0 || on > 2) return fail(c, PSX_ERR_INVALID_ARG, "timing mode is 0, 1 or 2");
  c->timing = on;
  return PSX_OK;
}

psx_status psx_timing_read(psx_ctx *c, const char *kernel, double *total_ms, int64_t *launches) {
  if (!c || !kernel || !total_ms || !launches) return PSX_ERR_INVALID_ARG;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  collect_timing(c);
  auto it = c->times.find(kernel);
  *total_ms = it == c->times.end() ? 0.0 : it->second.first;
  *launches = it == c->times.end() ? 0 : it->second.second;
  return PSX_OK;
}

psx_status psx_ctx_stats(psx_ctx *c, psx_apply_stats *out, int32_t reset) {
  if (!c) return PSX_ERR_INVALID_ARG;
  if (out) *out = c->stats;
  if (reset) {
    c->stats = psx_apply_stats{};
    // the open interval's calls went out with the reset: restart it, so the next sync adds
    // only the device time of calls made after the reset
    if (c->stats_open) c->ev_pool.push_back(c->stats_open);
    c->stats_open = nullptr;
    c->stats_open_calls = 0;
  }
  return PSX_OK;
}

psx_status psx_timing_reset(psx_ctx *c) {
  if (!c) return PSX_ERR_INVALID_ARG;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(c->stream));
  collect_timing(c);
  c->times.clear();
  return PSX_OK;
}

}  // extern "C"

// ---- kernel selectors (include/psx_debug.h) ------------------------------------
#include "../../include/psx_debug.h"
namespace psx {
extern int g_apply_variant;
extern int g_dense_last;
extern int g_classify_blocks;
extern int g_classify_dry;
extern int g_ord_split;
extern int g_offsets_blocks;
extern int g_dry_blocks;
}  // namespace psx

static int *variant_slot(int32_t which) {
  switch (which) {
    case PSX_VARIANT_DENSE_APPLY: return &psx::g_apply_variant;
    case PSX_VARIANT_ORD_SPLIT: return &psx::g_ord_split;
    case PSX_VARIANT_DECODE: return &psx::g_decode_walk;
    case PSX_STAT_WALK_CALLS: return &psx::g_walk_calls;
    case PSX_STAT_DENSE_LAST: return &psx::g_dense_last;
    case PSX_VARIANT_PREP_HALVES: return &psx::g_prep_halves;
    case PSX_VARIANT_CLASSIFY_GRID: return &psx::g_classify_blocks;
    case PSX_VARIANT_CLASSIFY_DRY: return &psx::g_classify_dry;
    case PSX_VARIANT_WALK_CUS_PIPELINED: return &psx::g_walk_cus_pipelined;
    case PSX_VARIANT_STREAM_PRIORITY: return &psx::g_stream_priority;
    case PSX_VARIANT_ORD_BUCKET: return &psx::g_ord_bucket;
    case PSX_VARIANT_PIPE_SLOTS: return &psx::g_pipe_slots;
    case PSX_VARIANT_SIDE_CU_MASK: return &psx::g_side_cu_mask;
    case PSX_VARIANT_EVENT_SCOPE: return &psx::g_event_scope;
    case PSX_VARIANT_DENSE_STORE: return &psx::g_dense_store_nt;
    case PSX_DEBUG_WALK_TRACE: return &psx::g_walk_trace;
    case PSX_VARIANT_WALK_CUS: return &psx::g_walk_all_cus;
    case PSX_VARIANT_WALK_COUNT: return &psx::g_walk_count;
    case PSX_VARIANT_FOLD_FINISH: return &psx::g_fold_finish;
    case PSX_VARIANT_WALK_LEVELS: return &psx::g_walk_levels;
    case PSX_DEBUG_WALK_SKEW: return &psx::g_walk_skew;
    case PSX_VARIANT_ORD_LITE: return &psx::g_ord_lite;
#ifdef PSX_DEBUG_BUILD
    case PSX_DEBUG_ORD_PROBE: return &psx::g_ord_probe;   // timing probes: results wrong
#endif
    case PSX_VARIANT_WALK_SHAPE: return &psx::g_walk_shape;
    case PSX_VARIANT_CALL_EVENTS: return &psx::g_call_events;
    case PSX_VARIANT_OFFSETS_GRID: return &psx::g_offsets_blocks;
    case PSX_VARIANT_DRY_GRID: return &psx::g_dry_blocks;
    case PSX_VARIANT_WALK_RANK: return &psx::g_walk_rank;
    default: return nullptr;
  }
}

extern "C" int32_t psx_debug_set_variant(int32_t which, int32_t variant) {
  int *v = variant_slot(which);
  if (!v) return -1;
  int old = *v;
  *v = variant;
  return old;
}

extern "C" int32_t psx_debug_get_variant(int32_t which) {
  int *v = variant_slot(which);
  return v ? *v : -1;
}

extern "C" int64_t psx_debug_walk_trace(psx_ctx *c, uint64_t *out, int64_t max_items) {
  if (!c || !out || max_items < 0) return -1;
  const int k = c->walk_last_slot;
  const uint64_t items = c->walk_last_items;
  if (!c->d_walk[k] || !items) return 0;
  if (hipStreamSynchronize(c->stream) != hipSuccess || hipStreamSynchronize(c->side) != hipSuccess) return -1;
  const uint64_t n = std::min<uint64_t>(items, (uint64_t)max_items);
  if (hipMemcpy(out, reinterpret_cast<uint8_t *>(c->d_walk[k]) + psx::walk_trace_offset(items), n * 10 * sizeof(uint64_t),
                hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (int64_t)items;
}

#ifdef PSX_DEBUG_BUILD
namespace {
// Debug build only (`make debug` -> libpsx_debug.so, loaded through PSX_LIB): the
// PSX_* variables override the kernel selectors at load time, for the A/B runs of
// tools/gpu_run.sh.  The shipped libpsx.so reads no such variable (a stray
// variable in a user's environment must not change an apply); there the selectors are
// reachable only through psx_debug_set_variant.
struct VariantEnv {
  VariantEnv() {
    if (const char *v = getenv("PSX_APPLY_VARIANT")) psx::g_apply_variant = atoi(v);
    if (const char *v = getenv("PSX_ORD_SPLIT")) psx::g_ord_split = atoi(v);
    if (const char *v = getenv("PSX_ORD_LITE")) psx::g_ord_lite = atoi(v);
    if (const char *v = getenv("PSX_PREP_HALVES")) psx::g_prep_halves = atoi(v);
    if (const char *v = getenv("PSX_CLASSIFY_DRY")) psx::g_classify_dry = atoi(v);
    if (const char *v = getenv("PSX_ORD_BUCKET")) psx::g_ord_bucket = atoi(v);
    if (const char *v = getenv("PSX_PIPE_SLOTS")) psx::g_pipe_slots = atoi(v);
    if (const char *v = getenv("PSX_ORD_PROBE")) psx::g_ord_probe = atoi(v);
    if (const char *v = getenv("PSX_DECODE_WALK")) psx::g_decode_walk = atoi(v);
    if (const char *v = getenv("PSX_DENSE_STORE_NT")) psx::g_dense_store_nt = atoi(v);
    if (const char *v = getenv("PSX_WALK_CUS")) psx::g_walk_all_cus = atoi(v);
    if (const char *v = getenv("PSX_WALK_COUNT")) psx::g_walk_count = atoi(v);
    if (const char *v = getenv("PSX_FOLD_FINISH")) psx::g_fold_finish = atoi(v);
    if (const char *v = getenv("PSX_WALK_LEVELS")) psx::g_walk_levels = atoi(v);
    if (const char *v = getenv("PSX_WALK_SHAPE")) psx::g_walk_shape = atoi(v);
  }
} variant_env;
}  // namespace
#endif  // PSX_DEBUG_BUILD
