// psx_walk.hip — window-parallel decode of walked messages that hold sparse tables.
//
// The record chain of a sparse table (SerializedOpLogReader::Next,
// src/petuum_ps/server/serialized_oplog_reader.hpp:50-85: each record's size comes from its
// own n, so record k+1 starts where record k ends) is sequential.  decode_streams walks it
// with one workgroup per message, one 32 KiB window after another.  Here every 96 KiB window of
// every message is its own work item, and the work that does not depend on where the chain
// enters the window runs in parallel, before the chain arrives:
//
//   walk_head   one small block per message: per-call resets, the table headers up to the
//               first sparse table with records (dense tables are O(1) each), the message's
//               window range, the walker state at that table's first record.
//   walk        persistent blocks of 1,024 threads take (window, message) tickets in
//               window-major order.  Per window, speculatively for EVERY word q as a record
//               start: the 1- and 16-record jump tables, then pointer jumping to the LAST
//               record start on q's chain inside the window and the record count up to it
//               (the window's exit map).  Then one wave waits for the predecessor window's
//               walker state (8-byte {tag, value} granules written by atomics: the data is
//               the flag, no fence — cdna_hip_programming.md, publish/consume recipe R2),
//               resolves its own state in O(1) per table (one exit-map lookup per sparse
//               table, headers read directly), publishes, and only then expands its records'
//               offsets into recoff with the jump tables.
//
// The chain between windows costs one granule hand-off per window instead of a full window
// walk.  Output (segs, recoff, counters, the status bits) is exactly decode_streams'.
// Eligible calls (psx_runtime.cpp): no producer record offsets, every sparse table of the
// context with one value size (the speculation uses that record pair size), and at most
// kWalkMaxItems window items; the others run decode_streams.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "psx_device.hpp"

namespace psx {

// Walk shapes (PSX_VARIANT_WALK_SHAPE): threads per block x words per window.  A window's
// speculative work is LDS-bound inside its CU, so smaller windows spread one call's work
// over more CUs (several blocks per CU) at the price of more window-to-window hand-offs.
struct WalkShape {
  int threads, words, cand;   // cand: entry candidates (exit maps), at most threads
};
constexpr WalkShape kWalkShapes[] = {{1024, 24576, 1024}, {1024, 8192, 1024}, {512, 6144, 512}, {256, 4096, 256},
                                     {512, 12288, 512},   {512, 12288, 256},  {512, 12288, 128}};
constexpr int kNumWalkShapes = (int)(sizeof(kWalkShapes) / sizeof(kWalkShapes[0]));
uint64_t walk_window_bytes(int shape) {
  return (uint64_t)kWalkShapes[shape >= 0 && shape < kNumWalkShapes ? shape : 0].words * 4;
}
constexpr uint16_t kNo = 0xFFFFu;               // next record outside the window / bad header
// n16: the record count word after q (q's n as a record start), clipped to 16 bits
constexpr uint16_t kNBig = 0xFFFDu;             // n >= kNBig (read the word itself)
constexpr uint16_t kNNeg = 0xFFFEu;             // n < 0
constexpr uint16_t kNNone = 0xFFFFu;            // no such word (past the window and its halo)
constexpr int kGran = 14;                       // granules per published walker state
constexpr int kMaxSegs = kMaxTables;            // sparse tables with records in one window

typedef unsigned long long __attribute__((address_space(1))) gu64;

// Workspace of one call slot: [WalkCtl][WalkHead][granules: kGran per window item].
// walk_head resets the ticket for its call; the granules carry the call's epoch as tag.
constexpr size_t kWalkHeadOff = 256;

// Walker state between windows.  mode 0: the next table header is at pos; 1: inside sparse
// table t, `left` records still to walk, the next one at pos; 2: message done (or failed).
struct WalkState {
  uint64_t pos, left, rk, kk, seen;   // rk: next recoff index; kk: records before pos (all tables);
  int32_t k, t, mode, ntab;           // seen: bit t = table t met in this message (duplicate check)
};

struct WalkCtl {      // reset by walk_head for the walk of the same call
  uint32_t ticket;
  uint32_t lost;      // 1 once a hand-off timed out; dbg then holds the first one:
  uint32_t dbg[6];    // {ticket, message, window, epoch expected, tag seen (lane 0), lanes tagged}
};

struct WalkHead {     // written by walk_head, read by the first window of each message
  WalkState st[kMaxFused];
  uint32_t wfirst[kMaxFused];   // the message's first window (window grid from byte 0)
  uint32_t nwin[kMaxFused];     // its window count (0: nothing left to walk)
};
constexpr size_t kWalkGranOff = kWalkHeadOff + (sizeof(WalkHead) + 255) / 256 * 256;

// After the granules: a trace region of kTraceWords 64-bit timestamps per window item
// (s_memrealtime, 100 MHz), written only when the launch asks for it (psx_debug_walk_trace).
constexpr int kTraceWords = 10;  // ticket taken, counts loaded, exit map done, predecessor seen, published, expanded,
                                 // the composed exit's outcome (walk_trace.py decodes it), n16 done, jump table done,
                                 // candidates' exits done
size_t walk_trace_offset(uint64_t items) { return kWalkGranOff + items * kGran * 8; }
// After the trace region: the composed exit maps (walk levels > 0), kCand tagged entries
// per (item, level).
constexpr int kCandW = 1024;
size_t walk_maps_offset(uint64_t items) { return walk_trace_offset(items) + items * kTraceWords * 8; }
size_t walk_ws_bytes(uint64_t items, int levels) {
  return walk_maps_offset(items) + items * (uint64_t)(levels > 0 ? levels : 0) * kCandW * 8;
}

// One table header at s.pos (SerializedOpLogReader::StartNewTable, :87-121), read directly
// from the message.  Returns false when the message is done or failed (s.mode = 2).
// Run by every lane of a wave on the same state (the state stays wave-uniform); only the
// `writer` lane stores the segment and raises status bits.
__device__ bool walk_header(const uint8_t *p, uint64_t size, const TableDir &dir, Seg *segs_b, WalkState &s,
                            uint32_t *call_status, bool writer = true) {
  if (s.k >= s.ntab) { s.mode = 2; return false; }
  uint64_t off = s.pos;
  if (off + 16 > size) { if (writer) atomicOr(call_status, kStMalformed); s.mode = 2; return false; }
  const int32_t tid = *reinterpret_cast<const int32_t *>(p + off);
  const uint64_t usz = (uint64_t) * reinterpret_cast<const uint32_t *>(p + off + 4) |
                       ((uint64_t) * reinterpret_cast<const uint32_t *>(p + off + 8) << 32);
  const int32_t nrows = *reinterpret_cast<const int32_t *>(p + off + 12);
  off += 16;
  int t = -1;
  for (int i = 0; i < dir.n; ++i)
    if (dir.table_id[i] == tid) t = i;
  if (t < 0) { if (writer) atomicOr(call_status, kStUnknownTable); s.mode = 2; return false; }
  if (usz != (uint64_t)dir.vsize[t] || nrows < 0) { if (writer) atomicOr(call_status, kStMalformed); s.mode = 2; return false; }
  if ((s.seen >> t) & 1ull) { if (writer) atomicOr(call_status, kStUnsupported); s.mode = 2; return false; }
  s.seen |= 1ull << t;
  Seg *sg = &segs_b[t];
  if (dir.dense_serialized[t]) {
    const uint64_t stride = 4 + (uint64_t)dir.dense_body[t];
    const uint64_t need = (uint64_t)nrows * stride;
    if (off + need > size) { if (writer) atomicOr(call_status, kStMalformed); s.mode = 2; return false; }
    Seg v;
    v.rec0 = (int64_t)off;
    v.num_rows = nrows;
    v.sparse = 0;
    v.ord0 = (int64_t)s.kk;
    if (writer) *sg = v;
    s.pos = off + need;
    s.k += 1;
    s.kk += (uint64_t)nrows;
    return true;
  }
  if (off & 3) { if (writer) atomicOr(call_status, kStUnsupported); s.mode = 2; return false; }
  Seg v;
  v.rec0 = (int64_t)s.rk;
  v.num_rows = nrows;
  v.sparse = 1;
  v.ord0 = (int64_t)s.kk;
  if (writer) *sg = v;
  s.pos = off;
  if (nrows) {
    s.mode = 1;
    s.t = t;
    s.left = (uint64_t)nrows;
  } else {
    s.k += 1;
  }
  return true;
}

__global__ void __launch_bounds__(256) walk_head_kernel(StreamSet ss, TableDir dir, Seg *segs, uint32_t *call_status,
                                                        uint32_t *counters, uint32_t *ntouched, WalkCtl *ctl,
                                                        WalkHead *head, const WalkCount *wc, uint64_t wbytes) {
  const int b = blockIdx.x;
  for (int t = threadIdx.x; t < kMaxTables; t += blockDim.x) {
    Seg s;
    s.rec0 = -1;
    s.num_rows = 0;
    s.sparse = 0;
    s.ord0 = 0;
    segs[b * kMaxTables + t] = s;
    counters[t * kMaxFused + b] = 0;
    if (b == 0) ntouched[t] = 0;
    if (b == 0 && wc && t < dir.n && wc[t].on) {   // ordered_count's reset of ordered_offsets' counters
#pragma unroll
      for (int i = 0; i < 5; ++i) wc[t].nsplit[i * kNsStride] = 0;
      wc[t].tsum[0] = 0;
    }
  }
  if (b == 0 && threadIdx.x == 0) {
    ctl->ticket = 0;
    ctl->lost = 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint8_t *p = ss.data[b];
  const uint64_t size = ss.size[b];
  WalkState s{};
  s.pos = 4;
  s.rk = ss.recoff_base[b];
  s.mode = 2;
  if (size == 0) {
    // empty message (server.cpp:128)
  } else if (size < 4 || *reinterpret_cast<const int32_t *>(p) < 0) {
    atomicOr(call_status, kStMalformed);
  } else {
    s.ntab = *reinterpret_cast<const int32_t *>(p);
    s.mode = 0;
    while (s.mode == 0 && walk_header(p, size, dir, segs + b * kMaxTables, s, call_status)) {
    }
  }
  uint32_t nwin = 0, wf = 0;
  if (s.mode == 1 && s.pos + 8 > size) {   // the first record's header past the message end
    atomicOr(call_status, kStMalformed);
    s.mode = 2;
  }
  if (s.mode == 1) {
    wf = (uint32_t)(s.pos / wbytes);
    nwin = (uint32_t)((size + wbytes - 1) / wbytes) - wf;
  }
  head->st[b] = s;
  head->wfirst[b] = wf;
  head->nwin[b] = nwin;
}

// The next record start after a speculative record at word q with count word c (n16), or
// kNo when it lies outside the window or past the message (a count >= kNBig always does).
// (32-bit: c < kNBig and spec_wpr <= 3 keep q + 2 + c * spec_wpr far below 2^32; nw never
// passes the message's end, so a start before nw is inside the message.)
__device__ __forceinline__ uint16_t next_of(uint32_t q, uint16_t c, uint32_t nw, uint64_t W0, uint64_t size,
                                            uint32_t spec_wpr) {
  (void)W0;
  (void)size;
  if (c >= kNBig) return kNo;
  const uint32_t nxt = q + 2 + (uint32_t)c * spec_wpr;
  return nxt < nw ? (uint16_t)nxt : kNo;
}

// entry candidates per window: the block's thread count (at most kCandW, the exit maps'
// 10-bit entry field)

// The exit map entry of word q: the last record start on q's chain inside the window and
// the records from q up to it, packed (16 | 16 bits): 16 records a step on jt4, then
// single records.
__device__ __forceinline__ uint32_t exit_walk(uint32_t q, const uint16_t *jt4, const uint16_t *n16, uint32_t nw,
                                              uint64_t W0, uint64_t size, uint32_t spec_wpr) {
  uint32_t w = q, cnt = 0;
  for (uint16_t j = jt4[w]; j != kNo; j = jt4[w]) {
    w = j;
    cnt += 16;
  }
  for (uint16_t j = next_of(w, n16[w], nw, W0, size, spec_wpr); j != kNo; j = next_of(w, n16[w], nw, W0, size, spec_wpr)) {
    w = j;
    cnt += 1;
  }
  return w | (cnt << 16);
}

// The resolve's (wave-uniform) lookup: the candidates' table, or the walk itself for a
// later entry.
template <int kCand>
__device__ __forceinline__ uint32_t exit_at(uint32_t q, const uint32_t *xc, const uint16_t *jt4, const uint16_t *n16,
                                            uint32_t nw, uint64_t W0, uint64_t size, uint32_t spec_wpr) {
  if (q < (uint32_t)kCand) return (uint32_t)__builtin_amdgcn_readfirstlane((int)xc[q]);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)exit_walk(q, jt4, n16, nw, W0, size, spec_wpr));
}

__device__ __forceinline__ uint32_t gran_value(const WalkState &s, int i) {
  switch (i) {
    case 0: return (uint32_t)s.pos;
    case 1: return (uint32_t)(s.pos >> 32);
    case 2: return (uint32_t)s.left;
    case 3: return (uint32_t)(s.left >> 32);
    case 4: return (uint32_t)s.rk;
    case 5: return (uint32_t)(s.rk >> 32);
    case 6: return (uint32_t)s.kk;
    case 7: return (uint32_t)(s.kk >> 32);
    case 8: return (uint32_t)s.seen;
    case 9: return (uint32_t)(s.seen >> 32);
    case 10: return (uint32_t)s.k;
    case 11: return (uint32_t)s.t;
    case 12: return (uint32_t)s.mode;
    default: return (uint32_t)s.ntab;
  }
}

// ordered_count for one record of a walk-counted split table (WalkCount): the record's row
// id and pair count at p (a record the walk accepted: its header lies inside the message).
__device__ __forceinline__ void walk_count(const uint8_t *p, const WalkCount &w, uint32_t *call_status,
                                           uint64_t idx, uint64_t ref) {
  const int32_t rid = *reinterpret_cast<const int32_t *>(p);
  const int32_t n = *reinterpret_cast<const int32_t *>(p + 4);
  int64_t d = (int64_t)rid - w.row_offset;
  bool ok = d >= 0;
  if (ok && w.row_stride != 1) {
    ok = d % w.row_stride == 0;
    d /= w.row_stride;
  }
  if (!ok || d >= w.max_rows) {
    atomicOr(call_status, kStRowRange);
    if (w.wfill) w.wfill[idx] = int2{-1, 0};
    return;
  }
  // bucket lists: no growth atomic (the pair count goes beside the list entry below and the
  // ordered prep sums them, psx_ordered.hip o_grow)
  if (!w.bucket) atomicAdd(&w.grow[d], n);
#ifdef PSX_DEBUG_BUILD
  // timing probes (PSX_ORD_PROBE bits 8, 9): one more fire-and-forget count atomic, or one
  // more returning one, that change nothing
  if (w.pad2 & 1) atomicAdd(&w.grow[d], 0);
  if (w.pad2 & 2) {
    const int32_t z = atomicAdd(&w.cnt[d], 0);
    if (z == -12345) atomicOr(call_status, 0u);
  }
#endif
  if (w.wfill) {
    // the count's returned value is the record's place in its slot's list (the apply sorts
    // each list into message order, so any order of these atomics is as good)
    const int32_t k = atomicAdd(&w.cnt[d], 1);
    w.wfill[idx] = int2{(int32_t)d, k};
    if (w.bucket) {   // bucket lists: the list entry itself, no ordered_fill
      if (k < w.bucket_m) {
        w.bucket[d * w.bucket_m + k] = ref;
        // its pair count beside the entries (psx_ordered.hip bucket_pairs, o_grow)
        reinterpret_cast<int32_t *>(w.bucket + w.max_rows * w.bucket_m)[d * w.bucket_m + k] = n;
      } else {
        atomicOr(call_status, kStDuplicateRow);   // more records than a bucket holds: replay
      }
    }
  } else {
    atomicAdd(&w.cnt[d], 1);
  }
}

template <int T_, int WW_, int C_>
__global__ void __launch_bounds__(T_) walk_kernel(StreamSet ss, TableDir dir, Seg *segs, uint64_t *recoff,
                                                            uint32_t *call_status, WalkCtl *ctl, const WalkHead *head,
                                                            unsigned long long *gran_p, uint32_t spec_wpr,
                                                            uint32_t epoch, unsigned long long *trace,
                                                            const WalkCount *wc, unsigned long long *maps_p,
                                                            int levels_arg) {
  // levels_arg: the composed exit-map levels (low byte); bit 8 (PSX_DEBUG_WALK_SKEW, tests
  // only) skews every early-published exit state by one record, which the cross-check
  // after the resolve must catch
  const int levels = levels_arg & 0xff;
  const bool skew = (levels_arg >> 8) & 1;
  constexpr int kWalkThreads = T_, kWW = WW_, kCand = C_;
  static_assert(C_ <= T_ && C_ % 64 == 0, "candidates");
  constexpr uint64_t kWBytes = (uint64_t)WW_ * 4;
  static_assert(kWW % kWalkThreads == 0 && ((kWW / kWalkThreads) % 8 == 0 || (kWW / kWalkThreads) % 12 == 0) && kWW < 0xFFF0 && kCand <= kCandW,
                "walk shape");
  gu64 *gran = (gu64 *)gran_p;
  gu64 *maps = (gu64 *)maps_p;
  // Windows of kWW words (96 KiB for shape 0), everything but the hand-off done before it.
  // n16 keeps the clipped record count after each word, loaded straight from the message
  // (single-record steps are computed from it, next_of); wbuf's two halves (sa, sb) take the
  // 16-bit squarings of the next-record link — 2, 4, 8, 16 records — and sb ends as jt4, the
  // 16-record jump table; xc is the exit map of the entry candidates (packed: low 16 bits the
  // last record start on q's chain inside the window, high 16 the records from q up to it,
  // exclusive).
  __shared__ uint32_t wbuf[kWW];
  __shared__ __align__(16) uint16_t n16[kWW];
  __shared__ uint32_t xc[kCand];   // exit map of the first kCand words (the entry candidates)
  uint16_t *const sa = reinterpret_cast<uint16_t *>(wbuf);
  uint16_t *const sb = sa + kWW;
  uint16_t *const jt4 = sb;
  __shared__ uint16_t seg_q[kMaxSegs];
  __shared__ uint16_t seg_n[kMaxSegs];
  __shared__ uint64_t seg_rk[kMaxSegs];
  __shared__ uint8_t seg_t[kMaxSegs];   // the segment's table (walk-counted tables: WalkCount)
  __shared__ uint16_t a16[kWW / 32 + 1], a1[16];
  __shared__ uint32_t sh_nseg, sh_n16, sh_n1, sh_ticket;
  const int tid = threadIdx.x;
  const int B = ss.n;
  uint32_t maxwin = 0;
  for (int i = 0; i < B; ++i) maxwin = head->nwin[i] > maxwin ? head->nwin[i] : maxwin;
  const uint32_t items = (uint32_t)B * maxwin;

  for (;;) {
    if (tid == 0) sh_ticket = atomicAdd(&ctl->ticket, 1u);
    __syncthreads();
    const uint32_t tk = sh_ticket;
    if (tk >= items) break;
    const int b = (int)(tk % (uint32_t)B);
    const uint32_t j = tk / (uint32_t)B;
    const uint32_t nwin_b = head->nwin[b];
    if (j >= nwin_b) {
      __syncthreads();   // sh_ticket is rewritten at the top
      continue;
    }
    unsigned long long *tr = trace ? trace + (uint64_t)tk * kTraceWords : nullptr;
    if (tr && tid == 0) tr[0] = __builtin_amdgcn_s_memrealtime();
    const uint8_t *p = ss.data[b];
    const uint64_t size = ss.size[b];
    const uint64_t W0 = ((uint64_t)head->wfirst[b] + j) * kWBytes;
    const uint64_t tot = (size - W0) / 4;                   // whole words from W0
    const uint32_t nw = (uint32_t)(tot < (uint64_t)kWW ? tot : (uint64_t)kWW);
    const bool halo = tot > nw;
    const bool last = j + 1 == nwin_b;
    // 1) every word a speculative record start: n16[q], the clipped count word after q,
    //    straight from the message (coalesced loads, one word ahead; the words themselves are
    //    not kept — the resolve reads headers from the message)
    {
      const uint32_t *src = reinterpret_cast<const uint32_t *>(p + W0);
      const uint32_t lim = halo ? nw + 1 : nw;   // words readable from W0 (with the halo word)
      constexpr int PER = (kWW / kWalkThreads) % 12 == 0 ? 12 : 8;   // loads in flight per thread
#pragma unroll
      for (int h = 0; h < kWW / (PER * kWalkThreads); ++h) {
        uint32_t r[PER];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const uint32_t q = (uint32_t)tid + (uint32_t)(h * PER + k) * kWalkThreads;
          r[k] = q + 1 < lim ? src[q + 1] : 0u;
        }
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const uint32_t q = (uint32_t)tid + (uint32_t)(h * PER + k) * kWalkThreads;
          const int32_t n = (int32_t)r[k];
          n16[q] = q + 1 >= lim ? kNNone : n < 0 ? kNNeg : (n >= (int32_t)kNBig ? kNBig : (uint16_t)n);
        }
      }
    }
    __syncthreads();
    if (tr && tid == 0) tr[1] = __builtin_amdgcn_s_memrealtime();
    if (tr && tid == 0) tr[7] = __builtin_amdgcn_s_memrealtime();
    // 2) the 16-record jump table by four squarings of the next-record link in 16 bits,
    //    one barrier each; a thread takes two neighbouring words at a time (32-bit LDS reads
    //    and writes of the sequential side, 16-bit gathers of the links)
    {
      constexpr int PER = kWW / kWalkThreads;
      static_assert(PER % 2 == 0, "word pairs");
      // next_of inside the window: n < kNBig and the next start before nw (nw <= the
      // message's words from W0, so such a start is inside the message too)
      auto nx = [&](uint32_t q, uint32_t c) -> uint32_t {
        if (c >= kNBig) return kNo;
        const uint32_t nxt = q + 2 + c * spec_wpr;
        return nxt < nw ? nxt : kNo;
      };
      const uint32_t *const n16w = reinterpret_cast<const uint32_t *>(n16);
#pragma unroll
      for (int lv = 0; lv < 4; ++lv) {
        const uint16_t *src = (lv & 1) ? sa : sb;   // lv 0 reads n16, not sb
        uint16_t *dst = (lv & 1) ? sb : sa;
        const uint32_t *srcw = reinterpret_cast<const uint32_t *>(src);
        uint32_t *dstw = reinterpret_cast<uint32_t *>(dst);
#pragma unroll
        for (int k = 0; k < PER / 2; ++k) {
          const uint32_t i = (uint32_t)tid + (uint32_t)k * kWalkThreads;   // words 2i, 2i + 1
          uint32_t a0, a1;
          if (lv == 0) {
            const uint32_t cc = n16w[i];
            a0 = nx(2 * i, cc & 0xFFFFu);
            a1 = nx(2 * i + 1, cc >> 16);
          } else {
            const uint32_t aa = srcw[i];
            a0 = aa & 0xFFFFu;
            a1 = aa >> 16;
          }
          uint32_t r0 = kNo, r1 = kNo;
          if (lv == 0) {
            if (a0 != kNo) r0 = nx(a0, n16[a0]);
            if (a1 != kNo) r1 = nx(a1, n16[a1]);
          } else {
            if (a0 != kNo) r0 = src[a0];
            if (a1 != kNo) r1 = src[a1];
          }
          dstw[i] = r0 | (r1 << 16);
        }
        __syncthreads();
      }
    }
    if (tr && tid == 0) tr[8] = __builtin_amdgcn_s_memrealtime();
    //    The exit map for the window's first kCand words only — the chain enters a window
    //    inside the record that crosses its start, so in practice within its first few
    //    hundred bytes (a later entry, a record longer than kCand words, is walked by the
    //    resolve itself): thread q walks q's chain, 16 records a step, then single ones.
    if ((uint32_t)tid < (uint32_t)kCand) xc[tid] = exit_walk((uint32_t)tid, jt4, n16, nw, W0, size, spec_wpr);
    __syncthreads();
    if (tr && tid == 0) tr[9] = __builtin_amdgcn_s_memrealtime();
    // 4') composed exit maps (levels > 0): the window's forward map F[q] — from entry
    //     candidate q, the records up to and including the one that crosses the window's
    //     end, and the word where the next window's chain starts (a candidate of it, < kCand)
    //     — then, level by level, P_l(j) = P_{l-1}(j) o P_{l-1}(j - 2^(l-1)): the map over the
    //     2^l windows ending here (from the message's first window when fewer precede).
    //     Partner maps come from the blocks of earlier windows of the same message (earlier
    //     tickets), as epoch-tagged entries.  With them the exit state of window j follows
    //     from the exit state 2^levels windows back in one lookup (step 4 below), so the
    //     chain between windows hops 2^levels windows at a time.  Encoding: count << 10 |
    //     entry word, kNoMap where the chain leaves the table's records, a header or the message.
    uint32_t *pm = reinterpret_cast<uint32_t *>(sa);          // (sa is free after the squarings)
    uint32_t *pm2 = pm + kCand;
    constexpr uint32_t kNoMap = 0xFFFFFFFFu;
    if (levels > 0) {
      if ((uint32_t)tid < (uint32_t)kCand) {
        const uint32_t q = (uint32_t)tid;
        uint32_t f = kNoMap;
        if (!last) {
          const uint32_t x = xc[q];
          const uint32_t T = x & 0xFFFFu, cnt = (x >> 16) + 1;
          if (T + 1 < nw || (T + 1 == nw && halo)) {   // T's count word in the window or its halo
            const uint16_t cT = n16[T];
            if (cT < kNBig) {
              const uint64_t endw = (uint64_t)T + 2 + (uint64_t)cT * spec_wpr;
              if (endw >= (uint64_t)kWW && W0 + endw * 4 <= size && endw - kWW < (uint64_t)kCand && cnt < (1u << 22) - 1)
                f = (cnt << 10) | (uint32_t)(endw - kWW);
            }
          }
        }
        pm[q] = f;
        __hip_atomic_store(maps + ((uint64_t)tk * levels + 0) * kCand + q, ((uint64_t)epoch << 32) | f,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      for (int l = 1; l <= levels; ++l) {
        const uint32_t d = 1u << (l - 1);
        const uint32_t q = (uint32_t)tid;
        const bool cq = q < (uint32_t)kCand;   // (the block's other threads only keep the barriers)
        uint32_t v = cq ? pm[q] : kNoMap;
        if (cq && j >= d) {
          // the partner's P_{l-1} covers the windows just before this one's P_{l-1}
          const gu64 *g = maps + ((uint64_t)(tk - d * (uint32_t)B) * levels + (l - 1)) * kCand + q;
          uint64_t x = 0;
          bool ok = false;
          for (uint32_t spins = 0; spins <= (1u << 20); ++spins) {
            x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((uint32_t)(x >> 32) == epoch) { ok = true; break; }
            __builtin_amdgcn_s_sleep(1);
          }
          if (!ok) atomicOr(call_status, kStWalkLost);
          const uint32_t u = ok ? (uint32_t)x : kNoMap;
          v = kNoMap;
          if (u != kNoMap) {
            const uint32_t w = pm[u & 1023u];
            if (w != kNoMap) {
              const uint32_t c = (u >> 10) + (w >> 10);
              if (c < (1u << 22) - 1) v = (c << 10) | (w & 1023u);
            }
          }
        }
        if (cq) pm2[q] = v;
        __syncthreads();
        if (cq) {
          pm[q] = v;
          if (l < levels)
            __hip_atomic_store(maps + ((uint64_t)tk * levels + l) * kCand + q, ((uint64_t)epoch << 32) | v,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
      }
    }
    if (tr && tid == 0) tr[2] = __builtin_amdgcn_s_memrealtime();
    // 4) wave 0: wait for the predecessor's state, resolve this window (every lane on the
    //    same state, lane 0 writing), publish (lane i its granule i)
    if (tid < 64) {
      // read before the wait (a scalar-cache miss here would sit on the chain's critical
      // path): this message's record-offset range (psx_runtime.cpp sizes it size / 8 + 1)
      const uint64_t rk_lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)ss.recoff_base[b]) |
                             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(ss.recoff_base[b] >> 32)) << 32);
      const uint64_t rk_hi = rk_lo + size / 8 + 1;
      const int lane = tid;
      // The composed exit: window j's exit state from the exit state of window a - 1, a the
      // first window P_levels(j) covers (the message's head when a == 0), when that state
      // enters window a as a candidate inside a sparse table that goes on past window j.
      bool pub_early = false;
      uint32_t mine_early = 0;   // this lane's granule of the early-published state
      uint64_t t_early = 0;
      uint64_t xdbg = 0;   // trace word 6: bit 0 tried, 1 ok0, 2 mode 1, 3 entry in range, 4 map, 5 left; hi: map
      if (levels > 0 && !last) {
        xdbg = 1;
        const uint32_t span = 1u << levels;
        const uint32_t a0 = j + 1 >= span ? j + 1 - span : 0u;
        WalkState s0;
        bool ok0 = true;
        if (a0 == 0) {
          s0 = head->st[b];
        } else {
          const gu64 *g = gran + (uint64_t)(tk - (j - a0 + 1) * (uint32_t)B) * kGran;
          uint32_t v = 0;
          ok0 = false;
          for (uint32_t spins = 0;; ++spins) {
            uint64_t x = (uint64_t)epoch << 32;
            if (lane < kGran) x = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            v = (uint32_t)x;
            if (__all((uint32_t)(x >> 32) == epoch)) { ok0 = true; break; }
            if (spins > (1u << 20)) break;
            __builtin_amdgcn_s_sleep(1);
          }
          if (!ok0 && lane == 0) atomicOr(call_status, kStWalkLost);
          auto rl = [&](int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); };
          auto lo_hi = [&](int i) { return (uint64_t)rl(i) | ((uint64_t)rl(i + 1) << 32); };
          s0.pos = lo_hi(0);
          s0.left = lo_hi(2);
          s0.rk = lo_hi(4);
          s0.kk = lo_hi(6);
          s0.seen = lo_hi(8);
          s0.k = (int32_t)rl(10);
          s0.t = (int32_t)rl(11);
          s0.mode = (int32_t)rl(12);
          s0.ntab = (int32_t)rl(13);
        }
        const uint64_t Wa = ((uint64_t)head->wfirst[b] + a0) * kWBytes;
        xdbg |= (ok0 ? 2u : 0u) | (s0.mode == 1 ? 4u : 0u);
        if (ok0 && s0.mode == 1 && s0.pos >= Wa && s0.pos - Wa < (uint64_t)kCand * 4 && s0.rk >= rk_lo &&
            s0.rk + s0.left <= rk_hi) {
          const uint32_t q0 = (uint32_t)((s0.pos - Wa) / 4);
          const uint32_t m = (uint32_t)__builtin_amdgcn_readfirstlane((int)pm[q0]);
          xdbg |= 8u | (m != kNoMap ? 16u : 0u) | (m != kNoMap && s0.left > (uint64_t)(m >> 10) ? 32u : 0u) |
                  ((uint64_t)m << 32);
          if (m != kNoMap && s0.left > (uint64_t)(m >> 10)) {
            WalkState e = s0;
            const uint64_t c = m >> 10;
            e.pos = W0 + kWBytes + (uint64_t)(m & 1023u) * 4;
            e.rk += c;
            e.kk += c;
            e.left -= c;
            if (skew) e.rk += 1;
            uint32_t mine = 0;
#pragma unroll
            for (int i = 0; i < kGran; ++i) mine = lane == i ? gran_value(e, i) : mine;
            if (lane < kGran)
              __hip_atomic_store(gran + (uint64_t)tk * kGran + lane, ((uint64_t)epoch << 32) | (uint64_t)mine,
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            mine_early = mine;
            pub_early = true;
            if (tr) t_early = __builtin_amdgcn_s_memrealtime();
          }
        }
      }
      WalkState s;
      if (j == 0) {
        s = head->st[b];
      } else {
        const gu64 *g = gran + (uint64_t)(tk - (uint32_t)B) * kGran;
        uint32_t v = 0, tag = 0;
        bool ok = false;
        for (uint32_t spins = 0;; ++spins) {
          uint64_t x = (uint64_t)epoch << 32;
          if (lane < kGran) x = __hip_atomic_load(g + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v = (uint32_t)x;
          tag = (uint32_t)(x >> 32);
          if (__all(tag == epoch)) { ok = true; break; }
          if (spins > (1u << 20)) break;        // bounded (~1 s; a call takes ~0.1 ms): a lost hand-off fails the call
          __builtin_amdgcn_s_sleep(1);
        }
        if (!ok) {
          // record the first lost hand-off of the call (psx_last_error reports it)
          const uint64_t tagged = __ballot(lane < kGran && tag == epoch);
          const uint32_t tag0 = (uint32_t)__shfl((int)tag, 0);
          if (lane == 0) {
            atomicOr(call_status, kStWalkLost);
            if (atomicCAS(&ctl->lost, 0u, 1u) == 0u) {
              ctl->dbg[0] = tk;
              ctl->dbg[1] = (uint32_t)b;
              ctl->dbg[2] = j;
              ctl->dbg[3] = epoch;
              ctl->dbg[4] = tag0;
              ctl->dbg[5] = (uint32_t)tagged;
            }
          }
        }
        // readlane: the state lands in scalar registers, wave-uniform for the resolve
        auto rl = [&](int i) { return (uint32_t)__builtin_amdgcn_readlane((int)v, i); };
        auto lo_hi = [&](int i) { return (uint64_t)rl(i) | ((uint64_t)rl(i + 1) << 32); };
        s.pos = lo_hi(0);
        s.left = lo_hi(2);
        s.rk = lo_hi(4);
        s.kk = lo_hi(6);
        s.seen = lo_hi(8);
        s.k = (int32_t)rl(10);
        s.t = (int32_t)rl(11);
        s.mode = (int32_t)rl(12);
        s.ntab = (int32_t)rl(13);
        if (!ok) s.mode = 2;
      }
      // (stamps held in registers and stored together after the publish: a store here
      // would put its own completion wait inside the resolve)
      const uint64_t t_seen = tr ? __builtin_amdgcn_s_memrealtime() : 0;
      const bool w0 = lane == 0;
      {
        // Wave-uniform scalar code: every value read back through readfirstlane, so the
        // loop branches on SCC; status bits gathered in `bad` and raised once.
        const uint64_t Wend = W0 + kWBytes;
        uint32_t nseg = 0, bad = 0;
        Seg *segs_b = segs + b * kMaxTables;
        // Fast path (almost every window of a large sparse table): the table's records
        // continue past this window — one exit-map lookup, the last record's count, done.
        // Anything else (a table or the message ending here, a header, a bad state) takes
        // the general loop below from the unchanged state.
        bool done = false;
        if (s.mode == 1 && !last && s.pos >= W0 && s.pos - W0 < (uint64_t)nw * 4 && s.rk >= rk_lo &&
            s.rk + s.left <= rk_hi) {
          const uint32_t q = (uint32_t)((s.pos - W0) / 4);
          const uint32_t x = exit_at<kCand>(q, xc, jt4, n16, nw, W0, size, spec_wpr);
          const uint32_t T = x & 0xFFFFu;
          const uint64_t c = (uint64_t)(x >> 16) + 1;
          if (s.left > c && (T + 1 < nw || (T + 1 == nw && halo))) {
            const uint32_t cT = (uint32_t)__builtin_amdgcn_readfirstlane((int)n16[T]);
            if (cT < kNBig) {
              const uint64_t endT = W0 + ((uint64_t)T + 2 + (uint64_t)cT * spec_wpr) * 4;
              if (endT >= Wend && endT <= size) {
                if (w0) {
                  seg_q[0] = (uint16_t)q;
                  seg_n[0] = (uint16_t)c;
                  seg_rk[0] = s.rk;
                  seg_t[0] = (uint8_t)s.t;
                }
                nseg = 1;
                s.rk += c;
                s.kk += c;
                s.left -= c;
                s.pos = endT;
                done = true;
              }
            }
          }
        }
        for (; !done;) {
          if (s.mode == 2) break;
          if (s.mode == 1 && (s.pos < W0 || s.rk < rk_lo || s.rk + s.left > rk_hi)) {
            // a state no walk of this message can reach: never expand from it
            bad |= kStWalkBound;
            s.mode = 2;
            break;
          }
          if (s.pos >= Wend && !last) break;          // the walk continues in a later window
          if (s.mode == 0) {
            walk_header(p, size, dir, segs_b, s, call_status, w0);
            continue;
          }
          // sparse records from s.pos: one exit-map lookup
          const uint32_t q = (uint32_t)((s.pos - W0) / 4);
          if (s.pos - W0 >= (uint64_t)nw * 4) { bad |= kStMalformed; s.mode = 2; break; }   // header past the end
          const uint32_t x = exit_at<kCand>(q, xc, jt4, n16, nw, W0, size, spec_wpr);
          const uint32_t T = x & 0xFFFFu;
          const uint64_t c = (uint64_t)(x >> 16) + 1;                                // records q .. T
          const uint64_t take = s.left < c ? s.left : c;
          uint64_t endT = 0;
          if (take == c) {
            // the table holds T's record (before T every link is a checked jump-table link;
            // past the table's end the speculative chain may be garbage): its header inside
            // the message, n >= 0, its end inside the message
            if (T + 1 > nw || (T + 1 == nw && !halo)) { bad |= kStMalformed; s.mode = 2; break; }
            const uint32_t cT = (uint32_t)__builtin_amdgcn_readfirstlane((int)n16[T]);
            if (cT == kNNeg || cT == kNNone) { bad |= kStMalformed; s.mode = 2; break; }
            const int32_t nT = cT == kNBig ? __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int32_t *>(p + W0 + ((uint64_t)T + 1) * 4))
                                           : (int32_t)cT;
            endT = W0 + ((uint64_t)T + 2 + (uint64_t)nT * spec_wpr) * 4;
            if (endT > size) { bad |= kStMalformed; s.mode = 2; break; }
          }
          if (w0) {
            seg_q[nseg] = (uint16_t)q;
            seg_n[nseg] = (uint16_t)take;
            seg_rk[nseg] = s.rk;
            seg_t[nseg] = (uint8_t)s.t;
          }
          ++nseg;
          s.rk += take;
          s.kk += take;
          s.left -= take;
          if (take == c) {
            s.pos = endT;
          } else {
            // the table ends inside the chain: the record `take` on from q — 16 records a
            // step on jt4, then single records (every link before it is a checked
            // in-window link: n16 holds its exact n)
            uint32_t w = q;
            uint64_t r = take;
            for (; r >= 16; r -= 16) w = (uint32_t)__builtin_amdgcn_readfirstlane((int)jt4[w]);
            for (; r; --r) w = w + 2 + (uint32_t)__builtin_amdgcn_readfirstlane((int)n16[w]) * spec_wpr;
            s.pos = W0 + (uint64_t)w * 4;
          }
          if (s.left == 0) {
            s.k += 1;
            s.mode = 0;
          }
        }
        if (bad && w0) atomicOr(call_status, bad);
        if (w0) sh_nseg = nseg;
      }
      // lane i publishes granule i of the (wave-uniform) state
      // lane i's granule: a select chain over the wave-uniform state (no divergent switch)
      uint32_t mine = 0;
#pragma unroll
      for (int i = 0; i < kGran; ++i) mine = lane == i ? gran_value(s, i) : mine;
      if (!last && !pub_early && lane < kGran) {
        gu64 *g = gran + (uint64_t)tk * kGran;
        __hip_atomic_store(g + lane, ((uint64_t)epoch << 32) | (uint64_t)mine, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
      // The state published early (from the composed maps) must be the one the resolve
      // reached: later windows started from it.  Any difference fails the call before an
      // offset is used (kStWalkBound is fatal; the apply stages are gated on it).
      if (pub_early && __ballot(lane < kGran && mine != mine_early) && lane == 0)
        atomicOr(call_status, kStWalkBound);
      if (tr) {
        const uint64_t t_pub = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
          tr[3] = t_seen;
          tr[4] = pub_early ? t_early : t_pub;   // when this window's exit state went out
          tr[6] = xdbg;
        }
      }
    }
    __syncthreads();
    // 5) expand the window's record offsets: thread 0 collects the 16-record hop starts,
    //    one thread per hop lists its 16 records' word offsets in LDS (sa: free once the
    //    state is out), then one thread per record writes its offset (coalesced) and, for a
    //    walk-counted table, does ordered_count's work for it
    const uint32_t nseg = sh_nseg;
    uint16_t *const recq = sa;
    for (uint32_t si = 0; si < nseg; ++si) {
      if (si) __syncthreads();   // recq and a16 held the previous segment's
      if (tid == 0) {
        uint32_t w = seg_q[si];
        uint32_t rem = seg_n[si];
        uint32_t nh = 0, n1 = 0;
        while (rem >= 16) {
          a16[nh++] = (uint16_t)w;
          rem -= 16;
          if (rem) w = jt4[w];
        }
        while (rem) {
          a1[n1++] = (uint16_t)w;
          if (--rem) w = next_of(w, n16[w], nw, W0, size, spec_wpr);
        }
        sh_n16 = nh;
        sh_n1 = n1;
      }
      __syncthreads();
      const uint32_t nh = sh_n16, n1 = sh_n1;
      const uint64_t rk = seg_rk[si];
      for (uint32_t i = tid; i < nh; i += kWalkThreads) {   // one thread per 16-record hop
        uint32_t q = a16[i];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          recq[16 * i + k] = (uint16_t)q;
          if (k < 15) q = next_of(q, n16[q], nw, W0, size, spec_wpr);
        }
      }
      if (tid < n1) recq[16 * nh + tid] = a1[tid];
      __syncthreads();
      const uint32_t nrec = 16 * nh + n1;
      const int t = seg_t[si];
      const bool counted = wc && wc[t].on;
      for (uint32_t r = (uint32_t)tid; r < nrec; r += kWalkThreads) {
        const uint64_t off = W0 + (uint64_t)recq[r] * 4;
        recoff[rk + r] = off;
        if (counted && off + 8 <= size) walk_count(p + off, wc[t], call_status, rk + r, ((uint64_t)b << 56) | off);
      }
    }
    if (tr && tid == 0) tr[5] = __builtin_amdgcn_s_memrealtime();
  }
}

// idx_verify: the indexed messages' record chains (psx_kernels.hip decode_streams found
// each indexed table's segment and checked its first and last offsets).  Grid (G, B): the
// G blocks of message b take its records in a grid stride: each record's offset aligned,
// its header and pairs inside the message, the next offset where it ends; the offset goes
// to recoff and, for a walk-counted split table, ordered_count's work is done here
// (walk_count).  A bad record fails the call (kStMalformed) and marks the message
// (idxw[4 b + 1]); idx_settle then releases the header errors decode_streams held back
// (idxw[4 b]) for the messages whose index was sound.
__global__ void __launch_bounds__(256) idx_verify_kernel(StreamSet ss, TableDir dir, const Seg *segs, IdxSet ix,
                                                         uint64_t *recoff, uint32_t *call_status, uint32_t *idxw,
                                                         const WalkCount *wc) {
  const int b = blockIdx.y;
  const uint8_t *p = ss.data[b];
  const uint64_t size = ss.size[b];
  const uint64_t *idx = ix.p[b];
  if (wc && blockIdx.x == 0 && b == 0) {   // ordered_count's reset of ordered_offsets' counters
    // (walk_head's job on walked calls; nothing in this launch reads them)
    for (int t = threadIdx.x; t < dir.n; t += blockDim.x)
      if (wc[t].on) {
        for (int i = 0; i < 5; ++i) wc[t].nsplit[i * kNsStride] = 0;
        wc[t].tsum[0] = 0;
      }
  }
  bool bad = false;
  if (idx) {
    for (int t = 0; t < dir.n; ++t) {
      const Seg sg = segs[b * kMaxTables + t];
      if (sg.rec0 < 0 || !sg.sparse || sg.num_rows <= 0) continue;
      const uint64_t *ofs = idx + sg.ord0;
      const uint64_t nrec = (uint64_t)sg.num_rows, rk = (uint64_t)sg.rec0, pair = 4 + (uint64_t)dir.vsize[t];
      const bool counted = wc && wc[t].on;
      for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nrec;
           i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t o = ofs[i];
        bool ok = (o & 3) == 0 && o + 8 <= size;
        uint64_t end = 0;
        if (ok) {
          const int32_t n = *reinterpret_cast<const int32_t *>(p + o + 4);
          end = o + 8 + (uint64_t)(n < 0 ? 0 : n) * pair;
          ok = n >= 0 && end <= size;
        }
        if (ok && i + 1 < nrec) ok = ofs[i + 1] == end;
        recoff[rk + i] = o;
        if (!ok) bad = true;
        else if (counted) walk_count(p + o, wc[t], call_status, rk + i, ((uint64_t)b << 56) | o);
      }
    }
  }
  if (bad) {
    atomicOr(call_status, kStMalformed);
    atomicOr(&idxw[4 * b + 1], 1u);
  }
}

// After idx_verify (a kernel boundary): message b's held-back header errors reach the call
// only when its index was sound.
__global__ void __launch_bounds__(64) idx_settle_kernel(IdxSet ix, int B, uint32_t *call_status, const uint32_t *idxw) {
  const int b = threadIdx.x;
  if (b < B && ix.p[b] && !idxw[4 * b + 1] && idxw[4 * b + 0]) atomicOr(call_status, idxw[4 * b + 0]);
}

hipError_t launch_idx_verify(StreamSet ss, const TableDir &dir, const Seg *segs, const IdxSet &ix, uint64_t *recoff,
                             uint32_t *call_status, uint32_t *idxw, const WalkCount *wc, hipStream_t st) {
  const unsigned B = (unsigned)(ss.n < 1 ? 1 : ss.n);
  const unsigned G = (512u + B - 1) / B;   // ~512 blocks in all (grid stride over larger messages)
  hipLaunchKernelGGL(idx_verify_kernel, dim3(G, B), dim3(256), 0, st, ss, dir, segs, ix, recoff, call_status, idxw, wc);
  hipLaunchKernelGGL(idx_settle_kernel, dim3(1), dim3(64), 0, st, ix, (int)B, call_status, idxw);
  return hipGetLastError();
}

// ws: walk_ws_bytes(items) bytes (items >= B x the largest message's window count at `shape`);
// epoch: nonzero, different from the previous call's on this workspace (granule tags);
// trace_items: nonzero = write the per-item timestamps (the workspace's item count);
// wc: null, or per table (TableDir index) the walk-counted split tables' WalkCount.
hipError_t launch_walk(StreamSet ss, const TableDir &dir, Seg *segs, uint64_t *recoff, uint32_t *call_status,
                       uint32_t *counters, uint32_t *ntouched, void *ws, uint32_t spec_wpr, unsigned blocks,
                       uint32_t epoch, uint64_t trace_items, const WalkCount *wc, uint64_t items, int levels_arg,
                       int shape, hipStream_t st) {
  const int levels = levels_arg & 0xff;
  if (shape < 0 || shape >= kNumWalkShapes) shape = 0;
  WalkCtl *ctl = reinterpret_cast<WalkCtl *>(ws);
  WalkHead *head = reinterpret_cast<WalkHead *>(reinterpret_cast<uint8_t *>(ws) + kWalkHeadOff);
  unsigned long long *gran = reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(ws) + kWalkGranOff);
  hipLaunchKernelGGL(walk_head_kernel, dim3(ss.n), dim3(256), 0, st, ss, dir, segs, call_status, counters, ntouched,
                     ctl, head, wc, walk_window_bytes(shape));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  unsigned long long *trace =
      trace_items ? reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(ws) + walk_trace_offset(trace_items))
                  : nullptr;
  unsigned long long *maps =
      levels > 0 ? reinterpret_cast<unsigned long long *>(reinterpret_cast<uint8_t *>(ws) + walk_maps_offset(items))
                 : nullptr;
#define PSX_WALK_LAUNCH(S)                                                                                    \
  hipLaunchKernelGGL((walk_kernel<kWalkShapes[S].threads, kWalkShapes[S].words, kWalkShapes[S].cand>), dim3(blocks), \
                     dim3(kWalkShapes[S].threads), 0, st, ss, dir, segs, recoff, call_status, ctl, head, gran, spec_wpr, \
                     epoch, trace, wc, maps, levels_arg)
  switch (shape) {
    case 1: PSX_WALK_LAUNCH(1); break;
    case 2: PSX_WALK_LAUNCH(2); break;
    case 3: PSX_WALK_LAUNCH(3); break;
    case 4: PSX_WALK_LAUNCH(4); break;
    case 5: PSX_WALK_LAUNCH(5); break;
    case 6: PSX_WALK_LAUNCH(6); break;
    default: PSX_WALK_LAUNCH(0); break;
  }
#undef PSX_WALK_LAUNCH
  return hipGetLastError();
}

}  // namespace psx
