// psx_ordered.hip — the ordered apply path (counting sort by slot, then one wave per row).
//
// Used for every table whose records are sparse ({int32 n; int32 cols[n]; V vals[n]},
// AbstractRowOpLog::ParseSparseSerializedOpLog, abstract_row_oplog.hpp:64-78) and, as a
// replay, for dense tables when a row occurs twice inside one message.
//
//   ordered_count  cnt[slot] += 1 per record (also validates row range / columns)
//   scan_*         off = exclusive prefix of cnt (max_rows + 1 entries)
//   ordered_fill   list[off[slot] + --cnt[slot]] = flattened record number r
//                  (r orders records by (message, position) = reference apply order;
//                  cnt returns to zero, the invariant between calls)
//   capacity check (sorted/map tables whose keys ever left [0, max_entries)): a dry run of
//                  the apply on the rows whose entries + the call's record entries exceed
//                  max_entries; a row that would overflow fails the whole call
//                  (kStCapacity) before anything is applied
//   ordered_apply  one wave per touched slot: sort the slot's r-list, then apply the
//                  records in order with the reference store semantics:
//                    DenseRow     VectorStore::Inc          vector_store.hpp:100-102
//                    SortedMapRow SortedVectorMapStore::Inc sorted_vector_map_store.hpp:175-197,305-337
//                    SparseRow    MapStore::Inc             map_store.hpp:60-65
//                  Sorted-map rows are staged in LDS and updated with wave-parallel
//                  find / bubble / compact, reproducing the reference's entry ORDER
//                  byte for byte (it is history dependent: found keys are not re-sorted).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include "psx_device.hpp"
#include "psx_scan.hpp"

namespace psx {

// The register apply's timing probes (PSX_DEBUG_ORD_PROBE, results wrong) exist only in the
// debug build (`make debug`); in libpsx.so the branches are compiled out.
#ifdef PSX_DEBUG_BUILD
constexpr bool kOrdProbe = true;
#else
constexpr bool kOrdProbe = false;
#endif


__device__ __forceinline__ int32_t o_ld32(const uint8_t *p) { return *reinterpret_cast<const int32_t *>(p); }

__device__ __forceinline__ int64_t o_slot(int32_t rid, const OrdArgs &a) {
  int64_t d = (int64_t)rid - a.row_offset;
  if (d < 0) return -1;
  if (a.row_stride != 1) {
    if (d % a.row_stride) return -1;
    d /= a.row_stride;
  }
  return d < a.max_rows ? d : -1;
}

__device__ __forceinline__ bool o_gate(const OrdArgs &a) {
  const uint32_t st = *a.call_status, sk = *a.sticky;   // both words in flight at once
  return !(st & (kStFatal | kStDuplicateRow)) && (a.force || !(sk & kStDuplicateRow));
}

__device__ __forceinline__ uint64_t shfl64_up(uint64_t x, int o) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)x, o, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(x >> 32), o, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Flattened record space r in [0, pre[B]) in (message, position) order.
struct RecSpace {
  int64_t pre[kMaxFused + 1];
  int64_t first[kMaxFused];   // dense: byte offset of record 0; sparse: index into recoff
  int32_t sparse[kMaxFused];
};

// Run by the block's first wave: lane b reads message b's segment (the B loads in flight
// together), a wave prefix of the record counts places them.
__device__ void build_space(const OrdArgs &a, RecSpace &rs) {
  const int lane = threadIdx.x & 63;
  int64_t nr = 0, first = 0;
  int32_t sp = 0;
  if (lane < kMaxFused && lane < a.B) {
    const Seg sg = a.segs[lane * kMaxTables + a.t];
    if (sg.rec0 >= 0) {
      nr = sg.num_rows;
      first = sg.rec0;
      sp = sg.sparse;
    }
  }
  int64_t incl = nr;
#pragma unroll
  for (int o = 1; o < kMaxFused; o <<= 1) {
    const int64_t y = (int64_t)shfl64_up((uint64_t)incl, o);
    if (lane >= o) incl += y;
  }
  if (lane < kMaxFused) {
    rs.pre[lane] = incl - nr;
    rs.first[lane] = first;
    rs.sparse[lane] = sp;
  }
  if (lane == kMaxFused - 1) rs.pre[kMaxFused] = incl;
}

// Locate record r: message b and the byte offset of its row id.
__device__ __forceinline__ void locate(const OrdArgs &a, const RecSpace &rs, int64_t r, int &b, uint64_t &off) {
  b = 0;
  while (b + 1 < a.B && rs.pre[b + 1] <= r) ++b;
  const int64_t k = r - rs.pre[b];
  off = rs.sparse[b] ? a.recoff[rs.first[b] + k] : (uint64_t)(rs.first[b] + k * a.stride);
}

// A record list entry: (message << 56) | byte offset of the record's row id.  Sorting
// entries as integers orders the records as the reference applies them (message, then
// position), and the apply reaches a record without the record-offset table.
constexpr uint64_t kRefOffMask = (1ull << 56) - 1;
__device__ __forceinline__ uint64_t rec_ref(int b, uint64_t off) { return ((uint64_t)b << 56) | off; }
__device__ __forceinline__ const uint8_t *rec_ptr(const OrdArgs &a, uint64_t e) {
  return a.ss.data[e >> 56] + (e & kRefOffMask);
}

// Entries slot s's c records can add: the sum of their pair counts.  Prefix lists: the
// count's atomic sum (grow).  Bucket lists: the count adds nothing to grow — one
// device-scope atomic per record less in the walk, its costliest step (an extra one costs
// the C3 walk 8.5 us, profiles/r06/s15) — but stores each record's pair count beside its
// list entry (bucket_pairs), summed here: one 64-B line per slot.
__device__ __forceinline__ const int32_t *bucket_pairs(uint64_t *bucket, int64_t max_rows, int32_t m) {
  return reinterpret_cast<const int32_t *>(bucket + max_rows * m);
}
__device__ __forceinline__ const int4 *bucket_pairs4(const OrdArgs &a, int64_t s) {
  static_assert(kMaxFused == 16, "four int4 per slot");
  return reinterpret_cast<const int4 *>(bucket_pairs(a.list, a.max_rows, a.bucket_m) + s * kMaxFused);
}
// the sum of the first min(c, 16) pair counts of a slot's line
__device__ __forceinline__ int32_t pairs_sum(const int4 (&v)[4], int32_t c) {
  const int m = c < kMaxFused ? c : kMaxFused;   // (more records: the call replays, any value)
  int32_t g = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    g += (4 * k < m ? v[k].x : 0) + (4 * k + 1 < m ? v[k].y : 0) + (4 * k + 2 < m ? v[k].z : 0) +
         (4 * k + 3 < m ? v[k].w : 0);
  return g;
}
__device__ __forceinline__ int32_t o_grow(const OrdArgs &a, int64_t s, int32_t c) {
  if (!a.bucket_m) return a.grow[s];
  const int m = c < kMaxFused ? c : kMaxFused;
  const int4 *q = bucket_pairs4(a, s);
  int4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = 4 * k < m ? q[k] : int4{0, 0, 0, 0};
  return pairs_sum(v, c);
}

// Does any column of the sparse record at p lie outside [0, lim)?  Eight loads in flight
// per step, no early exit (the columns are one record's, a few cache lines).
__device__ __forceinline__ bool cols_outside(const uint8_t *p, int64_t lim) {
  const int32_t n = o_ld32(p + 4);
  const int32_t *cols = reinterpret_cast<const int32_t *>(p + 8);
  const uint32_t ul = lim > 0x7fffffff ? 0xffffffffu : (uint32_t)lim;
  bool bad = false;
  int32_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] = (uint32_t)cols[i + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) bad |= c[k] >= ul;   // negative columns wrap above lim
  }
  for (; i < n; ++i) bad |= (uint32_t)cols[i] >= ul;
  return bad;
}

// ---------------------------------------------------------------------------
// wfill (counted == 3, split tables): the count's returned value is also the record's place
// in its slot's list, stored per record (its recoff index) for ordered_fill.
__global__ void __launch_bounds__(256) ordered_count_kernel(OrdArgs a, int2 *wfill) {
  __shared__ RecSpace rs;
  if (a.grow && blockIdx.x == 0 && threadIdx.x < 6) {   // ordered_offsets' counters
    if (threadIdx.x < 5) a.nsplit[threadIdx.x * kNsStride] = 0;
    else a.tsum[0] = 0;
  }
  // a call whose decode failed has no trustworthy record offsets or sizes: nothing to count
  if (!o_gate(a)) return;
  if (threadIdx.x < 64) build_space(a, rs);
  __syncthreads();
  const int64_t total = rs.pre[kMaxFused];
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  // every lane runs the same trip count so the wave-aggregated append below sees the
  // whole wave
  const int64_t base0 = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63);
  for (int64_t r0 = base0; r0 < total; r0 += G) {
    const int64_t r = r0 + lane;
    bool first = false;
    int64_t s = -1;
    if (r < total) {
      int b;
      uint64_t off;
      locate(a, rs, r, b, off);
      const uint8_t *p = a.ss.data[b] + off;
      s = o_slot(o_ld32(p), a);
      if (s < 0) {
        atomicOr(a.call_status, kStRowRange);
        if (wfill) wfill[rs.first[b] + (r - rs.pre[b])] = int2{-1, 0};
      } else {
        if (!a.dense_records && a.kind == 0) {
          // sparse record into a dense row: every column must lie inside the row
          if (cols_outside(p, a.row_cap)) atomicOr(a.call_status, kStCapacity);
        } else if (a.kind != 0 && a.keyflag && !*a.keyflag && !a.grow) {
          // sorted/map rows: while every key stays in [0, max_entries) no row can hold
          // more than max_entries entries and the capacity dry run is skipped (split
          // tables bound each row by its Incs instead, ordered_offsets, and check the
          // key map's columns in the apply: no column scan here)
          if (cols_outside(p, a.max_entries)) atomicOr(a.keyflag, 1u);
        }
        if (a.grow && !(wfill && a.bucket_m))   // (bucket lists: o_grow sums the pairs later)
          atomicAdd(&a.grow[s], a.dense_records ? (int32_t)a.cap : o_ld32(p + 4));
        if (a.grow && wfill) {   // split tables, ranked: the record's place comes back with the count
          const int32_t k = atomicAdd(&a.cnt[s], 1);
          wfill[rs.first[b] + (r - rs.pre[b])] = int2{(int32_t)s, k};
          if (a.bucket_m) {   // bucket lists: the list entry itself, no ordered_fill
            if (k < a.bucket_m) {
              a.list[s * a.bucket_m + k] = rec_ref(b, off);
              const_cast<int32_t *>(bucket_pairs(a.list, a.max_rows, a.bucket_m))[s * a.bucket_m + k] = o_ld32(p + 4);
            } else {
              atomicOr(a.call_status, kStDuplicateRow);   // more than a bucket holds: replay
            }
          }
        } else if (a.grow)   // split tables: ordered_offsets finds the touched rows from the counts
          atomicAdd(&a.cnt[s], 1);
        else
          first = atomicAdd(&a.cnt[s], 1) == 0;
      }
    }
    // append first-touched slots to the touched list, one atomic per wave
    const uint64_t m = __ballot(first);
    if (m) {
      const int leader = __builtin_ctzll(m);
      uint32_t base = 0;
      if (lane == leader) base = atomicAdd(a.ntouched, (uint32_t)__builtin_popcountll(m));
      base = __builtin_amdgcn_readlane(base, leader);
      if (first) {
        const uint32_t rank = (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
        a.touched[base + rank] = (int32_t)s;
      }
    }
  }
}

// wfill (ranked split tables, counted >= 2): each record's {slot, place} from the walk or
// ordered_count;
// the list entry is written without an atomic and the counts were zeroed by ordered_offsets.
__global__ void __launch_bounds__(256) ordered_fill_kernel(OrdArgs a, const int2 *wfill) {
  __shared__ RecSpace rs;
  const bool gate = o_gate(a);   // (its words in flight beside the record space's)
  if (threadIdx.x < 64) build_space(a, rs);
  __syncthreads();
  const int64_t total = rs.pre[kMaxFused];
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  if (!gate) {
    // A failed call: ordered_count may have counted some records before a block of it set
    // a fatal bit (and blocks that started after that counted none), and ordered_offsets
    // skipped.  Restore the invariant (cnt and grow zero between calls) over every slot;
    // O(max_rows), failed calls only.
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < a.max_rows; s += G) {
      a.cnt[s] = 0;
      if (a.grow) a.grow[s] = 0;
    }
    return;
  }
  if (wfill) {
    for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < total; r += G) {
      int b = 0;
      while (b + 1 < a.B && rs.pre[b + 1] <= r) ++b;
      const int64_t idx = rs.first[b] + (r - rs.pre[b]);   // ranked tables are sparse
      const int2 sk = wfill[idx];
      const uint64_t off = a.recoff[idx];
      if (sk.x < 0) continue;
      a.list[a.off[sk.x] + sk.y] = rec_ref(b, off);
    }
    return;
  }
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < total; r += G) {
    int b;
    uint64_t off;
    locate(a, rs, r, b, off);
    const int64_t s = o_slot(o_ld32(a.ss.data[b] + off), a);
    if (s < 0) continue;
    const int32_t p = atomicSub(&a.cnt[s], 1) - 1;
    a.list[a.off[s] + p] = rec_ref(b, off);
  }
}

// ordered_offsets (split tables, instead of the exclusive scan): each block takes a
// contiguous range of slots and, over its touched ones (count > 0), gives every row its
// record-list range and its descriptor {slot, list begin, list end, image size} in three
// lists: the 256-entry and the 1,024-entry apply lists (a row whose image can outgrow 256
// entries in this call: entries now + its records' entries) and, in slot order, the list
// the capacity dry run walks (its length is the table's touched count).  A block adds its
// four totals to the call counters once (ranges need not follow slot order), so the
// counters see a few hundred atomics instead of one per wave of touched rows; the count
// kernel then needs no first-touch atomics.  grow returns to 0.
__device__ __forceinline__ int32_t block_excl_sum(int32_t v, int32_t *sh, int32_t &total) {
  // 256 threads: exclusive prefix of v in thread order; sh holds 4 ints (one per wave)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) sh[w] = incl;
  __syncthreads();
  int32_t pre = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (k < w) pre += sh[k];
    total += sh[k];
  }
  __syncthreads();
  return pre + incl - v;
}

// N exclusive prefix sums at once (one LDS exchange, two barriers instead of 2N).
template <int N>
__device__ __forceinline__ void block_excl_sumN(const int32_t (&v)[N], int32_t (&pre)[N], int32_t (&total)[N],
                                                int32_t (*sh)[4]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int32_t incl[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    incl[i] = v[i];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(incl[i], o, 64);
      if (lane >= o) incl[i] += y;
    }
    if (lane == 63) sh[i][w] = incl[i];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < N; ++i) {
    int32_t p = 0, t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k < w) p += sh[i][k];
      t += sh[i][k];
    }
    pre[i] = p + incl[i] - v[i];
    total[i] = t;
  }
  __syncthreads();
}

// Which apply launch a touched row starts on.  Default: the 1,024-entry one when its image
// can outgrow 256 entries in this call (entries now + the call's Incs).  Spill mode: only
// an image already 7/8 full; the rest start on the 256-entry launch and spill if they
// outgrow it (rare).  Heavy-first (spill bit 1): 256-entry rows with >= kHeavyRecords
// records are listed apart and taken first, so the longest chains start at time zero.
constexpr int32_t kHeavyRecords = 4;
__device__ __forceinline__ bool starts_big(const OrdArgs &a, int32_t nen, int32_t grow) {
  return (int64_t)nen + grow > 256 && (!a.spill || nen > 224);
}
__device__ __forceinline__ bool starts_heavy(const OrdArgs &a, int32_t c) {
  return (a.spill & 2) && c >= kHeavyRecords;
}

// Light rows (OrdArgs.lite): the 256-entry launch takes them four to a wave, sixteen lanes
// each (lite_quad below): few records and an image that stays within 64 entries whatever
// the call's Incs insert, so a row's dependent chain of loads runs beside three others.
constexpr int32_t kLiteRecords = 3;
constexpr int32_t kLiteEntries = 64;
__device__ __forceinline__ bool starts_lite(const OrdArgs &a, int32_t c, int32_t nen, int32_t grow) {
  return a.lite && c <= kLiteRecords && (int64_t)nen + grow <= kLiteEntries;
}

// The capacity dry run's rows: those whose image can outgrow max_entries in this call
// (entries now + the call's Incs).  Any other row cannot overflow, whatever its keys.
__device__ __forceinline__ bool may_overflow(const OrdArgs &a, int32_t nen, int32_t grow) {
  return (int64_t)nen + grow > a.max_entries;
}

__global__ void __launch_bounds__(256) ordered_offsets_kernel(OrdArgs a) {
  __shared__ int32_t sh[7][4];
  __shared__ int32_t base[7];   // touched, records, 256-entry list, 1,024-entry list, heavy rows, dry run, light rows
  const int64_t R = a.max_rows;
  const int64_t per = (R + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = (int64_t)blockIdx.x * per;
  const int64_t c1 = c0 + per < R ? c0 + per : R;
  int4 *const desc = reinterpret_cast<int4 *>(a.split);
  if (per <= (int64_t)blockDim.x) {
    // one slot per thread (the usual grid): the slot's words loaded once (beside the gate's
    // words), one scan gives both the block's totals (one atomic per counter) and each
    // row's place
    const int64_t s = c0 + threadIdx.x;
    int32_t c = 0, nen = 0, g = 0;
    if (s < c1) {
      c = a.cnt[s];
      nen = a.nent[s];
      if (!a.bucket_m) g = a.grow[s];
    }
    if (!o_gate(a)) {
      // bucket lists have no ordered_fill to restore the counts of a failed call: each block
      // clears its own slots (cnt and grow zero between calls)
      if (a.bucket_m && s < c1) {
        a.cnt[s] = 0;
        a.grow[s] = 0;
      }
      return;
    }
    const bool t = c > 0;
    if (t && a.bucket_m) g = o_grow(a, s, c);   // (behind the gate)
    const bool big = t && starts_big(a, nen, g);
    const bool heavy = t && !big && starts_heavy(a, c);
    const bool lite = t && !big && !heavy && starts_lite(a, c, nen, g);
    const bool risky = t && may_overflow(a, nen, g);
    int32_t pre[7], tot[7];
    block_excl_sumN<7>({t ? 1 : 0, c, t && !big && !heavy && !lite ? 1 : 0, big ? 1 : 0, heavy ? 1 : 0,
                        risky ? 1 : 0, lite ? 1 : 0},
                       pre, tot, sh);
    if (threadIdx.x == 0) {
      base[0] = tot[0] ? (int32_t)atomicAdd(a.ntouched, (uint32_t)tot[0]) : 0;
      base[1] = tot[1] && !a.bucket_m ? atomicAdd(&a.tsum[0], tot[1]) : 0;
      base[2] = tot[2] ? (int32_t)atomicAdd(&a.nsplit[0 * kNsStride], (uint32_t)tot[2]) : 0;
      base[3] = tot[3] ? (int32_t)atomicAdd(&a.nsplit[1 * kNsStride], (uint32_t)tot[3]) : 0;
      base[4] = tot[4] ? (int32_t)atomicAdd(&a.nsplit[2 * kNsStride], (uint32_t)tot[4]) : 0;
      base[5] = tot[5] ? (int32_t)atomicAdd(&a.nsplit[3 * kNsStride], (uint32_t)tot[5]) : 0;
      base[6] = tot[6] ? (int32_t)atomicAdd(&a.nsplit[4 * kNsStride], (uint32_t)tot[6]) : 0;
    }
    __syncthreads();
    if (t) {
      if (!a.bucket_m) a.grow[s] = 0;
      if (a.counted >= 2) a.cnt[s] = 0;   // ranked: ordered_fill takes no count back
      const int32_t beg = a.bucket_m ? (int32_t)(s * a.bucket_m) : base[1] + pre[1];
      const int4 d = int4{(int32_t)s, beg, beg + c, nen};
      a.off[s] = beg;
      if (risky) desc[2 * R + base[5] + pre[5]] = d;
      if (big) desc[R + base[3] + pre[3]] = d;
      else if (heavy) desc[R - 1 - (base[4] + pre[4])] = d;
      else if (lite) desc[3 * R + base[6] + pre[6]] = d;
      else desc[base[2] + pre[2]] = d;
    }
    return;
  }
  if (!o_gate(a)) {
    if (a.bucket_m)   // bucket lists: clear this block's slots (no ordered_fill follows)
      for (int64_t s = c0 + threadIdx.x; s < c1; s += blockDim.x) {
        a.cnt[s] = 0;
        a.grow[s] = 0;
      }
    return;
  }
  // pass 1: the block's totals, one atomic per counter
  int32_t nt = 0, nr = 0, ns = 0, nb = 0, nh = 0, nd = 0, nl = 0;
  for (int64_t s = c0 + threadIdx.x; s < c1; s += blockDim.x) {
    const int32_t c = a.cnt[s];
    if (c > 0) {
      ++nt;
      nr += c;
      const int32_t nen = a.nent[s], g = o_grow(a, s, c);
      if (starts_big(a, nen, g)) ++nb;
      else if (starts_heavy(a, c)) ++nh;
      else if (starts_lite(a, c, nen, g)) ++nl;
      else ++ns;
      if (may_overflow(a, nen, g)) ++nd;
    }
  }
  int32_t pre1[7], tot1[7];
  block_excl_sumN<7>({nt, nr, ns, nb, nh, nd, nl}, pre1, tot1, sh);
  const int32_t tt = tot1[0], tr = tot1[1], ts = tot1[2], tb = tot1[3], th = tot1[4], td = tot1[5], tl = tot1[6];
  if (threadIdx.x == 0) {
    base[0] = tt ? (int32_t)atomicAdd(a.ntouched, (uint32_t)tt) : 0;
    base[1] = tr && !a.bucket_m ? atomicAdd(&a.tsum[0], tr) : 0;
    base[2] = ts ? (int32_t)atomicAdd(&a.nsplit[0 * kNsStride], (uint32_t)ts) : 0;
    base[3] = tb ? (int32_t)atomicAdd(&a.nsplit[1 * kNsStride], (uint32_t)tb) : 0;
    base[4] = th ? (int32_t)atomicAdd(&a.nsplit[2 * kNsStride], (uint32_t)th) : 0;
    base[5] = td ? (int32_t)atomicAdd(&a.nsplit[3 * kNsStride], (uint32_t)td) : 0;
    base[6] = tl ? (int32_t)atomicAdd(&a.nsplit[4 * kNsStride], (uint32_t)tl) : 0;
  }
  __syncthreads();
  // pass 2: tiles of 256 slots in slot order, block prefix sums place each touched row.
  // Heavy rows fill the 256-entry list's region [0, R) from its end: small and heavy rows
  // are distinct touched rows, so the two never meet.  The 1,024-entry region [R, 2R) holds
  // the big rows and, appended behind them by the 256-entry launch, the spilled rows (small
  // or heavy, each at most once): at most the touched count in all.
  int32_t ar = base[1], as = base[2], ab = base[3], ah = base[4], ad = base[5], al = base[6];
  for (int64_t t0 = c0; t0 < c1; t0 += blockDim.x) {
    const int64_t s = t0 + threadIdx.x;
    int32_t c = 0, nen = 0;
    bool big = false, heavy = false, risky = false, lite = false;
    if (s < c1) {
      c = a.cnt[s];
      if (c > 0) {
        nen = a.nent[s];
        const int32_t g = o_grow(a, s, c);
        big = starts_big(a, nen, g);
        heavy = !big && starts_heavy(a, c);
        lite = !big && !heavy && starts_lite(a, c, nen, g);
        risky = may_overflow(a, nen, g);
        if (!a.bucket_m) a.grow[s] = 0;
        if (a.counted >= 2) a.cnt[s] = 0;   // ranked: ordered_fill takes no count back
      }
    }
    const bool t = c > 0;
    int32_t pre[7], tot[7];
    block_excl_sumN<7>({t ? 1 : 0, c, t && !big && !heavy && !lite ? 1 : 0, t && big ? 1 : 0, t && heavy ? 1 : 0,
                        t && risky ? 1 : 0, t && lite ? 1 : 0},
                       pre, tot, sh);
    const int32_t pr = pre[1], ps = pre[2], pb = pre[3], ph = pre[4], pd = pre[5], pl = pre[6];
    const int32_t sr = tot[1], ss2 = tot[2], sb = tot[3], sh2 = tot[4], sd = tot[5], sl = tot[6];
    if (t) {
      const int32_t beg = a.bucket_m ? (int32_t)(s * a.bucket_m) : ar + pr;
      const int4 d = int4{(int32_t)s, beg, beg + c, nen};
      a.off[s] = beg;
      if (risky) desc[2 * R + ad + pd] = d;   // the capacity dry run's list
      if (big) desc[R + ab + pb] = d;
      else if (heavy) desc[R - 1 - (ah + ph)] = d;
      else if (lite) desc[3 * R + al + pl] = d;
      else desc[as + ps] = d;
    }
    ar += sr;
    as += ss2;
    ab += sb;
    ah += sh2;
    ad += sd;
    al += sl;
  }
}

// ---------------------------------------------------------------------------
// Pipelined split tables: ordered_offsets in two halves.
//
// ordered_place is the half that depends only on the call's records: each touched row's
// record-list range (a block prefix over the counts, one atomic per block for its base) and
// one compact entry {slot, list begin, records, entries its records can add} per touched
// row in the call slot's list `plist`; counts (when ranked) and growth return to zero.  It
// runs on the prep stream after the walk and before ordered_fill, beside the previous
// call's apply: nothing it reads or writes is the previous call's (count state, offsets and
// record lists are per call slot or prep-stream only).
//
// ordered_classify is the half that depends on the rows' images after that apply (nent):
// it reads the compact list only — the touched rows, not every slot — and files each row in
// the apply launches' descriptor lists (256-entry, 1,024-entry, heavy, light) and the
// capacity dry run's list, as ordered_offsets does, on the context stream.
__global__ void __launch_bounds__(256) ordered_place_kernel(OrdArgs a, int4 *plist) {
  __shared__ int32_t sh[2][4];
  __shared__ int32_t base[2];   // touched, records
  const int64_t R = a.max_rows;
  const int64_t per = (R + gridDim.x - 1) / gridDim.x;
  const int64_t c0 = (int64_t)blockIdx.x * per;
  const int64_t c1 = c0 + per < R ? c0 + per : R;
  if (!o_gate(a)) {
    if (a.bucket_m)   // bucket lists: clear this block's slots (no ordered_fill follows)
      for (int64_t s = c0 + threadIdx.x; s < c1; s += blockDim.x) {
        a.cnt[s] = 0;
        a.grow[s] = 0;
      }
    return;
  }
  if (per <= (int64_t)blockDim.x) {   // one slot per thread (the usual grid)
    const int64_t s = c0 + threadIdx.x;
    const int32_t c = s < c1 ? a.cnt[s] : 0;
    const bool t = c > 0;
    int32_t pre[2], tot[2];
    block_excl_sumN<2>({t ? 1 : 0, c}, pre, tot, sh);
    if (threadIdx.x == 0) {
      base[0] = tot[0] ? (int32_t)atomicAdd(a.ntouched, (uint32_t)tot[0]) : 0;
      base[1] = tot[1] && !a.bucket_m ? atomicAdd(&a.tsum[0], tot[1]) : 0;
    }
    __syncthreads();
    if (t) {
      const int32_t beg = a.bucket_m ? (int32_t)(s * a.bucket_m) : base[1] + pre[1];
      a.off[s] = beg;
      plist[base[0] + pre[0]] = int4{(int32_t)s, beg, c, o_grow(a, s, c)};
      if (!a.bucket_m) a.grow[s] = 0;
      if (a.counted >= 2) a.cnt[s] = 0;   // ranked: ordered_fill takes no count back
    }
    return;
  }
  int32_t nt = 0, nr = 0;   // pass 1: the block's totals, one atomic per counter
  for (int64_t s = c0 + threadIdx.x; s < c1; s += blockDim.x) {
    const int32_t c = a.cnt[s];
    nt += c > 0;
    nr += c > 0 ? c : 0;
  }
  int32_t pre1[2], tot1[2];
  block_excl_sumN<2>({nt, nr}, pre1, tot1, sh);
  if (threadIdx.x == 0) {
    base[0] = tot1[0] ? (int32_t)atomicAdd(a.ntouched, (uint32_t)tot1[0]) : 0;
    base[1] = tot1[1] && !a.bucket_m ? atomicAdd(&a.tsum[0], tot1[1]) : 0;
  }
  __syncthreads();
  int32_t at = base[0], ar = base[1];
  for (int64_t t0 = c0; t0 < c1; t0 += blockDim.x) {   // pass 2: tiles of 256 slots in slot order
    const int64_t s = t0 + threadIdx.x;
    const int32_t c = s < c1 ? a.cnt[s] : 0;
    const bool t = c > 0;
    int32_t pre[2], tot[2];
    block_excl_sumN<2>({t ? 1 : 0, c}, pre, tot, sh);
    if (t) {
      const int32_t beg = a.bucket_m ? (int32_t)(s * a.bucket_m) : ar + pre[1];
      a.off[s] = beg;
      plist[at + pre[0]] = int4{(int32_t)s, beg, c, o_grow(a, s, c)};
      if (!a.bucket_m) a.grow[s] = 0;
      if (a.counted >= 2) a.cnt[s] = 0;
    }
    at += tot[0];
    ar += tot[1];
  }
}

__global__ void __launch_bounds__(256) ordered_classify_kernel(OrdArgs a, const int4 *plist) {
  __shared__ int32_t sh[5][4];
  __shared__ int32_t base[5];   // 256-entry list, 1,024-entry list, heavy rows, dry run, light rows
  const int64_t R = a.max_rows;
  const int64_t n = (int64_t)*a.ntouched;
  if (!o_gate(a)) return;
  int4 *const desc = reinterpret_cast<int4 *>(a.split);
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t0 = (int64_t)blockIdx.x * blockDim.x; t0 < n; t0 += G) {   // block-uniform trips
    const int64_t i = t0 + threadIdx.x;
    const bool t = i < n;
    int4 e = int4{0, 0, 0, 0};
    int32_t nen = 0;
    if (t) {
      e = plist[i];
      nen = a.nent[e.x];
    }
    const int32_t c = e.z, g = e.w;
    const bool big = t && starts_big(a, nen, g);
    const bool heavy = t && !big && starts_heavy(a, c);
    const bool lite = t && !big && !heavy && starts_lite(a, c, nen, g);
    const bool risky = t && may_overflow(a, nen, g);
    int32_t pre[5], tot[5];
    block_excl_sumN<5>({t && !big && !heavy && !lite ? 1 : 0, big ? 1 : 0, heavy ? 1 : 0, risky ? 1 : 0,
                        lite ? 1 : 0},
                       pre, tot, sh);
    if (threadIdx.x == 0) {
#pragma unroll
      for (int k = 0; k < 5; ++k) base[k] = tot[k] ? (int32_t)atomicAdd(&a.nsplit[k * kNsStride], (uint32_t)tot[k]) : 0;
    }
    __syncthreads();
    if (t) {
      const int4 d = int4{e.x, e.y, e.y + c, nen};
      if (risky) desc[2 * R + base[3] + pre[3]] = d;
      if (big) desc[R + base[1] + pre[1]] = d;
      else if (heavy) desc[R - 1 - (base[2] + pre[2])] = d;
      else if (lite) desc[3 * R + base[4] + pre[4]] = d;
      else desc[base[0] + pre[0]] = d;
    }
    __syncthreads();   // base[] is rewritten by the next tile
  }
}

// ---------------------------------------------------------------------------
// Wave-level helpers.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int32_t wave_sum_i32(int32_t x) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
  return x;
}

template <typename V> struct OV;
template <> struct OV<float> {
  __device__ static float add(float x, float y) { return x + y; }
};
template <> struct OV<double> {
  __device__ static double add(double x, double y) { return x + y; }
};
template <> struct OV<int32_t> {
  __device__ static int32_t add(int32_t x, int32_t y) { return (int32_t)((uint32_t)x + (uint32_t)y); }
};
template <> struct OV<int64_t> {
  __device__ static int64_t add(int64_t x, int64_t y) { return (int64_t)((uint64_t)x + (uint64_t)y); }
};

// Records hold V values at 4-byte alignment: read/write them bytewise-safe.
template <typename V>
__device__ __forceinline__ V ldv(const uint8_t *p) {
  V v;
  __builtin_memcpy(&v, p, sizeof(V));
  return v;
}
template <typename V>
__device__ __forceinline__ void stv(uint8_t *p, V v) {
  __builtin_memcpy(p, &v, sizeof(V));
}

// Element e of a dense record body: V, or binary16 for kDenseRowOpLogFloat16 records
// (f32 tables only; dense_row_oplog_float16.hpp:144-157).
template <typename V>
__device__ __forceinline__ V rec_val(const uint8_t *body, int64_t e, int f16) {
  if constexpr (sizeof(V) == 4) {
    if (f16) {
      uint16_t h;
      __builtin_memcpy(&h, body + e * 2, 2);
      return __builtin_bit_cast(V, half_to_f32_bits(h));
    }
  }
  return ldv<V>(body + e * (int64_t)sizeof(V));
}

// Entry<V>{int32 first; V second} with the C++ layout: 8 bytes, or 16 with 4 pad bytes.
template <typename V> struct Ent {
  static constexpr int ES = sizeof(V) == 4 ? 8 : 16;
  static constexpr int VO = sizeof(V) == 4 ? 4 : 8;
};

__device__ __forceinline__ uint64_t shfl64(uint64_t x, int k) {
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)x, k, 64), hi = (uint32_t)__shfl((int)(uint32_t)(x >> 32), k, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Sort the record list of one slot (L <= 64) by value, one entry per lane: rank = number
// of smaller entries (entries are distinct).
__device__ __forceinline__ uint64_t wave_rank_sort(uint64_t r, int L, int lane, uint64_t *scratch) {
  int rank = 0;
  for (int k = 0; k < L; ++k) {
    const uint64_t x = shfl64(r, k);
    rank += (x < r) ? 1 : 0;
  }
  if (lane < L) scratch[rank] = r;
  wave_sync();
  const uint64_t out = lane < L ? scratch[lane] : 0;
  wave_sync();
  return out;
}

// A wave's global stores visible to its own later loads (other lanes' addresses included).
__device__ __forceinline__ void wave_sync_global() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// Sort the record list of one slot with L > 64 entries (distinct) ascending, in place:
// O(L log^2 L / 64) loads per lane, never O(L^2).  A row named by many records of one call
// (a row repeated inside messages: legal input no reference packer emits, or a corrupted
// message) used to take lane 0's insertion sort over the list in global memory, which ran
// for minutes at 500K records.  Runs of 64 are rank-sorted in registers, then bottom-up
// merge passes place every entry at (its index in its run) + (the entries of the partner
// run below it), found by a branch-free binary search; kG searches per lane are in flight
// together.  tmp: scratch of L entries (the list's mirror region).
__device__ __forceinline__ void wave_sort_long(uint64_t *lst, uint64_t *tmp, int32_t L, int lane, uint64_t *scratch) {
  for (int32_t c0 = 0; c0 < L; c0 += 64) {
    const int32_t n = L - c0 < 64 ? L - c0 : 64;
    uint64_t x = lane < n ? lst[c0 + lane] : ~0ull;
    x = wave_rank_sort(x, n, lane, scratch);
    if (lane < n) lst[c0 + lane] = x;
  }
  wave_sync_global();
  constexpr int kG = 4;
  uint64_t *src = lst, *dst = tmp;
  for (int32_t w = 64; w < L; w <<= 1) {
    int steps = 0;
    while ((1 << steps) <= w) ++steps;   // lower_bound over <= w entries: <= steps halvings
    for (int32_t i0 = 0; i0 < L; i0 += 64 * kG) {
      uint64_t x[kG];
      int32_t base[kG], len[kG], at[kG];
#pragma unroll
      for (int g = 0; g < kG; ++g) {
        const int32_t i = i0 + g * 64 + lane;
        const int32_t ii = i < L ? i : L - 1;
        const int32_t lo = ii / (2 * w) * (2 * w);
        const int32_t mid = lo + w < L ? lo + w : L;
        const int32_t hi = lo + 2 * w < L ? lo + 2 * w : L;
        const bool inA = ii < mid;
        x[g] = src[ii];
        base[g] = inA ? mid : lo;                 // the partner run [base, base + len)
        len[g] = inA ? hi - mid : mid - lo;
        at[g] = lo + (inA ? ii - lo : ii - mid);  // + the partner entries below x
        if (i >= L) len[g] = -1;                  // (no store)
      }
      int32_t b0[kG];
#pragma unroll
      for (int g = 0; g < kG; ++g) b0[g] = base[g];
      for (int st = 0; st < steps; ++st) {
#pragma unroll
        for (int g = 0; g < kG; ++g) {
          if (len[g] > 0) {
            const int32_t half = len[g] >> 1;
            if (src[base[g] + half] < x[g]) {
              base[g] += half + 1;
              len[g] -= half + 1;
            } else {
              len[g] = half;
            }
          }
        }
      }
#pragma unroll
      for (int g = 0; g < kG; ++g)
        if (len[g] >= 0) dst[at[g] + (base[g] - b0[g])] = x[g];
    }
    wave_sync_global();
    uint64_t *t = src;
    src = dst;
    dst = t;
  }
  if (src != lst) {
    for (int32_t i = lane; i < L; i += 64) lst[i] = src[i];
    wave_sync_global();
  }
}

// NSSumImpCalc::ApplyBatchIncGetImportance (ns_sum_imp_calc.hpp:57-77): sum of |u_i|
// over a sparse record's values, lane-parallel then a wave butterfly.
template <typename V>
__device__ __forceinline__ double sparse_importance(const uint8_t *vals, int32_t nn, int lane) {
  double p = 0.0;
  for (int32_t i = lane; i < nn; i += 64) p += __builtin_fabs((double)ldv<V>(vals + (int64_t)i * sizeof(V)));
  return wave_sum_f64(p);
}

// DRY: the capacity dry run — same walk on the LDS image, nothing written back; only rows
// whose entries plus the call's record entries exceed max_entries are simulated.
// finish_call folded into the call's last apply launch (OrdArgs.fin_done set): every block,
// once all its waves are done, counts itself; the last one folds the call's status into the
// sticky word, logs it and frees the ring slot — what finish_call_kernel does, without a
// launch of its own (an empty launch costs ~4.6 µs per call, profiles/r03/s26).
// (derived from call_status and the ring slot, not read from the OrdArgs: the extra pointers
// live through the row loop spilled the C3 kernel to scratch).  Only the blocks that take
// rows count themselves (`working`, from the launch's row count, which no block of it
// changes); a launch with no rows finishes in block 0 alone — an empty spill launch's 768
// blocks all counting cost ~11 µs (profiles/r04/s8).
__device__ __forceinline__ void finish_tail(uint32_t *call_status, int32_t ring, uint32_t working) {
  __syncthreads();
  if (threadIdx.x == 0 && (working == 0 ? blockIdx.x == 0 : blockIdx.x < working)) {
    uint32_t *status = call_status - 1 - ring;
    uint32_t *done = status + 1 + 2 * kCallRing;
    __threadfence();
    if (working == 0 || atomicAdd(done, 1u) == working - 1) {
      __threadfence();
      const uint32_t st = atomicOr(call_status, 0u);   // the L2 value: every block's bits
      atomicOr(status, st);                            // the sticky word
      status[1 + kCallRing + ring] = st;               // the call log
      atomicExch(call_status, 0u);
      atomicExch(done, 0u);
    }
  }
}

template <typename V, int KIND, bool DRY = false>
__global__ void __launch_bounds__(256) ordered_apply_kernel(OrdArgs a, int wpb) {
  extern __shared__ __align__(16) uint8_t dyn[];
  __shared__ uint64_t sort_scratch[4][64];
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  if (wib >= wpb) goto done;
  {
  const bool go = o_gate(a) && (!DRY || *a.keyflag);
  constexpr int ES = Ent<V>::ES, VO = Ent<V>::VO;
  uint8_t *E = dyn + (size_t)wib * (size_t)a.max_entries * ES;   // this wave's row image
  const int64_t wave_g = (int64_t)blockIdx.x * wpb + wib;
  const int64_t nwaves = (int64_t)gridDim.x * wpb;

  // one touched row per wave at a time (rows are independent; hot rows spread out)
  const int64_t nt = go ? (int64_t)*a.ntouched : 0;
  for (int64_t ti = wave_g; ti < nt; ti += nwaves) {
    // per-row scalars are wave-uniform: readfirstlane keeps them in SGPRs so the row's
    // loops branch on SCC instead of running under exec masks
    const int64_t slot = __builtin_amdgcn_readfirstlane(a.touched[ti]);
    if (!DRY && lane == 0) a.flags[slot] = 3;
    {
      const int32_t beg = __builtin_amdgcn_readfirstlane(a.off[slot]);
      const int32_t L = __builtin_amdgcn_readfirstlane(a.off[slot + 1]) - beg;
      uint64_t *lst = a.list + beg;
      if constexpr (DRY) {
        int32_t grow = 0;
        for (int32_t q = lane; q < L; q += 64) grow += o_ld32(rec_ptr(a, lst[q]) + 4);
        grow = wave_sum_i32(grow);
        if ((int64_t)a.nent[slot] + grow <= a.max_entries) continue;
      }
      // order the slot's records by (message, position)
      uint64_t mine = 0;
      if (L <= 64) {
        mine = wave_rank_sort(lane < L ? lst[lane] : ~0ull, L, lane, sort_scratch[wib]);
      } else {   // rare: > 64 records for one row in one call
        wave_sort_long(lst, a.list_tmp + beg, L, lane, sort_scratch[wib]);
      }

      // stage the row
      int32_t n = 0;
      if (KIND != 0) {
        n = a.nent[slot];
        const uint32_t *src = reinterpret_cast<const uint32_t *>(a.entries + slot * a.max_entries * ES);
        uint32_t *dst = reinterpret_cast<uint32_t *>(E);
        for (int32_t w = lane; w < n * (ES / 4); w += 64) dst[w] = src[w];
        wave_sync();
      }
      uint8_t *drow = reinterpret_cast<uint8_t *>(a.dense) + slot * a.row_cap * (int64_t)sizeof(V);
      double impt = a.imp ? a.imp[slot] : 0.0;

      if (a.dense_records && !a.imp) {
        // duplicate-row replay of dense records: the row in registers, kCh elements a lane
        // per pass, every record added in message order (records in flight together; the
        // row is loaded and stored once a pass, not once a record)
        constexpr int kCh = 8;
        for (int64_t e0 = 0; e0 < a.cap; e0 += 64 * kCh) {
          V x[kCh];
#pragma unroll
          for (int k = 0; k < kCh; ++k) {
            const int64_t e = e0 + k * 64 + lane;
            x[k] = e < a.cap ? ldv<V>(drow + e * sizeof(V)) : V(0);
          }
          for (int32_t q0 = 0; q0 < L; q0 += 64) {
            const uint64_t blk = L <= 64 ? mine : (q0 + lane < L ? lst[q0 + lane] : 0ull);
            const int32_t m = L - q0 < 64 ? L - q0 : 64;
            for (int32_t qq = 0; qq < m; ++qq) {
              const uint64_t r = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(blk >> 32), qq) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)blk, qq);
              const uint8_t *body = rec_ptr(a, r) + 4;
#pragma unroll
              for (int k = 0; k < kCh; ++k) {
                const int64_t e = e0 + k * 64 + lane;
                if (e < a.cap) x[k] = OV<V>::add(x[k], rec_val<V>(body, e, a.rec_f16));
              }
            }
          }
#pragma unroll
          for (int k = 0; k < kCh; ++k) {
            const int64_t e = e0 + k * 64 + lane;
            if (e < a.cap) stv<V>(drow + e * sizeof(V), x[k]);
          }
        }
        if (a.ver && lane == 0) a.ver[slot] += (uint64_t)L;   // VersionServerRow: +1 per record
        continue;
      }
      bool over = false;   // DRY: this row would exceed max_entries
      for (int32_t q = 0; q < L && !over; ++q) {
        const uint64_t r = L <= 64 ? shfl64(mine, q) : lst[q];
        const uint8_t *rec = rec_ptr(a, r);
        if (a.dense_records) {
          // duplicate-row replay of a dense record: row[e] += rec[e] (lane owns e)
          double p = 0.0;
          for (int64_t e = lane; e < a.cap; e += 64) {
            V x = ldv<V>(drow + e * sizeof(V));
            const V u = rec_val<V>(rec + 4, e, a.rec_f16);
            if (a.imp) p += imp_term<V>(x, u);
            x = OV<V>::add(x, u);
            stv<V>(drow + e * sizeof(V), x);
          }
          if (a.imp) impt += wave_sum_f64(p);
          continue;
        }
        const int32_t nn = o_ld32(rec + 4);
        const uint8_t *cols = rec + 8;
        const uint8_t *vals = rec + 8 + (int64_t)nn * 4;
        if (a.imp) impt += sparse_importance<V>(vals, nn, lane);
        if (KIND == 0) {
          // VectorStore::Inc per (col, val), in record order.  Lanes run in parallel
          // when the record's columns are strictly ascending (what both reference
          // packers emit); otherwise lane 0 walks it.
          bool asc = true;
          for (int32_t c0 = 0; c0 < nn; c0 += 64) {
            const int32_t i = c0 + lane;
            const bool bad = i < nn && i > 0 && o_ld32(cols + i * 4) <= o_ld32(cols + (i - 1) * 4);
            if (__ballot(bad)) asc = false;
          }
          if (asc) {
            for (int32_t c0 = 0; c0 < nn; c0 += 64) {
              const int32_t i = c0 + lane;
              if (i < nn) {
                uint8_t *p = drow + (int64_t)o_ld32(cols + i * 4) * sizeof(V);
                stv<V>(p, OV<V>::add(ldv<V>(p), ldv<V>(vals + (int64_t)i * sizeof(V))));
              }
            }
          } else if (lane == 0) {
            for (int32_t i = 0; i < nn; ++i) {
              uint8_t *p = drow + (int64_t)o_ld32(cols + i * 4) * sizeof(V);
              stv<V>(p, OV<V>::add(ldv<V>(p), ldv<V>(vals + (int64_t)i * sizeof(V))));
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
          __builtin_amdgcn_wave_barrier();
          continue;
        }
        // sorted-map / map rows: each Inc(col, delta) in order, wave-parallel over entries
        for (int32_t i = 0; i < nn && !over; ++i) {
          const int32_t key = o_ld32(cols + i * 4);
          const V delta = ldv<V>(vals + (int64_t)i * sizeof(V));
          if (delta == V(0)) continue;                         // :306
          int32_t idx = -1;                                    // FindIndex :230-238
          for (int32_t c0 = 0; c0 < n && idx < 0; c0 += 64) {
            const int32_t j = c0 + lane;
            const bool m = j < n && o_ld32(E + j * ES) == key;
            const uint64_t bal = __ballot(m);
            if (bal) idx = c0 + __builtin_ctzll(bal);
          }
          if (idx < 0) {
            if (n >= a.max_entries) {
              if (lane == 0) atomicOr(a.call_status, kStCapacity);
              over = DRY;
              continue;
            }
            int32_t p = n;
            if (KIND == 1) {
              // LinearSearchAndMove backward (:264-285): the new entry lands after the
              // last entry whose value is not strictly smaller than delta.
              int32_t pmax = -1;
              for (int32_t c0 = 0; c0 < n; c0 += 64) {
                const int32_t j = c0 + lane;
                const bool m = j < n && !(delta > ldv<V>(E + j * ES + VO));
                const uint64_t bal = __ballot(m);
                if (bal) pmax = c0 + 63 - __builtin_clzll(bal);
              }
              p = pmax + 1;
              for (int32_t c = n - 1; c >= p; c -= 64) {       // shift [p, n) right by one
                const int32_t j = c - lane;
                uint32_t w[ES / 4];
                const bool act = j >= p;
                if (act)
                  for (int x = 0; x < ES / 4; ++x) w[x] = reinterpret_cast<const uint32_t *>(E + j * ES)[x];
                wave_sync();
                if (act)
                  for (int x = 0; x < ES / 4; ++x) reinterpret_cast<uint32_t *>(E + (j + 1) * ES)[x] = w[x];
                wave_sync();
              }
            }
            if (lane == 0) {
              for (int x = 0; x < ES / 4; ++x) reinterpret_cast<uint32_t *>(E + p * ES)[x] = 0;
              *reinterpret_cast<int32_t *>(E + p * ES) = key;
              stv<V>(E + p * ES + VO, delta);
            }
            wave_sync();
            ++n;
          } else {
            // found: add in place (no re-sort, :325-327); remove on zero (:329-334)
            V nv = OV<V>::add(ldv<V>(E + idx * ES + VO), delta);
            wave_sync();
            if (lane == 0) stv<V>(E + idx * ES + VO, nv);
            wave_sync();
            if (nv == V(0)) {
              if (KIND == 1) {
                for (int32_t c = idx + 1; c < n; c += 64) {    // shift (idx, n) left by one
                  const int32_t j = c + lane;
                  uint32_t w[ES / 4];
                  const bool act = j < n;
                  if (act)
                    for (int x = 0; x < ES / 4; ++x) w[x] = reinterpret_cast<const uint32_t *>(E + j * ES)[x];
                  wave_sync();
                  if (act)
                    for (int x = 0; x < ES / 4; ++x) reinterpret_cast<uint32_t *>(E + (j - 1) * ES)[x] = w[x];
                  wave_sync();
                }
              } else if (idx != n - 1) {
                // MapStore::Inc erases (map_store.hpp:63-64); unordered: move last into hole
                if (lane < ES / 4)
                  reinterpret_cast<uint32_t *>(E + idx * ES)[lane] =
                      reinterpret_cast<const uint32_t *>(E + (n - 1) * ES)[lane];
                wave_sync();
              }
              --n;
            }
          }
        }
      }
      if (DRY) {
        wave_sync();
        continue;
      }
      if (KIND != 0) {
        uint32_t *dst = reinterpret_cast<uint32_t *>(a.entries + slot * a.max_entries * ES);
        const uint32_t *src = reinterpret_cast<const uint32_t *>(E);
        for (int32_t w = lane; w < n * (ES / 4); w += 64) dst[w] = src[w];
        if (lane == 0) a.nent[slot] = n;
        wave_sync();
      }
      if (a.imp && lane == 0) a.imp[slot] = impt;
      if (a.ver && lane == 0) a.ver[slot] += (uint64_t)L;   // VersionServerRow: +1 per record
    }
  }
  }
done:
  if (a.fin_ring >= 0) finish_tail(a.call_status, a.fin_ring, gridDim.x);
}

// ---------------------------------------------------------------------------
// Register-resident row image for sorted/map rows of <= 64*J entries: entry i lives in
// lane i % 64, register i / 64 ("striped").  FindIndex and the insert position are J
// compares + ballots; the one-slot shifts of LinearSearchAndMove / RemoveOneEntryAndCompact
// are wave rotates (DPP wave_ror:1 / wave_rol:1) plus a select — no LDS round trips.
template <typename T>
__device__ __forceinline__ T dpp_rot(T x, bool right) {
  if constexpr (sizeof(T) == 4) {
    int v = __builtin_bit_cast(int, x);
    v = right ? __builtin_amdgcn_update_dpp(0, v, 0x13C, 0xf, 0xf, false)    // wave_ror:1: lane l <- l-1
              : __builtin_amdgcn_update_dpp(0, v, 0x134, 0xf, 0xf, false);   // wave_rol:1: lane l <- l+1
    return __builtin_bit_cast(T, v);
  } else {
    long long v = __builtin_bit_cast(long long, x);
    int lo = (int)v, hi = (int)(v >> 32);
    if (right) {
      lo = __builtin_amdgcn_update_dpp(0, lo, 0x13C, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, hi, 0x13C, 0xf, 0xf, false);
    } else {
      lo = __builtin_amdgcn_update_dpp(0, lo, 0x134, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, hi, 0x134, 0xf, 0xf, false);
    }
    return __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  }
}

template <typename T>
__device__ __forceinline__ T bcast(T x, int src) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), src));
  } else {
    long long v = __builtin_bit_cast(long long, x);
    int lo = __builtin_amdgcn_readlane((int)v, src), hi = __builtin_amdgcn_readlane((int)(v >> 32), src);
    return __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  }
}

// ---------------------------------------------------------------------------
// Light rows, four to a wave (OrdArgs.lite, starts_lite): lane group g = lane / 16 takes
// row 4q + g of the light list, and its 16 lanes hold the row's image striped as the
// register kernel's (entry i in lane i % 16 of the group, register i / 16; <= 64 entries
// for the whole call).  The row's dependent loads (descriptor, record references, headers,
// image) go out beside three other rows', which is the point: one row per wave left the
// SIMDs waiting on those chains (DESIGN.md §5, C3 counters).  Control that depends on the
// row (its records, Incs, found / insert / removal) is group-uniform: groups diverge as
// wholes, and the one-slot shifts are DPP rotates within a 16-lane row.  FindIndex is four
// compares and a ballot (no key map at 64 entries).  SortedVectorMapStore::Inc
// (sorted_vector_map_store.hpp:175-197,305-337) and MapStore::Inc (map_store.hpp:60-65)
// semantics as the register kernel, Inc by Inc.
template <typename T>
__device__ __forceinline__ T row_rot(T x, bool right) {
  // row_ror:1 (lane l <- l-1 within its row of 16) / row_ror:15 (lane l <- l+1)
  if constexpr (sizeof(T) == 4) {
    int v = __builtin_bit_cast(int, x);
    v = right ? __builtin_amdgcn_update_dpp(0, v, 0x121, 0xf, 0xf, false)
              : __builtin_amdgcn_update_dpp(0, v, 0x12F, 0xf, 0xf, false);
    return __builtin_bit_cast(T, v);
  } else {
    long long v = __builtin_bit_cast(long long, x);
    int lo = (int)v, hi = (int)(v >> 32);
    const int c = right ? 0x121 : 0x12F;
    if (right) {
      lo = __builtin_amdgcn_update_dpp(0, lo, 0x121, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, hi, 0x121, 0xf, 0xf, false);
    } else {
      lo = __builtin_amdgcn_update_dpp(0, lo, 0x12F, 0xf, 0xf, false);
      hi = __builtin_amdgcn_update_dpp(0, hi, 0x12F, 0xf, 0xf, false);
    }
    (void)c;
    return __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  }
}

// Lane src (0..15) of the caller's 16-lane group.
template <typename T>
__device__ __forceinline__ T gshfl(T x, int src) {
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, __shfl(__builtin_bit_cast(int, x), src, 16));
  } else {
    long long v = __builtin_bit_cast(long long, x);
    const int lo = __shfl((int)v, src, 16), hi = __shfl((int)(v >> 32), src, 16);
    return __builtin_bit_cast(T, (long long)(((unsigned long long)(unsigned)hi << 32) | (unsigned)lo));
  }
}

// Remove entry idx of a group's striped image (the Inc that made it zero): sorted maps move
// entries (idx, n) down one (RemoveOneEntryAndCompact, sorted_vector_map_store.hpp:289-303,
// :329-334), maps move the last entry into the hole (MapStore erase, map_store.hpp:63-64).
// pos: the group's key map (null: none) — the removed key leaves it, moved keys follow.
template <typename V, int KIND>
__device__ __forceinline__ void lite_remove(int32_t (&key)[4], V (&val)[4], int32_t &n, int32_t idx, int gl,
                                            int8_t *pos) {
  if (pos) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j * 16 + gl == idx) pos[key[j]] = -1;
  }
  if constexpr (KIND == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t kl = row_rot(key[j], false);
      const V vl = row_rot(val[j], false);
      int32_t kn = 0;
      V vn = V(0);
      if (j + 1 < 4) {
        kn = row_rot(key[j + 1], false);
        vn = row_rot(val[j + 1], false);
      }
      const int32_t i = j * 16 + gl;
      if (i >= idx && i < n - 1) {
        key[j] = gl == 15 ? kn : kl;
        val[j] = gl == 15 ? vn : vl;
        if (pos) pos[key[j]] = (int8_t)i;
      }
    }
  } else {
    const int jl = (n - 1) >> 4, lla = (n - 1) & 15;
    int32_t lk = 0;
    V lv = V(0);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j == jl) {
        lk = gshfl(key[j], lla);
        lv = gshfl(val[j], lla);
      }
    if (idx != n - 1) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (j * 16 + gl == idx) {
          key[j] = lk;
          val[j] = lv;
          if (pos) pos[lk] = (int8_t)idx;
        }
    }
  }
  --n;
}

// One Inc(c, dd) on a group's striped image (the inserts between found runs, and every Inc
// of a row whose keys leave [0, 1024), where the key map cannot index them).
template <typename V, int KIND>
__device__ __forceinline__ void lite_inc(int32_t (&key)[4], V (&val)[4], int32_t &n, int32_t c, V dd, int gl, int gb,
                                         int8_t *pos, const OrdArgs &a) {
  int32_t idx = -1;                                   // FindIndex :230-238
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t gm = (uint32_t)(__ballot(j * 16 + gl < n && key[j] == c) >> gb) & 0xffffu;
    if (idx < 0 && gm) idx = j * 16 + __builtin_ctz(gm);
  }
  if (idx >= 0) {
    // found: add in place (no re-sort, :325-327); the owner lane tells the group if it hit 0
    bool z = false;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j * 16 + gl == idx) {
        val[j] = OV<V>::add(val[j], dd);
        z = val[j] == V(0);
      }
    if ((__ballot(z) >> gb) & 0xffffu) lite_remove<V, KIND>(key, val, n, idx, gl, pos);
    return;
  }
  if (n >= a.max_entries) {
    if (gl == 0) atomicOr(a.call_status, kStCapacity);
    return;
  }
  int32_t p = n;
  if constexpr (KIND == 1) {
    // LinearSearchAndMove backward (:264-285): after the last entry whose value is not
    // strictly smaller than the delta
    int32_t pmax = -1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t gm = (uint32_t)(__ballot(j * 16 + gl < n && !(dd > val[j])) >> gb) & 0xffffu;
      if (gm) pmax = j * 16 + 31 - __builtin_clz(gm);
    }
    p = pmax + 1;
    // entries [p, n) move up one: descending registers, rotate right within the row
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      const int32_t kr = row_rot(key[j], true);
      const V vr = row_rot(val[j], true);
      int32_t kp = 0;
      V vp = V(0);
      if (j > 0) {
        kp = row_rot(key[j - 1], true);
        vp = row_rot(val[j - 1], true);
      }
      const int32_t i = j * 16 + gl;
      if (i > p && i <= n) {
        key[j] = gl == 0 ? kp : kr;
        val[j] = gl == 0 ? vp : vr;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (j * 16 + gl == p) {
      key[j] = c;
      val[j] = dd;
    }
  ++n;
  if (pos) {   // entries [p, n) have new indices
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t i = j * 16 + gl;
      if (i >= p && i < n) pos[key[j]] = (int8_t)i;
    }
  }
}

// A light row's group (16 lanes of the caller's wave) applies its row.  pos: the group's
// key map (int8 per key of [0, 1024), -1 between rows), sv: its 64-value delta scratch
// (zero between runs), scr: the wave's 64-entry sort scratch (16 per group).
// Per record chunk of <= 16 pairs (lane t: pair t), as the register kernel's found_run:
// every lane looks its key up in the map at once; the pairs up to the chunk's next insert
// are found keys, applied together (each adds in place, sorted_vector_map_store.hpp:325-327;
// their deltas scattered by entry index, one add per register; the entries that reached
// zero removed afterwards, which leaves the same image as removing them in Inc order); the
// insert then goes Inc by Inc (LinearSearchAndMove, :264-285) and the next run starts.
template <typename V, int KIND>
__device__ __forceinline__ void lite_quad(const OrdArgs &a, int64_t q, int64_t nl, uint64_t *scr, int8_t *pos, V *sv,
                                          int32_t *pc, V *pv, const uint8_t *const *sdata, int lane) {
  // a record reference's bytes: the messages' base pointers from LDS (an index that differs
  // across the wave's groups into the kernel arguments would be one more dependent global load)
  auto rptr = [&](uint64_t e) { return sdata[e >> 56] + (e & kRefOffMask); };
  constexpr int ES = Ent<V>::ES, VO = Ent<V>::VO;
  const int gl = lane & 15, gb = lane & 48;
  const int64_t r = q * 4 + (lane >> 4);
  int4 d = int4{0, 0, 0, 0};
  if (r < nl) d = reinterpret_cast<const int4 *>(a.light)[r];
  const int64_t slot = d.x;
  const int32_t beg = d.y, L = d.z - d.y;
  int32_t n = d.w;
  const bool live = L > 0;
  // the record references, each record's pair count and the image go out together
  const uint64_t ref = gl < L ? a.list[beg + gl] : ~0ull;
  int32_t hn = 0;
  if (gl < L) hn = o_ld32(rptr(ref) + 4);
  const uint8_t *row = a.entries + slot * a.max_entries * ES;
  int32_t key[4];
  V val[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int32_t i = j * 16 + gl;
    key[j] = live && i < n ? o_ld32(row + (int64_t)i * ES) : 0;
    val[j] = live && i < n ? ldv<V>(row + (int64_t)i * ES + VO) : V(0);
  }
  if (live && gl == 0) a.flags[slot] = 3;
  // records in (message, position) order: a rank sort of the <= kLiteRecords references
  int rank = 0;
#pragma unroll
  for (int k = 0; k < kLiteRecords; ++k) {
    const uint64_t x = gshfl(ref, k);
    rank += (k < L && x < ref) ? 1 : 0;
  }
  if (gl < L) {
    scr[gb + rank] = ref;
    scr[gb + 8 + rank] = (uint64_t)(uint32_t)hn;
  }
  // the key map while every key of the row stays in [0, 1024) (group-uniform)
  bool out = false;
#pragma unroll
  for (int j = 0; j < 4; ++j) out = out || (j * 16 + gl < n && (uint32_t)key[j] >= 1024u);
  bool use_pos = live && ((__ballot(out) >> gb) & 0xffffu) == 0;
  if (use_pos) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j * 16 + gl < n) pos[key[j]] = (int8_t)(j * 16 + gl);
  }
  wave_sync();
  const uint64_t mine = gl < L ? scr[gb + gl] : 0ull;
  const int32_t mn = gl < L ? (int32_t)scr[gb + 8 + gl] : 0;
  wave_sync();
  // Every pair of the row's records (<= 64: the image plus them stays within 64 entries)
  // loaded at once into the group's LDS staging, in record order: one memory round trip
  // instead of one per record chunk.
  const int32_t n0 = gshfl(mn, 0), n1 = L > 1 ? gshfl(mn, 1) : 0, n2 = L > 2 ? gshfl(mn, 2) : 0;
  const int32_t total = n0 + n1 + n2;
  {
    const uint64_t r0 = gshfl(mine, 0), r1 = gshfl(mine, 1), r2 = gshfl(mine, 2);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int32_t k = m * 16 + gl;
      if (k < total) {
        const int qq = k >= n0 + n1 ? 2 : k >= n0 ? 1 : 0;
        const int32_t o = qq == 2 ? k - n0 - n1 : qq == 1 ? k - n0 : k;
        const int32_t nq = qq == 2 ? n2 : qq == 1 ? n1 : n0;
        const uint8_t *rp = rptr(qq == 2 ? r2 : qq == 1 ? r1 : r0);
        pc[k] = o_ld32(rp + 8 + (int64_t)o * 4);
        pv[k] = ldv<V>(rp + 8 + (int64_t)nq * 4 + (int64_t)o * sizeof(V));
      }
    }
  }
  wave_sync();
  for (int q2 = 0; q2 < kLiteRecords; ++q2) {
    if (q2 >= L) break;   // group-uniform
    const int32_t nn = q2 == 0 ? n0 : q2 == 1 ? n1 : n2;
    const int32_t pbase = q2 == 0 ? 0 : q2 == 1 ? n0 : n0 + n1;
    for (int32_t c0 = 0; c0 < nn; c0 += 16) {
      const int32_t pi = c0 + gl;
      const int32_t col = pi < nn ? pc[pbase + pi] : 0;
      const V dv = pi < nn ? pv[pbase + pi] : V(0);
      const int32_t cnt = nn - c0 < 16 ? nn - c0 : 16;
      if (use_pos && ((__ballot(gl < cnt && (uint32_t)col >= 1024u) >> gb) & 0xffffu)) {
        // a key the map cannot index: clear the map (every mapped key is in the image) and
        // finish the row Inc by Inc
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j * 16 + gl < n) pos[key[j]] = -1;
        wave_sync();
        use_pos = false;
      }
      if (!use_pos) {
        for (int32_t t = 0; t < cnt; ++t) {
          const int32_t c = gshfl(col, t);
          const V dd = gshfl(dv, t);
          if (dd == V(0)) continue;                       // :306
          lite_inc<V, KIND>(key, val, n, c, dd, gl, gb, nullptr, a);
        }
        continue;
      }
      for (int32_t t = 0; t < cnt;) {
        wave_sync();
        const int32_t my_idx = gl < cnt ? (int32_t)pos[col] : -1;
        const bool lv = gl >= t && gl < cnt && dv != V(0);
        const uint32_t ins = (uint32_t)(__ballot(lv && my_idx < 0) >> gb) & 0xffffu;
        const int32_t run_end = ins ? __builtin_ctz(ins) : cnt;
        if (run_end > t) {
          // the found run [t, run_end): distinct keys (a record's columns are distinct)
          const bool run = lv && gl < run_end;
          if (run) sv[my_idx] = dv;
          wave_sync();
          uint32_t rmm[4];
          bool anyrm = false;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int32_t i = j * 16 + gl;
            bool z = false;
            if (i < n) {
              const V x = sv[i];
              if (x != V(0)) {
                val[j] = OV<V>::add(val[j], x);
                sv[i] = V(0);
                z = val[j] == V(0);
              }
            }
            rmm[j] = (uint32_t)(__ballot(z) >> gb) & 0xffffu;
            anyrm = anyrm || rmm[j] != 0;
          }
          if (anyrm) {
            // highest index first: the lower removed indices stay where they are
            for (int j = 3; j >= 0; --j) {
              while (rmm[j]) {
                const int32_t b = 31 - __builtin_clz(rmm[j]);
                rmm[j] &= ~(1u << b);
                lite_remove<V, KIND>(key, val, n, j * 16 + b, gl, pos);
              }
            }
          }
          t = run_end;
          continue;
        }
        // an insert: pair t is not in the image
        const int32_t c = gshfl(col, t);
        const V dd = gshfl(dv, t);
        lite_inc<V, KIND>(key, val, n, c, dd, gl, gb, pos, a);
        ++t;
      }
    }
  }
  if (use_pos) {   // back to all -1: every key the row still maps is in its image
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j * 16 + gl < n) pos[key[j]] = -1;
  }
  wave_sync();
  if (live) {
    // the row image back (Entry<V> layout; 8-byte V entries carry 4 zero pad bytes)
    uint8_t *wrow = a.entries + slot * a.max_entries * ES;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int32_t i = j * 16 + gl;
      if (i < n) {
        *reinterpret_cast<int32_t *>(wrow + (int64_t)i * ES) = key[j];
        if (ES == 16) *reinterpret_cast<int32_t *>(wrow + (int64_t)i * ES + 4) = 0;
        stv<V>(wrow + (int64_t)i * ES + VO, val[j]);
      }
    }
    if (gl == 0) {
      a.nent[slot] = n;
      if (a.ver) a.ver[slot] += (uint64_t)L;   // VersionServerRow: +1 per record
    }
  }
}

// The light rows as a launch of their own: wave w takes quads w, w + nwaves, ...
template <typename V, int KIND>
__global__ void __launch_bounds__(256) ordered_apply_lite_kernel(OrdArgs a) {
  __shared__ uint64_t sort_scratch[4][64];
  __shared__ int8_t s_pos[16][1024];   // per group: key -> entry index, -1 absent
  __shared__ V s_sv[16][64];           // per group: found-run deltas by entry index
  __shared__ int32_t s_pc[16][64];     // per group: the row's (column, delta) pairs, record order
  __shared__ V s_pv[16][64];
  __shared__ const uint8_t *s_data[kMaxFused];   // the call's message base pointers
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const uint32_t st0 = *a.call_status, sk0 = *a.sticky, nl0 = *a.nlight;
  const bool go = !(st0 & (kStFatal | kStDuplicateRow)) && (a.force || !(sk0 & kStDuplicateRow));
  const int64_t nq = ((int64_t)nl0 + 3) / 4;
  if (!go || (int64_t)blockIdx.x * 4 >= nq) return;
  const int g = wib * 4 + (lane >> 4);
  if (threadIdx.x < kMaxFused) s_data[threadIdx.x] = a.ss.data[threadIdx.x];
  for (int k = lane & 15; k < 1024; k += 16) s_pos[g][k] = -1;
  for (int k = lane & 15; k < 64; k += 16) s_sv[g][k] = V(0);
  __syncthreads();
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  for (int64_t q = (int64_t)blockIdx.x * 4 + wib; q < nq; q += nwaves)
    lite_quad<V, KIND>(a, q, (int64_t)nl0, sort_scratch[wib], s_pos[g], s_sv[g], s_pc[g], s_pv[g], s_data, lane);
}

// Found-key update of a striped image: entry (jj, l) += d, returning its new value.  jj
// is wave-uniform, so a binary search over the J registers costs log2(J) uniform branches
// instead of J guarded blocks.  (A branch-free form — one compare of every register's
// entry index against idx — was slower: 420 vs 380 ns per Inc on the 1,024-entry image,
// C3 apply 0.248 vs 0.230 ms.)
template <int LO, int HI, int J, typename V>
__device__ __forceinline__ V add_at(V (&val)[J], int jj, int l, int lane, V d) {
  if constexpr (HI - LO == 1) {
    if (lane == l) val[LO] = OV<V>::add(val[LO], d);
    return bcast(val[LO], l);
  } else {
    constexpr int MID = (LO + HI) / 2;
    if (jj < MID) return add_at<LO, MID, J, V>(val, jj, l, lane, d);
    return add_at<MID, HI, J, V>(val, jj, l, lane, d);
  }
}

// A run of found-key Incs of one record chunk (lanes with distinct keys, all present,
// delta != 0, before the chunk's next insert), applied at once.  Sequentially each adds in
// place (sorted_vector_map_store.hpp:325-327) and an entry that reaches zero is removed with
// an order-preserving memmove (:329-334, RemoveOneEntryAndCompact :289-303): the adds touch
// distinct entries and move nothing, and the removals of several entries leave the same
// sequence in any order, so the run equals: every delta added to its entry, then every
// entry of the run that reached zero removed by one stable compaction.  sv (V[J*64], zero
// between runs) and ck (int32[J*64]) are the wave's LDS scratch; pos is the key map.
template <typename V, int J>
__device__ __forceinline__ int32_t found_run(int32_t (&key)[J], V (&val)[J], int32_t n, bool run, int32_t my_idx,
                                             V my_d, int lane, V *sv, int32_t *ck, int16_t *pos, bool &stale) {
  if (run) sv[my_idx] = my_d;
  wave_sync();
  uint64_t rmm[J];
  // every register at once, selects instead of branches (sv is zero outside the run's
  // entries, so a miss adds nothing and rewrites the zero it read)
  uint64_t anym = 0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int32_t i = j * 64 + lane;
    const V dv = sv[i];
    const bool hit = dv != V(0);
    const V nv = OV<V>::add(val[j], dv);
    val[j] = hit ? nv : val[j];
    sv[i] = V(0);
    rmm[j] = __ballot(hit && nv == V(0));
    anym |= rmm[j];
  }
  const bool anyrm = anym != 0;
  if (!anyrm) return n;
  // stable compaction: kept entries to LDS at their new index, the key map updated
  int32_t gone = 0;
  const uint64_t lt = (1ull << lane) - 1;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (j * 64 < n) {
      const int32_t i = j * 64 + lane;
      if (i < n) {
        if ((rmm[j] >> lane) & 1ull) {
          pos[key[j]] = -1;
        } else {
          const int32_t ni = i - gone - __builtin_popcountll(rmm[j] & lt);
          ck[ni] = key[j];
          sv[ni] = val[j];
          pos[key[j]] = (int16_t)ni;
        }
      }
      gone += __builtin_popcountll(rmm[j]);
    }
  }
  wave_sync();
  const int32_t n2 = n - gone;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    if (j * 64 < n) {
      const int32_t i = j * 64 + lane;
      if (i < n2) {
        key[j] = ck[i];
        val[j] = sv[i];
        sv[i] = V(0);
      }
    }
  }
  wave_sync();
  stale = true;
  return n2;
}

// Split tables run two launches of this kernel concurrently, over the touched rows
// ordered_offsets put in the 256- and the 1,024-entry list (a.touched / a.ntouched point
// at one list each).
// DRY: the capacity dry run (see ordered_apply_kernel); J must hold max_entries.
// Occupancy targets: 7 waves/SIMD for the 256-entry image (its rows are bound by their
// setup's dependent loads, so more rows in flight pays: C3 apply 0.123 -> 0.114 ms), the
// VGPR file's limit for J = 16.
// FIN: this instantiation may carry the call's folded finish (a.fin_ring >= 0); the others
// do not compile the tail (it costs the 7-wave kernel registers it does not have).
template <typename V, int KIND, int J, bool DRY = false, bool FIN = false>
__global__ void __launch_bounds__(256, (J <= 4 ? 7 : (sizeof(V) == 4 ? 3 : 2))) ordered_apply_reg_kernel(OrdArgs a) {
  __shared__ uint64_t sort_scratch[4][64];
  // Key -> entry-index map of the wave's row (FindIndex in one LDS read instead of J
  // ballots), usable while every key lies in [0, max_entries) (keyflag clear, and checked
  // per row at load): int16 per key, -1 = absent.
  __shared__ int16_t s_pos[4][1024 + 64];   // keys < 1,024 (the register kernels' max_entries), then one spare per lane
  __shared__ V s_sv[4][J * 64];        // found_run: deltas by entry (zero between runs), compaction values
  __shared__ int32_t s_ck[4][J * 64];  // found_run: compaction keys
  __shared__ const uint8_t *s_data[kMaxFused];   // the call's message base pointers
  // classify + dry run in one launch (DRY with a.plist): the block's risky rows, in LDS
  constexpr bool kLocal = DRY && J == 16;   // the only dry run of split tables
  __shared__ int4 s_risky[kLocal ? 256 : 1];
  __shared__ int32_t s_cls[kLocal ? 5 : 1][4];
  __shared__ int32_t s_base[6];
  const int lane = threadIdx.x & 63;
  const int wib = threadIdx.x >> 6;
  // the gate's words and the launch's row counts read at once (not one after another)
  const uint32_t st0 = *a.call_status, sk0 = *a.sticky;
  const uint32_t kf0 = DRY && a.keyflag ? *a.keyflag : 0u;
  // slots mode: the slot's count, image size and bucket pair counts loaded beside the gate's
  // words (all in bounds; the pairs are used only for a counted slot behind a passing gate)
  int32_t pc = 0, pnen = 0;
  int4 pv[kLocal ? 4 : 1];
  if constexpr (kLocal) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (a.classify_slots && i < a.max_rows) {
      pc = a.cnt[i];
      pnen = a.nent[i];
      const int4 *q = bucket_pairs4(a, i);
#pragma unroll
      for (int k = 0; k < 4; ++k) pv[k] = q[k];
    }
  }
  // slots: the classification reads the slots themselves (cnt, grow; bucket lists, whose
  // ranges need no prefix) instead of ordered_place's compact list
  const bool slots = kLocal && a.classify_slots;
  const bool local = kLocal && (a.plist || slots);
  const uint32_t nt0 = slots ? 0u : local ? *a.nplist : *a.ntouched, nh0 = a.nheavy ? *a.nheavy : 0u;
  const bool go = !(st0 & (kStFatal | kStDuplicateRow)) && (a.force || !(sk0 & kStDuplicateRow)) &&
                  (!DRY || a.grow || kf0);
  // blocks past the touched rows leave before any setup (the grid is sized by max_rows); the
  // row count is final when the launch starts (the folded finish counts the blocks below it)
  const int64_t launch_rows = slots ? a.max_rows : (int64_t)nt0 + (int64_t)nh0;
  if (kLocal && slots && !go) {
    // a failed call: no ordered_offsets or ordered_fill restores the count state, so each
    // block clears its own slots (cnt and grow zero between calls)
    const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (s < a.max_rows) {
      a.cnt[s] = 0;
      a.grow[s] = 0;
    }
  }
  if (!go || (int64_t)blockIdx.x * (local ? 256 : 4) >= launch_rows) goto done;
  if constexpr (kLocal) {
    if (local) {
      // ordered_classify's work for the block's 256 entries of the compact touched list
      // (ordered_place_kernel): each row filed in the apply launches' descriptor lists on the
      // images the previous call left; the rows whose image can outgrow max_entries stay in
      // LDS and this block's waves dry-run them below (one launch instead of two).
      const int64_t R = a.max_rows;
      int4 *const desc = reinterpret_cast<int4 *>(a.split);
      const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
      int4 e = int4{0, 0, 0, 0};
      int32_t nen = 0;
      bool t;
      if (slots) {   // slot i itself: its count state is read and cleared here (ordered_offsets')
        t = false;
        if (i < a.max_rows) {
          const int32_t c = pc;
          nen = pnen;
          t = c > 0;
          if (t) {
            e = int4{(int32_t)i, (int32_t)(i * a.bucket_m), c, pairs_sum(pv, c)};
            if (!a.bucket_m) a.grow[i] = 0;
            if (a.counted >= 2) a.cnt[i] = 0;
          }
        }
      } else {
        t = i < (int64_t)nt0;
        if (t) {
          e = a.plist[i];
          nen = a.nent[e.x];
        }
      }
      const int32_t c = e.z, g = e.w;
      const bool big = t && starts_big(a, nen, g);
      const bool heavy = t && !big && starts_heavy(a, c);
      const bool lite = t && !big && !heavy && starts_lite(a, c, nen, g);
      const bool risky = t && may_overflow(a, nen, g);
      int32_t pre[5], tot[5];
      block_excl_sumN<5>({t && !big && !heavy && !lite ? 1 : 0, big ? 1 : 0, heavy ? 1 : 0, lite ? 1 : 0,
                          risky ? 1 : 0},
                         pre, tot, s_cls);
      if (threadIdx.x == 0) {
        s_base[0] = tot[0] ? (int32_t)atomicAdd(&a.nsplit[0 * kNsStride], (uint32_t)tot[0]) : 0;
        s_base[1] = tot[1] ? (int32_t)atomicAdd(&a.nsplit[1 * kNsStride], (uint32_t)tot[1]) : 0;
        s_base[2] = tot[2] ? (int32_t)atomicAdd(&a.nsplit[2 * kNsStride], (uint32_t)tot[2]) : 0;
        s_base[3] = tot[3] ? (int32_t)atomicAdd(&a.nsplit[4 * kNsStride], (uint32_t)tot[3]) : 0;
        s_base[4] = tot[4];
      }
      __syncthreads();
      if (t) {
        const int4 d = int4{e.x, e.y, e.y + c, nen};
        if (risky) s_risky[pre[4]] = d;
        if (big) desc[R + s_base[1] + pre[1]] = d;
        else if (heavy) desc[R - 1 - (s_base[2] + pre[2])] = d;
        else if (lite) desc[3 * R + s_base[3] + pre[3]] = d;
        else desc[s_base[0] + pre[0]] = d;
      }
      __syncthreads();
      if (s_base[4] == 0) goto done;   // no risky row in the block (block-uniform)
    }
  }
  {
#pragma unroll
  for (int j = 0; j < J; ++j) s_sv[wib][j * 64 + lane] = V(0);
  for (int32_t k = lane; k < 1024; k += 64) s_pos[wib][k] = -1;
  if (threadIdx.x < kMaxFused) s_data[threadIdx.x] = a.ss.data[threadIdx.x];
  __syncthreads();
  // split tables check each record chunk's columns here instead (cols_checked below)
  const bool pos_ok = a.keyflag && (a.grow || !*a.keyflag) && a.max_entries <= 1024;
  int16_t *pos = s_pos[wib];
  constexpr int ES = Ent<V>::ES, VO = Ent<V>::VO;
  // (local: this block's own waves over its risky rows in LDS)
  const int64_t wave_g = local ? (int64_t)wib : (int64_t)blockIdx.x * 4 + wib;
  const int64_t nwaves = local ? 4 : (int64_t)gridDim.x * 4;
  const int32_t cap = (int32_t)a.max_entries;

  // one touched row per wave at a time (rows are independent; hot rows spread out);
  // heavy-first: the heavy rows' list (descending from heavy_end) before the rest
  const int64_t nh = go && !local ? (int64_t)nh0 : 0;
  const int64_t nt = !go ? 0 : local ? (int64_t)s_base[4] : nh + (int64_t)nt0;
  // Descriptor lists: the wave's next row's descriptor is loaded a row ahead (a scalar load:
  // the index is wave-uniform), so a row's setup starts from its record list, not from its
  // descriptor.
  auto desc_at = [&](int64_t t) -> int4 {
    t = (int64_t)__builtin_amdgcn_readfirstlane((int32_t)t);   // t < nt < 2^31
    if (kLocal && local) {   // written by this block above: LDS, not the scalar cache
      const int4 d = s_risky[kLocal ? t : 0];
      return int4{__builtin_amdgcn_readfirstlane(d.x), __builtin_amdgcn_readfirstlane(d.y),
                  __builtin_amdgcn_readfirstlane(d.z), __builtin_amdgcn_readfirstlane(d.w)};
    }
    const int4 *p = t < nh ? reinterpret_cast<const int4 *>(a.heavy_end) - 1 - t
                           : reinterpret_cast<const int4 *>(a.touched) + (t - nh);
    const __attribute__((address_space(4))) int32_t *q = (const __attribute__((address_space(4))) int32_t *)p;
    return int4{q[0], q[1], q[2], q[3]};
  };
  int4 d_next = int4{0, 0, 0, 0};
  if (a.desc && wave_g < nt) d_next = desc_at(wave_g);
  for (int64_t ti = wave_g; ti < nt; ti += nwaves) {
    // per-row scalars are wave-uniform: readfirstlane keeps them in SGPRs so the row's
    // loops branch on SCC instead of running under exec masks
    int64_t slot;
    int32_t beg, L, n;
    if (a.desc) {
      const int4 d = d_next;
      if (ti + nwaves < nt) d_next = desc_at(ti + nwaves);
      slot = __builtin_amdgcn_readfirstlane(d.x);
      beg = __builtin_amdgcn_readfirstlane(d.y);
      L = __builtin_amdgcn_readfirstlane(d.z) - beg;
      n = __builtin_amdgcn_readfirstlane(d.w);
    } else {
      slot = __builtin_amdgcn_readfirstlane(a.touched[ti]);
      beg = __builtin_amdgcn_readfirstlane(a.off[slot]);
      L = __builtin_amdgcn_readfirstlane(a.off[slot + 1]) - beg;
      n = __builtin_amdgcn_readfirstlane(a.nent[slot]);
    }
    if (!DRY && lane == 0) a.flags[slot] = 3;
    if (!DRY && (kOrdProbe && (a.probe & 4))) L = 0;   // timing probe: no record references, headers or pairs
    {
      uint64_t *lst = a.list + beg;
      uint64_t mine = 0;
      if (L <= 64) {
        mine = wave_rank_sort(lane < L ? lst[lane] : ~0ull, L, lane, sort_scratch[wib]);
      } else {   // rare: > 64 records for one row in one call
        wave_sort_long(lst, a.list_tmp + beg, L, lane, sort_scratch[wib]);
      }
      if constexpr (DRY) {
        int32_t grow = 0;
        for (int32_t q = lane; q < L; q += 64) grow += o_ld32(rec_ptr(a, L <= 64 ? mine : lst[q]) + 4);
        if ((int64_t)n + wave_sum_i32(grow) <= (int64_t)cap) continue;
      }
      // Record headers fetched for all of the row's records at once (lane q: record q in
      // message order; rows with <= 64 records in the call), issued before the row image so
      // that the first record's chunk loads below wait on the headers only (loads return in
      // order); each record's first 64 (column, value) pairs are loaded one record ahead, so
      // the Inc chain does not wait on a dependent global load per record.
      // lane q: record q's address (its message's base from LDS: no per-record kernel
      // argument load) and pair count
      uint64_t hp = 0;
      int32_t hn = 0;
      if (L <= 64 && lane < L) {
        hp = (uint64_t)(uintptr_t)(s_data[mine >> 56] + (mine & kRefOffMask));
        hn = o_ld32(reinterpret_cast<const uint8_t *>((uintptr_t)hp) + 4);
      }
      // load the row image
      const uint8_t *row = a.entries + slot * a.max_entries * ES;
      int32_t key[J];
      V val[J];
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int32_t i = j * 64 + lane;
        key[j] = i < n ? o_ld32(row + (int64_t)i * ES) : 0;
        val[j] = i < n ? ldv<V>(row + (int64_t)i * ES + VO) : V(0);
      }
      auto rec_at = [&](int32_t q, const uint8_t *&rec, int32_t &nn) {
        int b;
        uint64_t off;
        if (L <= 64) {
          const uint64_t p = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(hp >> 32), q) << 32) |
                             (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)hp, q);
          nn = __builtin_amdgcn_readlane(hn, q);
          rec = reinterpret_cast<const uint8_t *>((uintptr_t)p);
          return;
        } else {
          const uint64_t e = lst[q];
          const uint64_t eu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(e >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int32_t)(uint32_t)e);
          b = (int)(eu >> 56);
          off = eu & kRefOffMask;
          nn = __builtin_amdgcn_readfirstlane(o_ld32(a.ss.data[b] + off + 4));
        }
        rec = a.ss.data[b] + off;
      };
      const uint8_t *rec_n = nullptr;
      int32_t nn_n = 0, col_n = 0;
      V d_n = V(0);
      if (L > 0) {
        rec_at(0, rec_n, nn_n);
        col_n = lane < nn_n ? o_ld32(rec_n + 8 + (int64_t)lane * 4) : 0;
        d_n = lane < nn_n ? ldv<V>(rec_n + 8 + (int64_t)nn_n * 4 + (int64_t)lane * sizeof(V)) : V(0);
      }
      bool use_pos = pos_ok;
      bool pos_dirty = false;   // sorted rows: inserts not yet written to the key map
      if (use_pos) {
        bool out = false;
#pragma unroll
        for (int j = 0; j < J; ++j)
          out = out || (j * 64 + lane < n && (key[j] < 0 || key[j] >= (int32_t)a.max_entries));
        use_pos = __ballot(out) == 0;
      }
      if (use_pos) {   // the map is all -1 between rows (cleared once, then per row below)
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (j * 64 < n) pos[j * 64 + lane < n ? key[j] : 1024 + lane] = (int16_t)(j * 64 + lane);
        wave_sync();
      }
      double impt = a.imp ? a.imp[slot] : 0.0;
      bool over = false;   // DRY: this row would exceed max_entries
      bool spilled = false;
      const int32_t n0 = n;
      int32_t Lq = L;
      if (!DRY && (kOrdProbe && (a.probe & 1))) {   // timing probe: the setup's loads arrive, no record is applied
        asm volatile("" ::"v"(col_n), "v"(d_n));
        Lq = 0;
      }
      for (int32_t q = 0; q < Lq && !over; ++q) {
        const uint8_t *rec = rec_n;
        const int32_t nn = nn_n;
        int32_t col0 = col_n;
        V d0 = d_n;
        if (q + 1 < L) {
          rec_at(q + 1, rec_n, nn_n);
          col_n = lane < nn_n ? o_ld32(rec_n + 8 + (int64_t)lane * 4) : 0;
          d_n = lane < nn_n ? ldv<V>(rec_n + 8 + (int64_t)nn_n * 4 + (int64_t)lane * sizeof(V)) : V(0);
        }
        const uint8_t *cols = rec + 8;
        const uint8_t *vals = rec + 8 + (int64_t)nn * 4;
        if (a.imp) impt += sparse_importance<V>(vals, nn, lane);
        // (a do-while: a record's one chunk, the usual case, pays no entry test; an empty
        // record runs it once with no live lane)
        int32_t c0 = 0;
        do {
          const int32_t pi = c0 + lane;
          const int32_t my_col = c0 == 0 ? col0 : (pi < nn ? o_ld32(cols + (int64_t)pi * 4) : 0);
          const V my_d = c0 == 0 ? d0 : (pi < nn ? ldv<V>(vals + (int64_t)pi * sizeof(V)) : V(0));
          const int32_t cnt = nn - c0 < 64 ? nn - c0 : 64;
          // With the key map, lane t looks up its own column once for the whole chunk
          // (a record's columns are distinct, so an Inc moves no other key except by an
          // insert/remove shift, after which the chunk's lookups are re-read).
          int32_t my_idx = -1;
          bool stale = true;
          if constexpr (KIND == 1) {
            if (use_pos) {
              // the usual chunk: every live key is in the image — one lookup, one found run,
              // none of the Inc loop's control; a column the map cannot index (split
              // tables check here) or an insert takes the Inc loop below
              const bool bad = a.grow && lane < cnt && (uint32_t)my_col >= (uint32_t)a.max_entries;
              if (pos_dirty) {
                wave_sync();
#pragma unroll
                for (int j = 0; j < J; ++j) {
                  const int32_t i = j * 64 + lane;
                  if (j * 64 < n) pos[i < n ? key[j] : 1024 + lane] = (int16_t)i;
                }
                wave_sync();
                pos_dirty = false;
              }
              const int32_t pv = (int32_t)pos[bad ? 0 : my_col];   // lanes past the chunk hold column 0
              const bool live = lane < cnt && my_d != V(0);
              my_idx = lane < cnt ? pv : -1;
              if (__ballot((live && my_idx < 0) || bad) == 0) {
                stale = false;
                if (__ballot(live)) {
                  n = found_run<V, J>(key, val, n, live, my_idx, my_d, lane, s_sv[wib], s_ck[wib], pos, stale);
                  if (stale) pos_dirty = false;   // the compaction rewrote the whole map
                }
                continue;
              }
              my_idx = -1;   // the Inc loop looks the chunk up again
            }
          }
          if (use_pos && a.grow &&
              __ballot(lane < cnt && (uint32_t)my_col >= (uint32_t)a.max_entries)) {
            // a column outside [0, max_entries) (split tables: no column scan before the
            // apply): the key map cannot index it — clear it (every mapped key is in the
            // image) and finish the row on ballots
            wave_sync();
#pragma unroll
            for (int j = 0; j < J; ++j)
              if (j * 64 < n && j * 64 + lane < n) pos[key[j]] = -1;
            wave_sync();
            use_pos = false;
            pos_dirty = false;
          }
          for (int32_t t = 0; t < cnt && !over; ++t) {
            if constexpr (KIND == 1) {
              if (use_pos) {
                // the found keys up to the chunk's next insert, at once (found_run)
                if (stale) {
                  if (pos_dirty) {   // inserts since the map was last written: rewrite it
                    wave_sync();
#pragma unroll
                    for (int j = 0; j < J; ++j) {
                      const int32_t i = j * 64 + lane;
                      if (j * 64 < n && i < n) pos[key[j]] = (int16_t)i;
                    }
                    wave_sync();
                    pos_dirty = false;
                  }
                  my_idx = lane < cnt ? (int32_t)pos[my_col] : -1;
                  stale = false;
                }
                const bool live = lane >= t && lane < cnt && my_d != V(0);
                const uint64_t ins = __ballot(live && my_idx < 0);
                const int32_t run_end = ins ? (int32_t)__builtin_ctzll(ins) : cnt;
                if (run_end > t) {
                  const bool run = live && lane < run_end;
                  if (__ballot(run)) {
                    n = found_run<V, J>(key, val, n, run, my_idx, my_d, lane, s_sv[wib], s_ck[wib], pos, stale);
                    if (stale) pos_dirty = false;   // the compaction rewrote the whole map
                  }
                  t = run_end - 1;
                  continue;
                }
              }
            }
            const int32_t c = __builtin_amdgcn_readlane(my_col, t);
            const V d = bcast(my_d, t);
            if (d == V(0)) continue;                                  // :306
            int32_t idx = -1;                                         // FindIndex :230-238
            if (use_pos) {
              if (stale) {
                my_idx = lane < cnt ? (int32_t)pos[my_col] : -1;
                stale = false;
              }
              idx = __builtin_amdgcn_readlane(my_idx, t);
            } else {
#pragma unroll
              for (int j = 0; j < J; ++j) {
                if (j * 64 < n && idx < 0) {
                  const uint64_t bal = __ballot(j * 64 + lane < n && key[j] == c);
                  if (bal) idx = j * 64 + __builtin_ctzll(bal);
                }
              }
            }
            if (idx < 0) {
              // outgrows this image: hand the row on (only the 256-entry launch of a split
              // table spills; the 1,024-entry image holds every entry max_entries allows)
              if (!DRY && a.spill && a.spill_list && J * 64 < a.max_entries && n >= J * 64) {
                spilled = true;
                over = true;
                continue;
              }
              if (n >= cap) {
                if (lane == 0) atomicOr(a.call_status, kStCapacity);
                over = DRY;
                continue;
              }
              int32_t p = n;
              if (KIND == 1) {
                // LinearSearchAndMove backward (:264-285)
                int32_t pmax = -1;
#pragma unroll
                for (int j = 0; j < J; ++j) {
                  if (j * 64 < n) {
                    const uint64_t bal = __ballot(j * 64 + lane < n && !(d > val[j]));
                    if (bal) pmax = j * 64 + 63 - __builtin_clzll(bal);
                  }
                }
                p = pmax + 1;
                // entries [p, n) move to i + 1: descending j, rotate right by one lane
                const int jhi = n >> 6, jlo = p >> 6;   // chunks holding entries p+1 .. n
#pragma unroll
                for (int j = J - 1; j >= 0; --j) {
                  if (j <= jhi && j >= jlo) {
                    const int32_t kr = dpp_rot(key[j], true);
                    const V vr = dpp_rot(val[j], true);
                    int32_t kp = 0;
                    V vp = V(0);
                    if (j > 0) {
                      kp = dpp_rot(key[j - 1], true);
                      vp = dpp_rot(val[j - 1], true);
                    }
                    const int32_t i = j * 64 + lane;
                    const int32_t ks = lane == 0 ? kp : kr;
                    const V vs = lane == 0 ? vp : vr;
                    if (i > p && i <= n) {
                      key[j] = ks;
                      val[j] = vs;
                    }
                  }
                }
              }
#pragma unroll
              for (int j = 0; j < J; ++j)
                if (j * 64 + lane == p) {
                  key[j] = c;
                  val[j] = d;
                }
              ++n;
              if (KIND == 1 && use_pos) {
                // entries [p, n) moved up one: the chunk's other looked-up indices follow
                // arithmetically; the key map is rewritten before the next lookup
                my_idx += my_idx >= p ? 1 : 0;
                pos_dirty = true;
              } else if (use_pos) {   // entries [p, n) moved or arrived: their new indices
                stale = true;
                wave_sync();
#pragma unroll
                for (int j = 0; j < J; ++j) {
                  const int32_t i = j * 64 + lane;
                  if (i >= p && i < n) pos[key[j]] = (int16_t)i;
                }
                wave_sync();
              }
            } else {
              // found: add in place (:325-327), remove on zero (:329-334)
              const V nv = add_at<0, J>(val, idx >> 6, idx & 63, lane, d);
              if (nv == V(0)) {
                if (KIND == 1) {
                  // entries (idx, n) move to i - 1: ascending j, rotate left by one lane
                  const int jlo = idx >> 6, jhi = (n - 1) >> 6;   // chunks holding idx .. n-2
#pragma unroll
                  for (int j = 0; j < J; ++j) {
                    if (j >= jlo && j <= jhi) {
                      const int32_t kl = dpp_rot(key[j], false);
                      const V vl = dpp_rot(val[j], false);
                      int32_t kn = 0;
                      V vn = V(0);
                      if (j + 1 < J) {
                        kn = dpp_rot(key[j + 1], false);
                        vn = dpp_rot(val[j + 1], false);
                      }
                      const int32_t i = j * 64 + lane;
                      const int32_t ks = lane == 63 ? kn : kl;
                      const V vs = lane == 63 ? vn : vl;
                      if (i >= idx && i < n - 1) {
                        key[j] = ks;
                        val[j] = vs;
                      }
                    }
                  }
                  if (use_pos) {   // c leaves; entries (idx, n) moved down one
                    stale = true;
                    wave_sync();
                    if (lane == 0) pos[c] = -1;
                    wave_sync();
#pragma unroll
                    for (int j = 0; j < J; ++j) {
                      const int32_t i = j * 64 + lane;
                      if (i >= idx && i < n - 1) pos[key[j]] = (int16_t)i;
                    }
                    wave_sync();
                  }
                } else {
                  // MapStore erase; unordered: the last entry fills the hole
                  int32_t lk = 0;
                  V lv = V(0);
#pragma unroll
                  for (int j = 0; j < J; ++j)
                    if (j == ((n - 1) >> 6)) {
                      lk = __builtin_amdgcn_readlane(key[j], (n - 1) & 63);
                      lv = bcast(val[j], (n - 1) & 63);
                    }
#pragma unroll
                  for (int j = 0; j < J; ++j)
                    if (j * 64 + lane == idx) {
                      key[j] = lk;
                      val[j] = lv;
                    }
                  if (use_pos) {   // c leaves; the last entry takes its index
                    stale = true;
                    wave_sync();
                    if (lane == 0) {
                      pos[c] = -1;
                      if (idx != n - 1) pos[lk] = (int16_t)idx;
                    }
                    wave_sync();
                  }
                }
                --n;
              }
            }
          }
        } while ((c0 += 64) < nn && !over);
      }
      if (use_pos) {
        // back to all -1: every key the row ever mapped is in the final image or was
        // unmapped when it left
        wave_sync();
#pragma unroll
        for (int j = 0; j < J; ++j)
          if (j * 64 < n) pos[j * 64 + lane < n ? key[j] : 1024 + lane] = -1;
        wave_sync();
      }
      if (DRY) continue;
      if (spilled) {   // nothing of the row was written: the 1,024-entry launch redoes it
        if (lane == 0) {
          const uint32_t k = atomicAdd(a.nspill, 1u);
          reinterpret_cast<int4 *>(a.spill_list)[k] = int4{(int32_t)slot, beg, beg + L, n0};
        }
        continue;
      }
      if (kOrdProbe && (a.probe & 2)) continue;   // timing probe: no write-back
      // write the row image back (Entry<V> layout; 8-byte V entries carry 4 zero pad bytes)
      uint8_t *wrow = a.entries + slot * a.max_entries * ES;
#pragma unroll
      for (int j = 0; j < J; ++j) {
        const int32_t i = j * 64 + lane;
        if (i < n) {
          *reinterpret_cast<int32_t *>(wrow + (int64_t)i * ES) = key[j];
          if (ES == 16) *reinterpret_cast<int32_t *>(wrow + (int64_t)i * ES + 4) = 0;
          stv<V>(wrow + (int64_t)i * ES + VO, val[j]);
        }
      }
      if (lane == 0) a.nent[slot] = n;
      if (a.imp && lane == 0) a.imp[slot] = impt;
      if (a.ver && lane == 0) a.ver[slot] += (uint64_t)L;
    }
  }
  }
done:
  if constexpr (FIN) {
    if (a.fin_ring >= 0) {
      const int64_t wk = (launch_rows + 3) / 4;
      finish_tail(a.call_status, a.fin_ring, (uint32_t)(wk < (int64_t)gridDim.x ? wk : (int64_t)gridDim.x));
    }
  }
}

// ---------------------------------------------------------------------------
// Serve-back of sorted/map rows: gather (count, entries) for a list of slots.
template <int ES>
__global__ void gather_entries_kernel(const int32_t *nent, const uint8_t *entries, int64_t max_entries,
                                      const int64_t *slots, int32_t n, int32_t *out_n, uint8_t *out) {
  const int r = blockIdx.x;
  if (r >= n) return;
  const int64_t s = slots[r];
  const int32_t k = s >= 0 ? nent[s] : 0;
  if (threadIdx.x == 0) out_n[r] = k;
  const uint32_t *src = reinterpret_cast<const uint32_t *>(entries + s * max_entries * ES);
  uint32_t *dst = reinterpret_cast<uint32_t *>(out + (int64_t)r * max_entries * ES);
  for (int32_t w = threadIdx.x; w < k * (ES / 4); w += blockDim.x) dst[w] = src[w];
}

// ---------------------------------------------------------------------------
int g_ord_split = 3;  // rows of > 256-entry tables: 3 spill mode with heavy rows first (default),
                      // 2 spill mode, 1 classified into concurrent 256- / 1,024-entry launches,
                      // 0 one 1,024-entry launch (C3 apply 0.088 / 0.059 / 0.051 ms for 1 / 2 / 3,
                      // profiles/r03/s12)

// One touched row per wave at a time: the grid is sized by rows (the touched count is on
// the device), not by 64-row tiles — 100K rows as tiles gave 1,564 waves for ~35K touched
// rows, 1.5 waves per SIMD (profiles/r01/exp_c3_grid.txt).
static unsigned row_blocks(int64_t n, int wpb) {
  int64_t blocks = (n + wpb - 1) / wpb;
  if (blocks > 4096) blocks = 4096;
  return (unsigned)(blocks < 1 ? 1 : blocks);
}

// Launches that usually find few rows or none — the capacity dry run (only when a key
// lies outside [0, max_entries)) and the 1,024-entry launch of spill mode (rows already
// 7/8 full, and spills) — take the J = 16 kernel's resident grid (3 waves per SIMD: 768
// blocks of 4 waves on 256 CUs) and loop over their rows: an empty 4,096-block launch
// cost 4.7-4.9 µs per C3 step (profiles/r03/s26/c3_kernel_stats.csv).
static unsigned few_row_blocks(int64_t n) { return std::min(row_blocks(n, 4), 768u); }
int g_offsets_blocks = 1024;   // PSX_VARIANT_OFFSETS_GRID: ordered_offsets' grid cap
int g_dry_blocks = 128;        // PSX_VARIANT_DRY_GRID: the capacity dry run's grid cap
int g_classify_blocks = 256;   // PSX_VARIANT_CLASSIFY_GRID: ordered_classify's grid cap
int g_classify_dry = 1;        // PSX_VARIANT_CLASSIFY_DRY: ordered_classify as the dry run's prologue

static void lds_geometry(int dtype, const OrdArgs &a, int *wpb, size_t *lds) {
  const int esz = (dtype == 0 || dtype == 2) ? 8 : 16;
  const int64_t per_wave = a.kind == 0 ? 0 : a.max_entries * esz;
  int w = 4;
  while (w > 1 && per_wave * w > 150 * 1024) --w;
  *wpb = w;
  *lds = (size_t)per_wave * w;
}

template <typename V, int KIND>
static void launch_dry(const OrdArgs &a0, int dtype, hipStream_t st) {
  OrdArgs a = a0;
  if (a.grow) {   // split tables: the rows that may overflow (ordered_offsets), as descriptors
    a.touched = a.split + 2 * 4 * a.max_rows;
    a.ntouched = a.nsplit + 3 * kNsStride;
    a.desc = 1;
  }
  // (the rows are rare — keys outside [0, max_entries), images about to overflow — and the
  // launch runs on every call of a split table: a small grid keeps the empty case cheap)
  const unsigned blocks = std::min(few_row_blocks(a.max_rows), (unsigned)std::max(1, g_dry_blocks));
  if (a.max_entries <= 64)
    hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 1, true>), dim3(blocks), dim3(256), 0, st, a);
  else if (a.max_entries <= 256)
    hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 4, true>), dim3(blocks), dim3(256), 0, st, a);
  else if (a.max_entries <= 1024)
    hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 16, true>), dim3(blocks), dim3(256), 0, st, a);
  else {
    int wpb;
    size_t lds;
    lds_geometry(dtype, a, &wpb, &lds);
    hipLaunchKernelGGL((ordered_apply_kernel<V, KIND, true>), dim3(row_blocks(a.max_rows, wpb)), dim3(256), lds, st,
                       a, wpb);
  }
}

// Stage 1 of the ordered path (before any table of the call is applied): record lists by
// slot, every validation, and the capacity dry run of sorted/map tables.
hipError_t launch_ordered_prep(int dtype, const OrdArgs &a, int2 *wfill, hipStream_t st) {
  if (a.counted == 0 || a.counted == 3)
    hipLaunchKernelGGL(ordered_count_kernel, dim3(1024), dim3(256), 0, st, a, a.counted == 3 ? wfill : nullptr);
  if (a.grow)
    hipLaunchKernelGGL(ordered_offsets_kernel, dim3(std::min(row_blocks(a.max_rows, 256), (unsigned)std::max(1, g_offsets_blocks))),
                       dim3(256), 0, st, a);
  else
    launch_exclusive_scan<int32_t>(a.cnt, a.max_rows, a.off, a.tsum, st);
  if (!a.bucket_m) hipLaunchKernelGGL(ordered_fill_kernel, dim3(1024), dim3(256), 0, st, a, wfill);
  if (a.kind != 0 && !a.dense_records && a.keyflag) {
#define PSX_DRY(V) do { if (a.kind == 1) launch_dry<V, 1>(a, dtype, st); else launch_dry<V, 2>(a, dtype, st); } while (0)
    switch (dtype) {
      case 0: PSX_DRY(float); break;
      case 1: PSX_DRY(double); break;
      case 2: PSX_DRY(int32_t); break;
      default: PSX_DRY(int64_t); break;
    }
#undef PSX_DRY
  }
  return hipGetLastError();
}

// The pipelined split-table prep in its two halves (ordered_place_kernel above): the records'
// half on the prep stream (ordered_count where the walk did not count, ordered_place,
// ordered_fill), the rows' half on the context stream (ordered_classify, the capacity dry
// run).  A split table only (a.grow).
hipError_t launch_ordered_prep_records(const OrdArgs &a, int2 *wfill, int4 *plist, hipStream_t st) {
  if (a.counted == 0 || a.counted == 3)
    hipLaunchKernelGGL(ordered_count_kernel, dim3(1024), dim3(256), 0, st, a, a.counted == 3 ? wfill : nullptr);
  hipLaunchKernelGGL(ordered_place_kernel,
                     dim3(std::min(row_blocks(a.max_rows, 256), (unsigned)std::max(1, g_offsets_blocks))), dim3(256), 0,
                     st, a, plist);
  if (!a.bucket_m) hipLaunchKernelGGL(ordered_fill_kernel, dim3(1024), dim3(256), 0, st, a, wfill);
  return hipGetLastError();
}

// The dry run's kernel (J = 16: split tables have 256 < max_entries <= 1,024) with
// ordered_classify's work as its prologue, one block per 256 compact-list entries.
template <typename V, int KIND>
static void launch_classify_dry(const OrdArgs &a0, const int4 *plist, hipStream_t st) {
  OrdArgs a = a0;
  a.plist = plist;
  a.nplist = a0.ntouched;       // ordered_place's count
  a.desc = 1;
  const unsigned blocks = (unsigned)((a.max_rows + 255) / 256);
  hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 16, true>), dim3(blocks), dim3(256), 0, st, a);
}

// Bucket lists of a ranked split table (a.bucket_m, a.counted >= 2): no prefix is needed, so
// the whole prep after the count is the dry run's kernel classifying its 256 slots as its
// prologue (ordered_offsets' classification) — one launch where the prefix form has
// ordered_offsets, ordered_fill and the dry run.
bool ordered_prep_in_dry_run(const OrdArgs &a) {
  return g_classify_dry && a.bucket_m && a.counted >= 2 && a.kind != 0 && !a.dense_records && a.keyflag &&
         a.max_entries <= 1024 && (a.max_rows + 255) / 256 <= 65535;
}

template <typename V, int KIND>
static void launch_slots_dry(const OrdArgs &a0, hipStream_t st) {
  OrdArgs a = a0;
  a.classify_slots = 1;
  a.plist = nullptr;
  a.desc = 1;
  const unsigned blocks = (unsigned)((a.max_rows + 255) / 256);
  hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 16, true>), dim3(blocks), dim3(256), 0, st, a);
}

hipError_t launch_ordered_count(const OrdArgs &a, int2 *wfill, hipStream_t st) {
  hipLaunchKernelGGL(ordered_count_kernel, dim3(1024), dim3(256), 0, st, a, wfill);
  return hipGetLastError();
}

hipError_t launch_ordered_prep_slots(int dtype, const OrdArgs &a, int2 *wfill, bool with_count, hipStream_t st) {
  if (with_count && a.counted == 3)   // ordered_count ranks and fills the buckets
    hipLaunchKernelGGL(ordered_count_kernel, dim3(1024), dim3(256), 0, st, a, wfill);
#define PSX_SD(V) do { if (a.kind == 1) launch_slots_dry<V, 1>(a, st); else launch_slots_dry<V, 2>(a, st); } while (0)
  switch (dtype) {
    case 0: PSX_SD(float); break;
    case 1: PSX_SD(double); break;
    case 2: PSX_SD(int32_t); break;
    default: PSX_SD(int64_t); break;
  }
#undef PSX_SD
  return hipGetLastError();
}

hipError_t launch_ordered_prep_rows(int dtype, const OrdArgs &a, const int4 *plist, hipStream_t st) {
  if (g_classify_dry && a.kind != 0 && !a.dense_records && a.keyflag && a.max_entries <= 1024 &&
      (a.max_rows + 255) / 256 <= 65535) {
#define PSX_CD(V) do { if (a.kind == 1) launch_classify_dry<V, 1>(a, plist, st); else launch_classify_dry<V, 2>(a, plist, st); } while (0)
    switch (dtype) {
      case 0: PSX_CD(float); break;
      case 1: PSX_CD(double); break;
      case 2: PSX_CD(int32_t); break;
      default: PSX_CD(int64_t); break;
    }
#undef PSX_CD
    return hipGetLastError();
  }
  hipLaunchKernelGGL(ordered_classify_kernel,
                     dim3(std::min(row_blocks(a.max_rows, 256), (unsigned)std::max(1, g_classify_blocks))), dim3(256),
                     0, st, a, plist);
  if (a.kind != 0 && !a.dense_records && a.keyflag) {
#define PSX_DRY(V) do { if (a.kind == 1) launch_dry<V, 1>(a, dtype, st); else launch_dry<V, 2>(a, dtype, st); } while (0)
    switch (dtype) {
      case 0: PSX_DRY(float); break;
      case 1: PSX_DRY(double); break;
      case 2: PSX_DRY(int32_t); break;
      default: PSX_DRY(int64_t); break;
    }
#undef PSX_DRY
  }
  return hipGetLastError();
}

// Stage 2: the apply (after every table's stage 1 and the duplicate-row gate).  Split
// tables (a.grow set): the 1,024-entry launch on `aux` (its long
// per-row chains start first) beside the 256-entry launch on `st`; `st` joins `aux`.
hipError_t launch_ordered_apply(int dtype, const OrdArgs &a, hipStream_t st, const Fork &fk) {
  if (a.kind != 0 && a.max_entries <= 1024) {
    const unsigned blocks = row_blocks(a.max_rows, 4);
    OrdArgs small = a, big = a;
    if (a.grow) small.fin_ring = -1;   // a folded finish goes with the last launch (big)
    if (a.grow && !a.spill) big.fin_ring = -1;   // concurrent launches: finish_call after the join
    if (a.grow) {   // ordered_offsets wrote the two descriptor lists
      small.touched = a.split;
      small.ntouched = a.nsplit;   // counter 0
      big.touched = a.split + 4 * a.max_rows;
      big.ntouched = a.nsplit + 1 * kNsStride;
      small.desc = big.desc = 1;
      small.spill_list = big.touched;
      small.nspill = big.ntouched;
      if (a.spill & 2) {   // heavy rows: listed backwards
        small.heavy_end = a.split + 4 * a.max_rows;   // end of the 256-entry list's region
        small.nheavy = a.nsplit + 2 * kNsStride;
      }
      if (a.lite) {   // light rows, four to a wave, in a launch of their own
        small.light = a.split + 12 * a.max_rows;
        small.nlight = a.nsplit + 4 * kNsStride;
      }
      if (!a.spill) {   // concurrent launches: the side stream starts behind the prep
        hipError_t e = hipEventRecord(fk.fork, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(fk.aux, fk.fork, 0);
        if (e != hipSuccess) return e;
      }
    }

#define PSX_REG(V, KIND)                                                                           \
  do {                                                                                             \
    if (a.max_entries <= 64)                                                                       \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 1, false, true>), dim3(blocks), dim3(256), 0, st, a); \
    else if (a.max_entries <= 256)                                                                 \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 4, false, true>), dim3(blocks), dim3(256), 0, st, a); \
    else if (a.grow && a.spill) {                                                                  \
      if (a.lite)   /* the light rows, four to a wave, before the 256-entry launch */              \
        hipLaunchKernelGGL((ordered_apply_lite_kernel<V, KIND>), dim3(row_blocks((a.max_rows + 3) / 4, 4)), \
                           dim3(256), 0, st, small);                                               \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 4>), dim3(blocks), dim3(256), 0, st, small); \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 16, false, true>), dim3(few_row_blocks(a.max_rows)), dim3(256), 0, st, big); \
    } else if (a.grow) {                                                                           \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 16>), dim3(blocks), dim3(256), 0, fk.aux, big); \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 4>), dim3(blocks), dim3(256), 0, st, small); \
    } else                                                                                         \
      hipLaunchKernelGGL((ordered_apply_reg_kernel<V, KIND, 16, false, true>), dim3(blocks), dim3(256), 0, st, a); \
  } while (0)
#define PSX_REGK(V) do { if (a.kind == 1) PSX_REG(V, 1); else PSX_REG(V, 2); } while (0)
    switch (dtype) {
      case 0: PSX_REGK(float); break;
      case 1: PSX_REGK(double); break;
      case 2: PSX_REGK(int32_t); break;
      default: PSX_REGK(int64_t); break;
    }
#undef PSX_REGK
#undef PSX_REG
    if (a.grow && !a.spill) {
      hipError_t e = hipEventRecord(fk.join, fk.aux);
      if (e == hipSuccess) e = hipStreamWaitEvent(st, fk.join, 0);
      if (e != hipSuccess) return e;
    }
    return hipGetLastError();
  }
  // LDS row images (max_entries > 1024) or dense rows
  int wpb;
  size_t lds;
  lds_geometry(dtype, a, &wpb, &lds);
  const unsigned blocks = row_blocks(a.max_rows, wpb);
#define PSX_ORD(V)                                                                                 \
  do {                                                                                             \
    if (a.kind == 0)                                                                               \
      hipLaunchKernelGGL((ordered_apply_kernel<V, 0>), dim3(blocks), dim3(256), lds, st, a, wpb);  \
    else if (a.kind == 1)                                                                          \
      hipLaunchKernelGGL((ordered_apply_kernel<V, 1>), dim3(blocks), dim3(256), lds, st, a, wpb);  \
    else                                                                                           \
      hipLaunchKernelGGL((ordered_apply_kernel<V, 2>), dim3(blocks), dim3(256), lds, st, a, wpb);  \
  } while (0)
  switch (dtype) {
    case 0: PSX_ORD(float); break;
    case 1: PSX_ORD(double); break;
    case 2: PSX_ORD(int32_t); break;
    default: PSX_ORD(int64_t); break;
  }
#undef PSX_ORD
  return hipGetLastError();
}

hipError_t launch_gather_entries(int dtype, const int32_t *nent, const uint8_t *entries, int64_t max_entries,
                                 const int64_t *slots, int32_t n, int32_t *out_n, uint8_t *out,
                                 hipStream_t st) {
  if (n <= 0) return hipSuccess;
  if (dtype == 0 || dtype == 2)
    hipLaunchKernelGGL(gather_entries_kernel<8>, dim3(n), dim3(256), 0, st, nent, entries, max_entries, slots,
                       n, out_n, out);
  else
    hipLaunchKernelGGL(gather_entries_kernel<16>, dim3(n), dim3(256), 0, st, nent, entries, max_entries, slots,
                       n, out_n, out);
  return hipGetLastError();
}

// Gate: a duplicate row inside any message of a fast-path dense table turns the whole
// call into a replay (nothing is applied now).
__global__ void gate_kernel(const Seg *segs, const uint32_t *counters, TableMask m, int B, uint32_t *call_status) {
  if (threadIdx.x != 0) return;
  for (int i = 0; i < m.n; ++i) {
    const int t = m.t[i];
    for (int b = 0; b < B; ++b) {
      const Seg sg = segs[b * kMaxTables + t];
      if (sg.rec0 >= 0 && !sg.sparse && counters[t * kMaxFused + b] != (uint32_t)sg.num_rows) {
        atomicOr(call_status, kStDuplicateRow);
        return;
      }
    }
  }
}

hipError_t launch_gate(const Seg *segs, const uint32_t *counters, const TableMask &m, int B,
                       uint32_t *call_status, hipStream_t st) {
  hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, st, segs, counters, m, B, call_status);
  return hipGetLastError();
}

}  // namespace psx
