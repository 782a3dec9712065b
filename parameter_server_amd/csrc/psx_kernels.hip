// psx_kernels.hip — CDNA4 (gfx950) kernels of the row-update apply path.
//
// Pipeline for one psx_apply_streams_device call (B messages, applied in order):
//   decode_streams   one workgroup per message walks the Appendix-A headers
//                    (SerializedOpLogReader::Restart/Next/StartNewTable,
//                    src/petuum_ps/server/serialized_oplog_reader.hpp:30-133) and writes
//                    one Seg per (message, table).
//   dense_index      inv[slot][b] = record number, one 4-byte row-id read per record.
//   dense_verify     per-message count of claimed slots; a shortfall means a row occurs
//                    twice in one message (or out of range) -> the fused apply is skipped.
//   dense_apply      one wave per 64-slot tile; per touched slot it streams the table row
//                    and the B records and adds them IN MESSAGE ORDER
//                    (NumericStoreRow::ApplyDenseBatchIncUnsafe,
//                    src/petuum_ps_common/storage/numeric_store_row.hpp:177-185, once per
//                    message), so f32/f64 results are bit-identical to the reference loop.
//   finish_call      folds the per-call status into the sticky word.
// No MFMA: this is an HBM-bound element-wise add (roofline).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "psx_device.hpp"

namespace psx {

__device__ __forceinline__ int32_t ld32(const uint8_t *p) {
  return *reinterpret_cast<const int32_t *>(p);
}
__device__ __forceinline__ uint64_t ld64_a4(const uint8_t *p) {
  // size_t fields sit at 4-byte-aligned offsets (Appendix A): two dword loads.
  uint64_t lo = *reinterpret_cast<const uint32_t *>(p);
  uint64_t hi = *reinterpret_cast<const uint32_t *>(p + 4);
  return lo | (hi << 32);
}

// ---------------------------------------------------------------------------
// decode_streams: grid = B workgroups of 1024 threads; thread 0 walks one message's
// headers.  Sparse tables' variable-length records form a dependency chain (each size
// comes from its n), so the walk is sequential: the block stages the table's records
// through LDS in 32 KiB windows of a fixed grid (the next one prefetched into registers
// while the current one is walked), builds 1/2/4/8/16-record jump tables in parallel, and
// thread 0 hops the chain 16 records per dependent LDS read.
constexpr int kDecodeThreads = 1024;
constexpr int kDecodeWindowWords = 8192;    // 32 KiB window
constexpr uint64_t kWinBytes = (uint64_t)kDecodeWindowWords * 4;
constexpr int kJumpLevels = 5;              // 1, 2, 4, 8, 16 records
constexpr uint16_t kU16 = 0xFFFFu;          // chain leaves the window / bad header

// Indexed messages (ix.p[b] set, psx_apply_indexed): a sparse table's record offsets come
// from the producer's index.  This kernel (one workgroup per message) checks only the
// table's first and last offsets and steps to the table's end; idx_verify (psx_walk.hip,
// a grid over every record) checks the chain (each record ends where the next begins,
// inside the message), writes the offsets and, for walk-counted split tables, does
// ordered_count's work.  What this kernel finds wrong after an indexed table of the
// message may come from a bad index: those status bits wait in idxw[4 b] and reach the
// call only if idx_verify finds the message's index sound (a bad index is kStMalformed).
// idxw: 4 words per message ([0] pending bits, [1] bad index).
__global__ void __launch_bounds__(kDecodeThreads) decode_streams_kernel(StreamSet ss, TableDir dir, Seg *segs,
                                                                        uint64_t *recoff, uint32_t *call_status,
                                                                        uint32_t *counters, uint32_t *ntouched,
                                                                        IdxSet ix, uint32_t *idxw) {
  __shared__ uint32_t win[kDecodeWindowWords + 1];                 // + 1 halo word
  __shared__ uint16_t jt[kJumpLevels][kDecodeWindowWords];          // jt[l]: 2^l records on
  __shared__ uint16_t a16[kDecodeWindowWords / 32];                 // starts of 16-record hops
  __shared__ uint16_t a4[8], a1s[16];                               // 4-record hops (<= 3), single records (<= 4)
  __shared__ uint32_t sh_n16, sh_n4, sh_ns;
  __shared__ int32_t sh_bad;
  __shared__ uint64_t sh_off, sh_rk, sh_left, sh_kk, sh_t0;
  uint32_t pf[kDecodeWindowWords / kDecodeThreads];                 // the prefetched window
  uint64_t pf_w0 = ~0ull;
  __shared__ int32_t sh_state;   // 0 walking headers, 1 sparse walk needs a window, 2 done, 3 indexed sparse table
  __shared__ int32_t sh_t, sh_ntab, sh_k;
  __shared__ uint32_t *sh_err;   // where header errors go: call_status, or idxw[4 b] after an indexed table
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
  }
  const uint8_t *p = ss.data[b];
  const uint64_t size = ss.size[b];
  if (threadIdx.x == 0) {
    sh_err = call_status;
    if (ix.p[b]) {
      idxw[4 * b + 0] = 0;
      idxw[4 * b + 1] = 0;
    }
    sh_state = 2;
    sh_off = 4;
    sh_k = 0;
    sh_rk = ss.recoff_base[b];
    sh_kk = 0;
    if (size == 0) {
      // empty message (server.cpp:128)
    } else if (size < 4 || ld32(p) < 0) {
      atomicOr(call_status, kStMalformed);
    } else {
      sh_ntab = ld32(p);
      sh_state = 0;
    }
  }
  for (;;) {
    // A) thread 0 advances over table headers until a sparse table needs the window
    //    walk or the message ends.  (Nobody else touches the shared state here.)
    if (threadIdx.x == 0) {
      while (sh_state == 0) {
        // next table header (SerializedOpLogReader::StartNewTable, :87-121)
        if (sh_k >= sh_ntab) { sh_state = 2; break; }
        uint64_t off = sh_off;
        if (off + 16 > size) { atomicOr(sh_err, kStMalformed); sh_state = 2; break; }
        const int32_t tid = ld32(p + off);
        const uint64_t usz = ld64_a4(p + off + 4);
        const int32_t nrows = ld32(p + off + 12);
        off += 16;
        int t = -1;
        for (int i = 0; i < dir.n; ++i)
          if (dir.table_id[i] == tid) t = i;
        if (t < 0) { atomicOr(sh_err, kStUnknownTable); sh_state = 2; break; }
        if (usz != (uint64_t)dir.vsize[t] || nrows < 0) { atomicOr(sh_err, kStMalformed); sh_state = 2; break; }
        Seg *sg = &segs[b * kMaxTables + t];
        if (sg->rec0 >= 0) { atomicOr(sh_err, kStUnsupported); sh_state = 2; break; }
        if (dir.dense_serialized[t]) {
          const uint64_t stride = 4 + (uint64_t)dir.dense_body[t];
          const uint64_t need = (uint64_t)nrows * stride;
          if (off + need > size) { atomicOr(sh_err, kStMalformed); sh_state = 2; break; }
          sg->rec0 = (int64_t)off;
          sg->num_rows = nrows;
          sg->sparse = 0;
          sg->ord0 = (int64_t)sh_kk;
          sh_off = off + need;
          sh_k = sh_k + 1;
          sh_kk = sh_kk + (uint64_t)nrows;
        } else if (off & 3) {
          // the sparse walk stages 4-byte words: a sparse table behind a version table's
          // odd-sized records (9-byte trailers) is not supported
          atomicOr(sh_err, kStUnsupported); sh_state = 2; break;
        } else {
          sg->rec0 = (int64_t)sh_rk;   // index of the first record offset
          sg->num_rows = nrows;
          sg->sparse = 1;
          sg->ord0 = (int64_t)sh_kk;
          sh_t = t;
          sh_off = off;
          sh_t0 = off;
          sh_left = (uint64_t)nrows;
          sh_bad = 0;
          if (nrows) sh_state = ix.p[b] ? 3 : 1;
          else sh_k = sh_k + 1;
        }
      }
    }
    __syncthreads();
    if (sh_state == 2) break;
    if (sh_state == 3) {
      // A') indexed sparse table: its first and last offsets here (the first at the
      // table's first byte, the last record inside the message, every record >= 8 bytes),
      // the chain in idx_verify; later header errors of this message wait for its verdict
      if (threadIdx.x == 0) {
        const uint64_t *ofs = ix.p[b] + sh_kk;
        const uint64_t nrec = sh_left, start = sh_off;
        const uint64_t pair = 4 + (uint64_t)dir.vsize[sh_t];
        bool ok = start < size && nrec <= (size - start) / 8;
        uint64_t end = 0;
        if (ok) {
          const uint64_t o0 = ofs[0], ol = ofs[nrec - 1];
          ok = o0 == start && (ol & 3) == 0 && ol >= start && ol + 8 <= size;
          if (ok) {
            const int32_t n = ld32(p + ol + 4);
            end = ol + 8 + (uint64_t)(n < 0 ? 0 : n) * pair;
            ok = n >= 0 && end <= size;
          }
        }
        if (!ok) {
          atomicOr(call_status, kStMalformed);
          segs[b * kMaxTables + sh_t].num_rows = 0;   // idx_verify skips it (the call fails)
          sh_state = 2;
        } else {
          sh_off = end;
          sh_rk = sh_rk + nrec;
          sh_kk = sh_kk + nrec;
          sh_k = sh_k + 1;
          sh_err = idxw + 4 * b;
          sh_state = 0;
        }
      }
      __syncthreads();
      continue;
    }
    // B) the window of the fixed grid (from the table's first record) that holds the
    //    current record, plus one halo word; window k+1 was prefetched into registers
    //    while window k was walked.
    const uint64_t t0 = sh_t0;
    const uint64_t w0 = t0 + (sh_off - t0) / kWinBytes * kWinBytes;
    const uint64_t tot = (size - w0) / 4;                       // whole words from w0
    const uint32_t nw = (uint32_t)(tot < (uint64_t)kDecodeWindowWords ? tot : (uint64_t)kDecodeWindowWords);
    const bool halo = tot > nw;
    {
      constexpr int PER = kDecodeWindowWords / kDecodeThreads;
      const uint32_t *src = reinterpret_cast<const uint32_t *>(p + w0);
      if (pf_w0 != w0) {
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const uint32_t i = threadIdx.x + (uint32_t)k * kDecodeThreads;
          pf[k] = i < nw ? src[i] : 0u;
        }
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint32_t i = threadIdx.x + (uint32_t)k * kDecodeThreads;
        if (i < nw) win[i] = pf[k];
      }
      if (threadIdx.x == 0) win[nw] = halo ? src[nw] : 0u;
      // prefetch the next grid window (used if the walk continues there)
      const uint64_t n0 = w0 + kWinBytes;
      pf_w0 = ~0ull;
      if (n0 + 8 <= size) {
        const uint64_t ntot = (size - n0) / 4;
        const uint32_t nnw = (uint32_t)(ntot < (uint64_t)kDecodeWindowWords ? ntot : (uint64_t)kDecodeWindowWords);
        const uint32_t *nsrc = reinterpret_cast<const uint32_t *>(p + n0);
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const uint32_t i = threadIdx.x + (uint32_t)k * kDecodeThreads;
          pf[k] = i < nnw ? nsrc[i] : 0u;
        }
        pf_w0 = n0;
      }
    }
    __syncthreads();
    // C) jump tables over the window (all threads, 16-bit word indices): j1[q] = word of
    //    the record after a record starting at word q; j2 = j1 o j1, ..., j16; kU16 where
    //    the next record leaves the window or the header is bad (thread 0 resolves those
    //    one record at a time from the words themselves).
    const uint64_t wpr = 1 + (uint64_t)dir.vsize[sh_t] / 4;   // words per (col, val) pair
    for (uint32_t q = threadIdx.x; q < nw; q += blockDim.x) {
      uint16_t v = kU16;
      if (q + 1 < nw) {
        const int32_t n = (int32_t)win[q + 1];
        if (n >= 0) {
          const uint64_t nxt = (uint64_t)q + 2 + (uint64_t)n * wpr;
          if (nxt < nw && w0 + nxt * 4 <= size) v = (uint16_t)nxt;
        }
      }
      jt[0][q] = v;
    }
    __syncthreads();
#pragma unroll
    for (int lv = 1; lv < kJumpLevels; ++lv) {
      for (uint32_t q = threadIdx.x; q < nw; q += blockDim.x) {
        const uint16_t a1 = jt[lv - 1][q];
        jt[lv][q] = a1 != kU16 ? jt[lv - 1][a1] : kU16;
      }
      __syncthreads();
    }
    // D) thread 0 hops the chain 16 records at a time, then 4, then singly (the record
    //    that leaves the window, a bad header or the table's last records)
    if (threadIdx.x == 0) {
      uint64_t left = sh_left;
      uint32_t w = (uint32_t)((sh_off - w0) / 4);
      uint32_t n16 = 0, n4 = 0, ns = 0;
      int bad = w >= nw;   // the table's first record header lies past the message end
      if (bad) left = 0;
      while (left >= 16 && jt[4][w] != kU16) {
        a16[n16++] = (uint16_t)w;
        w = jt[4][w];
        left -= 16;
      }
      while (left >= 4 && jt[2][w] != kU16) {
        a4[n4++] = (uint16_t)w;
        w = jt[2][w];
        left -= 4;
      }
      bool out = false;   // the walk left the window (sh_off already set)
      while (left) {
        if (w + 1 > nw || (w + 1 == nw && !halo)) { bad = 1; break; }   // header cut by the message end
        const int32_t n = (int32_t)win[w + 1];
        if (n < 0) { bad = 1; break; }
        const uint64_t nxt = (uint64_t)w + 2 + (uint64_t)n * wpr;
        if (w0 + nxt * 4 > size) { bad = 1; break; }
        a1s[ns++] = (uint16_t)w;
        --left;
        if (nxt >= nw) { out = true; sh_off = w0 + nxt * 4; break; }
        w = (uint32_t)nxt;
      }
      if (!out) sh_off = w0 + (uint64_t)w * 4;
      sh_n16 = n16;
      sh_n4 = n4;
      sh_ns = ns;
      sh_bad = bad;
      sh_left = left;
    }
    __syncthreads();
    // E) expand the hops into record offsets (all threads)
    {
      const uint32_t n16 = sh_n16, n4 = sh_n4, ns = sh_ns;
      const uint64_t rk = sh_rk;
      for (uint32_t i = threadIdx.x; i < n16 * 4; i += blockDim.x) {   // 4 threads per 16-hop
        uint32_t q = a16[i >> 2];
        const uint32_t sub = i & 3;
        for (uint32_t k = 0; k < sub; ++k) q = jt[2][q];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          recoff[rk + 16 * (uint64_t)(i >> 2) + 4 * sub + k] = w0 + (uint64_t)q * 4;
          q = jt[0][q];
        }
      }
      const uint64_t r4 = rk + 16 * (uint64_t)n16;
      for (uint32_t i = threadIdx.x; i < n4; i += blockDim.x) {
        uint32_t q = a4[i];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          recoff[r4 + 4 * (uint64_t)i + k] = w0 + (uint64_t)q * 4;
          q = jt[0][q];
        }
      }
      const uint64_t r1 = r4 + 4 * (uint64_t)n4;
      for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) recoff[r1 + i] = w0 + (uint64_t)a1s[i] * 4;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (sh_bad) {
        atomicOr(call_status, kStMalformed);
        sh_state = 2;
      } else {
        sh_rk = sh_rk + 16 * (uint64_t)sh_n16 + 4 * (uint64_t)sh_n4 + sh_ns;
        if (!sh_left) {
          sh_state = 0;
          sh_k = sh_k + 1;
          sh_kk = sh_kk + (uint64_t)segs[b * kMaxTables + sh_t].num_rows;
        } else if (sh_off + 8 > size) {
          atomicOr(call_status, kStMalformed);
          sh_state = 2;
        }
      }
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// Shard geometry: row r -> slot (r - row_offset) / row_stride (context.hpp:291-304).
struct Geo {
  int64_t row_offset;
  int64_t row_stride;
  int64_t max_rows;
};

__device__ __forceinline__ int64_t slot_of(int32_t rid, const Geo &g) {
  int64_t d = (int64_t)rid - g.row_offset;
  if (d < 0) return -1;
  if (g.row_stride != 1) {
    if (d % g.row_stride) return -1;
    d /= g.row_stride;
  }
  return d < g.max_rows ? d : -1;
}

// dense_verify: counters[t][b] = number of slots claimed by message b.
__global__ void __launch_bounds__(256) dense_verify_kernel(const int32_t *inv, InvLayout L, int t, int B,
                                                          int64_t max_rows, uint32_t *counters) {
  __shared__ uint32_t part[kMaxFused];
  if (threadIdx.x < kMaxFused) part[threadIdx.x] = 0;
  __syncthreads();
  uint32_t cnt[kMaxFused];
#pragma unroll
  for (int b = 0; b < kMaxFused; ++b) cnt[b] = 0;
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < max_rows; s += gsz) {
    const int32_t *row = inv + s * L.ss;
#pragma unroll
    for (int b = 0; b < kMaxFused; ++b)
      if (b < B) cnt[b] += row[b * L.sb] >= 0 ? 1u : 0u;
  }
#pragma unroll
  for (int b = 0; b < kMaxFused; ++b) {
    if (b < B) {
      uint32_t v = cnt[b];
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      if ((threadIdx.x & 63) == 0 && v) atomicAdd(&part[b], v);
    }
  }
  __syncthreads();
  if (threadIdx.x < B && part[threadIdx.x]) atomicAdd(&counters[t * kMaxFused + threadIdx.x], part[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// Element helpers.  Records are only 4-byte aligned (a 4-byte row id precedes every
// payload), so 8-byte values are read as two dwords.
template <typename V> struct Elem;
template <> struct Elem<float> {
  __device__ static float load_rec(const uint8_t *p) { return *reinterpret_cast<const float *>(p); }
  __device__ static float add(float a, float b) { return a + b; }
};
template <> struct Elem<double> {
  __device__ static double load_rec(const uint8_t *p) {
    uint64_t lo = *reinterpret_cast<const uint32_t *>(p);
    uint64_t hi = *reinterpret_cast<const uint32_t *>(p + 4);
    return __longlong_as_double((long long)(lo | (hi << 32)));
  }
  __device__ static double add(double a, double b) { return a + b; }
};
template <> struct Elem<int32_t> {
  __device__ static int32_t load_rec(const uint8_t *p) { return *reinterpret_cast<const int32_t *>(p); }
  __device__ static int32_t add(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
};
template <> struct Elem<int64_t> {
  __device__ static int64_t load_rec(const uint8_t *p) {
    uint64_t lo = *reinterpret_cast<const uint32_t *>(p);
    uint64_t hi = *reinterpret_cast<const uint32_t *>(p + 4);
    return (int64_t)(lo | (hi << 32));
  }
  __device__ static int64_t add(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
};

// ---------------------------------------------------------------------------
// dense_apply_v2: 16 bytes per lane per load.  Record payloads start 4 bytes after a
// row id, so they are only 4-byte aligned: the loads are unaligned global_load_dwordx4
// (gfx950 runs HSA in unaligned-access mode; hipcc emits dwordx4 for align-4 memcpy).
// Record loads may be non-temporal (read once).  TILE slots per wave-tile; PAIR touched
// slots in flight per wave; the grid is sized to the resident capacity and strides
// over tiles, so the tail is one tile, not one wave-lifetime.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

template <bool NT>
__device__ __forceinline__ u32x4 load16(const uint8_t *p) {
  if constexpr (NT) {
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4 *>(p));
  } else {
    u32x4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
  }
}
// Table-row loads and stores (DenseArgs.store_nt, PSX_VARIANT_DENSE_STORE): bit 0 stores
// the row non-temporally (a streaming write instead of a dirty L2 line evicted later amid
// the record gathers), bit 1 loads it non-temporally.  In tools/probe_apply.hip (the C2
// pattern alone) the 1.07 GB of row writes cost ~0.6-0.8 ms of a 2.2-2.4 ms launch (reads
// alone: 1.60 ms) and the policy mattered there: nt store 2.20 ms, plain 2.38-2.41
// (profiles/r03/s10).  In this kernel it does not: policies 0, 1 and 3 all measured
// 2.290-2.293 ms walked and 2.316-2.320 ms with record rows on one box (s10, 5 rounds
// each); 1 is the default.  Rows are 4-byte aligned.
__device__ __forceinline__ void store16(uint8_t *p, u32x4 v, int mode) {
  if (mode & 1)
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4_a4, v), reinterpret_cast<u32x4_a4 *>(p));
  else
    __builtin_memcpy(p, &v, 16);
}
__device__ __forceinline__ u32x4 load_row16(const uint8_t *p, int mode) {
  return (mode & 2) ? load16<true>(p) : load16<false>(p);
}

// Four binary16 record values (8 bytes, 2-byte aligned) -> four f32 bit patterns, by the
// hardware conversion (NaN payloads kept and quieted; every value then goes through
// `row += u`, which quiets anyway).
typedef uint32_t u32x2_a2 __attribute__((ext_vector_type(2), aligned(2)));
template <bool NT>
__device__ __forceinline__ u32x4 load_h4(const uint8_t *p) {
  uint32_t w0, w1;
  if constexpr (NT) {
    const u32x2_a2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2_a2 *>(p));
    w0 = v[0];
    w1 = v[1];
  } else {
    __builtin_memcpy(&w0, p, 4);
    __builtin_memcpy(&w1, p + 4, 4);
  }
  return u32x4{half_to_f32_bits_hw(w0 & 0xffffu), half_to_f32_bits_hw(w0 >> 16), half_to_f32_bits_hw(w1 & 0xffffu),
               half_to_f32_bits_hw(w1 >> 16)};
}

template <typename V> struct Vec;
template <> struct Vec<float> {
  __device__ static u32x4 add(u32x4 a, u32x4 b) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(__uint_as_float(a[i]) + __uint_as_float(b[i]));
    return r;
  }
};
template <> struct Vec<int32_t> {
  __device__ static u32x4 add(u32x4 a, u32x4 b) { return a + b; }
};
template <> struct Vec<double> {
  __device__ static u32x4 add(u32x4 a, u32x4 b) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      double x = __longlong_as_double((long long)(((uint64_t)a[2 * i + 1] << 32) | a[2 * i]));
      double y = __longlong_as_double((long long)(((uint64_t)b[2 * i + 1] << 32) | b[2 * i]));
      uint64_t z = (uint64_t)__double_as_longlong(x + y);
      r[2 * i] = (uint32_t)z;
      r[2 * i + 1] = (uint32_t)(z >> 32);
    }
    return r;
  }
};
template <> struct Vec<int64_t> {
  __device__ static u32x4 add(u32x4 a, u32x4 b) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      uint64_t z = (((uint64_t)a[2 * i + 1] << 32) | a[2 * i]) + (((uint64_t)b[2 * i + 1] << 32) | b[2 * i]);
      r[2 * i] = (uint32_t)z;
      r[2 * i + 1] = (uint32_t)(z >> 32);
    }
    return r;
  }
};

// Importance terms (ns_sum_imp_calc.hpp:87-90) of the 16/sizeof(V) elements of one lane
// vector: old values a, record values b.
template <typename V>
__device__ __forceinline__ double vec_imp(u32x4 a, u32x4 b) {
  double r = 0.0;
  if constexpr (sizeof(V) == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // copy the lanes out first: __builtin_bit_cast applied directly to a vector
      // subscript a[i] reads element 0 for every i (observed with this clang)
      const uint32_t ai = a[i], bi = b[i];
      r += imp_term<V>(__builtin_bit_cast(V, ai), __builtin_bit_cast(V, bi));
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
      r += imp_term<V>(__builtin_bit_cast(V, ((uint64_t)a[2 * i + 1] << 32) | a[2 * i]),
                       __builtin_bit_cast(V, ((uint64_t)b[2 * i + 1] << 32) | b[2 * i]));
  }
  return r;
}

// IMP: also accumulate each record's NSSumImpCalc importance, sum_i |u_i / v_i| with v_i
// the value before that record's add (ns_sum_imp_calc.hpp:79-98), into imp[slot]; here
// all of a row's terms of one call share one f64 accumulator (non-negative terms: within
// (cap*B-1)*2^-53 relative of the reference's record-by-record sum).
// H16 (f32 tables with kDenseRowOpLogFloat16 records): record payloads are binary16, so a
// lane's 4 elements come from one 8-byte load and are decompressed before the add
// (2: the hardware conversion).
template <typename V, int BMAX, int TILE, bool NT, int PAIR, bool IMP, int H16 = 0>
__global__ void __launch_bounds__(256) dense_apply_v2_kernel(DenseArgs a) {
  constexpr int VS = (int)sizeof(V);
  constexpr int EPV = 16 / VS;        // elements per 16-byte lane vector
  constexpr int CHUNK = 64 * EPV;     // elements per wave-wide vector pass
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int B = a.B;

  bool skip = (*a.call_status & (kStFatal | kStDuplicateRow)) != 0 || (*a.sticky & kStDuplicateRow) != 0;
  bool dup = false;
  const uint8_t *pay0[BMAX];   // payload of record 0 of message b (nullptr: table absent)
#pragma unroll
  for (int b = 0; b < BMAX; ++b) {
    pay0[b] = nullptr;
    if (b < B) {
      const Seg sg = a.segs[b * kMaxTables + a.t];
      if (sg.rec0 >= 0 && !sg.sparse) {
        pay0[b] = a.ss.data[b] + sg.rec0 + 4;
        if (a.counters[a.t * kMaxFused + b] != (uint32_t)sg.num_rows) dup = true;
      }
    }
  }
  if (dup && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.call_status, kStDuplicateRow);
  skip = skip || dup;

  const int64_t vec_elems = (a.cap / EPV) * EPV;   // elements covered by full lane vectors
  const int64_t row_bytes = a.row_cap * VS;
  uint8_t *table = reinterpret_cast<uint8_t *>(a.table);
  const int64_t ntiles = (a.max_rows + TILE - 1) / TILE;

  for (int64_t tile = wave_g; tile < ntiles; tile += nwaves) {
    const int64_t s0 = tile * TILE;
    const int64_t my_slot = s0 + lane;
    const bool mine = lane < TILE && my_slot < a.max_rows;
    int32_t idx[BMAX];
    bool touched = false;
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
      idx[b] = -1;
      if (b < B && mine) {
        idx[b] = a.inv[my_slot * a.inv_ss + b * a.inv_sb];
        if (idx[b] >= 0) {
          touched = true;
          a.inv[my_slot * a.inv_ss + b * a.inv_sb] = -1;
        }
      }
    }
    if (skip) continue;
    if (touched) {
      a.flags[my_slot] = 3;   // exists | dirty
      if (a.ver) {            // VersionServerRow: version_++ per applied record (version_server_row.hpp:44-53)
        uint64_t n = 0;
#pragma unroll
        for (int b = 0; b < BMAX; ++b) n += idx[b] >= 0 ? 1u : 0u;
        a.ver[my_slot] += n;
      }
    }
    uint64_t live = __ballot(touched);

    while (live) {
      int ks[PAIR];
      bool has[PAIR];
#pragma unroll
      for (int q = 0; q < PAIR; ++q) {
        has[q] = live != 0;
        ks[q] = has[q] ? __builtin_ctzll(live) : 0;
        if (has[q]) live &= live - 1;
      }
      const uint8_t *rp[PAIR][BMAX];
      bool pres[PAIR][BMAX];
      uint8_t *trow[PAIR];
#pragma unroll
      for (int q = 0; q < PAIR; ++q) {
        trow[q] = table + (s0 + ks[q]) * row_bytes;
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
          const int32_t i = __builtin_amdgcn_readlane(idx[b], ks[q]);
          pres[q][b] = has[q] && pay0[b] != nullptr && i >= 0;
          rp[q][b] = pres[q][b] ? pay0[b] + (int64_t)i * a.stride : a.zero_chunk;
        }
      }
      // IMP: one f64 accumulator per row (all of its records this call) and the row's
      // current importance fetched up front, so its latency hides under the row loads.
      double ib[IMP ? PAIR : 1], imp0[IMP ? PAIR : 1];
#pragma unroll
      for (int q = 0; q < (IMP ? PAIR : 1); ++q) {
        ib[q] = 0.0;
        if constexpr (IMP) imp0[q] = has[q] ? a.imp[s0 + ks[q]] : 0.0;
      }
      for (int64_t c0 = 0; c0 < vec_elems; c0 += CHUNK) {
        const int64_t e0 = c0 + (int64_t)lane * EPV;
        const bool full = e0 < vec_elems;
        u32x4 t[PAIR];
        u32x4 u[PAIR][BMAX];
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          t[q] = (full && has[q]) ? load_row16(trow[q] + e0 * VS, a.store_nt) : u32x4{0, 0, 0, 0};
#pragma unroll
          for (int b = 0; b < BMAX; ++b) {
            if constexpr (H16) {
              const uint8_t *src = pres[q][b] ? rp[q][b] + e0 * 2 : a.zero_chunk + lane * 8;
              u[q][b] = full ? load_h4<NT>(src) : u32x4{0, 0, 0, 0};
            } else {
              const uint8_t *src = pres[q][b] ? rp[q][b] + e0 * VS : a.zero_chunk + lane * 16;
              u[q][b] = full ? load16<NT>(src) : u32x4{0, 0, 0, 0};
            }
          }
        }
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          u32x4 acc = t[q];
#pragma unroll
          for (int b = 0; b < BMAX; ++b)
            if (pres[q][b]) {
              if constexpr (IMP) {
                if (full) ib[q] += vec_imp<V>(acc, u[q][b]);
              }
              acc = Vec<V>::add(acc, u[q][b]);
            }
          if (full && has[q]) store16(trow[q] + e0 * VS, acc, a.store_nt);
        }
      }
      // ragged tail (cap % EPV elements): element-wise on the first lanes
      const int64_t tail = a.cap - vec_elems;
      if (tail) {
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          if (has[q] && lane < tail) {
            const int64_t e = vec_elems + lane;
            V acc = *reinterpret_cast<const V *>(trow[q] + e * VS);
#pragma unroll
            for (int b = 0; b < BMAX; ++b)
              if (pres[q][b]) {
                V u;
                if constexpr (H16) {
                  uint16_t h;
                  __builtin_memcpy(&h, rp[q][b] + e * 2, 2);
                  u = __builtin_bit_cast(V, half_to_f32_bits_hw(h));
                } else {
                  u = Elem<V>::load_rec(rp[q][b] + e * VS);
                }
                if constexpr (IMP) ib[q] += imp_term<V>(acc, u);
                acc = Elem<V>::add(acc, u);
              }
            *reinterpret_cast<V *>(trow[q] + e * VS) = acc;
          }
        }
      }
      if constexpr (IMP) {
        // ServerRow::AccumImportance (server_row.hpp:56-62,124-126)
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          const double tot = imp0[q] + wave_sum_f64(ib[q]);
          if (has[q] && lane == 0) a.imp[s0 + ks[q]] = tot;
        }
      }
    }
  }
}

// dense_apply_v3: dense_apply_v2 with the record addresses kept as one wave-uniform
// base per message (its first record's payload, in SGPRs) plus a 32-bit UNSIGNED per-lane
// offset.  v2 keeps PAIR x BMAX uniform 64-bit record pointers, which overflow the SGPR
// file and spill to VGPR lanes (~500 v_readlane/v_writelane per row pair).  Streams must be
// < 4 GiB.  The offset is zero-extended wherever the address is formed (the compiler builds
// 64-bit VGPR addresses with v_lshl_add_u64; tests/test_isa.py checks that no v3
// instantiation sign-extends a per-lane value, tests/test_configs_gpu.py runs offsets with
// bit 31 set on the GPU).
typedef const uint8_t __attribute__((address_space(1))) *gbyte_p;
typedef const u32x4_a4 __attribute__((address_space(1))) *gu32x4_p;
typedef uint32_t u32x2_a2g __attribute__((ext_vector_type(2), aligned(2)));
typedef const u32x2_a2g __attribute__((address_space(1))) *gu32x2_p;

template <bool NT>
__device__ __forceinline__ u32x4 gload16(const uint8_t *base, uint32_t off) {
  const gu32x4_p p = (gu32x4_p)((gbyte_p)base + off);
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

template <bool NT>
__device__ __forceinline__ u32x4 gload_h4(const uint8_t *base, uint32_t off) {
  const gu32x2_p p = (gu32x2_p)((gbyte_p)base + off);
  u32x2_a2g v;
  if constexpr (NT) v = __builtin_nontemporal_load(p);
  else v = *p;
  const uint32_t w0 = v[0], w1 = v[1];
  return u32x4{half_to_f32_bits_hw(w0 & 0xffffu), half_to_f32_bits_hw(w0 >> 16), half_to_f32_bits_hw(w1 & 0xffffu),
               half_to_f32_bits_hw(w1 >> 16)};
}

template <typename V, int BMAX, int TILE, bool NT, int PAIR, bool IMP, int H16 = 0>
__global__ void __launch_bounds__(256) dense_apply_v3_kernel(DenseArgs a) {
  static_assert(PAIR * BMAX <= 32, "presence mask is 32 bits");
  constexpr int VS = (int)sizeof(V);
  constexpr int EPV = 16 / VS;
  constexpr int CHUNK = 64 * EPV;
  constexpr int RB = H16 ? 2 : VS;    // record bytes per element
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int B = a.B;

  bool skip = (*a.call_status & (kStFatal | kStDuplicateRow)) != 0 || (*a.sticky & kStDuplicateRow) != 0;
  bool dup = false;
  const uint8_t *pay0[BMAX];
  uint32_t real = 0;   // bit b: message b holds this table
#pragma unroll
  for (int b = 0; b < BMAX; ++b) {
    pay0[b] = a.zero_chunk;
    if (b < B) {
      const Seg sg = a.segs[b * kMaxTables + a.t];
      if (sg.rec0 >= 0 && !sg.sparse) {
        pay0[b] = a.ss.data[b] + sg.rec0 + 4;
        real |= 1u << b;
        if (a.counters[a.t * kMaxFused + b] != (uint32_t)sg.num_rows) dup = true;
      }
    }
  }
  if (dup && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.call_status, kStDuplicateRow);
  skip = skip || dup;
  const bool rows_mode = a.rows_mask != 0;
  const int wib = threadIdx.x >> 6;
  __shared__ int32_t s_idx[4][TILE * BMAX];     // rows mode: the tile's record numbers
  __shared__ const uint8_t *s_pay0[BMAX];
#pragma unroll
  for (int b = 0; b < BMAX; ++b)
    if (threadIdx.x == b) s_pay0[b] = pay0[b];
  __syncthreads();

  const int64_t vec_elems = (a.cap / EPV) * EPV;
  const int64_t row_bytes = a.row_cap * VS;
  const uint32_t stride = (uint32_t)a.stride;
  const uint32_t lane_off = (uint32_t)(lane * EPV * RB);
  uint8_t *table = reinterpret_cast<uint8_t *>(a.table);
  const int64_t ntiles = (a.max_rows + TILE - 1) / TILE;

  for (int64_t tile = wave_g; tile < ntiles; tile += nwaves) {
    const int64_t s0 = tile * TILE;
    const int64_t my_slot = s0 + lane;
    const bool mine = lane < TILE && my_slot < a.max_rows;
    int32_t idx[BMAX];
    bool touched = false;
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
      idx[b] = -1;
      if (b < B && mine) {
        idx[b] = a.inv[my_slot * a.inv_ss + b * a.inv_sb];
        if (idx[b] >= 0) {
          touched = true;
          a.inv[my_slot * a.inv_ss + b * a.inv_sb] = -1;
        }
      }
    }
    if (skip) continue;
    // Rows mode (records placed from the producer's record-row lists): the tile's record
    // numbers go to LDS so that, per row pair, lane q*BMAX + b can load the row id of
    // record (q, b) right beside the pair's payload loads (same first cache line: no added
    // DRAM traffic); a row any of whose records names another row is neither written nor
    // marked.  Loading each slot's row ids in the tile prologue instead needs no LDS but
    // re-fetches ~half of those lines (PMC 11.32 vs 10.77 GB read per launch: evicted before
    // the pair that uses them), and a 16-way select chain for the addressing costs 1.7% of
    // the apply (profiles/r02/ab_rows_check.json).
    if (rows_mode && mine) {
#pragma unroll
      for (int b = 0; b < BMAX; ++b) s_idx[wib][lane * BMAX + b] = idx[b];
    }
    if (touched && !rows_mode) {
      a.flags[my_slot] = 3;
      if (a.ver) {
        uint64_t n = 0;
#pragma unroll
        for (int b = 0; b < BMAX; ++b) n += idx[b] >= 0 ? 1u : 0u;
        a.ver[my_slot] += n;
      }
    }
    uint64_t live = __ballot(touched);

    while (live) {
      int ks[PAIR];
      bool has[PAIR];
#pragma unroll
      for (int q = 0; q < PAIR; ++q) {
        has[q] = live != 0;
        ks[q] = has[q] ? __builtin_ctzll(live) : 0;
        if (has[q]) live &= live - 1;
      }
      uint32_t presm = 0;
      uint32_t voff[PAIR][BMAX];   // per-lane byte offset of the lane's first element
      uint8_t *trow[PAIR];
#pragma unroll
      for (int q = 0; q < PAIR; ++q) {
        trow[q] = table + (s0 + ks[q]) * row_bytes;
#pragma unroll
        for (int b = 0; b < BMAX; ++b) {
          const int32_t i = __builtin_amdgcn_readlane(idx[b], ks[q]);
          if (has[q] && ((real >> b) & 1u) && i >= 0) presm |= 1u << (q * BMAX + b);
          voff[q][b] = (uint32_t)i * stride + lane_off;
        }
      }
      uint32_t okq = (1u << PAIR) - 1;   // bit q: row q may be stored (rows mode)
      bool chk = false;
      int32_t rid = 0, rid_want = 0;
      if (rows_mode) {
        const int qj = lane / BMAX, bj = lane % BMAX;
        int ksj = ks[0];
#pragma unroll
        for (int q = 1; q < PAIR; ++q)
          if (qj == q) ksj = ks[q];
        chk = lane < PAIR * BMAX && ((presm >> lane) & 1u) && ((a.rows_mask >> bj) & 1u);
        rid_want = (int32_t)(a.row_offset + (s0 + ksj) * a.row_stride);
        if (chk) {
          const int32_t i = s_idx[wib][ksj * BMAX + bj];
          rid = *reinterpret_cast<const int32_t *>(s_pay0[bj] + (uint32_t)i * stride - 4);
        }
      }
      bool verified = !rows_mode;
      auto verify = [&]() {
        const uint64_t badm = __ballot(chk && rid != rid_want);
        if (badm && lane == 0) atomicOr(a.call_status, kStRowsMismatch);
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          if ((badm >> (q * BMAX)) & ((1ull << BMAX) - 1)) okq &= ~(1u << q);
          if (lane == 0 && has[q] && ((okq >> q) & 1u)) {
            a.flags[s0 + ks[q]] = 3;
            if (a.ver) a.ver[s0 + ks[q]] += (uint64_t)__builtin_popcount((presm >> (q * BMAX)) & ((1u << BMAX) - 1));
          }
        }
        verified = true;
      };
      double ib[IMP ? PAIR : 1], imp0[IMP ? PAIR : 1];
#pragma unroll
      for (int q = 0; q < (IMP ? PAIR : 1); ++q) {
        ib[q] = 0.0;
        if constexpr (IMP) imp0[q] = has[q] ? a.imp[s0 + ks[q]] : 0.0;
      }
      for (int64_t c0 = 0; c0 < vec_elems; c0 += CHUNK) {
        const int64_t e0 = c0 + (int64_t)lane * EPV;
        const bool full = e0 < vec_elems;
        const uint32_t coff = (uint32_t)(c0 * RB);
        // Branch-free loads (no exec-mask saves): every address is in bounds — a lane
        // past the row's vector part reads element 0, an absent record reads the
        // message's first record (or the zero chunk) — and absent values are never added.
        const int64_t te = full ? e0 : 0;
        u32x4 t[PAIR];
        u32x4 u[PAIR][BMAX];
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          t[q] = load_row16(trow[q] + te * VS, a.store_nt);
#pragma unroll
          for (int b = 0; b < BMAX; ++b) {
            const bool pr = (presm >> (q * BMAX + b)) & 1u;
            // an absent record reads its message's first chunk (or the 4 KiB zero chunk):
            // never past the first CHUNK bytes, whatever the row width
            const uint32_t off = full ? (pr ? voff[q][b] + coff : lane_off) : 0u;
            if constexpr (H16)
              u[q][b] = gload_h4<NT>(pay0[b], off);
            else
              u[q][b] = gload16<NT>(pay0[b], off);
          }
        }
        if (!verified) verify();
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          u32x4 acc = t[q];
#pragma unroll
          for (int b = 0; b < BMAX; ++b)
            if ((presm >> (q * BMAX + b)) & 1u) {
              if constexpr (IMP) {
                if (full) ib[q] += vec_imp<V>(acc, u[q][b]);
              }
              acc = Vec<V>::add(acc, u[q][b]);
            }
          if (full && has[q] && ((okq >> q) & 1u)) store16(trow[q] + e0 * VS, acc, a.store_nt);
        }
      }
      if (!verified) verify();
      const int64_t tail = a.cap - vec_elems;
      if (tail) {
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          if (has[q] && ((okq >> q) & 1u) && lane < tail) {
            const int64_t e = vec_elems + lane;
            V acc = *reinterpret_cast<const V *>(trow[q] + e * VS);
#pragma unroll
            for (int b = 0; b < BMAX; ++b)
              if ((presm >> (q * BMAX + b)) & 1u) {
                const uint8_t *rec = pay0[b] + (int64_t)__builtin_amdgcn_readlane(idx[b], ks[q]) * a.stride;
                V u;
                if constexpr (H16) {
                  uint16_t h;
                  __builtin_memcpy(&h, rec + e * 2, 2);
                  u = __builtin_bit_cast(V, half_to_f32_bits_hw(h));
                } else {
                  u = Elem<V>::load_rec(rec + e * VS);
                }
                if constexpr (IMP) ib[q] += imp_term<V>(acc, u);
                acc = Elem<V>::add(acc, u);
              }
            *reinterpret_cast<V *>(trow[q] + e * VS) = acc;
          }
        }
      }
      if constexpr (IMP) {
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          const double tot = imp0[q] + wave_sum_f64(ib[q]);
          if (has[q] && ((okq >> q) & 1u) && lane == 0) a.imp[s0 + ks[q]] = tot;
        }
      }
    }
  }
}

// dense_apply_v4 (compact): for partially covered calls (a row present in few of the B
// messages).  v2/v3 keep PAIR rows x BMAX record slots in flight, most of them empty when
// coverage is sparse; v4 packs up to PAIR rows whose present records total <= M into a
// per-wave LDS slot list (row-major, message order within a row), so a wave keeps up to
// PAIR table rows + M records in flight whatever the coverage.
template <typename V, int BMAX, int TILE, bool NT, int PAIR, int M>
__global__ void __launch_bounds__(256) dense_apply_v4_kernel(DenseArgs a) {
  static_assert(M >= BMAX, "a row's records must fit the slot list");
  constexpr int VS = (int)sizeof(V);
  constexpr int EPV = 16 / VS;
  constexpr int CHUNK = 64 * EPV;
  __shared__ const uint8_t *s_rec[4][M];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + w;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int B = a.B;

  bool skip = (*a.call_status & (kStFatal | kStDuplicateRow)) != 0 || (*a.sticky & kStDuplicateRow) != 0;
  bool dup = false;
  const uint8_t *pay0[BMAX];
#pragma unroll
  for (int b = 0; b < BMAX; ++b) {
    pay0[b] = nullptr;
    if (b < B) {
      const Seg sg = a.segs[b * kMaxTables + a.t];
      if (sg.rec0 >= 0 && !sg.sparse) {
        pay0[b] = a.ss.data[b] + sg.rec0 + 4;
        if (a.counters[a.t * kMaxFused + b] != (uint32_t)sg.num_rows) dup = true;
      }
    }
  }
  if (dup && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.call_status, kStDuplicateRow);
  skip = skip || dup;

  const int64_t vec_elems = (a.cap / EPV) * EPV;
  const int64_t row_bytes = a.row_cap * VS;
  uint8_t *table = reinterpret_cast<uint8_t *>(a.table);
  const int64_t ntiles = (a.max_rows + TILE - 1) / TILE;

  for (int64_t tile = wave_g; tile < ntiles; tile += nwaves) {
    const int64_t s0 = tile * TILE;
    const int64_t my_slot = s0 + lane;
    const bool mine = lane < TILE && my_slot < a.max_rows;
    int32_t idx[BMAX];
    int cnt = 0;
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
      idx[b] = -1;
      if (b < B && mine && pay0[b]) {
        idx[b] = a.inv[my_slot * a.inv_ss + b * a.inv_sb];
        if (idx[b] >= 0) {
          ++cnt;
          a.inv[my_slot * a.inv_ss + b * a.inv_sb] = -1;
        }
      }
    }
    if (skip) continue;
    if (cnt) {
      a.flags[my_slot] = 3;
      if (a.ver) a.ver[my_slot] += (uint64_t)cnt;
    }
    uint64_t live = __ballot(cnt > 0);

    while (live) {
      // take rows while their records fit the slot list
      int ks[PAIR], beg[PAIR + 1];
      int nrows = 0, nslot = 0;
      beg[0] = 0;
#pragma unroll
      for (int q = 0; q < PAIR; ++q) {
        ks[q] = 0;
        if (live) {
          const int k = __builtin_ctzll(live);
          const int c = __builtin_amdgcn_readlane(cnt, k);
          if (nslot + c <= M) {
            live &= live - 1;
            ks[q] = k;
            int j = nslot;
#pragma unroll
            for (int b = 0; b < BMAX; ++b) {
              const int32_t i = __builtin_amdgcn_readlane(idx[b], k);
              if (i >= 0) {
                s_rec[w][j] = pay0[b] + (int64_t)i * a.stride;   // same value from every lane
                ++j;
              }
            }
            nslot = j;
            nrows = q + 1;
          }
        }
        beg[q + 1] = nslot;
      }
      for (int64_t c0 = 0; c0 < vec_elems; c0 += CHUNK) {
        const int64_t e0 = c0 + (int64_t)lane * EPV;
        const bool full = e0 < vec_elems;
        const int64_t te = full ? e0 : 0;
        u32x4 t[PAIR], u[M];
#pragma unroll
        for (int q = 0; q < PAIR; ++q)
          if (q < nrows) t[q] = load_row16(table + (s0 + ks[q]) * row_bytes + te * VS, a.store_nt);
#pragma unroll
        for (int j = 0; j < M; ++j)
          if (j < nslot) u[j] = load16<NT>(s_rec[w][j] + te * VS);
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          if (q < nrows) {
            u32x4 acc = t[q];
#pragma unroll
            for (int j = 0; j < M; ++j)
              if (j >= beg[q] && j < beg[q + 1]) acc = Vec<V>::add(acc, u[j]);
            if (full) store16(table + (s0 + ks[q]) * row_bytes + e0 * VS, acc, a.store_nt);
          }
        }
      }
      const int64_t tail = a.cap - vec_elems;
      if (tail) {
#pragma unroll
        for (int q = 0; q < PAIR; ++q) {
          if (q < nrows && lane < tail) {
            const int64_t e = vec_elems + lane;
            uint8_t *tr = table + (s0 + ks[q]) * row_bytes;
            V acc = *reinterpret_cast<const V *>(tr + e * VS);
            for (int j = beg[q]; j < beg[q + 1]; ++j)
              acc = Elem<V>::add(acc, Elem<V>::load_rec(s_rec[w][j] + e * VS));
            *reinterpret_cast<V *>(tr + e * VS) = acc;
          }
        }
      }
    }
  }
}

// dense_index_v2: flattened (message, record) space, UNROLL row-id loads in flight per
// thread before any store.  A message in rows_mask takes its row ids from the producer's
// record-row list (contiguous int32s, psx_apply_indexed_rows) instead of the stream.
// Every 4-byte row id read from the stream costs one 128-B L2->DRAM request (PMC,
// profiles/r02/pmc_request_sizes_index_apply.json): 1.07 GB on C2 for 32 MB of row ids.
// Plain loads, loads issued one lane at a time, sc0/sc1/nt scope hints (still 128-B
// requests) and scalar s_load_dword (64-B requests, but 0.51 vs 0.26 ms) were no faster
// than the non-temporal vector loads kept here (profiles/r02/ab_index_loads.json,
// ab_index_policy.json).
template <int UNROLL>
__global__ void __launch_bounds__(256) dense_index_v2_kernel(StreamSet ss, IdxSet ix, uint32_t rows_mask,
                                                            const Seg *segs, int t, int B, int64_t stride, Geo g,
                                                            int32_t *inv, InvLayout L, uint32_t *call_status) {
  __shared__ int64_t pre[kMaxFused + 1];
  __shared__ const uint8_t *base[kMaxFused];
  __shared__ int64_t sstr[kMaxFused];
  if (threadIdx.x == 0) {
    int64_t acc = 0;
    for (int b = 0; b < kMaxFused; ++b) {
      pre[b] = acc;
      base[b] = nullptr;
      sstr[b] = stride;
      if (b < B) {
        const Seg sg = segs[b * kMaxTables + t];
        if (sg.rec0 >= 0 && !sg.sparse) {
          acc += sg.num_rows;
          if ((rows_mask >> b) & 1u) {
            base[b] = reinterpret_cast<const uint8_t *>(ix.rows[b] + sg.ord0);
            sstr[b] = 4;
          } else {
            base[b] = ss.data[b] + sg.rec0;
          }
        }
      }
    }
    pre[kMaxFused] = acc;
  }
  __syncthreads();
  const int64_t total = pre[kMaxFused];
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  for (int64_t r0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r0 < total; r0 += G * UNROLL) {
    int32_t rid[UNROLL];
    int32_t bi[UNROLL];
    int64_t ii[UNROLL];
    const int32_t *ptr[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int64_t r = r0 + u * G;
      bi[u] = -1;
      ii[u] = 0;
      rid[u] = 0;
      ptr[u] = nullptr;
      if (r < total) {
        int b = 0;
        while (b + 1 < B && pre[b + 1] <= r) ++b;
        bi[u] = b;
        ii[u] = r - pre[b];
        ptr[u] = reinterpret_cast<const int32_t *>(base[b] + ii[u] * sstr[b]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      if (ptr[u]) rid[u] = __builtin_nontemporal_load(ptr[u]);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (bi[u] < 0) continue;
      const int64_t s = slot_of(rid[u], g);
      if (s < 0) {
        // a listed row outside the shard only drops the claim: the short count replays the
        // call from the stream, whose own row ids decide (as for a duplicate row)
        if (!((rows_mask >> bi[u]) & 1u)) atomicOr(call_status, kStRowRange);
        continue;
      }
      inv[s * L.ss + bi[u] * L.sb] = (int32_t)ii[u];
    }
  }
}

// finish_call: fold the per-call status into the sticky word and free the ring slot.
__global__ void finish_call_kernel(uint32_t *sticky, uint32_t *call_status, uint32_t *call_log) {
  if (threadIdx.x == 0) {
    *sticky |= *call_status;
    *call_log = *call_status;
    *call_status = 0;
  }
}

// flags_or: mark num slots starting at first as present (psx_table_load_rows).
__global__ void flags_or_kernel(uint8_t *flags, int64_t first, int64_t num, uint8_t bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < num) flags[first + i] |= bits;
}

__global__ void flags_and_kernel(uint8_t *flags, int64_t num, uint8_t bits) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < num) flags[i] &= bits;
}

// gather_dense_rows: copy rows for a list of slots into a compact buffer (serve-back).
template <typename V>
__global__ void gather_rows_kernel(const V *table, const int64_t *slots, int32_t n, int64_t row_cap,
                                   V *out) {
  const int r = blockIdx.x;
  if (r >= n) return;
  const int64_t s = slots[r];
  for (int64_t e = threadIdx.x; e < row_cap; e += blockDim.x)
    out[(int64_t)r * row_cap + e] = s >= 0 ? table[s * row_cap + e] : V(0);
}

__global__ void fill_u64_kernel(uint64_t *p, int64_t n, uint64_t v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

__global__ void gather_u64_kernel(const uint64_t *src, const int64_t *slots, int32_t n, uint64_t *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = slots[i] >= 0 ? src[slots[i]] : 0;
}

__global__ void gather_flags_kernel(const uint8_t *flags, const int64_t *slots, int32_t n, uint8_t *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = slots[i] >= 0 ? flags[slots[i]] : 0;
}

// ---------------------------------------------------------------------------
// Host-side launchers (internal to libpsx).
hipError_t launch_idx_verify(StreamSet ss, const TableDir &dir, const Seg *segs, const IdxSet &ix, uint64_t *recoff,
                             uint32_t *call_status, uint32_t *idxw, const WalkCount *wc, hipStream_t st);

// idxw: 4 words per message (indexed messages); wc: null, or the walk-counted split tables'
// WalkCount (idx_verify counts their records, as the window-parallel walk does)
hipError_t launch_decode(StreamSet ss, const TableDir &dir, Seg *segs, uint64_t *recoff,
                         uint32_t *call_status, uint32_t *counters, uint32_t *ntouched, const IdxSet &ix,
                         uint32_t *idxw, const WalkCount *wc, hipStream_t st) {
  hipLaunchKernelGGL(decode_streams_kernel, dim3(ss.n), dim3(kDecodeThreads), 0, st, ss, dir, segs, recoff,
                     call_status, counters, ntouched, ix, idxw);
  hipError_t e = hipGetLastError();
  bool any = false;
  for (int b = 0; b < ss.n; ++b) any = any || ix.p[b];
  if (e == hipSuccess && any) e = launch_idx_verify(ss, dir, segs, ix, recoff, call_status, idxw, wc, st);
  return e;
}

// Resident-capacity grid for a persistent-style kernel (blocks per CU x CUs).
template <typename K>
static unsigned resident_blocks(K kernel, int64_t want) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu <= 0)
    per_cu = 2;
  int64_t cap = (int64_t)per_cu * cus;
  if (want < cap) cap = want;
  return (unsigned)(cap < 1 ? 1 : cap);
}

// Run-time selectors (include/psx_debug.h): the defaults are the measured winners; the
// alternatives stay selectable so the parity suite runs every kernel the product can
// launch (v2 is the >= 4 GiB fallback, v4 the partial-coverage kernel).
int g_apply_variant = 0;   // 0: auto, 1: force v2, 2: force v4 (compact)
int g_dense_last = 0;      // PSX_STAT_DENSE_LAST: the dense apply kernel last launched (2, 3, 4)

hipError_t launch_dense_index(StreamSet ss, const IdxSet &ix, uint32_t rows_mask, const Seg *segs, int t, int B,
                              int64_t stride, int64_t row_offset, int64_t row_stride, int64_t max_rows,
                              int32_t *inv, InvLayout L, uint32_t *call_status, hipStream_t st) {
  // Listed messages read their row ids from the record-row lists (contiguous).  An
  // XCD-local form of the scatter (each XCD writing only its eighth of the slots) was
  // slower, 0.21 vs 0.13 ms on C2 (profiles/r02/ab_index_rows.json).
  Geo g{row_offset, row_stride, max_rows};
  hipLaunchKernelGGL((dense_index_v2_kernel<8>), dim3(2048), dim3(256), 0, st, ss, ix, rows_mask, segs, t, B, stride,
                     g, inv, L, call_status);
  return hipGetLastError();
}

hipError_t launch_dense_verify(const int32_t *inv, InvLayout L, int t, int B, int64_t max_rows,
                               uint32_t *counters, hipStream_t st) {
  int64_t blocks = (max_rows + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dense_verify_kernel, dim3((unsigned)blocks), dim3(256), 0, st, inv, L, t, B, max_rows,
                     counters);
  return hipGetLastError();
}

template <typename V, int BMAX, int TILE, bool NT, int PAIR, bool IMP = false, int H16 = 0>
static void launch_v2(const DenseArgs &a, hipStream_t st) {
  auto k = dense_apply_v2_kernel<V, BMAX, TILE, NT, PAIR, IMP, H16>;
  g_dense_last = 2;
  const int64_t tiles = (a.max_rows + TILE - 1) / TILE;
  const unsigned blocks = resident_blocks(k, (tiles + 3) / 4);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, st, a);
}

template <typename V, int BMAX, int TILE, bool NT, int PAIR, bool IMP = false, int H16 = 0>
static void launch_v3(const DenseArgs &a, hipStream_t st) {
  auto k = dense_apply_v3_kernel<V, BMAX, TILE, NT, PAIR, IMP, H16>;
  g_dense_last = 3;
  const int64_t tiles = (a.max_rows + TILE - 1) / TILE;
  const unsigned blocks = resident_blocks(k, (tiles + 3) / 4);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, st, a);
}

// BMAX is the next power of two >= B and the rows in flight per wave grow as B shrinks,
// so every wave keeps ~8-18 16-byte loads in flight whatever the batch width.
template <typename V, bool IMP, int H16>
static void launch_adaptive_v3(const DenseArgs &a, hipStream_t st) {
  if (a.B <= 1) launch_v3<V, 1, 16, true, 8, IMP, H16>(a, st);
  else if (a.B <= 2) launch_v3<V, 2, 16, true, 4, IMP, H16>(a, st);
  else if (a.B <= 4) launch_v3<V, 4, 16, true, 3, IMP, H16>(a, st);
  else if (a.B <= 8) launch_v3<V, 8, 16, true, 2, IMP, H16>(a, st);
  else launch_v3<V, 16, 16, true, 1, IMP, H16>(a, st);
}

// v2 (64-bit record pointers): streams of >= 4 GiB, which v3's 32-bit offsets cannot reach.
template <typename V, int H16>
static void launch_adaptive_v2(const DenseArgs &a, hipStream_t st) {
  if (a.B <= 1) launch_v2<V, 1, 16, true, 8, false, H16>(a, st);
  else if (a.B <= 2) launch_v2<V, 2, 16, true, 4, false, H16>(a, st);
  else if (a.B <= 4) launch_v2<V, 4, 16, true, 3, false, H16>(a, st);
  else if (a.B <= 8) launch_v2<V, 8, 16, true, 2, false, H16>(a, st);
  else launch_v2<V, 16, 16, true, 1, false, H16>(a, st);
}

// Importance tables: the f64 terms cost registers, so fewer rows in flight per wave buys
// back occupancy.
template <typename V, int H16>
static void launch_adaptive_imp(const DenseArgs &a, hipStream_t st) {
  if (a.B <= 1) launch_v2<V, 1, 16, true, 4, true, H16>(a, st);
  else if (a.B <= 2) launch_v2<V, 2, 16, true, 2, true, H16>(a, st);
  else if (a.B <= 4) launch_v2<V, 4, 16, true, 2, true, H16>(a, st);
  else if (a.B <= 8) launch_v2<V, 8, 16, true, 1, true, H16>(a, st);
  else launch_v2<V, 16, 16, true, 1, true, H16>(a, st);
}

template <typename V>
static void launch_v4(const DenseArgs &a, hipStream_t st) {
  g_dense_last = 4;
  if (a.B > 8) {
    auto k = dense_apply_v4_kernel<V, 16, 16, true, 8, 16>;
    hipLaunchKernelGGL(k, dim3(resident_blocks(k, ((a.max_rows + 15) / 16 + 3) / 4)), dim3(256), 0, st, a);
  } else {
    auto k = dense_apply_v4_kernel<V, 8, 16, true, 4, 12>;
    hipLaunchKernelGGL(k, dim3(resident_blocks(k, ((a.max_rows + 15) / 16 + 3) / 4)), dim3(256), 0, st, a);
  }
}

// v3 addresses records by 32-bit offsets from each message's first record.
static bool v3_ok(const DenseArgs &a) {
  for (int b = 0; b < a.B; ++b)
    if ((uint64_t)a.ss.size[b] >= 0xffff0000ull) return false;
  return true;
}

// Sparse coverage: at most ~2 records per row on average (estimated from the message
// sizes, which over-count when messages carry other tables — erring towards v3).  v4
// compact is 5% faster than v3 at 12.5% density and 11% slower at full density
// (profiles/r01/exp_density125_variants.txt).
static bool sparse_coverage(const DenseArgs &a) {
  uint64_t bytes = 0;
  for (int b = 0; b < a.B; ++b) bytes += a.ss.size[b];
  return a.B <= 8 && bytes / (uint64_t)a.stride <= 2 * (uint64_t)a.max_rows;
}

template <typename V>
static hipError_t launch_dense_apply_t(const DenseArgs &a, hipStream_t st) {
  if (a.imp) launch_adaptive_imp<V, 0>(a, st);
  else if (g_apply_variant == 1 || !v3_ok(a)) launch_adaptive_v2<V, 0>(a, st);
  else if (g_apply_variant == 2 || (g_apply_variant == 0 && sparse_coverage(a))) launch_v4<V>(a, st);
  else launch_adaptive_v3<V, false, 0>(a, st);
  return hipGetLastError();
}

// True when launch_dense_apply runs v3 on these arguments: the only apply kernel that
// checks producer-placed records (DenseArgs::rows_mask); other tables index from the stream.
bool dense_apply_checks_rows(const DenseArgs &a, bool rec_f16) {
  if (a.imp || g_apply_variant == 1 || !v3_ok(a)) return false;
  if (rec_f16) return true;
  // v4 (partial coverage) does not check lists: a form that did (lane j checking slot-list
  // entry j before the group's payload loads) made its apply 40% slower on the 12.5%-density
  // C2 variant, 0.907 vs 0.65 ms (profiles/r02/ab_v4_rows.json)
  return !(g_apply_variant == 2 || (g_apply_variant == 0 && sparse_coverage(a)));
}

hipError_t launch_dense_apply(int dtype, const DenseArgs &a, hipStream_t st, bool rec_f16) {
  if (rec_f16) {   // f32 tables only (checked at table creation)
    // binary16 records decompressed by the hardware conversion (H16 = 2): it keeps NaN
    // payloads and quiets them, and every decompressed value goes through `row += u`,
    // which quiets anyway, so rows are bit-identical to the payload-exact decompression
    // at 23% less time on C2 (VALU-bound, profiles/r01/exp_f16_variants.txt).
    if (a.imp) launch_adaptive_imp<float, 2>(a, st);
    else if (g_apply_variant == 1 || !v3_ok(a)) launch_adaptive_v2<float, 2>(a, st);
    else launch_adaptive_v3<float, false, 2>(a, st);
    return hipGetLastError();
  }
  switch (dtype) {
    case 0: return launch_dense_apply_t<float>(a, st);
    case 1: return launch_dense_apply_t<double>(a, st);
    case 2: return launch_dense_apply_t<int32_t>(a, st);
    default: return launch_dense_apply_t<int64_t>(a, st);
  }
}

hipError_t launch_finish(uint32_t *sticky, uint32_t *call_status, uint32_t *call_log, hipStream_t st) {
  hipLaunchKernelGGL(finish_call_kernel, dim3(1), dim3(64), 0, st, sticky, call_status, call_log);
  return hipGetLastError();
}

hipError_t launch_flags_or(uint8_t *flags, int64_t first, int64_t num, uint8_t bits, hipStream_t st) {
  if (num <= 0) return hipSuccess;
  hipLaunchKernelGGL(flags_or_kernel, dim3((unsigned)((num + 255) / 256)), dim3(256), 0, st, flags, first,
                     num, bits);
  return hipGetLastError();
}

hipError_t launch_flags_and(uint8_t *flags, int64_t num, uint8_t bits, hipStream_t st) {
  if (num <= 0) return hipSuccess;
  hipLaunchKernelGGL(flags_and_kernel, dim3((unsigned)((num + 255) / 256)), dim3(256), 0, st, flags, num,
                     bits);
  return hipGetLastError();
}

hipError_t launch_gather_rows(int dtype, const void *table, const int64_t *slots, int32_t n,
                              int64_t row_cap, void *out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  switch (dtype) {
    case 0: hipLaunchKernelGGL(gather_rows_kernel<float>, dim3(n), dim3(256), 0, st,
                               (const float *)table, slots, n, row_cap, (float *)out); break;
    case 1: hipLaunchKernelGGL(gather_rows_kernel<double>, dim3(n), dim3(256), 0, st,
                               (const double *)table, slots, n, row_cap, (double *)out); break;
    case 2: hipLaunchKernelGGL(gather_rows_kernel<int32_t>, dim3(n), dim3(256), 0, st,
                               (const int32_t *)table, slots, n, row_cap, (int32_t *)out); break;
    default: hipLaunchKernelGGL(gather_rows_kernel<int64_t>, dim3(n), dim3(256), 0, st,
                                (const int64_t *)table, slots, n, row_cap, (int64_t *)out); break;
  }
  return hipGetLastError();
}

hipError_t launch_fill_u64(uint64_t *p, int64_t n, uint64_t v, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_u64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, n, v);
  return hipGetLastError();
}

hipError_t launch_gather_u64(const uint64_t *src, const int64_t *slots, int32_t n, uint64_t *out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_u64_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, slots, n, out);
  return hipGetLastError();
}

hipError_t launch_gather_flags(const uint8_t *flags, const int64_t *slots, int32_t n, uint8_t *out,
                               hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(gather_flags_kernel, dim3((n + 255) / 256), dim3(256), 0, st, flags, slots, n, out);
  return hipGetLastError();
}

}  // namespace psx
