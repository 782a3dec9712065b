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
// decode_streams: grid = B workgroups of 64 threads; lane 0 walks one message.
__global__ void __launch_bounds__(64) decode_streams_kernel(StreamSet ss, TableDir dir, Seg *segs,
                                                            uint64_t *recoff, uint32_t *call_status,
                                                            uint32_t *counters) {
  const int b = blockIdx.x;
  for (int t = threadIdx.x; t < kMaxTables; t += blockDim.x) {
    Seg s;
    s.rec0 = -1;
    s.num_rows = 0;
    s.sparse = 0;
    segs[b * kMaxTables + t] = s;
    counters[t * kMaxFused + b] = 0;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  const uint8_t *p = ss.data[b];
  const uint64_t size = ss.size[b];
  if (size == 0) return;                       // empty message (server.cpp:128)
  if (size < 4) { atomicOr(call_status, kStMalformed); return; }
  const int32_t ntab = ld32(p);
  if (ntab < 0) { atomicOr(call_status, kStMalformed); return; }
  uint64_t off = 4;
  uint64_t rk = ss.recoff_base[b];
  for (int32_t k = 0; k < ntab; ++k) {
    if (off + 16 > size) { atomicOr(call_status, kStMalformed); return; }
    const int32_t tid = ld32(p + off);
    const uint64_t usz = ld64_a4(p + off + 4);
    const int32_t nrows = ld32(p + off + 12);
    off += 16;
    int t = -1;
    for (int i = 0; i < dir.n; ++i)
      if (dir.table_id[i] == tid) t = i;
    if (t < 0) { atomicOr(call_status, kStUnknownTable); return; }
    if (usz != (uint64_t)dir.vsize[t] || nrows < 0) { atomicOr(call_status, kStMalformed); return; }
    Seg &sg = segs[b * kMaxTables + t];
    if (sg.rec0 >= 0) { atomicOr(call_status, kStUnsupported); return; }
    if (dir.dense_serialized[t]) {
      const uint64_t stride = 4 + (uint64_t)dir.oplog_cap[t] * dir.vsize[t];
      const uint64_t need = (uint64_t)nrows * stride;
      if (off + need > size) { atomicOr(call_status, kStMalformed); return; }
      sg.rec0 = (int64_t)off;
      sg.num_rows = nrows;
      sg.sparse = 0;
      off += need;
    } else {
      // Sparse records {int32 row; int32 n; int32 cols[n]; V vals[n]}
      // (AbstractRowOpLog::ParseSparseSerializedOpLog, abstract_row_oplog.hpp:64-78):
      // sizes chain, so the walk is sequential.
      sg.rec0 = (int64_t)rk;   // index of the first record offset
      sg.num_rows = nrows;
      sg.sparse = 1;
      const uint64_t per = 4 + (uint64_t)dir.vsize[t];
      for (int32_t r = 0; r < nrows; ++r) {
        if (off + 8 > size) { atomicOr(call_status, kStMalformed); return; }
        const int32_t n = ld32(p + off + 4);
        if (n < 0) { atomicOr(call_status, kStMalformed); return; }
        const uint64_t rs = 8 + (uint64_t)n * per;
        if (off + rs > size) { atomicOr(call_status, kStMalformed); return; }
        recoff[rk++] = off;
        off += rs;
      }
    }
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

// dense_index: grid-stride over every record of every message containing table t.
__global__ void __launch_bounds__(256) dense_index_kernel(StreamSet ss, const Seg *segs, int t, int B,
                                                         int64_t stride, Geo g, int32_t *inv,
                                                         uint32_t *call_status) {
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x;
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int b = 0; b < B; ++b) {
    const Seg sg = segs[b * kMaxTables + t];
    if (sg.rec0 < 0 || sg.sparse) continue;
    const uint8_t *base = ss.data[b] + sg.rec0;
    for (int64_t i = gid; i < sg.num_rows; i += gsz) {
      const int32_t rid = ld32(base + i * stride);
      const int64_t s = slot_of(rid, g);
      if (s < 0) { atomicOr(call_status, kStRowRange); continue; }
      inv[s * B + b] = (int32_t)i;
    }
  }
}

// dense_verify: counters[t][b] = number of slots claimed by message b.
__global__ void __launch_bounds__(256) dense_verify_kernel(const int32_t *inv, int t, int B,
                                                          int64_t max_rows, uint32_t *counters) {
  __shared__ uint32_t part[kMaxFused];
  if (threadIdx.x < kMaxFused) part[threadIdx.x] = 0;
  __syncthreads();
  uint32_t cnt[kMaxFused];
#pragma unroll
  for (int b = 0; b < kMaxFused; ++b) cnt[b] = 0;
  const int64_t gsz = (int64_t)gridDim.x * blockDim.x;
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < max_rows; s += gsz) {
    const int32_t *row = inv + s * B;
#pragma unroll
    for (int b = 0; b < kMaxFused; ++b)
      if (b < B) cnt[b] += row[b] >= 0 ? 1u : 0u;
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


// dense_apply: each wave owns a tile of 64 consecutive slots.  Lane k reads the B
// inverse-index entries of slot k (and restores them to -1), writes the slot's flags,
// then the wave walks the touched slots; for each, 4 elements per lane per 256-element
// chunk: 1 table load + B record loads issued back to back, then the in-order sum.
template <typename V, int BMAX>
__global__ void __launch_bounds__(256) dense_apply_kernel(DenseArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int B = a.B;

  // Per-call gate: fatal errors, a duplicate row in any message, or a duplicate still
  // pending from an earlier call (ordering) => apply nothing, just restore the index.
  bool skip = (*a.call_status & kStFatal) != 0 || (*a.sticky & kStDuplicateRow) != 0;
  bool dup = false;
  int64_t rec0[BMAX];
#pragma unroll
  for (int b = 0; b < BMAX; ++b) {
    rec0[b] = -1;
    if (b < B) {
      const Seg sg = a.segs[b * kMaxTables + a.t];
      if (sg.rec0 >= 0 && !sg.sparse) {
        rec0[b] = sg.rec0;
        if (a.counters[a.t * kMaxFused + b] != (uint32_t)sg.num_rows) dup = true;
      }
    }
  }
  if (dup && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.call_status, kStDuplicateRow);
  skip = skip || dup;

  const int64_t s0 = tile * 64;
  if (s0 >= a.max_rows) return;
  const int64_t my_slot = s0 + lane;
  const bool in_range = my_slot < a.max_rows;
  int32_t idx[BMAX];
  bool touched = false;
#pragma unroll
  for (int b = 0; b < BMAX; ++b) {
    idx[b] = -1;
    if (b < B && in_range) {
      idx[b] = a.inv[my_slot * B + b];
      if (idx[b] >= 0) {
        touched = true;
        a.inv[my_slot * B + b] = -1;
      }
    }
  }
  if (skip) return;
  if (touched) a.flags[my_slot] = 3;   // exists | dirty

  uint64_t live = __ballot(touched);
  V *table = reinterpret_cast<V *>(a.table);
  while (live) {
    const int k = __builtin_ctzll(live);
    live &= live - 1;
    const int64_t slot = s0 + k;
    V *trow = table + slot * a.row_cap;
    const uint8_t *rb[BMAX];
    bool present[BMAX];
#pragma unroll
    for (int b = 0; b < BMAX; ++b) {
      const int32_t i = __builtin_amdgcn_readlane(idx[b], k);
      present[b] = (b < B) && i >= 0;
      rb[b] = present[b] ? a.ss.data[b] + rec0[b] + (int64_t)i * a.stride + 4 : a.zero_chunk;
    }
    for (int64_t c0 = 0; c0 < a.cap; c0 += 256) {
      V t[4];
      V u[BMAX][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t e = c0 + lane + 64 * j;
        t[j] = e < a.cap ? trow[e] : V(0);
      }
#pragma unroll
      for (int b = 0; b < BMAX; ++b) {
        const uint8_t *base = present[b] ? rb[b] + c0 * (int64_t)sizeof(V) : a.zero_chunk;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t e = c0 + lane + 64 * j;
          u[b][j] = e < a.cap ? Elem<V>::load_rec(base + (lane + 64 * j) * sizeof(V)) : V(0);
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        V acc = t[j];
#pragma unroll
        for (int b = 0; b < BMAX; ++b)
          if (present[b]) acc = Elem<V>::add(acc, u[b][j]);
        const int64_t e = c0 + lane + 64 * j;
        if (e < a.cap) trow[e] = acc;
      }
    }
  }
}

// finish_call: fold the per-call status into the sticky word and free the ring slot.
__global__ void finish_call_kernel(uint32_t *sticky, uint32_t *call_status) {
  if (threadIdx.x == 0) {
    *sticky |= *call_status;
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

// ---------------------------------------------------------------------------
// Host-side launchers (internal to libpsx).
hipError_t launch_decode(StreamSet ss, const TableDir &dir, Seg *segs, uint64_t *recoff,
                         uint32_t *call_status, uint32_t *counters, hipStream_t st) {
  hipLaunchKernelGGL(decode_streams_kernel, dim3(ss.n), dim3(64), 0, st, ss, dir, segs, recoff,
                     call_status, counters);
  return hipGetLastError();
}

hipError_t launch_dense_index(StreamSet ss, const Seg *segs, int t, int B, int64_t stride,
                              int64_t row_offset, int64_t row_stride, int64_t max_rows,
                              int32_t *inv, uint32_t *call_status, hipStream_t st) {
  Geo g{row_offset, row_stride, max_rows};
  hipLaunchKernelGGL(dense_index_kernel, dim3(4096), dim3(256), 0, st, ss, segs, t, B, stride, g,
                     inv, call_status);
  return hipGetLastError();
}

hipError_t launch_dense_verify(const int32_t *inv, int t, int B, int64_t max_rows, uint32_t *counters,
                               hipStream_t st) {
  int64_t blocks = (max_rows + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dense_verify_kernel, dim3((unsigned)blocks), dim3(256), 0, st, inv, t, B, max_rows,
                     counters);
  return hipGetLastError();
}

template <typename V>
static hipError_t launch_dense_apply_t(const DenseArgs &a, hipStream_t st) {
  const int64_t tiles = (a.max_rows + 63) / 64;
  const int64_t blocks = (tiles + 3) / 4;
  if (a.B <= 8)
    hipLaunchKernelGGL((dense_apply_kernel<V, 8>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((dense_apply_kernel<V, 16>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_dense_apply(int dtype, const DenseArgs &a, hipStream_t st) {
  switch (dtype) {
    case 0: return launch_dense_apply_t<float>(a, st);
    case 1: return launch_dense_apply_t<double>(a, st);
    case 2: return launch_dense_apply_t<int32_t>(a, st);
    default: return launch_dense_apply_t<int64_t>(a, st);
  }
}

hipError_t launch_finish(uint32_t *sticky, uint32_t *call_status, hipStream_t st) {
  hipLaunchKernelGGL(finish_call_kernel, dim3(1), dim3(64), 0, st, sticky, call_status);
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

}  // namespace psx
