// psx_split.hip — the client's per-server split of one packed message, on the device.
//
// AbstractBgWorker::CreateOpLogMsgs (abstract_bg_worker.cpp:590-649) builds one message per
// server from the rows each server owns (RowOpLogSerializer::AppendRowOpLog routes every
// row by GetPartitionServerID, row_oplog_serializer.hpp:100-124); psx_split_stream does the
// same for a message already packed on one GPU whose rows span the row-range shards of
// several (the one exchange step of the multi-GPU path).  Owner o's
// sub-stream is a complete Appendix-A message: its tables in the message's order (tables
// without records for o omitted), each table's records in message order.
//
// Records are flattened over the message's tables in stream order (record k) and dealt to
// waves in tiles of 64 (lane l: record 64t + l):
//   split_count    owner and size of every record; per tile the bytes of each owner (a
//                  stable partition's bucket counts), per (owner, table) the records and bytes
//   scan           exclusive scan of the tile bytes, owner-major
//   split_scatter  each record's destination = its owner's message base + the headers in
//                  front of its table + the owner's bytes before it (tile prefix + the wave's
//                  prefix over earlier lanes of the same owner); then the wave copies its 64
//                  records one after another (16-byte accesses, both sides 4-byte aligned)
//   put_words      the num_tables word and table headers of every owner's message
// Byte traffic: the message read twice (sizes, then the copy: the row id and n share the
// record's first line) and written once, plus 16 B of per-record metadata written and read.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "psx_device.hpp"
#include "psx_scan.hpp"

namespace psx {

typedef uint32_t sx_u32x4 __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ int split_table_of(const SplitArgs &a, int64_t k) {
  int j = 0;
  while (j + 1 < a.ntab && a.tabs[j + 1].k0 <= k) ++j;
  return j;
}

__device__ __forceinline__ int split_owner_of(const SplitArgs &a, int64_t row) {
  if (row < a.row_begin[0] || row >= a.row_begin[a.nowners]) return -1;
  int lo = 0, hi = a.nowners;   // row_begin[lo] <= row < row_begin[hi]
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (a.row_begin[mid] <= row) lo = mid;
    else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(256) split_count_kernel(SplitArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t t = wave; t < a.ntiles; t += nw) {
    const int64_t k = t * 64 + lane;
    int o = -1, j = 0;
    uint64_t size = 0;
    if (k < a.nrec) {
      j = split_table_of(a, k);
      const SplitTab &tb = a.tabs[j];
      const int64_t i = k - tb.k0;
      const uint64_t off = tb.sparse ? a.recoff[tb.rec0 + i] : (uint64_t)(tb.rec0 + i * tb.stride);
      const int32_t rid = *reinterpret_cast<const int32_t *>(a.msg + off);
      size = tb.sparse ? 8 + (uint64_t)(*reinterpret_cast<const int32_t *>(a.msg + off + 4)) * (4 + tb.vsize)
                       : (uint64_t)tb.stride;
      o = split_owner_of(a, rid);
      if (o < 0) atomicOr(a.status, kStRowRange);
      a.src_off[k] = off;
      a.meta[k] = ((uint64_t)(uint32_t)(o < 0 ? 0xFFFF : o) << 48) | ((uint64_t)j << 40) | size;
    }
    // per (owner, table) present in the tile: one atomic pair; per owner: the tile's bytes
    uint64_t todo = __ballot(o >= 0);
    while (todo) {
      const int leader = __builtin_ctzll(todo);
      const int lo = __builtin_amdgcn_readlane(o, leader), lj = __builtin_amdgcn_readlane(j, leader);
      const bool mine = o == lo && j == lj && o >= 0;
      const uint64_t m = __ballot(mine);
      uint64_t v = mine ? size : 0;
#pragma unroll
      for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
      if (lane == leader) {
        atomicAdd((unsigned long long *)&a.ot_count[lo * a.ntab + lj], (unsigned long long)__builtin_popcountll(m));
        atomicAdd((unsigned long long *)&a.ot_bytes[lo * a.ntab + lj], (unsigned long long)v);
      }
      todo &= ~m;
    }
    todo = __ballot(o >= 0);
    while (todo) {
      const int leader = __builtin_ctzll(todo);
      const int lo = __builtin_amdgcn_readlane(o, leader);
      const bool mine = o == lo;
      const uint64_t m = __ballot(mine);
      uint64_t v = mine ? size : 0;
#pragma unroll
      for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
      if (lane == leader) a.tile_bytes[(int64_t)lo * a.ntiles + t] = (int64_t)v;
      todo &= ~m;
    }
  }
}

__global__ void __launch_bounds__(256) split_scatter_kernel(SplitArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  if (*a.status & kStFatal) return;
  for (int64_t t = wave; t < a.ntiles; t += nw) {
    const int64_t k = t * 64 + lane;
    int o = -1, j = 0;
    uint64_t size = 0, src = 0;
    if (k < a.nrec) {
      const uint64_t m = a.meta[k];
      o = (int)(m >> 48);
      j = (int)((m >> 40) & 0xFF);
      size = m & ((1ull << 40) - 1);
      src = a.src_off[k];
    }
    // this record's byte offset inside its owner's records: earlier tiles + earlier lanes
    uint64_t dst = 0;
    uint64_t todo = __ballot(k < a.nrec);
    while (todo) {
      const int leader = __builtin_ctzll(todo);
      const int lo = __builtin_amdgcn_readlane(o, leader);
      const bool mine = o == lo && k < a.nrec;
      const uint64_t msk = __ballot(mine);
      uint64_t incl = mine ? size : 0;
#pragma unroll
      for (int s = 1; s < 64; s <<= 1) {
        const uint64_t y = __shfl_up(incl, s, 64);
        if (lane >= s) incl += y;
      }
      if (mine) {
        const int64_t tp = a.tile_pre[(int64_t)lo * a.ntiles + t] - a.tile_pre[(int64_t)lo * a.ntiles];
        dst = (uint64_t)(a.owner_base[lo] + a.hdr_shift[lo * a.ntab + j] + tp) + incl - size;
      }
      todo &= ~msk;
    }
    // copy the tile's records, one at a time with the whole wave
    const int64_t kend = (t + 1) * 64 < a.nrec ? (t + 1) * 64 : a.nrec;
    for (int64_t kk = t * 64; kk < kend; ++kk) {
      const int q = (int)(kk - t * 64);
      const uint64_t s_ = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(src >> 32), q) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)src, q);
      const uint64_t d_ = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(dst >> 32), q) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)dst, q);
      const uint64_t n_ = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(size >> 32), q) << 32) |
                          (uint32_t)__builtin_amdgcn_readlane((int32_t)(uint32_t)size, q);
      const uint8_t *sp = a.msg + s_;
      uint8_t *dp = a.out + d_;
      const uint64_t n16 = n_ & ~15ull;
      for (uint64_t b = (uint64_t)lane * 16; b < n16; b += 64 * 16)
        *reinterpret_cast<sx_u32x4 *>(dp + b) = *reinterpret_cast<const sx_u32x4 *>(sp + b);
      for (uint64_t b = n16 + (uint64_t)lane * 4; b < n_; b += 64 * 4)
        *reinterpret_cast<uint32_t *>(dp + b) = *reinterpret_cast<const uint32_t *>(sp + b);
    }
  }
}

__global__ void split_words_kernel(uint8_t *out, const int64_t *pos, const uint32_t *val, int32_t n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) *reinterpret_cast<uint32_t *>(out + pos[i]) = val[i];
}

hipError_t launch_split_count(const SplitArgs &a, hipStream_t st) {
  const unsigned blocks = (unsigned)((a.ntiles + 3) / 4 < 4096 ? (a.ntiles + 3) / 4 : 4096);
  hipLaunchKernelGGL(split_count_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  launch_exclusive_scan<int64_t>(a.tile_bytes, (int64_t)a.nowners * a.ntiles, a.tile_pre, a.scan_tmp, st);
  return hipGetLastError();
}

hipError_t launch_split_scatter(const SplitArgs &a, const int64_t *pos, const uint32_t *val, int32_t nwords,
                                hipStream_t st) {
  const unsigned blocks = (unsigned)((a.ntiles + 3) / 4 < 4096 ? (a.ntiles + 3) / 4 : 4096);
  hipLaunchKernelGGL(split_scatter_kernel, dim3(blocks ? blocks : 1), dim3(256), 0, st, a);
  if (nwords) hipLaunchKernelGGL(split_words_kernel, dim3((nwords + 255) / 256), dim3(256), 0, st, a.out, pos, val, nwords);
  return hipGetLastError();
}

}  // namespace psx
