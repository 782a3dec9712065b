// psx_client.hip — the client side of serve-back: a push (or row-request reply) body
// applied to a client's cached rows.
//
// SSPPushBgWorker::ApplyServerPushedRow (ssp_push_bg_worker.cpp:70-122) walks the body with
// SerializedRowReader (serialized_row_reader.hpp:30-100): per table int32 table_id, then
// records {int32 row_id; size_t size; bytes}, int32 -1 before the next table id, int32 -2
// at the end.  For a version table the last 8 bytes are the row version
// (AbstractBgWorker::ExtractRowVersion, abstract_bg_worker.cpp:1032-1040).  A record for a
// row the client caches replaces its data — UpdateExistingRow -> ResetRowData
// (abstract_bg_worker.cpp:775-800, numeric_store_row.hpp:142-145): VectorStore::ResetData
// copies the bytes over the row (vector_store.hpp:89-91); SortedVectorMapStore and
// MapStore take AbstractStore's default, Deserialize (abstract_store.hpp:30-32,
// sorted_vector_map_store.hpp:155-164, map_store.hpp:103-120).  Rows the client does not
// cache are skipped; a row-request reply inserts them (InsertNonexistentRow, :853-870).
//
//   push_walk    one workgroup: stages the body in LDS windows, computes every word's
//                chain successor in parallel, and thread 0 hops the record chain at LDS
//                latency, writing (table, row id, byte offset, size) per record
//   push_claim   validates every record (all-or-nothing) and picks, per row, the body's
//                last record for it (the reference resets in body order: last one wins)
//   push_reset   one wave per winning record: the store's ResetData
#include <hip/hip_runtime.h>
#include <cstdint>
#include "psx_device.hpp"

namespace psx {

constexpr int kWalkThreads = 1024;
constexpr int kWalkWords = 8192;              // 32 KiB window
constexpr uint32_t kNoNext = 0xFFFFFFFFu;

__device__ __forceinline__ int32_t c_ld32(const uint8_t *p) {
  int32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}
__device__ __forceinline__ uint64_t c_ld64(const uint8_t *p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

// Chain positions (word indices relative to the window): a record {row_id >= 0, size}
// continues at +3 + size/4; a separator -1 at +2 (the next table id follows); -2 ends.
__global__ void __launch_bounds__(kWalkThreads) push_walk_kernel(const uint8_t *body, uint64_t size,
                                                                 PushEntry *ent, uint32_t *nent, uint32_t max_ent,
                                                                 uint32_t *status) {
  __shared__ uint32_t win[kWalkWords];
  __shared__ uint32_t nxt[kWalkWords];
  __shared__ uint64_t sh_pos;      // byte offset of the next chain element (a row id / separator)
  __shared__ int32_t sh_table;     // current table id
  __shared__ uint32_t sh_n;
  __shared__ int32_t sh_state;     // 0 walking, 1 done
  if (threadIdx.x == 0) {
    sh_n = 0;
    sh_state = 1;
    if (size >= 4) {
      sh_table = c_ld32(body);
      sh_pos = 4;
      // Restart (:33-41): a body that opens with the end marker holds nothing
      if (sh_table != -2) sh_state = 0;
    } else if (size) {
      atomicOr(status, kStMalformed);
    }
  }
  __syncthreads();
  while (sh_state == 0) {
    const uint64_t w0 = sh_pos;
    uint64_t wbytes = size > w0 ? size - w0 : 0;
    if (wbytes > (uint64_t)kWalkWords * 4) wbytes = (uint64_t)kWalkWords * 4;
    const uint32_t nw = (uint32_t)(wbytes / 4);
    for (uint32_t i = threadIdx.x; i < nw; i += blockDim.x) win[i] = (uint32_t)c_ld32(body + w0 + 4ull * i);
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nw; q += blockDim.x) {
      const int32_t w = (int32_t)win[q];
      uint32_t v = kNoNext;
      if (w == -1) {
        v = q + 2;
      } else if (w >= 0 && q + 2 < nw) {
        const uint64_t sz = (uint64_t)win[q + 1] | ((uint64_t)win[q + 2] << 32);
        if ((sz & 3) == 0 && sz / 4 + q + 3 < kNoNext) v = (uint32_t)(q + 3 + sz / 4);
      }
      nxt[q] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const bool last = w0 + 4ull * nw >= size;   // this window reaches the end of the body
      uint32_t q = 0;
      uint32_t n = sh_n;
      int32_t tab = sh_table;
      int st = 0;                                 // 0 continue in the next window, 1 end, 2 malformed
      for (;;) {
        if (q >= nw) {                            // the chain leaves the window
          if (last) st = 2;                       // ... and the body: no -2 terminator
          break;
        }
        const int32_t w = (int32_t)win[q];
        if (w == -2) { st = 1; break; }
        if (w == -1) {                            // table separator: the next table id follows
          if (q + 1 >= nw) { if (last) st = 2; break; }
          tab = (int32_t)win[q + 1];
          q += 2;
          continue;
        }
        if (w < 0) { st = 2; break; }
        if (q + 2 >= nw) { if (last) st = 2; break; }   // header split by the window
        const uint64_t off = w0 + 4ull * q;
        const uint64_t sz = (uint64_t)win[q + 1] | ((uint64_t)win[q + 2] << 32);
        if ((sz & 3) || off + 12 + sz > size || nxt[q] == kNoNext || n >= max_ent) { st = 2; break; }
        PushEntry e;
        e.table_id = tab;
        e.row_id = w;
        e.offset = off + 12;
        e.size = sz;
        ent[n++] = e;
        q = nxt[q];
      }
      sh_n = n;
      sh_table = tab;
      sh_pos = w0 + 4ull * q;
      if (st == 2) atomicOr(status, kStMalformed);
      if (st) sh_state = 1;
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) *nent = sh_n;
}

// Validation and last-writer selection.  claim[slot] (zero between calls) receives
// 1 + the index of the body's last record for that row.
__global__ void __launch_bounds__(256) push_claim_kernel(const PushEntry *ent, const uint32_t *nent,
                                                         const ClientTable *ct, int nt, int insert, uint32_t *status) {
  const uint32_t n = *nent;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const PushEntry e = ent[i];
    int t = -1;
    for (int k = 0; k < nt; ++k)
      if (ct[k].table_id == e.table_id) t = k;
    if (t < 0) {   // "Cannot find table" (ssp_push_bg_worker.cpp:88)
      atomicOr(status, kStUnknownTable);
      continue;
    }
    const ClientTable &c = ct[t];
    int64_t d = (int64_t)e.row_id - c.row_offset;
    if (d < 0 || d % c.row_stride || d / c.row_stride >= c.max_rows) continue;   // not cached here
    const int64_t s = d / c.row_stride;
    if (!insert && !(c.flags[s] & 1)) continue;                                   // not in process storage
    uint64_t body = e.size;
    if (c.ver) {
      if (body < 8) { atomicOr(status, kStMalformed); continue; }
      body -= 8;
    }
    bool ok;
    if (c.kind == 0 && c.f16) ok = body % 2 == 0 && body <= (uint64_t)c.row_cap * 2;   // uint16[cap]
    else if (c.kind == 0) ok = body % c.vsize == 0 && body <= (uint64_t)c.row_cap * c.vsize;
    else if (c.kind == 1) ok = body % c.es == 0;
    else ok = body % (4 + c.vsize) == 0;
    if (!ok) { atomicOr(status, kStMalformed); continue; }
    const uint64_t cnt = c.kind == 0 ? 0 : (c.kind == 1 ? body / c.es : body / (4 + c.vsize));
    if (cnt > (uint64_t)c.max_entries) { atomicOr(status, kStCapacity); continue; }
    atomicMax(&c.claim[s], (int32_t)(i + 1));
  }
}

__global__ void __launch_bounds__(256) push_reset_kernel(const uint8_t *body, const PushEntry *ent,
                                                         const uint32_t *nent, const ClientTable *ct,
                                                         int nt, const uint32_t *status) {
  const int lane = threadIdx.x & 63;
  const uint32_t n = *nent;
  const bool go = (*status & kStFatal) == 0;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwv = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = w0; i < n; i += nwv) {
    const PushEntry e = ent[i];
    int t = -1;
    for (int k = 0; k < nt; ++k)
      if (ct[k].table_id == e.table_id) t = k;
    if (t < 0) continue;
    const ClientTable &c = ct[t];
    const int64_t d = (int64_t)e.row_id - c.row_offset;
    if (d < 0 || d % c.row_stride || d / c.row_stride >= c.max_rows) continue;
    const int64_t s = d / c.row_stride;
    if (c.claim[s] != (int32_t)(i + 1)) continue;    // an earlier record of the row, or skipped
    if (go) {
      const uint8_t *src = body + e.offset;
      const uint64_t bytes = c.ver ? e.size - 8 : e.size;
      if (c.kind == 0 && c.f16) {
        // VectorStoreFloat16::ResetData: Float16Compressor::decompress per value
        // (vector_store_float16.hpp:110-115)
        float *dst = reinterpret_cast<float *>(c.dense + s * (int64_t)c.row_cap * 4);
        for (uint64_t e = lane; e < bytes / 2; e += 64) {
          uint16_t h;
          __builtin_memcpy(&h, src + 2 * e, 2);
          dst[e] = __builtin_bit_cast(float, half_to_f32_bits(h));
        }
      } else if (c.kind == 0) {
        uint8_t *dst = c.dense + s * (int64_t)c.row_cap * c.vsize;
        for (uint64_t w = lane; w < bytes / 4; w += 64)
          reinterpret_cast<uint32_t *>(dst)[w] = (uint32_t)c_ld32(src + 4 * w);
      } else if (c.kind == 1) {   // Entry<V> bytes as stored
        uint8_t *dst = c.entries + s * c.max_entries * c.es;
        for (uint64_t w = lane; w < bytes / 4; w += 64)
          reinterpret_cast<uint32_t *>(dst)[w] = (uint32_t)c_ld32(src + 4 * w);
        if (lane == 0) c.nent[s] = (int32_t)(bytes / c.es);
      } else {                    // packed {int32 col; V val} -> Entry<V>
        const int64_t m = (int64_t)(bytes / (4 + c.vsize));
        uint8_t *dst = c.entries + s * c.max_entries * c.es;
        const int vo = c.vsize == 4 ? 4 : 8;
        for (int64_t k = lane; k < m; k += 64) {
          const uint8_t *p = src + k * (4 + c.vsize);
          uint8_t *q = dst + k * c.es;
          reinterpret_cast<int32_t *>(q)[0] = c_ld32(p);
          if (c.es == 16) reinterpret_cast<int32_t *>(q)[1] = 0;
          if (c.vsize == 4) {
            reinterpret_cast<uint32_t *>(q + vo)[0] = (uint32_t)c_ld32(p + 4);
          } else {
            const uint64_t v = c_ld64(p + 4);
            reinterpret_cast<uint32_t *>(q + vo)[0] = (uint32_t)v;
            reinterpret_cast<uint32_t *>(q + vo)[1] = (uint32_t)(v >> 32);
          }
        }
        if (lane == 0) c.nent[s] = (int32_t)m;
      }
      if (lane == 0) {
        if (c.ver) c.ver[s] = c_ld64(src + bytes);
        c.flags[s] |= 1;
      }
    }
    if (lane == 0) c.claim[s] = 0;   // the invariant between calls
  }
}

hipError_t launch_push_walk(const uint8_t *body, uint64_t size, PushEntry *ent, uint32_t *nent, uint32_t max_ent,
                            uint32_t *status, hipStream_t st) {
  hipLaunchKernelGGL(push_walk_kernel, dim3(1), dim3(kWalkThreads), 0, st, body, size, ent, nent, max_ent, status);
  return hipGetLastError();
}

hipError_t launch_push_apply(const uint8_t *body, const PushEntry *ent, const uint32_t *nent, uint32_t max_ent,
                             const ClientTable *ct, int nt, int insert, uint32_t *status, hipStream_t st) {
  unsigned blocks = (max_ent + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(push_claim_kernel, dim3(blocks), dim3(256), 0, st, ent, nent, ct, nt, insert, status);
  unsigned wblocks = (max_ent + 3) / 4;
  if (wblocks > 4096) wblocks = 4096;
  if (wblocks < 1) wblocks = 1;
  hipLaunchKernelGGL(push_reset_kernel, dim3(wblocks), dim3(256), 0, st, body, ent, nent, ct, nt, status);
  return hipGetLastError();
}

}  // namespace psx
