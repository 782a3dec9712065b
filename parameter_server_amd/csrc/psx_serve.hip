// psx_serve.hip — serve-back on the device: every dirty row of a table serialized as the
// reference's push-message records.
//
// Server::CreateSendServerPushRowMsgs (server.cpp:189-309) writes, per table,
// int32 table_id, then ServerTable::AppendTableToBuffs (server_table.cpp:197-261): every
// dirty (and subscribed) row as a RecordBuff record {int32 row_id; size_t size;
// ServerRow::Serialize bytes} (record_buff.hpp:41-53), resetting dirty_; tables are
// separated by int32 -1 and the body ends with -2 (context.hpp:123-129).
//
//   serve_sizes  sizes[s] = 12 + body bytes for dirty rows, 0 otherwise
//   scan         offs = exclusive prefix (int64, psx_scan.hpp)
//   serve_emit   one wave per dirty row writes its record at base + offs[s]
// Row bodies: DenseRow V[capacity] (vector_store.hpp:75-80); SortedVectorMapRow
// Entry<V>[n] in store order (sorted_vector_map_store.hpp:148-152); SparseRow packed
// {int32 col; V val}[n] (map_store.hpp:89-100).  Rows come out in ascending row id.
// Partial push (psx_serialize_partial, server.cpp:311-420): serve_sizes also writes a
// sort key per slot (importance, or 0, for dirty rows; -1 otherwise); a stable
// descending radix sort of (key, slot) puts the dirty rows in send order — importance
// descending, ties by ascending slot = ascending row id (server_table.cpp:272-287); the
// first upper_bound entries are the send list, emitted by serve_emit_list.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdint>
#include "psx_device.hpp"
#include "psx_scan.hpp"

namespace psx {


__device__ __forceinline__ int64_t row_bytes(const ServeArgs &a, int64_t s) {
  if (a.kind == 0) return a.row_cap * (a.f16 ? 2 : a.vsize);   // VectorStoreFloat16: uint16[cap]
  const int64_t es = a.vsize == 4 ? 8 : 16;
  const int64_t n = a.nent[s];
  return a.kind == 1 ? n * es : n * (4 + a.vsize);
}
// VersionServerRow::Serialize appends uint64 version_ (version_server_row.hpp:55-64).
__device__ __forceinline__ int64_t body_bytes(const ServeArgs &a, int64_t s) {
  return row_bytes(a, s) + (a.ver ? 8 : 0);
}

__global__ void __launch_bounds__(256) serve_sizes_kernel(ServeArgs a) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = s < a.max_rows;
  const bool dirty = in && (a.flags[s] & 3) == 3 && (!a.subs || (a.subs[s] & a.cmask) != 0);
  if (in) a.sizes[s] = dirty ? 12 + body_bytes(a, s) : 0;
  if (a.keys) {
    if (in) {
      a.keys[s] = dirty ? (a.imp ? a.imp[s] : 0.0) : -1.0;
      a.vals[s] = (int32_t)s;
    }
    const uint64_t bal = __ballot(dirty);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(a.ndirty, (uint32_t)__builtin_popcountll(bal));
  }
}

__global__ void __launch_bounds__(256) serve_list_sizes_kernel(ServeArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.nsel) a.lsizes[i] = a.sizes[a.sel[i]];
}

// A 32-bit word at a 2-byte-aligned address (records after binary16 rows of odd width).
__device__ __forceinline__ void st32_a2(uint8_t *p, uint32_t v) {
  reinterpret_cast<uint16_t *>(p)[0] = (uint16_t)v;
  reinterpret_cast<uint16_t *>(p)[1] = (uint16_t)(v >> 16);
}

// One record {int32 row_id; size_t size; row bytes} for slot s at rec (one wave); with
// flags_rw, ResetDirty and ResetImportance_ (server_table.cpp:234-235, :398-399).
__device__ void emit_row(const ServeArgs &a, int64_t s, uint8_t *rec, int lane) {
  const int64_t total = a.sizes[s] - 12;
  const int64_t body = total - (a.ver ? 8 : 0);   // row bytes before the version trailer
  if (a.f16) {
    // DenseRowFloat16: VectorStoreFloat16::Serialize, Float16Compressor::compress per value
    // (vector_store_float16.hpp:91-99); the record may start on a 2-byte boundary
    if (lane == 0) {
      const int32_t rid = (int32_t)(a.row_offset + s * a.row_stride);
      st32_a2(rec, (uint32_t)rid);
      st32_a2(rec + 4, (uint32_t)(uint64_t)total);
      st32_a2(rec + 8, (uint32_t)((uint64_t)total >> 32));
      if (a.ver) {
        const uint64_t v = a.ver[s];
        st32_a2(rec + 12 + body, (uint32_t)v);
        st32_a2(rec + 16 + body, (uint32_t)(v >> 32));
      }
    }
    const float *src = reinterpret_cast<const float *>(a.dense + s * a.row_cap * 4);
    uint16_t *dst = reinterpret_cast<uint16_t *>(rec + 12);
    for (int64_t e = lane; e < a.row_cap; e += 64) dst[e] = (uint16_t)f32_to_half_fc(src[e]);
    if (lane == 0 && a.flags_rw) {
      a.flags_rw[s] &= (uint8_t)~2u;
      if (a.imp_rw) a.imp_rw[s] = 0.0;
    }
    return;
  }
  // A record behind a binary16 row of odd width (another table earlier in the same push)
  // starts on a 2-byte boundary: then every word goes out as two 16-bit stores.
  // The test is per record, so wave-uniform.
  const bool a2 = ((uintptr_t)rec & 3) != 0;
  auto put = [&](uint8_t *p, uint32_t v) {
    if (a2) st32_a2(p, v);
    else *reinterpret_cast<uint32_t *>(p) = v;
  };
  if (lane == 0) {
    const int32_t rid = (int32_t)(a.row_offset + s * a.row_stride);
    put(rec, (uint32_t)rid);
    put(rec + 4, (uint32_t)(uint64_t)total);          // size_t
    put(rec + 8, (uint32_t)((uint64_t)total >> 32));
    if (a.ver) {
      const uint64_t v = a.ver[s];
      put(rec + 12 + body, (uint32_t)v);
      put(rec + 16 + body, (uint32_t)(v >> 32));
    }
  }
  uint8_t *dst = rec + 12;
  if (a.kind == 0) {
    const uint32_t *src = reinterpret_cast<const uint32_t *>(a.dense + s * a.row_cap * a.vsize);
    for (int64_t w = lane; w < body / 4; w += 64) put(dst + w * 4, src[w]);
  } else if (a.kind == 1) {
    const int64_t es = a.vsize == 4 ? 8 : 16;
    const uint32_t *src = reinterpret_cast<const uint32_t *>(a.entries + s * a.max_entries * es);
    for (int64_t w = lane; w < body / 4; w += 64) put(dst + w * 4, src[w]);
  } else {
    const int64_t es = a.vsize == 4 ? 8 : 16, vo = a.vsize == 4 ? 4 : 8;
    const uint8_t *src = a.entries + s * a.max_entries * es;
    const int32_t n = a.nent[s];
    const int wpe = 1 + a.vsize / 4;                  // words per packed {int32, V}
    for (int32_t e = lane; e < n; e += 64) {
      uint8_t *d = dst + (int64_t)e * wpe * 4;
      put(d, *reinterpret_cast<const uint32_t *>(src + e * es));
      put(d + 4, *reinterpret_cast<const uint32_t *>(src + e * es + vo));
      if (wpe == 3) put(d + 8, *reinterpret_cast<const uint32_t *>(src + e * es + vo + 4));
    }
  }
  if (lane == 0 && a.flags_rw) {
    a.flags_rw[s] &= (uint8_t)~2u;
    if (a.imp_rw) a.imp_rw[s] = 0.0;
  }
}

__global__ void __launch_bounds__(256) serve_emit_kernel(ServeArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t ntiles = (a.max_rows + 63) / 64;
  for (int64_t tile = wave_g; tile < ntiles; tile += nwaves) {
    const int64_t ms = tile * 64 + lane;
    const bool dirty = ms < a.max_rows && a.sizes[ms] != 0;
    uint64_t live = __ballot(dirty);
    while (live) {
      const int k = __builtin_ctzll(live);
      live &= live - 1;
      const int64_t s = tile * 64 + k;
      emit_row(a, s, a.out + a.offs[s], lane);
    }
  }
}


// Emit the send list: one wave per entry, records in list order.
__global__ void __launch_bounds__(256) serve_emit_list_kernel(ServeArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wave_g; i < a.nsel; i += nwaves) emit_row(a, a.sel[i], a.out + a.loffs[i], lane);
}

// After a per-client push: every dirty row some client subscribes to was sent — ResetDirty
// + ResetImportance_ (server_table.cpp:233-235); unsubscribed dirty rows stay dirty (:222-225).
__global__ void __launch_bounds__(256) serve_clear_kernel(uint8_t *flags, double *imp, const uint64_t *subs,
                                                         int64_t n) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n && (flags[s] & 3) == 3 && subs[s] != 0) {
    flags[s] &= (uint8_t)~2u;
    if (imp) imp[s] = 0.0;
  }
}

// FindCreateRow + CallBackSubs::Subscribe for a list of slots (server.cpp:46-60,
// callback_subs.hpp:21-28): the row exists from now on; the client's bit is set.
__global__ void __launch_bounds__(256) subscribe_kernel(uint8_t *flags, uint64_t *subs, const int64_t *slots,
                                                       int32_t n, uint64_t bit) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const int64_t s = slots[i];
    flags[s] |= 1;
    subs[s] |= bit;
  }
}

hipError_t launch_serve_clear(uint8_t *flags, double *imp, const uint64_t *subs, int64_t n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(serve_clear_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, flags, imp, subs, n);
  return hipGetLastError();
}

hipError_t launch_subscribe(uint8_t *flags, uint64_t *subs, const int64_t *slots, int32_t n, uint64_t bit,
                            hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(subscribe_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, flags, subs, slots, n,
                     bit);
  return hipGetLastError();
}

__global__ void put_words_kernel(uint8_t *out, Words w) {
  for (int i = threadIdx.x; i < w.n; i += blockDim.x) {
    if (w.pos[i] & 3) st32_a2(out + w.pos[i], (uint32_t)w.val[i]);   // after binary16 rows of odd width
    else *reinterpret_cast<int32_t *>(out + w.pos[i]) = w.val[i];
  }
}

hipError_t launch_serve_sizes(const ServeArgs &a, hipStream_t st) {
  const int64_t n = a.max_rows;
  hipLaunchKernelGGL(serve_sizes_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  launch_exclusive_scan<int64_t>(a.sizes, n, a.offs, a.offs + n + 1, st);
  return hipGetLastError();
}

hipError_t launch_serve_emit(const ServeArgs &a, hipStream_t st) {
  const int64_t tiles = (a.max_rows + 63) / 64;
  int64_t blocks = (tiles + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(serve_emit_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_serve_list_sizes(const ServeArgs &a, hipStream_t st) {
  if (a.nsel <= 0) return hipSuccess;
  hipLaunchKernelGGL(serve_list_sizes_kernel, dim3((unsigned)((a.nsel + 255) / 256)), dim3(256), 0, st, a);
  launch_exclusive_scan<int64_t>(a.lsizes, a.nsel, a.loffs, a.loffs + a.nsel + 1, st);
  return hipGetLastError();
}

hipError_t launch_serve_emit_list(const ServeArgs &a, hipStream_t st) {
  if (a.nsel <= 0) return hipSuccess;
  int64_t blocks = (a.nsel + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(serve_emit_list_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

// Stable descending sort of (key, slot) pairs.  temp == nullptr: *temp_bytes <- size.
hipError_t launch_sort_desc(void *temp, size_t *temp_bytes, const double *keys_in, double *keys_out,
                            const int32_t *vals_in, int32_t *vals_out, int64_t n, hipStream_t st) {
  return hipcub::DeviceRadixSort::SortPairsDescending(temp, *temp_bytes, keys_in, keys_out, vals_in, vals_out,
                                                      (int)n, 0, 64, st);
}

hipError_t launch_put_words(uint8_t *out, const Words &w, hipStream_t st) {
  if (w.n <= 0) return hipSuccess;
  hipLaunchKernelGGL(put_words_kernel, dim3(1), dim3(128), 0, st, out, w);
  return hipGetLastError();
}

}  // namespace psx
