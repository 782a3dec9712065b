// psx_pack.hip — client-side pack on the device: per-table oplog rows -> one Appendix-A
// message (the payload of a ClientSendOpLogMsg).
//
// Reference: CreateOpLogMsgs + OpLogSerializer (abstract_bg_worker.cpp:590-649,
// oplog_serializer.hpp:12-37) lay out
//   int32 num_tables; per table (ascending table_id): int32 table_id; size_t update_size;
//   int32 num_rows; records...
// with RowOpLogSerializer (row_oplog_serializer.hpp:139-166) writing each record as
// int32 row_id + DenseRowOpLog::SerializeDense (V[capacity], dense_row_oplog.hpp:133-136)
// or SerializeSparse (int32 n; int32 cols[n]; V vals[n], the non-zero columns in
// ascending order, dense_row_oplog.hpp:112-131; zero = `== V(0)`,
// numeric_store_row.hpp:312-314).
//
//   pack_count   sparse tables: one wave per row counts its non-zeros (ballots)
//   scan         record byte offsets (int64, psx_scan.hpp)
//   pack_dense   one wave per row: row id + 16-byte copies of the payload
//   pack_sparse  one wave per row: ballot compaction of the non-zero columns
//   pack_header  num_tables and the table headers
// Every kernel also writes the byte offset of each record's row id into the optional
// record-offset index (the producer-side index SURVEY §8(f)-2 asks for).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "psx_device.hpp"
#include "psx_scan.hpp"

namespace psx {

typedef uint32_t p32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t p32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

template <typename V>
__device__ __forceinline__ bool is_zero_at(const uint8_t *p) {
  return *reinterpret_cast<const V *>(p) == V(0);
}

template <typename V>
__global__ void __launch_bounds__(256) pack_count_kernel(PackTab t) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = w0; r < t.nrows; r += nw) {
    const uint8_t *row = t.oplogs + r * t.cap * (int64_t)sizeof(V);
    int64_t nnz = 0;
    for (int64_t c0 = 0; c0 < t.cap; c0 += 64) {
      const int64_t c = c0 + lane;
      const bool nz = c < t.cap && !is_zero_at<V>(row + c * sizeof(V));
      nnz += __builtin_popcountll(__ballot(nz));
    }
    if (lane == 0) t.sizes[r] = 8 + nnz * (4 + (int64_t)sizeof(V));
  }
}

__global__ void __launch_bounds__(256) pack_dense_kernel(PackTab t, uint8_t *out, uint64_t *recoff) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int64_t pay = t.cap * t.vsize;           // payload bytes, a multiple of 4
  const int64_t stride = 4 + pay;
  const int64_t n16 = (t.src16 ? pay / 16 : 0);
  for (int64_t r = w0; r < t.nrows; r += nw) {
    uint8_t *rec = out + t.rec0 + r * stride;
    const uint8_t *src = t.oplogs + r * pay;
    if (lane == 0) {
      *reinterpret_cast<int32_t *>(rec) = t.row_ids[r];
      if (recoff) recoff[t.rec_base + r] = (uint64_t)(t.rec0 + r * stride);
    }
    uint8_t *dst = rec + 4;
    for (int64_t i = lane; i < n16; i += 64) {
      const p32x4 v = __builtin_nontemporal_load(reinterpret_cast<const p32x4 *>(src) + i);
      *reinterpret_cast<p32x4_a4 *>(dst + i * 16) = v;
    }
    for (int64_t wd = n16 * 4 + lane; wd < pay / 4; wd += 64)
      reinterpret_cast<uint32_t *>(dst)[wd] = reinterpret_cast<const uint32_t *>(src)[wd];
  }
}

template <typename V>
__global__ void __launch_bounds__(256) pack_sparse_kernel(PackTab t, uint8_t *out, uint64_t *recoff) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t r = w0; r < t.nrows; r += nw) {
    const int64_t off = t.rec0 + t.offs[r];
    uint8_t *rec = out + off;
    const int32_t n = (int32_t)((t.sizes[r] - 8) / (4 + (int64_t)sizeof(V)));
    if (lane == 0) {
      reinterpret_cast<int32_t *>(rec)[0] = t.row_ids[r];
      reinterpret_cast<int32_t *>(rec)[1] = n;
      if (recoff) recoff[t.rec_base + r] = (uint64_t)off;
    }
    int32_t *cols = reinterpret_cast<int32_t *>(rec + 8);
    uint8_t *vals = rec + 8 + (int64_t)n * 4;
    const uint8_t *row = t.oplogs + r * t.cap * (int64_t)sizeof(V);
    int32_t k = 0;
    for (int64_t c0 = 0; c0 < t.cap; c0 += 64) {
      const int64_t c = c0 + lane;
      V v = V(0);
      if (c < t.cap) v = *reinterpret_cast<const V *>(row + c * sizeof(V));
      const bool nz = c < t.cap && !(v == V(0));
      const uint64_t bal = __ballot(nz);
      if (nz) {
        const int32_t p = k + __builtin_popcountll(bal & below);
        cols[p] = (int32_t)c;
        if constexpr (sizeof(V) == 4) {
          reinterpret_cast<uint32_t *>(vals)[p] = __builtin_bit_cast(uint32_t, v);
        } else {   // 8-byte values sit at 4-byte alignment in the stream
          const uint64_t b = __builtin_bit_cast(uint64_t, v);
          reinterpret_cast<uint32_t *>(vals)[2 * p] = (uint32_t)b;
          reinterpret_cast<uint32_t *>(vals)[2 * p + 1] = (uint32_t)(b >> 32);
        }
      }
      k += __builtin_popcountll(bal);
    }
  }
}

__global__ void pack_header_kernel(uint8_t *out, PackHdr h) {
  for (int i = threadIdx.x; i < h.n; i += blockDim.x) {
    uint32_t *p = reinterpret_cast<uint32_t *>(out + h.pos[i]);
    for (int k = 0; k < h.len[i]; ++k) p[k] = h.w[i][k];
  }
}

hipError_t launch_pack_count(int dtype, PackTab t, hipStream_t st) {
  if (t.nrows <= 0) return hipSuccess;
  int64_t blocks = (t.nrows + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (dtype == 0) hipLaunchKernelGGL(pack_count_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, st, t);
  else if (dtype == 1) hipLaunchKernelGGL(pack_count_kernel<double>, dim3((unsigned)blocks), dim3(256), 0, st, t);
  else if (dtype == 2) hipLaunchKernelGGL(pack_count_kernel<int32_t>, dim3((unsigned)blocks), dim3(256), 0, st, t);
  else hipLaunchKernelGGL(pack_count_kernel<int64_t>, dim3((unsigned)blocks), dim3(256), 0, st, t);
  launch_exclusive_scan<int64_t>(t.sizes, t.nrows, t.offs, t.offs + t.nrows + 1, st);
  return hipGetLastError();
}

hipError_t launch_pack_emit(int dtype, PackTab t, uint8_t *out, uint64_t *recoff, hipStream_t st) {
  if (t.nrows <= 0) return hipSuccess;
  int64_t blocks = (t.nrows + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  const dim3 g((unsigned)blocks), b(256);
  if (!t.sparse) {
    hipLaunchKernelGGL(pack_dense_kernel, g, b, 0, st, t, out, recoff);
  } else if (dtype == 0) {
    hipLaunchKernelGGL(pack_sparse_kernel<float>, g, b, 0, st, t, out, recoff);
  } else if (dtype == 1) {
    hipLaunchKernelGGL(pack_sparse_kernel<double>, g, b, 0, st, t, out, recoff);
  } else if (dtype == 2) {
    hipLaunchKernelGGL(pack_sparse_kernel<int32_t>, g, b, 0, st, t, out, recoff);
  } else {
    hipLaunchKernelGGL(pack_sparse_kernel<int64_t>, g, b, 0, st, t, out, recoff);
  }
  return hipGetLastError();
}

hipError_t launch_pack_header(uint8_t *out, const PackHdr &h, hipStream_t st) {
  hipLaunchKernelGGL(pack_header_kernel, dim3(1), dim3(64), 0, st, out, h);
  return hipGetLastError();
}

}  // namespace psx
