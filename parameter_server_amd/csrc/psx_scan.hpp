// psx_scan.hpp — three-phase exclusive prefix sum over n counters (tiles of 1024):
// off[i] = sum(cnt[0, i)), off[n] = total.  Used for the ordered path's per-slot record
// lists (int32) and the serve-back record offsets (int64).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace psx {

// Three-phase exclusive scan of cnt[0, n) into off[0, n]; tiles of 1024.
template <typename T>
__global__ void __launch_bounds__(256) scan_tiles_kernel(const T *cnt, int64_t n, T *off, T *tsum) {
  __shared__ T wsum[4];
  const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  T v[4];
  T s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    v[j] = base + j < n ? cnt[base + j] : 0;
    s += v[j];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T incl = s;
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  T wpre = 0;
  for (int i = 0; i < w; ++i) wpre += wsum[i];
  T run = wpre + incl - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (base + j < n) off[base + j] = run;
    run += v[j];
  }
  if (threadIdx.x == 255) tsum[blockIdx.x] = wpre + incl;
}

template <typename T>
__global__ void __launch_bounds__(1024) scan_sums_kernel(T *tsum, int64_t ntiles, T *off, int64_t n) {
  __shared__ T carry;
  __shared__ T wsum[16];
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int64_t c = 0; c < ntiles; c += 1024) {
    const int64_t i = c + threadIdx.x;
    const T x = i < ntiles ? tsum[i] : 0;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T incl = x;
    for (int o = 1; o < 64; o <<= 1) {
      T y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    T wpre = 0;
    for (int k = 0; k < w; ++k) wpre += wsum[k];
    const T excl = carry + wpre + incl - x;
    __syncthreads();
    if (i < ntiles) tsum[i] = excl;
    if (threadIdx.x == 1023) carry = excl + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) off[n] = carry;
}

template <typename T>
__global__ void __launch_bounds__(256) scan_add_kernel(T *off, int64_t n, const T *tsum) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) off[i] += tsum[i >> 10];
}

template <typename T>
inline void launch_exclusive_scan(const T *cnt, int64_t n, T *off, T *tsum, hipStream_t st) {
  const int64_t ntiles = (n + 1023) / 1024;
  hipLaunchKernelGGL(scan_tiles_kernel<T>, dim3((unsigned)ntiles), dim3(256), 0, st, cnt, n, off, tsum);
  hipLaunchKernelGGL(scan_sums_kernel<T>, dim3(1), dim3(1024), 0, st, tsum, ntiles, off, n);
  hipLaunchKernelGGL(scan_add_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, off, n, tsum);
}

}  // namespace psx
