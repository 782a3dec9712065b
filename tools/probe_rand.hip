// probe_rand.hip — random small-request behaviour of this GPU's memory, the access pattern of
// the C3 ordered apply (one row per wave, a chain of dependent loads per row, every load a
// few 64-128 B lines at a random place in a table far larger than the Infinity Cache).
//
//   chase  each active lane follows its own chain of dependent 4-byte loads, one 128-B line
//          per hop, at uniformly random lines of a 4 GiB buffer; M lanes per wave active
//          (1: one request per wave-hop, as a row's setup chain; 64: 64 lines per wave-hop);
//          G waves in the grid.  Reports the mean hop latency (launch time / hops) and the
//          line request rate (G * M * hops / launch time).
//   indep  the same lines, but every lane issues D independent loads per step (no chain):
//          the rate the memory system sustains with requests always in flight.
//   rows   each wave reads a 1,200-B row (150 8-byte entries, one load per 64 lanes) at a
//          random slot of a table of 100K slots of a given stride, the next slot from the
//          row's data (one row in flight per wave, the ordered apply's image load): does the
//          slot stride (8 KiB = max_entries 1,024 x 8 B) concentrate rows on few channels?
//
// One JSON object per line.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_rand tools/probe_rand.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

__host__ __device__ inline uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}

// line i's first word: the next line of a chain (a hash of i, so chains are random walks)
__global__ void init_kernel(uint32_t *buf, uint32_t lines) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x)
    buf[i * 32] = mix(i + 12345) % lines;
}

__global__ void __launch_bounds__(256) chase_kernel(const uint32_t *buf, uint32_t lines, int m, int hops, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (lane >= m) return;
  uint32_t cur = mix(w * 64 + lane) % lines;
  for (int h = 0; h < hops; ++h) cur = __builtin_nontemporal_load(buf + (uint64_t)cur * 32);
  if (cur == 0xffffffffu) sink[0] = cur;
}

// rows: each wave reads one row of R bytes (8-byte entries, lane i: entries i, i + 64, ...)
// at slot r * stride, then the next row's slot from what it read (one row in flight per
// wave, as the ordered apply's image load), `hops` rows per wave.
__global__ void __launch_bounds__(256) rows_kernel(const uint8_t *buf, uint32_t nrows, int64_t stride, int rbytes,
                                                   int hops, uint32_t magic, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint32_t r = mix(w) % nrows;
  const int ne = rbytes / 8;
  for (int h = 0; h < hops; ++h) {
    const uint8_t *row = buf + (int64_t)r * stride;
    uint32_t x = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = j * 64 + lane;
      if (i < ne) x += (uint32_t)__builtin_nontemporal_load(reinterpret_cast<const uint64_t *>(row) + i);
    }
    // every lane's words feed the next slot: the whole row must arrive first
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    r = mix((uint64_t)x + h + w * 977) % nrows;
  }
  if (r == magic) sink[0] = r;   // a run-time value: the chain cannot be folded away
}

template <int D>
__global__ void __launch_bounds__(256) indep_kernel(const uint32_t *buf, uint32_t lines, int steps, uint32_t *sink) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint32_t s = mix(t);
  for (int k = 0; k < steps; ++k) {
    uint32_t v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      s = s * 1664525u + 1013904223u;
      v[d] = __builtin_nontemporal_load(buf + (uint64_t)(s % lines) * 32);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) acc += v[d];
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 5;
  const uint64_t bytes = 4ull << 30;
  const uint32_t lines = (uint32_t)(bytes / 128);
  uint32_t *buf, *sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 64));
  hipLaunchKernelGGL(init_kernel, dim3(4096), dim3(256), 0, 0, buf, lines);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](auto launch) {
    launch();   // warm
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return (double)ms / reps;
  };
  const int hops = 64;
  const int waves_list[] = {256, 1024, 2048, 4096, 7168, 8192, 16384};
  for (int m : {1, 4, 16, 64}) {
    for (int g : waves_list) {
      const double ms = time([&] { hipLaunchKernelGGL(chase_kernel, dim3(g / 4), dim3(256), 0, 0, buf, lines, m, hops, sink); });
      const double req = (double)g * m * hops;
      printf("{\"probe\": \"chase\", \"lanes_per_wave\": %d, \"waves\": %d, \"hops\": %d, \"ms\": %.4f, "
             "\"hop_us\": %.3f, \"Greq_per_s\": %.2f, \"GBps_128B\": %.1f}\n",
             m, g, hops, ms, ms * 1e3 / hops, req / (ms * 1e-3) / 1e9, req * 128 / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  for (int g : {2048, 8192, 16384}) {
    const int steps = 16;
    const double ms4 = time([&] { hipLaunchKernelGGL((indep_kernel<4>), dim3(g / 4), dim3(256), 0, 0, buf, lines, steps, sink); });
    const double ms16 = time([&] { hipLaunchKernelGGL((indep_kernel<16>), dim3(g / 4), dim3(256), 0, 0, buf, lines, steps, sink); });
    const double r4 = (double)g * 64 * 4 * steps, r16 = (double)g * 64 * 16 * steps;
    printf("{\"probe\": \"indep\", \"waves\": %d, \"in_flight_per_lane\": 4, \"ms\": %.4f, \"Greq_per_s\": %.2f, \"GBps_128B\": %.1f}\n",
           g, ms4, r4 / (ms4 * 1e-3) / 1e9, r4 * 128 / (ms4 * 1e-3) / 1e9);
    printf("{\"probe\": \"indep\", \"waves\": %d, \"in_flight_per_lane\": 16, \"ms\": %.4f, \"Greq_per_s\": %.2f, \"GBps_128B\": %.1f}\n",
           g, ms16, r16 / (ms16 * 1e-3) / 1e9, r16 * 128 / (ms16 * 1e-3) / 1e9);
    fflush(stdout);
  }
  // the ordered apply's image loads: 150-entry rows (1,200 B) at 8 KiB slots (max_entries
  // 1,024 x 8 B) and at padded strides
  for (int64_t stride : {8192LL, 8192LL + 128, 8192LL + 256, 8192LL + 640, 12288LL, 1280LL}) {
    const uint32_t nrows = (uint32_t)std::min<int64_t>(100000, (int64_t)(bytes / stride) - 1);
    for (int g : {7168, 14336}) {
      const int rh = 16;
      const double ms = time([&] { hipLaunchKernelGGL(rows_kernel, dim3(g / 4), dim3(256), 0, 0, (const uint8_t *)buf, nrows,
                                                      stride, 1200, rh, 0xffffffffu, sink); });
      const double lines = (double)g * rh * 10;
      printf("{\"probe\": \"rows\", \"stride\": %lld, \"rows\": %u, \"row_bytes\": 1200, \"waves\": %d, \"hops\": %d, "
             "\"ms\": %.4f, \"hop_us\": %.3f, \"Glines_per_s\": %.2f}\n",
             (long long)stride, nrows, g, rh, ms, ms * 1e3 / rh, lines / (ms * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
