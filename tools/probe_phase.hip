// probe_phase.hip — does separating the C2 apply's row writes from its record reads in
// time, chip-wide, recover the write cost?  tools/probe_apply.hip measured the pattern at
// ≈2.2-2.4 ms per launch with its 1.07 GB of row writes and 1.57 ms without them (reads
// alone): the writes cost ~0.65 ms where a write-only stream would take ~0.2 ms.
//
// phase<RPW>: a persistent grid (every block resident); each wave computes RPW rows into
// LDS (reads only), then a grid-wide barrier, then every wave writes its buffered rows,
// another barrier, next phase.  The barrier is a monotonic arrival counter (zeroed per
// launch by hipMemsetAsync on the stream): arrive with one agent-scope atomic add per block,
// wait with an agent-scope load loop.  base: the same kernel shape with stores issued as
// each row completes (no LDS buffering, no barriers).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_phase tools/probe_phase.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const u32x4_a4 __attribute__((address_space(1))) *gcu32x4_p;
typedef u32x4 __attribute__((address_space(1))) *gu32x4_p;
typedef const uint8_t __attribute__((address_space(1))) *gbyte_p;

__device__ __forceinline__ u32x4 ld_nt(const uint8_t *p) { return __builtin_nontemporal_load((gcu32x4_p)(gbyte_p)p); }
__device__ __forceinline__ u32x4 ld_plain(const uint8_t *p) { return *(const u32x4_a4 *)p; }
__device__ __forceinline__ u32x4 addf(u32x4 a, u32x4 b) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(__uint_as_float(a[i]) + __uint_as_float(b[i]));
  return r;
}

struct Args {
  uint8_t *table;
  const uint8_t *stream;
  const int32_t *pos;
  int64_t R, stride, msg_bytes;
  unsigned int *bar;
};

constexpr int B = 8, D = 4;

// Bounded and abortable: bar[0] counts arrivals, bar[16] is the abort flag.  A block that
// waits more than ~20-40 ms (the grid is not all resident) sets the flag; every block checks
// it after each barrier and leaves, so a bad grid ends the launch in milliseconds.
__device__ __forceinline__ bool grid_barrier(unsigned int *bar, unsigned int target) {
  __shared__ int s_ok;
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = 1;
    __hip_atomic_fetch_add(bar, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    for (uint32_t spins = 0;; ++spins) {
      if (__hip_atomic_load(bar, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= target) break;
      if (__hip_atomic_load(bar + 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) { ok = 0; break; }
      if (spins > (1u << 14)) {
        __hip_atomic_store(bar + 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(10);
    }
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// Rows are dealt to waves in groups of D: group g = phase * (nw * RPW/D) + k * nw + wave.
template <int RPW, bool NTST>
__global__ void __launch_bounds__(256) phase_kernel(Args a) {
  extern __shared__ u32x4 buf[];   // [4 waves][RPW rows][64 lanes]
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wib;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t rows_per_phase = nw * RPW;
  const int64_t nphase = (a.R + rows_per_phase - 1) / rows_per_phase;
  u32x4 *mine = buf + (int64_t)wib * RPW * 64;
  // residency check first: every block must arrive (else all leave at once)
  if (!grid_barrier(a.bar, gridDim.x)) return;
  for (int64_t ph = 0; ph < nphase; ++ph) {
    const int64_t base = ph * rows_per_phase;
#pragma unroll 1
    for (int k = 0; k < RPW / D; ++k) {
      const int64_t r0 = base + ((int64_t)k * nw + wave) * D;
      u32x4 t[D], u[D][B];
#pragma unroll
      for (int q = 0; q < D; ++q) {
        const int64_t r = r0 + q < a.R ? r0 + q : a.R - 1;
        t[q] = ld_plain(a.table + r * 1024 + lane * 16);
#pragma unroll
        for (int b = 0; b < B; ++b)
          u[q][b] = ld_nt(a.stream + b * a.msg_bytes + (int64_t)a.pos[b * a.R + r] * a.stride + 24 + lane * 16);
      }
      __builtin_amdgcn_sched_barrier(0);   // every load of the D rows in flight before any add
#pragma unroll
      for (int q = 0; q < D; ++q) {
        u32x4 acc = t[q];
#pragma unroll
        for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
        mine[(k * D + q) * 64 + lane] = acc;
      }
    }
    if (!grid_barrier(a.bar, (unsigned)((2 * ph + 2) * gridDim.x))) return;
#pragma unroll 1
    for (int k = 0; k < RPW / D; ++k) {
      const int64_t r0 = base + ((int64_t)k * nw + wave) * D;
#pragma unroll
      for (int q = 0; q < D; ++q)
        if (r0 + q < a.R) {
          uint8_t *p = a.table + (r0 + q) * 1024 + lane * 16;
          const u32x4 v = mine[(k * D + q) * 64 + lane];
          if (NTST) __builtin_nontemporal_store(v, (gu32x4_p)p);
          else *(u32x4 *)p = v;
        }
    }
    if (!grid_barrier(a.bar, (unsigned)((2 * ph + 3) * gridDim.x))) return;
  }
}

// Same dealing of rows, stores as each row completes.
template <int RPW>
__global__ void __launch_bounds__(256) base_kernel(Args a) {
  const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
  const int64_t wave = (int64_t)blockIdx.x * 4 + wib;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t rows_per_phase = nw * RPW;
  const int64_t nphase = (a.R + rows_per_phase - 1) / rows_per_phase;
  for (int64_t ph = 0; ph < nphase; ++ph) {
    const int64_t base = ph * rows_per_phase;
#pragma unroll 1
    for (int k = 0; k < RPW / D; ++k) {
      const int64_t r0 = base + ((int64_t)k * nw + wave) * D;
      u32x4 t[D], u[D][B];
#pragma unroll
      for (int q = 0; q < D; ++q) {
        const int64_t r = r0 + q < a.R ? r0 + q : a.R - 1;
        t[q] = ld_plain(a.table + r * 1024 + lane * 16);
#pragma unroll
        for (int b = 0; b < B; ++b)
          u[q][b] = ld_nt(a.stream + b * a.msg_bytes + (int64_t)a.pos[b * a.R + r] * a.stride + 24 + lane * 16);
      }
#pragma unroll
      for (int q = 0; q < D; ++q) {
        u32x4 acc = t[q];
#pragma unroll
        for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
        if (r0 + q < a.R) *(u32x4 *)(a.table + (r0 + q) * 1024 + lane * 16) = acc;
      }
    }
  }
}

template <typename K>
static unsigned resident(K k, size_t lds) {
  int per = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, lds));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  return (unsigned)(per * cus);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int64_t R = 1 << 20;
  Args a{};
  a.R = R;
  a.stride = 1028;
  a.msg_bytes = 20 + R * 1028 + 64;
  uint8_t *stream;
  int32_t *pos;
  CK(hipMalloc(&a.table, R * 1024));
  CK(hipMalloc(&stream, B * a.msg_bytes));
  CK(hipMalloc(&pos, B * R * sizeof(int32_t)));
  CK(hipMalloc(&a.bar, 256));
  CK(hipMemset(a.bar, 0, 256));
  CK(hipMemset(a.table, 0, R * 1024));
  CK(hipMemset(stream, 0, B * a.msg_bytes));
  a.stream = stream;
  a.pos = pos;
  std::mt19937 rng(1234);
  std::vector<int32_t> h(B * R);
  for (int64_t m = 0; m < B; ++m) {
    std::vector<int32_t> perm(R);
    for (int64_t i = 0; i < R; ++i) perm[i] = (int32_t)i;
    std::shuffle(perm.begin(), perm.end(), rng);
    for (int64_t i = 0; i < R; ++i) h[m * R + perm[i]] = (int32_t)i;
  }
  CK(hipMemcpy(pos, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  const double alg = (double)B * (20 + R * 1028) + 2.0 * R * 1024 + (double)B * R * 4;
  hipStream_t st;
  CK(hipStreamCreate(&st));

  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  auto time_it = [&](const char *name, auto kern, int rpw, size_t lds, bool barrier, int per_cu = 0) {
    const unsigned api = resident(kern, lds);
    const unsigned g = per_cu ? std::min<unsigned>(api, (unsigned)(per_cu * cus)) : api;
    auto launch = [&] {
      if (barrier) CK(hipMemsetAsync(a.bar, 0, 256, st));
      kern<<<g, 256, lds, st>>>(a);
    };
    launch();
    CK(hipStreamSynchronize(st));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    unsigned int gave_up = 0;
    CK(hipMemcpy(&gave_up, a.bar + 16, 4, hipMemcpyDeviceToHost));
    if (gave_up) ms = -1.f;   // the launch left early: no measurement
    printf("{\"probe\": \"%s\", \"rows_per_wave_phase\": %d, \"grid\": %u, \"lds\": %zu, \"ms\": %.4f, \"GBps\": %.1f, "
           "\"barrier_gave_up\": %u}\n", name, rpw, g, lds, ms, alg / ms / 1e6, gave_up);
    fflush(stdout);
  };
  time_it("base", base_kernel<16>, 16, 0, false);
  // one block per CU first (resident by construction), then two
  time_it("phase", phase_kernel<32, false>, 32, 4 * 32 * 1024, true, 1);
  time_it("phase_nt", phase_kernel<32, true>, 32, 4 * 32 * 1024, true, 1);
  time_it("phase", phase_kernel<16, false>, 16, 4 * 16 * 1024, true, 1);
  time_it("phase", phase_kernel<16, false>, 16, 4 * 16 * 1024, true, 2);
  time_it("phase_nt", phase_kernel<16, true>, 16, 4 * 16 * 1024, true, 2);
  time_it("base", base_kernel<16>, 16, 0, false);
  return 0;
}
