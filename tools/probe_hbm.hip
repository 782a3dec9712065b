// probe_hbm.hip — what HBM gives each access pattern of the C2 apply, measured with the
// same machinery (hip events over repeated launches, grids sized to residency).
//
//   copy      float4 copy src -> dst, U loads in flight per lane, plain or non-temporal:
//             the box's sequential rate (the microarch guide: 6.29 TB/s float4 copy)
//   read      sequential read-only sweep of a buffer, U loads in flight per lane
//   gather    read-only: chunks of C bytes at uniformly random chunk slots of a buffer far
//             larger than the Infinity Cache, D chunks in flight per wave; C = 256 .. 4096,
//             and 1,024-B chunks at a 1,028-B stride (the wire format's 4-byte row id puts
//             every record payload 4 bytes off the line grid: 9 lines per record)
//   apply     the C2 access pattern itself: per row B = 8 records gathered + the table row
//             read and written, rows in slot order, D rows per wave, 1,028- or 1,024-B stride
//
// Each line is one JSON object: bytes moved (algorithmic), ms per launch, GB/s.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_hbm tools/probe_hbm.hip
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

template <bool NT>
__device__ __forceinline__ u32x4 ld(const uint8_t *p) {
  if (NT) return __builtin_nontemporal_load((gcu32x4_p)(gbyte_p)p);
  return *(const u32x4_a4 *)p;
}
template <bool NT>
__device__ __forceinline__ void st(uint8_t *p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, (gu32x4_p)p);
  else *(u32x4 *)p = v;
}

// Each block sweeps contiguous tiles of U * 4 KiB (256 threads x 16 B x U); tiles are
// handed out grid-stride.
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const uint8_t *src, uint8_t *dst, int64_t tiles) {
  const int64_t tb = (int64_t)U * 4096;
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + t * tb + (int64_t)u * 4096 + threadIdx.x * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(dst + t * tb + (int64_t)u * 4096 + threadIdx.x * 16, v[u]);
  }
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) read_kernel(const uint8_t *src, int64_t tiles, uint32_t *sink) {
  const int64_t tb = (int64_t)U * 4096;
  u32x4 acc = {0, 0, 0, 0};
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + t * tb + (int64_t)u * 4096 + threadIdx.x * 16);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1;
}

// Random chunks: a wave takes D "groups" at a time; a group is one wave-instruction of
// 1 KiB (lane l loads 16 B).  For C < 1 KiB a group holds 1024 / C chunks (lane l in chunk
// l / (C / 16)); for C >= 1 KiB a chunk is C / 1024 consecutive groups.  Chunk k lives at
// base + slot[k] * stride (+ 4 for the misaligned form).
template <int D, bool NT>
__global__ void __launch_bounds__(256) gather_kernel(const uint8_t *buf, const int32_t *slot, int64_t groups,
                                                     int32_t C, int64_t stride, int32_t off, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int per_group = C >= 1024 ? 1 : 1024 / C;     // chunks per group
  const int gpc = C >= 1024 ? C / 1024 : 1;           // groups per chunk
  u32x4 acc = {0, 0, 0, 0};
  for (int64_t g0 = wave * D; g0 < groups; g0 += nw * D) {
    u32x4 v[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int64_t g = g0 + d < groups ? g0 + d : groups - 1;
      int64_t chunk, inner;
      if (per_group > 1) {
        chunk = g * per_group + lane / (64 / per_group);
        inner = (int64_t)(lane % (64 / per_group)) * 16;
      } else {
        chunk = g / gpc;
        inner = (g % gpc) * 1024 + lane * 16;
      }
      v[d] = ld<NT>(buf + (int64_t)slot[chunk] * stride + off + inner);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) acc ^= v[d];
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1;
}

__device__ __forceinline__ u32x4 addf(u32x4 a, u32x4 b) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(__uint_as_float(a[i]) + __uint_as_float(b[i]));
  return r;
}

// The C2 pattern: D rows per wave at a time, rows in slot order; per row the table row
// and its B records (positions from a [B][R] map), adds in message order, one store.
template <int B, int D>
__global__ void __launch_bounds__(256) apply_kernel(uint8_t *table, const uint8_t *stream, const int32_t *pos,
                                                    int64_t R, int64_t stride, int64_t msg_bytes) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = wave * D; r0 < R; r0 += nw * D) {
    u32x4 t[D], u[D][B];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      const int64_t r = r0 + q < R ? r0 + q : R - 1;
      t[q] = ld<true>(table + r * 1024 + lane * 16);
#pragma unroll
      for (int b = 0; b < B; ++b)
        u[q][b] = ld<true>(stream + b * msg_bytes + (int64_t)pos[b * R + r] * stride + 24 + lane * 16);
    }
#pragma unroll
    for (int q = 0; q < D; ++q) {
      u32x4 acc = t[q];
#pragma unroll
      for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
      if (r0 + q < R) st<false>(table + (r0 + q) * 1024 + lane * 16, acc);
    }
  }
}

template <typename K>
static unsigned resident(K k) {
  int per = 0, cus = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, k, 256, 0));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  return (unsigned)(per * cus);
}

template <typename F>
static float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

static void line(const char *probe, const char *extra, double bytes, float ms) {
  printf("{\"probe\": \"%s\", %s, \"ms\": %.4f, \"bytes\": %.0f, \"GBps\": %.1f}\n", probe, extra, ms, bytes,
         bytes / ms / 1e6);
  fflush(stdout);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int64_t BIG = 8ll << 30;   // 8 GiB: far beyond the 256 MiB Infinity Cache
  uint8_t *a, *b;
  uint32_t *sink;
  const int64_t ABYTES = 9ll << 30;   // also holds the apply probe's 8 messages (8.62 GB)
  CK(hipMalloc(&a, ABYTES));
  CK(hipMalloc(&b, BIG + 8192));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 1, ABYTES));
  CK(hipMemset(b, 0, BIG + 8192));
  char ex[256];

  // 1) copy: 4 GiB -> 4 GiB (8 GiB moved), U in flight per lane, plain / nt
#define COPY(U, NT, MULT)                                                                              \
  {                                                                                                    \
    auto k = copy_kernel<U, NT>;                                                                       \
    const int64_t bytes = 4ll << 30, tiles = bytes / (U * 4096);                                       \
    const unsigned g = resident(k) * MULT;                                                             \
    const float ms = time_ms([&] { k<<<g, 256>>>(a, b, tiles); }, reps);                               \
    snprintf(ex, sizeof ex, "\"U\": %d, \"nt\": %d, \"grid\": %u", U, (int)NT, g);                      \
    line("copy", ex, 2.0 * bytes, ms);                                                                 \
  }
  COPY(1, false, 1) COPY(4, false, 1) COPY(8, false, 1) COPY(4, true, 1) COPY(8, true, 1) COPY(4, false, 4)
  COPY(16, true, 1)

  // 2) sequential read of 8 GiB
#define READ(U, NT)                                                                                    \
  {                                                                                                    \
    auto k = read_kernel<U, NT>;                                                                       \
    const int64_t tiles = BIG / (U * 4096);                                                            \
    const unsigned g = resident(k);                                                                    \
    const float ms = time_ms([&] { k<<<g, 256>>>(a, tiles, sink); }, reps);                            \
    snprintf(ex, sizeof ex, "\"U\": %d, \"nt\": %d, \"grid\": %u", U, (int)NT, g);                      \
    line("read", ex, (double)BIG, ms);                                                                 \
  }
  READ(4, false) READ(8, false) READ(8, true) READ(16, true)

  // 3) random chunks of C bytes over the 8 GiB buffer (each slot read once per launch)
  std::mt19937 rng(1234);
  int32_t *slot;
  const int64_t max_slots = BIG / 256;
  CK(hipMalloc(&slot, max_slots * sizeof(int32_t)));
  auto gather = [&](int32_t C, int64_t stride, int32_t off, auto kern, int D) {
    const int64_t nslots = (BIG - 4096) / stride;
    std::vector<int32_t> h(nslots);
    for (int64_t i = 0; i < nslots; ++i) h[i] = (int32_t)i;
    std::shuffle(h.begin(), h.end(), rng);
    CK(hipMemcpy(slot, h.data(), nslots * sizeof(int32_t), hipMemcpyHostToDevice));
    const int64_t groups = C >= 1024 ? nslots * (C / 1024) : nslots / (1024 / C);
    const unsigned g = resident(kern);
    const float ms = time_ms([&] { kern<<<g, 256>>>(a, slot, groups, C, stride, off, sink); }, reps);
    snprintf(ex, sizeof ex, "\"C\": %d, \"stride\": %lld, \"off\": %d, \"D\": %d, \"grid\": %u", C,
             (long long)stride, off, D, g);
    line("gather", ex, (double)groups * 1024 + (double)nslots * 4, ms);
  };
  for (int C : {256, 512, 1024, 2048, 4096}) {
    gather(C, C, 0, gather_kernel<4, true>, 4);
    gather(C, C, 0, gather_kernel<8, true>, 8);
  }
  gather(1024, 1028, 4, gather_kernel<4, true>, 4);
  gather(1024, 1028, 4, gather_kernel<8, true>, 8);
  gather(1024, 1028, 4, gather_kernel<16, true>, 16);
  gather(1024, 1024, 0, gather_kernel<16, true>, 16);
  gather(1024, 1028, 4, gather_kernel<8, false>, 8);
  CK(hipFree(slot));

  // 4) the C2 pattern (2^20 rows x 256 f32, 8 messages), 1,028- and 1,024-B record stride
  {
    const int64_t R = 1 << 20, B = 8;
    const int64_t msg_bytes = 20 + R * 1028 + 64;
    uint8_t *table = b, *stream = a;     // 1 GiB table in b, 8 messages in a
    int32_t *pos;
    CK(hipMalloc(&pos, B * R * sizeof(int32_t)));
    std::vector<int32_t> h(B * R);
    for (int64_t m = 0; m < B; ++m) {
      std::vector<int32_t> perm(R);
      for (int64_t i = 0; i < R; ++i) perm[i] = (int32_t)i;
      std::shuffle(perm.begin(), perm.end(), rng);
      for (int64_t i = 0; i < R; ++i) h[m * R + perm[i]] = (int32_t)i;
    }
    CK(hipMemcpy(pos, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
#define APPLY(D, STRIDE)                                                                               \
    {                                                                                                  \
      auto k = apply_kernel<8, D>;                                                                     \
      const unsigned g = resident(k);                                                                  \
      const float ms = time_ms([&] { k<<<g, 256>>>(table, stream, pos, R, STRIDE, msg_bytes); }, reps); \
      snprintf(ex, sizeof ex, "\"D\": %d, \"stride\": %d, \"grid\": %u", D, (int)(STRIDE), g);          \
      line("apply", ex, (double)B * (20 + R * (4 + 1024)) + 2.0 * R * 1024 + (double)B * R * 4, ms);    \
    }
    APPLY(1, 1028) APPLY(2, 1028) APPLY(4, 1028) APPLY(2, 1024) APPLY(4, 1024)
    CK(hipFree(pos));
  }
  return 0;
}
