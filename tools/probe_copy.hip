// probe_copy.hip — how the launch shape moves the HBM rate of a float4 copy, a write-only
// sweep and the C2 read/write mix ("bring the copy probe to the guide's rate").
//
//   copy  flat      one 16-B load + store per thread, one tile per block (grid = n / 256):
//                   the hardware dispatcher hands out the tiles (the guide's float4 copy)
//   copy  flatU     U float4 per thread, block = U x 4 KiB contiguous, one tile per block
//   copy  persist   grid sized to residency x M, tiles handed out grid-stride (probe_hbm's form)
//   write flat      16-B stores only (what the row stores alone can reach)
//   read  flat      16-B loads only
//   mixK  seq|split K 1-KiB reads per wave then one 1-KiB write, flat grid, one wave per
//                   row: "seq" reads K consecutive KiB of one sweep (two streams in all),
//                   "split" reads piece k from region k (K + 1 streams, the C2 apply's shape
//                   with records in slot order) — the read/write ratio without the gather
//   apply flat      the C2 pattern (8 records + table row read, row written), D rows per
//                   wave, one tile per block, rows in slot order — against probe_hbm's
//                   persistent apply of the same bytes
//
// Each line: one JSON object, algorithmic bytes, ms per launch (hip events, mean of reps).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_copy tools/probe_copy.hip
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
typedef const u32x4 __attribute__((address_space(1))) *gcu32x4_p;
typedef u32x4 __attribute__((address_space(1))) *gu32x4_p;

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if (NT) return __builtin_nontemporal_load((gcu32x4_p)p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, (gu32x4_p)p);
  else *p = v;
}

// flat: block k covers elements [k * 256 * U, (k + 1) * 256 * U), lane-contiguous per step
template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_flat(const u32x4 *src, u32x4 *dst) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + base + u * 256);
#pragma unroll
  for (int u = 0; u < U; ++u) st<NT>(dst + base + u * 256, v[u]);
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_persist(const u32x4 *src, u32x4 *dst, int64_t tiles) {
  for (int64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int64_t base = t * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld<NT>(src + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) st<NT>(dst + base + u * 256, v[u]);
  }
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) write_flat(u32x4 *dst, uint32_t seed) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  const u32x4 v = {seed, seed ^ 1u, (uint32_t)blockIdx.x, (uint32_t)threadIdx.x};
#pragma unroll
  for (int u = 0; u < U; ++u) st<NT>(dst + base + u * 256, v);
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) read_flat(const u32x4 *src, uint32_t *sink) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < U; ++u) acc ^= ld<NT>(src + base + u * 256);
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1;
}

typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const u32x4_a4 __attribute__((address_space(1))) *gcu32x4a4_p;
__device__ __forceinline__ u32x4 ldu(const uint8_t *p) {
  return __builtin_nontemporal_load((gcu32x4a4_p)(const __attribute__((address_space(1))) uint8_t *)p);
}
__device__ __forceinline__ u32x4 addf(u32x4 a, u32x4 b) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(__uint_as_float(a[i]) + __uint_as_float(b[i]));
  return r;
}

// The C2 pattern, one tile of 4 * D rows per block (each wave D consecutive rows).
template <int B, int D>
__global__ void __launch_bounds__(256) apply_flat(uint8_t *table, const uint8_t *stream, const int32_t *pos,
                                                  int64_t R, int64_t stride, int64_t msg_bytes) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * D;
  u32x4 t[D], u[D][B];
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const int64_t r = r0 + q < R ? r0 + q : R - 1;
    t[q] = ldu(table + r * 1024 + lane * 16);
#pragma unroll
    for (int b = 0; b < B; ++b)
      u[q][b] = ldu(stream + b * msg_bytes + (int64_t)pos[b * R + r] * stride + 24 + lane * 16);
  }
#pragma unroll
  for (int q = 0; q < D; ++q) {
    u32x4 acc = t[q];
#pragma unroll
    for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
    if (r0 + q < R) *(u32x4 *)(table + (r0 + q) * 1024 + lane * 16) = acc;
  }
}

// K reads of 1 KiB then 1 write of 1 KiB per wave (row w = one wave), plain loads, nt or plain store
template <int K, bool SPLIT>
__global__ void __launch_bounds__(256) mix_flat(const u32x4 *src, u32x4 *dst, int64_t rows) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  u32x4 v[K];
#pragma unroll
  for (int k = 0; k < K; ++k)
    v[k] = ld<true>(src + (SPLIT ? (int64_t)k * rows * 64 + w * 64 : (w * K + k) * 64) + lane);
  u32x4 acc = v[0];
#pragma unroll
  for (int k = 1; k < K; ++k) acc ^= v[k];
  st<false>(dst + w * 64 + lane, acc);
}

// 9:1 variants (seq streams, 2^20 rows): MODE 0 = plain loads, 1 = nt store, 2 = store before
// the loads (a constant), 3 = two rows per wave (18 loads, 2 stores), 4 = role split: of
// every 10 waves, 9 read 10 KiB each... (wave w % 10 == 9 writes the ten rows' 10 KiB)
template <int MODE>
__global__ void __launch_bounds__(256) mix9_var(const u32x4 *src, u32x4 *dst, int64_t rows, uint32_t *sink) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if constexpr (MODE == 4) {
    // 10 waves cover 9 rows' reads (81 KiB) and 9 rows' writes (9 KiB): waves 0..8 read
    // 9 KiB each, wave 9 writes 9 KiB
    const int64_t grp = w / 10, r = w % 10;
    if (grp * 9 >= rows) return;
    if (r < 9) {
      if (grp * 9 + r >= rows) return;
      u32x4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < 9; ++k) acc ^= ld<true>(src + ((grp * 9 + r) * 9 + k) * 64 + lane);
      if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x9e3779b9u) sink[0] = 1;
    } else {
      const u32x4 v = {(uint32_t)grp, 1u, 2u, 3u};
#pragma unroll
      for (int k = 0; k < 9; ++k)
        if (grp * 9 + k < rows) st<false>(dst + (grp * 9 + k) * 64 + lane, v);
    }
    return;
  }
  constexpr int RW = MODE == 3 ? 2 : 1;
  if (w * RW >= rows) return;
  if constexpr (MODE == 2) st<false>(dst + w * 64 + lane, u32x4{(uint32_t)w, 0u, 0u, 0u});
  u32x4 acc[RW];
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    acc[q] = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const u32x4 *p = src + ((w * RW + q) * 9 + k) * 64 + lane;
      acc[q] ^= MODE == 0 ? ld<false>(p) : ld<true>(p);
    }
  }
  if constexpr (MODE == 2) {
    if ((acc[0][0] ^ acc[0][1]) == 0x9e3779b9u) sink[0] = 1;
  } else {
#pragma unroll
    for (int q = 0; q < RW; ++q) {
      if (MODE == 1) st<true>(dst + (w * RW + q) * 64 + lane, acc[q]);
      else st<false>(dst + (w * RW + q) * 64 + lane, acc[q]);
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
  CK(hipGetLastError());
  return ms / reps;
}

static void line(const char *probe, const char *extra, double bytes, float ms) {
  printf("{\"probe\": \"%s\", %s, \"ms\": %.4f, \"bytes\": %.0f, \"GBps\": %.1f}\n", probe, extra, ms, bytes,
         bytes / ms / 1e6);
  fflush(stdout);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int64_t ABYTES = 9ll << 30, BBYTES = (4ll << 30) + 8192;
  uint8_t *a, *b;
  uint32_t *sink;
  CK(hipMalloc(&a, ABYTES));
  CK(hipMalloc(&b, BBYTES));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 1, ABYTES));
  CK(hipMemset(b, 0, BBYTES));
  char ex[256];

  const bool only_mix = argc > 2 && argv[2][0] == 'm';   // "mix": the ratio and apply forms only
  for (int64_t gib : {1, 4}) {
    if (only_mix) break;
    const int64_t bytes = gib << 30, n16 = bytes / 16;
#define FLAT(U, NT)                                                                                   \
    {                                                                                                 \
      const unsigned g = (unsigned)(n16 / (256 * U));                                                 \
      const float ms = time_ms([&] { copy_flat<U, NT><<<g, 256>>>((const u32x4 *)a, (u32x4 *)b); }, reps); \
      snprintf(ex, sizeof ex, "\"form\": \"flat\", \"GiB\": %lld, \"U\": %d, \"nt\": %d", (long long)gib, U, (int)NT); \
      line("copy", ex, 2.0 * bytes, ms);                                                              \
    }
    FLAT(1, false) FLAT(1, true) FLAT(2, false) FLAT(4, false) FLAT(4, true) FLAT(8, true)
#define PERSIST(U, NT, M)                                                                             \
    {                                                                                                 \
      auto k = copy_persist<U, NT>;                                                                   \
      const unsigned g = resident(k) * M;                                                             \
      const int64_t tiles = n16 / (256 * U);                                                          \
      const float ms = time_ms([&] { k<<<g, 256>>>((const u32x4 *)a, (u32x4 *)b, tiles); }, reps);    \
      snprintf(ex, sizeof ex, "\"form\": \"persist\", \"GiB\": %lld, \"U\": %d, \"nt\": %d, \"grid\": %u", \
               (long long)gib, U, (int)NT, g);                                                        \
      line("copy", ex, 2.0 * bytes, ms);                                                              \
    }
    PERSIST(8, true, 1) PERSIST(4, false, 1) PERSIST(4, false, 8)
#define WRITE(U, NT)                                                                                  \
    {                                                                                                 \
      const unsigned g = (unsigned)(n16 / (256 * U));                                                 \
      const float ms = time_ms([&] { write_flat<U, NT><<<g, 256>>>((u32x4 *)b, 7u); }, reps);        \
      snprintf(ex, sizeof ex, "\"form\": \"flat\", \"GiB\": %lld, \"U\": %d, \"nt\": %d", (long long)gib, U, (int)NT); \
      line("write", ex, (double)bytes, ms);                                                           \
    }
    WRITE(1, false) WRITE(4, false) WRITE(4, true)
#define READF(U, NT)                                                                                  \
    {                                                                                                 \
      const unsigned g = (unsigned)(n16 / (256 * U));                                                 \
      const float ms = time_ms([&] { read_flat<U, NT><<<g, 256>>>((const u32x4 *)a, sink); }, reps); \
      snprintf(ex, sizeof ex, "\"form\": \"flat\", \"GiB\": %lld, \"U\": %d, \"nt\": %d", (long long)gib, U, (int)NT); \
      line("read", ex, (double)bytes, ms);                                                            \
    }
    READF(1, false) READF(4, false) READF(4, true)
  }

  // read/write ratio K:1 with sequential streams, 2^20 rows (1 GiB written)
  {
    const int64_t R = 1 << 20;
#define MIX(K, SPLIT)                                                                                 \
    {                                                                                                 \
      const unsigned g = (unsigned)(R / 4);                                                          \
      const float ms = time_ms([&] { mix_flat<K, SPLIT><<<g, 256>>>((const u32x4 *)a, (u32x4 *)b, R); }, reps); \
      snprintf(ex, sizeof ex, "\"form\": \"%s\", \"K\": %d", SPLIT ? "split" : "seq", K);           \
      line("mix", ex, (double)(K + 1) * R * 1024, ms);                                               \
    }
    MIX(1, false) MIX(2, false) MIX(4, false) MIX(9, false) MIX(9, true) MIX(4, true)
#define MIXV(MODE, WAVES)                                                                             \
    {                                                                                                 \
      const unsigned g = (unsigned)((WAVES + 3) / 4);                                                \
      const float ms = time_ms([&] { mix9_var<MODE><<<g, 256>>>((const u32x4 *)a, (u32x4 *)b, R, sink); }, reps); \
      snprintf(ex, sizeof ex, "\"form\": \"seq9_mode%d\", \"K\": 9", MODE);                        \
      line("mix", ex, 10.0 * R * 1024, ms);                                                          \
    }
    MIXV(0, R) MIXV(1, R) MIXV(2, R) MIXV(3, R / 2) MIXV(4, (R / 9 + 1) * 10) MIX(9, false)
  }

  // the C2 pattern, one tile per block (2^20 rows x 256 f32, 8 messages, 1,028-B records)
  {
    const int64_t R = 1 << 20, B = 8;
    const int64_t msg_bytes = 20 + R * 1028 + 64;
    uint8_t *table = b, *stream = a;
    int32_t *pos;
    CK(hipMalloc(&pos, B * R * sizeof(int32_t)));
    std::mt19937 rng(1234);
    std::vector<int32_t> h(B * R);
    for (int64_t m = 0; m < B; ++m) {
      std::vector<int32_t> perm(R);
      for (int64_t i = 0; i < R; ++i) perm[i] = (int32_t)i;
      std::shuffle(perm.begin(), perm.end(), rng);
      for (int64_t i = 0; i < R; ++i) h[m * R + perm[i]] = (int32_t)i;
    }
    CK(hipMemcpy(pos, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
#define APPLYF(D)                                                                                     \
    {                                                                                                 \
      const unsigned g = (unsigned)((R + 4 * D - 1) / (4 * D));                                      \
      const float ms = time_ms([&] { apply_flat<8, D><<<g, 256>>>(table, stream, pos, R, 1028, msg_bytes); }, reps); \
      snprintf(ex, sizeof ex, "\"form\": \"flat\", \"D\": %d, \"grid\": %u", D, g);                    \
      line("apply", ex, (double)B * (20 + R * (4 + 1024)) + 2.0 * R * 1024 + (double)B * R * 4, ms);   \
    }
    APPLYF(1) APPLYF(2) APPLYF(4)
    CK(hipFree(pos));
  }
  return 0;
}
