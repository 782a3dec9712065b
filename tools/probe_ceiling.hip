// probe_ceiling.hip — the hardware ceiling of the C2 apply's access pattern, without the
// apply's bookkeeping (no stream walk, no inverse index build, no presence checks).
//
// C2: B = 8 messages of R = 2^20 records, each record = 4-byte row id +
// 256 f32 (1,028 B), rows in a random order per message; table R x 256 f32.  Per row the
// apply reads the table row and its B records and writes the row.  Variants, each timed
// with hip events over several launches:
//   copy       float4 stream copy of 1 GiB (the box's sequential HBM rate)
//   stream     sequential read of all B messages (no gather): the stream's own rate
//   gather     per row: B records gathered from their random positions, 1,028-B stride
//              (payload 4-byte aligned, 9 lines per record) + table row read + write
//   gather_al  the same with a 1,024-B record stride (payload 128-B aligned, 8 lines):
//              what the wire format's 4-byte row id costs in line over-fetch
//   norec_tab  table read + write only (the row sweep alone)
// Record positions come from a precomputed [B][R] int32 map (what dense_index builds);
// reading it is part of every gather variant, as in the apply.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/probe_ceiling tools/probe_ceiling.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>
#include <random>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
typedef const u32x4_a4 __attribute__((address_space(1))) *gu32x4_p;
typedef const uint8_t __attribute__((address_space(1))) *gbyte_p;

__device__ __forceinline__ u32x4 ld_nt(const uint8_t *base, uint64_t off) {
  return __builtin_nontemporal_load((gu32x4_p)((gbyte_p)base + off));
}
__device__ __forceinline__ u32x4 addf(u32x4 a, u32x4 b) {
  u32x4 r;
  for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(__uint_as_float(a[i]) + __uint_as_float(b[i]));
  return r;
}

__global__ void copy_kernel(const u32x4 *src, u32x4 *dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

__global__ void stream_kernel(const u32x4 *src, int64_t n, uint32_t *sink) {
  u32x4 acc = {0, 0, 0, 0};
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    acc ^= __builtin_nontemporal_load(src + i);
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;
}

// One wave per PAIR rows at a time, rows taken in slot order; lane l owns floats 4l..4l+3.
template <int B, int PAIR, bool REC>
__global__ void __launch_bounds__(256) gather_kernel(uint8_t *table, const uint8_t *stream, const int32_t *pos,
                                                     int64_t R, int64_t stride, int64_t msg_bytes) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = wave * PAIR; r0 < R; r0 += nw * PAIR) {
    u32x4 t[PAIR], u[PAIR][B];
#pragma unroll
    for (int q = 0; q < PAIR; ++q) {
      const int64_t r = r0 + q < R ? r0 + q : R - 1;
      t[q] = *(const u32x4 *)(table + r * 1024 + lane * 16);
      if (REC) {
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const int64_t p = pos[b * R + r];
          u[q][b] = ld_nt(stream, b * msg_bytes + p * stride + 4 + lane * 16);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PAIR; ++q) {
      u32x4 acc = t[q];
      if (REC) {
#pragma unroll
        for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
      } else {
        acc = addf(acc, acc);
      }
      if (r0 + q < R) *(u32x4 *)(table + (r0 + q) * 1024 + lane * 16) = acc;
    }
  }
}

// Rows in message 0's record order: message 0 is read sequentially (its row ids inline),
// the table rows and the other messages' records are gathered.
template <int B, int PAIR>
__global__ void __launch_bounds__(256) seq0_kernel(uint8_t *table, const uint8_t *stream, const int32_t *pos,
                                                   const int32_t *perm0, int64_t R, int64_t stride, int64_t msg_bytes) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t i0 = wave * PAIR; i0 < R; i0 += nw * PAIR) {
    u32x4 t[PAIR], u[PAIR][B];
    int64_t rr[PAIR];
#pragma unroll
    for (int q = 0; q < PAIR; ++q) {
      const int64_t i = i0 + q < R ? i0 + q : R - 1;
      rr[q] = perm0[i];
      t[q] = *(const u32x4 *)(table + rr[q] * 1024 + lane * 16);
      u[q][0] = ld_nt(stream, i * stride + 4 + lane * 16);
#pragma unroll
      for (int b = 1; b < B; ++b) {
        const int64_t p = pos[b * R + rr[q]];
        u[q][b] = ld_nt(stream, b * msg_bytes + p * stride + 4 + lane * 16);
      }
    }
#pragma unroll
    for (int q = 0; q < PAIR; ++q) {
      u32x4 acc = t[q];
#pragma unroll
      for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
      if (i0 + q < R) *(u32x4 *)(table + rr[q] * 1024 + lane * 16) = acc;
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
  return ms / reps;
}

int main(int argc, char **argv) {
  const int64_t R = 1 << 20, B = 8;
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int64_t row = 1024;
  const int64_t stride_w = 1028, stride_a = 1024;
  const int64_t msg_bytes = 20 + R * stride_w + 64;   // header room, 1,028-B records (the larger)
  uint8_t *table, *stream, *scratch;
  int32_t *pos;
  uint32_t *sink;
  CK(hipMalloc(&table, R * row));
  CK(hipMalloc(&scratch, R * row));
  CK(hipMalloc(&stream, B * msg_bytes));
  CK(hipMalloc(&pos, B * R * sizeof(int32_t)));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(table, 0, R * row));
  CK(hipMemset(stream, 0, B * msg_bytes));
  std::vector<int32_t> h(B * R), p0(R);
  std::mt19937 g(1234);
  for (int64_t b = 0; b < B; ++b) {
    std::vector<int32_t> perm(R);
    for (int64_t i = 0; i < R; ++i) perm[i] = (int32_t)i;
    std::shuffle(perm.begin(), perm.end(), g);
    for (int64_t i = 0; i < R; ++i) h[b * R + perm[i]] = (int32_t)i;   // row perm[i] is record i
    if (b == 0) p0 = perm;
  }
  CK(hipMemcpy(pos, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  int32_t *perm0;
  CK(hipMalloc(&perm0, R * sizeof(int32_t)));
  CK(hipMemcpy(perm0, p0.data(), R * sizeof(int32_t), hipMemcpyHostToDevice));

  const double tab_bytes = 2.0 * R * row;
  const double rec_bytes_w = (double)B * R * stride_w, rec_bytes_a = (double)B * R * stride_a;
  const double idx_bytes = (double)B * R * 4;
  float ms;

  ms = time_ms([&] { copy_kernel<<<4096, 256>>>((const u32x4 *)table, (u32x4 *)scratch, R * row / 16); }, reps);
  printf("{\"probe\": \"copy\", \"ms\": %.4f, \"GBps\": %.1f, \"bytes\": %.0f}\n", ms, tab_bytes / ms / 1e6, tab_bytes);
  ms = time_ms([&] { stream_kernel<<<8192, 256>>>((const u32x4 *)stream, B * msg_bytes / 16, sink); }, reps);
  printf("{\"probe\": \"stream\", \"ms\": %.4f, \"GBps\": %.1f, \"bytes\": %.0f}\n", ms,
         (double)B * msg_bytes / ms / 1e6, (double)B * msg_bytes);

#define GATHER(NAME, PAIR, REC, STRIDE, ALG)                                                          \
  {                                                                                                   \
    auto k = gather_kernel<8, PAIR, REC>;                                                             \
    const unsigned blocks = resident(k);                                                              \
    ms = time_ms([&] { k<<<blocks, 256>>>(table, stream, pos, R, STRIDE, msg_bytes); }, reps);        \
    printf("{\"probe\": \"%s\", \"pair\": %d, \"ms\": %.4f, \"GBps_alg\": %.1f, \"alg_bytes\": %.0f, " \
           "\"blocks\": %u}\n", NAME, PAIR, ms, (ALG) / ms / 1e6, (double)(ALG), blocks);             \
  }
  GATHER("gather", 1, true, stride_w, rec_bytes_w + tab_bytes + idx_bytes)
  GATHER("gather", 2, true, stride_w, rec_bytes_w + tab_bytes + idx_bytes)
  GATHER("gather", 4, true, stride_w, rec_bytes_w + tab_bytes + idx_bytes)
  GATHER("gather_al", 2, true, stride_a, rec_bytes_a + tab_bytes + idx_bytes)
  GATHER("gather_al", 4, true, stride_a, rec_bytes_a + tab_bytes + idx_bytes)
  GATHER("norec_tab", 4, false, stride_w, tab_bytes)
#define SEQ0(PAIR)                                                                                  \
  {                                                                                                 \
    auto k = seq0_kernel<8, PAIR>;                                                                  \
    const unsigned blocks = resident(k);                                                            \
    const double alg = rec_bytes_w + tab_bytes + idx_bytes;                                         \
    ms = time_ms([&] { k<<<blocks, 256>>>(table, stream, pos, perm0, R, stride_w, msg_bytes); }, reps); \
    printf("{\"probe\": \"seq0\", \"pair\": %d, \"ms\": %.4f, \"GBps_alg\": %.1f, \"blocks\": %u}\n", PAIR, ms, \
           alg / ms / 1e6, blocks);                                                                 \
  }
  SEQ0(2)
  SEQ0(4)
  return 0;
}
