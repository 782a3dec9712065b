// probe_apply.hip — variants of the C2 apply's access pattern, to find what separates it
// (≈4.9 TB/s algorithmic) from the random record gather alone (≈5.9 TB/s at the wire
// format's 1,028-B stride, tools/probe_hbm.hip) and the sequential read (≈6.9 TB/s).
//
// C2: B = 8 messages of R = 2^20 records (4-byte row id + 256 f32, 1,028 B), rows in a
// random order per message; table R x 256 f32.  Per row: the table row and its B records
// are read, the sum (message order) is stored.  One wave per D rows at a time, lane l owns
// floats 4l..4l+3.  Variants (the store and the load policies, the row order, pipelining):
//   base      nt loads, plain in-place store                        (≈ dense_apply_v3)
//   nostore   no store (reads only)
//   ntstore   nt store
//   sc1store  store with sc1 (the line leaves the XCD's L2)
//   outplace  store to a second table
//   tabplain  table rows loaded without nt
//   pipe      the next D rows' loads issued before this D rows' stores
//   blocked   each wave sweeps 16 consecutive rows (4 x D=4) before taking the next block
// With a second argument 1 (mixing probe): table-plain variants with the records in random
// order, then in slot order (every access a sequential sweep), then sequential and aligned.
// Each line is one JSON object: ms per launch and algorithmic GB/s (the apply's bytes).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe_apply tools/probe_apply.hip
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

enum { ST_PLAIN = 0, ST_NONE = 1, ST_NT = 2, ST_SC1 = 3 };

template <int ST>
__device__ __forceinline__ void store(uint8_t *p, u32x4 v) {
  if (ST == ST_PLAIN) *(u32x4 *)p = v;
  if (ST == ST_NT) __builtin_nontemporal_store(v, (gu32x4_p)p);
  if (ST == ST_SC1) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  }
  if (ST == ST_NONE) {
    if (v[0] == 0x7fc00001u && v[1] == 0x7fc00002u) *(u32x4 *)p = v;   // never true: keeps the loads live
  }
}

struct Args {
  uint8_t *table;
  uint8_t *out;
  const uint8_t *stream;
  const int32_t *pos;   // [B][R]: record index of row r in message b
  int64_t R, stride, msg_bytes;
  int64_t rec_off;   // payload offset of record 0 (24: the wire format's header + row id)
};

template <int B, int D>
__device__ __forceinline__ void load_rows(const Args &a, int64_t r0, int lane, bool tab_nt, u32x4 (&t)[D],
                                          u32x4 (&u)[D][B]) {
#pragma unroll
  for (int q = 0; q < D; ++q) {
    const int64_t r = r0 + q < a.R ? r0 + q : a.R - 1;
    t[q] = tab_nt ? ld_nt(a.table + r * 1024 + lane * 16) : ld_plain(a.table + r * 1024 + lane * 16);
#pragma unroll
    for (int b = 0; b < B; ++b)
      u[q][b] = ld_nt(a.stream + b * a.msg_bytes + (int64_t)a.pos[b * a.R + r] * a.stride + a.rec_off + lane * 16);
  }
}

template <int B, int D, int ST>
__device__ __forceinline__ void finish_rows(const Args &a, int64_t r0, int lane, bool outplace, u32x4 (&t)[D],
                                            u32x4 (&u)[D][B]) {
#pragma unroll
  for (int q = 0; q < D; ++q) {
    u32x4 acc = t[q];
#pragma unroll
    for (int b = 0; b < B; ++b) acc = addf(acc, u[q][b]);
    if (r0 + q < a.R) store<ST>((outplace ? a.out : a.table) + (r0 + q) * 1024 + lane * 16, acc);
  }
}

template <int B, int D, int ST, bool TAB_NT, bool OUTPLACE>
__global__ void __launch_bounds__(256) apply_kernel(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t r0 = wave * D; r0 < a.R; r0 += nw * D) {
    u32x4 t[D], u[D][B];
    load_rows<B, D>(a, r0, lane, TAB_NT, t, u);
    finish_rows<B, D, ST>(a, r0, lane, OUTPLACE, t, u);
  }
}

// Software-pipelined: the next group's loads are issued before this group's adds/stores.
template <int B, int D>
__global__ void __launch_bounds__(256) pipe_kernel(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  int64_t r0 = wave * D;
  if (r0 >= a.R) return;
  u32x4 t[D], u[D][B];
  load_rows<B, D>(a, r0, lane, true, t, u);
  for (;;) {
    const int64_t r1 = r0 + nw * D;
    u32x4 sum[D];
#pragma unroll
    for (int q = 0; q < D; ++q) {
      sum[q] = t[q];
#pragma unroll
      for (int b = 0; b < B; ++b) sum[q] = addf(sum[q], u[q][b]);
    }
    if (r1 < a.R) load_rows<B, D>(a, r1, lane, true, t, u);
#pragma unroll
    for (int q = 0; q < D; ++q)
      if (r0 + q < a.R) *(u32x4 *)(a.table + (r0 + q) * 1024 + lane * 16) = sum[q];
    if (r1 >= a.R) break;
    r0 = r1;
  }
}

// Blocked: a wave takes a block of NB consecutive rows and sweeps it D rows at a time.
template <int B, int D, int NB>
__global__ void __launch_bounds__(256) blocked_kernel(Args a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t blk = wave * NB; blk < a.R; blk += nw * NB) {
    for (int64_t r0 = blk; r0 < blk + NB && r0 < a.R; r0 += D) {
      u32x4 t[D], u[D][B];
      load_rows<B, D>(a, r0, lane, true, t, u);
      finish_rows<B, D, ST_PLAIN>(a, r0, lane, false, t, u);
    }
  }
}

// Pseudo-random f32 data (|x| < 1, full mantissa entropy) for the data-dependence check.
__global__ void fill_random(uint32_t *p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 15; x *= 2246822519u; x ^= x >> 13; x *= 3266489917u; x ^= x >> 16;
    p[i] = (x & 0x807fffffu) | 0x3e000000u;   // sign and mantissa random, exponent fixed: 0.125..0.25
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

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const int64_t R = 1 << 20, B = 8;
  Args a{};
  a.R = R;
  a.stride = 1028;
  a.rec_off = 24;
  a.msg_bytes = 20 + R * 1028 + 64;
  uint8_t *stream;
  int32_t *pos;
  CK(hipMalloc(&a.table, R * 1024));
  CK(hipMalloc(&a.out, R * 1024));
  CK(hipMalloc(&stream, B * a.msg_bytes));
  CK(hipMalloc(&pos, B * R * sizeof(int32_t)));
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

  auto run = [&](const char *name, auto kern, int D, unsigned mult) {
    const unsigned g = resident(kern) * mult;
    const float ms = time_ms([&] { kern<<<g, 256>>>(a); }, reps);
    printf("{\"probe\": \"%s\", \"D\": %d, \"grid\": %u, \"ms\": %.4f, \"GBps\": %.1f}\n", name, D, g, ms,
           alg / ms / 1e6);
    fflush(stdout);
  };
  const char *order = "random";
  auto variants = [&] {
    printf("{\"order\": \"%s\"}\n", order);
    run("tabplain", apply_kernel<8, 4, ST_PLAIN, false, false>, 4, 1);
    run("tabplain_nostore", apply_kernel<8, 4, ST_NONE, false, false>, 4, 1);
    run("tabplain_outplace", apply_kernel<8, 4, ST_PLAIN, false, true>, 4, 1);
    run("tabplain_ntstore", apply_kernel<8, 4, ST_NT, false, false>, 4, 1);
    run("tabplain", apply_kernel<8, 4, ST_PLAIN, false, false>, 4, 1);
  };
  if (argc > 2 && atoi(argv[2]) == 1) {
    // Mixing probe: the same variants with every message's records in slot order (record r
    // of every message belongs to row r), so all reads and writes are sequential sweeps —
    // the same bytes, read/write ratio and kernel; only the randomness is gone.
    variants();
    for (int64_t m = 0; m < B; ++m)
      for (int64_t i = 0; i < R; ++i) h[m * R + i] = (int32_t)i;
    CK(hipMemcpy(pos, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    order = "sequential";
    variants();
    a.stride = 1024;   // sequential and line-aligned records (no 9th line per record)
    a.rec_off = 0;
    order = "sequential_aligned";
    variants();
    // the same, random order, with random data in the table and every record (the runs
    // above add zeros to zeros): does the data itself change the rate?
    a.stride = 1028;
    a.rec_off = 24;
    std::mt19937 rng2(1234);
    for (int64_t m = 0; m < B; ++m) {
      std::vector<int32_t> perm(R);
      for (int64_t i = 0; i < R; ++i) perm[i] = (int32_t)i;
      std::shuffle(perm.begin(), perm.end(), rng2);
      for (int64_t i = 0; i < R; ++i) h[m * R + perm[i]] = (int32_t)i;
    }
    CK(hipMemcpy(pos, h.data(), h.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    fill_random<<<4096, 256>>>(reinterpret_cast<uint32_t *>(a.table), R * 256, 17u);
    fill_random<<<4096, 256>>>(reinterpret_cast<uint32_t *>(stream), B * a.msg_bytes / 4, 91u);
    CK(hipDeviceSynchronize());
    order = "random_data";
    variants();
    return 0;
  }
  // the same variant twice, first and last, brackets the run's drift
  run("base", apply_kernel<8, 4, ST_PLAIN, true, false>, 4, 1);
  run("nostore", apply_kernel<8, 4, ST_NONE, true, false>, 4, 1);
  run("ntstore", apply_kernel<8, 4, ST_NT, true, false>, 4, 1);
  run("sc1store", apply_kernel<8, 4, ST_SC1, true, false>, 4, 1);
  run("outplace", apply_kernel<8, 4, ST_PLAIN, true, true>, 4, 1);
  run("tabplain", apply_kernel<8, 4, ST_PLAIN, false, false>, 4, 1);
  run("tabplain_ntstore", apply_kernel<8, 4, ST_NT, false, false>, 4, 1);
  run("base_x2grid", apply_kernel<8, 4, ST_PLAIN, true, false>, 4, 2);
  run("base_d2", apply_kernel<8, 2, ST_PLAIN, true, false>, 2, 1);
  run("base_d8", apply_kernel<8, 8, ST_PLAIN, true, false>, 8, 1);
  run("pipe", pipe_kernel<8, 2>, 2, 1);
  run("pipe_d4", pipe_kernel<8, 4>, 4, 1);
  run("blocked16", blocked_kernel<8, 4, 16>, 4, 1);
  run("blocked64", blocked_kernel<8, 4, 64>, 4, 1);
  run("base", apply_kernel<8, 4, ST_PLAIN, true, false>, 4, 1);
  return 0;
}
