// Probe: byte-aligned global_load_dword / dwordx4 on the GPU box (unaligned access mode).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstring>
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
__global__ void k(const uint8_t *p, uint32_t *o) {
  const int t = threadIdx.x;            // offsets 0..63
  uint32_t v; __builtin_memcpy(&v, p + t, 4);
  u4 w; __builtin_memcpy(&w, p + 100 + t, 16);
  o[t * 5] = v;
  for (int i = 0; i < 4; ++i) o[t * 5 + 1 + i] = w[i];
}
int main() {
  uint8_t h[256];
  for (int i = 0; i < 256; ++i) h[i] = (uint8_t)(i * 37 + 11);
  uint8_t *d; uint32_t *o;
  if (hipMalloc(&d, 256) || hipMalloc(&o, 64 * 5 * 4)) return 2;
  hipMemcpy(d, h, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
  if (hipDeviceSynchronize() != hipSuccess) { printf("FAULT\n"); return 3; }
  uint32_t r[320];
  hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int t = 0; t < 64; ++t) {
    uint32_t v; memcpy(&v, h + t, 4);
    uint32_t w[4]; memcpy(w, h + 100 + t, 16);
    bad += r[t * 5] != v;
    for (int i = 0; i < 4; ++i) bad += r[t * 5 + 1 + i] != w[i];
  }
  printf(bad ? "MISMATCH %d\n" : "unaligned loads OK\n", bad);
  return bad ? 1 : 0;
}
