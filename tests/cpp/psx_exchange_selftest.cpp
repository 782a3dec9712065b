// psx_exchange_selftest — libpsx's RCCL exchange from a C++ program with no torch in the
// process, so libpsx's -lrccl resolves to the ROCm image's own RCCL
// (/opt/rocm/lib/librccl.so.1) rather than the copy torch ships.  One rank exchanges a
// sub-stream with itself through psx_comm_* / psx_exchange_sizes / psx_exchange_streams_v:
// a size past 2 GiB (the single ~2 GiB point-to-point transfer RCCL 2.26 corrupted, which
// libpsx now sends in 512 MiB pieces, psx_exchange.cpp) must arrive byte for byte, at a
// receive displacement.  Reference: the per-server message transport it replaces,
// AbstractBgWorker::SendOpLogMsgs (abstract_bg_worker.cpp:651-689).
// Usage: psx_exchange_selftest [bytes]   (default 2 GiB + 12 KiB)
#include <hip/hip_runtime.h>
#include <link.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "psx.h"

static std::string g_rccl;
static int find_rccl(struct dl_phdr_info *info, size_t, void *) {
  if (info->dlpi_name && std::strstr(info->dlpi_name, "librccl")) g_rccl = info->dlpi_name;
  return 0;
}

#define HIPCK(x)                                                             \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
      return 2;                                                              \
    }                                                                        \
  } while (0)
#define PSXCK(c, x)                                                          \
  do {                                                                       \
    psx_status s_ = (x);                                                     \
    if (s_ != PSX_OK) {                                                      \
      std::fprintf(stderr, "%s: %s (%s)\n", #x, psx_status_string(s_),       \
                   psx_comm_last_error(c));                                  \
      return 3;                                                              \
    }                                                                        \
  } while (0)

int main(int argc, char **argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (2ull << 30) + (12ull << 10);
  const uint64_t displ = 4096;   // the sub-stream lands past a receive displacement
  if (n % 4) return 1;
  std::vector<uint32_t> host(n / 4);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto &w : host) {   // xorshift64: every word different, nothing repeating at 512 MiB
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    w = (uint32_t)(x >> 16);
  }
  uint8_t *send = nullptr, *recv = nullptr;
  HIPCK(hipSetDevice(0));
  HIPCK(hipMalloc(&send, n));
  HIPCK(hipMalloc(&recv, n + displ));
  HIPCK(hipMemcpy(send, host.data(), n, hipMemcpyHostToDevice));
  HIPCK(hipMemset(recv, 0, n + displ));
  hipStream_t st;
  HIPCK(hipStreamCreate(&st));

  char id[PSX_COMM_ID_BYTES];
  psx_comm *comm = nullptr;
  PSXCK(nullptr, psx_comm_unique_id(id));
  PSXCK(nullptr, psx_comm_create(id, 1, 0, 0, &comm));
  dl_iterate_phdr(find_rccl, nullptr);
  int32_t cn = 0, cr = -1, cd = -1, cv = 0;
  char cpath[512];
  PSXCK(comm, psx_comm_info(comm, &cn, &cr, &cd, &cv, cpath, sizeof cpath));
  std::printf("{\"comm_nranks\": %d, \"comm_rank\": %d, \"comm_device\": %d, \"rccl_version\": %d, "
              "\"comm_librccl\": \"%s\"}\n", cn, cr, cd, cv, cpath);
  if (cn != 1 || cr != 0 || cd != 0 || std::string(cpath) != g_rccl) return 6;
  uint64_t send_size = n, recv_size = 0, sdis = 0, rdis = displ;
  PSXCK(comm, psx_exchange_sizes(comm, &send_size, &recv_size, st));
  if (recv_size != n) {
    std::fprintf(stderr, "sizes: got %llu\n", (unsigned long long)recv_size);
    return 4;
  }
  PSXCK(comm, psx_exchange_streams_v(comm, send, &send_size, &sdis, recv, &recv_size, &rdis, st));
  HIPCK(hipStreamSynchronize(st));
  uint64_t psent = 0, precv = 0;
  PSXCK(comm, psx_comm_peer_bytes(comm, &psent, &precv, 1));
  if (psent != n || precv != n) return 7;
  std::vector<uint32_t> back(n / 4);
  HIPCK(hipMemcpy(back.data(), recv + displ, n, hipMemcpyDeviceToHost));
  uint32_t head[16];
  HIPCK(hipMemcpy(head, recv, sizeof(head), hipMemcpyDeviceToHost));
  uint64_t bad = 0, first = ~0ull;
  for (uint64_t i = 0; i < n / 4; ++i)
    if (back[i] != host[i]) {
      if (first == ~0ull) first = i;
      ++bad;
    }
  for (uint32_t h : head) bad += h != 0;   // nothing written before the displacement
  PSXCK(comm, psx_comm_destroy(comm));
  HIPCK(hipStreamDestroy(st));
  HIPCK(hipFree(send));
  HIPCK(hipFree(recv));
  std::printf("{\"bytes\": %llu, \"differing_words\": %llu, \"first_bad_word\": %lld, \"rccl\": \"%s\"}\n",
              (unsigned long long)n, (unsigned long long)bad, first == ~0ull ? -1ll : (long long)first,
              g_rccl.c_str());
  if (bad) return 5;
  std::printf("exchange ok\n");
  return 0;
}
