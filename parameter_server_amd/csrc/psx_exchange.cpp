// psx_exchange.cpp — the exchange step of the multi-GPU path, over RCCL (xGMI on one node).
//
// The reference moves a worker's per-server messages over ZeroMQ: the client splits its
// oplog by owning server while packing (AbstractBgWorker::CreateOpLogMsgs,
// abstract_bg_worker.cpp:590-649) and sends each server its message (SendOpLogMsgs,
// :651-689); each server thread receives and applies (server_thread.cpp:419-426).  On one
// MI355X node, when a worker's batch sits on one GPU and spans the row-range shards of
// several, the per-owner sub-streams (psx_split_stream) travel in one all-to-all-v of
// grouped ncclSend/ncclRecv: every GPU sends each owner its sub-stream and receives one
// from every worker, in source-rank order, which psx_apply_streams_device then applies in
// that order (bit-exact to the reference applying the same messages one by one).
//
// Why not reduce-scatter: the same bytes to 0.1% at full coverage, but it
// would sum the workers' updates before the table add (a different rounding) and needs
// dense full-width batches.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <link.h>

#include <cstring>
#include <string>
#include <vector>

#include "../../include/psx.h"

// psx_exchange_sizes_async stages the send sizes through a ring of page-locked slots, so a
// call returns before its sizes have crossed: slot k is reused only after its event.
constexpr int kSizeSlots = 8;

struct psx_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
  uint64_t *d_sizes = nullptr;   // [1 + kSizeSlots][2][nranks]: send sizes, received sizes
  uint64_t *h_send = nullptr;    // [kSizeSlots][nranks], page-locked
  hipEvent_t ev[kSizeSlots] = {};
  int next_slot = 0;
  std::vector<uint64_t> sent, recvd;   // bytes enqueued per peer (psx_comm_peer_bytes)
  std::string err;
};

namespace {

thread_local std::string t_err;

psx_status comm_fail(psx_comm *c, const std::string &m, psx_status st = PSX_ERR_DEVICE) {
  if (c) c->err = m;
  t_err = m;
  return st;
}

#define NCCL_TRY(c, x)                                                                     \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) return comm_fail(c, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)
// inside ncclGroupStart/End: close the group before reporting, so the next call does not
// nest into a half-built group
#define NCCL_TRY_G(c, x)                                                                   \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) {                                                               \
      ncclGroupEnd();                                                                      \
      return comm_fail(c, std::string(#x) + ": " + ncclGetErrorString(r_));                \
    }                                                                                      \
  } while (0)
#define HIPX_TRY(c, x)                                                                     \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) return comm_fail(c, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

}  // namespace

extern "C" {

psx_status psx_comm_unique_id(void *id) {
  static_assert(sizeof(ncclUniqueId) <= PSX_COMM_ID_BYTES, "ncclUniqueId size");
  if (!id) return PSX_ERR_INVALID_ARG;
  ncclUniqueId u;
  ncclResult_t r = ncclGetUniqueId(&u);
  if (r != ncclSuccess) return comm_fail(nullptr, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memset(id, 0, PSX_COMM_ID_BYTES);
  std::memcpy(id, &u, sizeof(u));
  return PSX_OK;
}

psx_status psx_comm_create(const void *id, int32_t nranks, int32_t rank, int32_t device, psx_comm **out) {
  if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) return PSX_ERR_INVALID_ARG;
  *out = nullptr;
  auto *c = new psx_comm();
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  auto cleanup = [&](psx_status st) {
    if (c->d_sizes) hipFree(c->d_sizes);
    if (c->h_send) hipHostFree(c->h_send);
    for (hipEvent_t &e : c->ev)
      if (e) hipEventDestroy(e);
    delete c;
    return st;
  };
  if (hipSetDevice(device) != hipSuccess) return cleanup(comm_fail(nullptr, "hipSetDevice", PSX_ERR_NO_DEVICE));
  if (hipMalloc(&c->d_sizes, sizeof(uint64_t) * 2 * (size_t)nranks * (1 + kSizeSlots)) != hipSuccess)
    return cleanup(comm_fail(nullptr, "hipMalloc", PSX_ERR_OOM));
  if (hipHostMalloc(&c->h_send, sizeof(uint64_t) * (size_t)nranks * kSizeSlots, 0) != hipSuccess)
    return cleanup(comm_fail(nullptr, "hipHostMalloc", PSX_ERR_OOM));
  for (hipEvent_t &e : c->ev)
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
      return cleanup(comm_fail(nullptr, "hipEventCreate", PSX_ERR_DEVICE));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) return cleanup(comm_fail(nullptr, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)));
  c->sent.assign((size_t)nranks, 0);
  c->recvd.assign((size_t)nranks, 0);
  *out = c;
  return PSX_OK;
}

psx_status psx_comm_destroy(psx_comm *c) {
  if (!c) return PSX_ERR_INVALID_ARG;
  hipSetDevice(c->device);
  // an async size exchange may still be queued: let every slot's work finish before the
  // communicator it runs on goes away
  for (hipEvent_t &e : c->ev)
    if (e) hipEventSynchronize(e);
  if (c->comm) ncclCommDestroy(c->comm);
  for (hipEvent_t &e : c->ev)
    if (e) hipEventDestroy(e);
  if (c->d_sizes) hipFree(c->d_sizes);
  if (c->h_send) hipHostFree(c->h_send);
  delete c;
  return PSX_OK;
}

const char *psx_comm_last_error(psx_comm *c) { return c ? c->err.c_str() : t_err.c_str(); }

psx_status psx_exchange_sizes(psx_comm *c, const uint64_t *send_sizes, uint64_t *recv_sizes, void *hip_stream) {
  if (!c || !send_sizes || !recv_sizes) return PSX_ERR_INVALID_ARG;
  for (int i = 0; i < c->nranks; ++i)
    if (send_sizes[i] % 4) return comm_fail(c, "sub-stream sizes are multiples of 4 bytes", PSX_ERR_INVALID_ARG);
  hipStream_t st = (hipStream_t)hip_stream;
  HIPX_TRY(c, hipSetDevice(c->device));
  const size_t n = (size_t)c->nranks;
  HIPX_TRY(c, hipMemcpyAsync(c->d_sizes, send_sizes, sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
  NCCL_TRY(c, ncclGroupStart());
  for (int p = 0; p < c->nranks; ++p) {
    NCCL_TRY_G(c, ncclSend(c->d_sizes + p, 1, ncclUint64, p, c->comm, st));
    NCCL_TRY_G(c, ncclRecv(c->d_sizes + n + p, 1, ncclUint64, p, c->comm, st));
  }
  NCCL_TRY(c, ncclGroupEnd());
  HIPX_TRY(c, hipMemcpyAsync(recv_sizes, c->d_sizes + n, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, st));
  HIPX_TRY(c, hipStreamSynchronize(st));
  return PSX_OK;
}

psx_status psx_exchange_sizes_async(psx_comm *c, const uint64_t *send_sizes, uint64_t *recv_sizes,
                                    void *hip_stream) {
  if (!c || !send_sizes || !recv_sizes) return PSX_ERR_INVALID_ARG;
  for (int i = 0; i < c->nranks; ++i)
    if (send_sizes[i] % 4) return comm_fail(c, "sub-stream sizes are multiples of 4 bytes", PSX_ERR_INVALID_ARG);
  HIPX_TRY(c, hipSetDevice(c->device));
  // recv_sizes is written by the stream: it must be page-locked for the copy to stay
  // asynchronous (a pageable destination would make the copy wait for the collective)
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, recv_sizes) != hipSuccess || at.type != hipMemoryTypeHost) {
    (void)hipGetLastError();
    return comm_fail(c, "exchange_sizes_async: recv_sizes must be page-locked host memory", PSX_ERR_INVALID_ARG);
  }
  hipStream_t st = (hipStream_t)hip_stream;
  const size_t n = (size_t)c->nranks;
  const int k = c->next_slot;
  c->next_slot = (k + 1) % kSizeSlots;
  HIPX_TRY(c, hipEventSynchronize(c->ev[k]));   // the slot's previous sizes have crossed
  uint64_t *hs = c->h_send + (size_t)k * n;
  std::memcpy(hs, send_sizes, sizeof(uint64_t) * n);
  uint64_t *ds = c->d_sizes + 2 * n * (size_t)(1 + k);
  HIPX_TRY(c, hipMemcpyAsync(ds, hs, sizeof(uint64_t) * n, hipMemcpyHostToDevice, st));
  NCCL_TRY(c, ncclGroupStart());
  for (int p = 0; p < c->nranks; ++p) {
    NCCL_TRY_G(c, ncclSend(ds + p, 1, ncclUint64, p, c->comm, st));
    NCCL_TRY_G(c, ncclRecv(ds + n + p, 1, ncclUint64, p, c->comm, st));
  }
  NCCL_TRY(c, ncclGroupEnd());
  HIPX_TRY(c, hipMemcpyAsync(recv_sizes, ds + n, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, st));
  HIPX_TRY(c, hipEventRecord(c->ev[k], st));
  return PSX_OK;
}

// One grouped all-to-all-v: peer p gets send_sizes[p] bytes from send + sdis[p] and this rank
// receives recv_sizes[p] bytes from p at recv + rdis[p].  Each sub-stream crosses in pieces
// of at most kPiece bytes (sends and receives to one peer match in issue order inside the
// group): this RCCL (2.26) delivers a single point-to-point transfer of ~2 GiB corrupted
// (measured: a 2,147,481,620-byte self send/recv arrived wrong while the same bytes in
// 512 MiB pieces arrive intact, tests/test_split_gpu.py::test_rccl_exchange_large_sub_stream_in_pieces).
static psx_status exchange_v(psx_comm *c, const void *send, const uint64_t *send_sizes, const uint64_t *sdis,
                             void *recv, const uint64_t *recv_sizes, const uint64_t *rdis, hipStream_t st) {
  constexpr uint64_t kPiece = (uint64_t)512 << 20;
  NCCL_TRY(c, ncclGroupStart());
  for (int p = 0; p < c->nranks; ++p) {
    for (uint64_t o = 0; o < send_sizes[p]; o += kPiece) {
      const uint64_t n = send_sizes[p] - o < kPiece ? send_sizes[p] - o : kPiece;
      NCCL_TRY_G(c, ncclSend((const uint8_t *)send + sdis[p] + o, n, ncclUint8, p, c->comm, st));
    }
    for (uint64_t o = 0; o < recv_sizes[p]; o += kPiece) {
      const uint64_t n = recv_sizes[p] - o < kPiece ? recv_sizes[p] - o : kPiece;
      NCCL_TRY_G(c, ncclRecv((uint8_t *)recv + rdis[p] + o, n, ncclUint8, p, c->comm, st));
    }
  }
  NCCL_TRY(c, ncclGroupEnd());
  for (int p = 0; p < c->nranks; ++p) {
    c->sent[p] += send_sizes[p];
    c->recvd[p] += recv_sizes[p];
  }
  return PSX_OK;
}

psx_status psx_exchange_streams(psx_comm *c, const void *send, const uint64_t *send_sizes, void *recv,
                                const uint64_t *recv_sizes, void *hip_stream) {
  if (!c || !send_sizes || !recv_sizes) return PSX_ERR_INVALID_ARG;
  for (int p = 0; p < c->nranks; ++p)
    if ((send_sizes[p] && !send) || (recv_sizes[p] && !recv))
      return comm_fail(c, "exchange_streams: null buffer with a nonzero size", PSX_ERR_INVALID_ARG);
  HIPX_TRY(c, hipSetDevice(c->device));
  std::vector<uint64_t> sdis((size_t)c->nranks), rdis((size_t)c->nranks);
  uint64_t so = 0, ro = 0;
  for (int p = 0; p < c->nranks; ++p) {
    sdis[p] = so;
    rdis[p] = ro;
    so += send_sizes[p];
    ro += recv_sizes[p];
  }
  return exchange_v(c, send, send_sizes, sdis.data(), recv, recv_sizes, rdis.data(), (hipStream_t)hip_stream);
}

psx_status psx_exchange_streams_v(psx_comm *c, const void *send, const uint64_t *send_sizes,
                                  const uint64_t *send_displs, void *recv, const uint64_t *recv_sizes,
                                  const uint64_t *recv_displs, void *hip_stream) {
  if (!c || !send_sizes || !recv_sizes || !send_displs || !recv_displs) return PSX_ERR_INVALID_ARG;
  for (int p = 0; p < c->nranks; ++p)
    if ((send_sizes[p] && !send) || (recv_sizes[p] && !recv))
      return comm_fail(c, "exchange_streams_v: null buffer with a nonzero size", PSX_ERR_INVALID_ARG);
  HIPX_TRY(c, hipSetDevice(c->device));
  return exchange_v(c, send, send_sizes, send_displs, recv, recv_sizes, recv_displs, (hipStream_t)hip_stream);
}

static int find_rccl(struct dl_phdr_info *info, size_t, void *out) {
  if (info->dlpi_name && std::strstr(info->dlpi_name, "librccl")) {
    *(std::string *)out = info->dlpi_name;
    return 1;
  }
  return 0;
}

psx_status psx_comm_info(psx_comm *c, int32_t *nranks, int32_t *rank, int32_t *device, int32_t *version,
                         char *path, size_t path_cap) {
  if (!c || !c->comm) return PSX_ERR_INVALID_ARG;
  int n = 0, r = 0, d = 0, v = 0;
  NCCL_TRY(c, ncclCommCount(c->comm, &n));
  NCCL_TRY(c, ncclCommUserRank(c->comm, &r));
  NCCL_TRY(c, ncclCommCuDevice(c->comm, &d));
  NCCL_TRY(c, ncclGetVersion(&v));
  if (nranks) *nranks = n;
  if (rank) *rank = r;
  if (device) *device = d;
  if (version) *version = v;
  if (path && path_cap) {
    std::string p;
    dl_iterate_phdr(find_rccl, &p);
    const size_t k = p.size() < path_cap - 1 ? p.size() : path_cap - 1;
    std::memcpy(path, p.data(), k);
    path[k] = 0;
  }
  return PSX_OK;
}

psx_status psx_comm_peer_bytes(psx_comm *c, uint64_t *sent, uint64_t *recv, int32_t reset) {
  if (!c) return PSX_ERR_INVALID_ARG;
  for (int p = 0; p < c->nranks; ++p) {
    if (sent) sent[p] = c->sent[p];
    if (recv) recv[p] = c->recvd[p];
  }
  if (reset) {
    c->sent.assign((size_t)c->nranks, 0);
    c->recvd.assign((size_t)c->nranks, 0);
  }
  return PSX_OK;
}

}  // extern "C"
