// psx_ada.hip — AdaRevision server-table logic on the device
// (src/petuum_ps/server/adarevision_server_table_logic.cpp:14-197; apps register it as
// TableInfo.server_table_logic, apps/matrixfact/src/matrixfact_adarevision.cpp:633-635).
//
// The per-row state (AdaRevisionRow, adarevision_server_table_logic.hpp:11-22:
// accum_gradients_, z_, z_max_, f32 [row_capacity] each) lives in HBM beside the table
// row; old_accum_gradients_ ((row, version) -> (accum_gradients_ when that version was
// sent, clients left), :64-67) is S slots per row: {version, count} + an f32 row image.
//
//   ada_check      (version records) every record's snapshot exists, in message order,
//                  before anything of the call is applied — kStState, all or nothing.
//   ada_new_rows   rows this call creates (touched, not present before), keyed by their
//                  first record (message, position): the order CreateRow runs in
//                  (server.cpp:154-178).  The host sorts the keys and draws each new row's
//                  N(0, 0.1) initial deltas from the table's mt19937(12345) (:30-34,43-46).
//   ada_init_rows  ServerRowCreated (:38-50): RowBatchInc_(deltas) into the zero row.
//   ada_apply      ApplyRowOpLog (:52-175): one wave per touched row, its records in
//                  message order; per element the AdaRevision step, then RowBatchInc_ of
//                  the delta (the row add, importance, VersionServerRow version_++).
//   ada_sent       ServerRowSent (:177-190): snapshot accum_gradients_ under
//                  (row, get_version()) unless that key is live (std::map::insert).
// Every f32 operation is the reference's, in its order (no contraction:
// -ffp-contract=off; sqrtf and division correctly rounded), so rows and state are
// bit-identical to the sequential reference.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <cstdint>
#include "psx_device.hpp"

namespace psx {

__device__ __forceinline__ bool ada_go(const AdaArgs &a) {
  return !(*a.call_status & (kStFatal | kStDuplicateRow)) && !(*a.sticky & kStDuplicateRow);
}

// Rows created by this call: touched by some message and not present before it.
__global__ void __launch_bounds__(256) ada_new_rows_kernel(AdaArgs a) {
  const int lane = threadIdx.x & 63;
  const bool go = ada_go(a);
  const int64_t G = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63); base < a.max_rows; base += G) {
    const int64_t s = base + lane;
    bool fresh = false;
    uint64_t key = 0;
    if (go && s < a.max_rows && !(a.flags[s] & 1)) {
      for (int b = 0; b < a.B; ++b) {
        const int32_t i = a.inv[s * a.inv_ss + b * a.inv_sb];
        if (i >= 0) {
          fresh = true;
          key = ((uint64_t)b << 32) | (uint32_t)i;
          break;
        }
      }
    }
    const uint64_t m = __ballot(fresh);
    if (m) {
      const int leader = __builtin_ctzll(m);
      uint32_t pos = 0;
      if (lane == leader) pos = atomicAdd(a.words + 1, (uint32_t)__builtin_popcountll(m));
      pos = __builtin_amdgcn_readlane(pos, leader);
      if (fresh) {
        const uint32_t r = pos + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1));
        a.new_keys[r] = key;
        a.new_slots[r] = (int32_t)s;
      }
    }
  }
}

// ServerRowCreated's RowBatchInc_ (:47-48): the new (zeroed) row += its initial deltas.
__global__ void __launch_bounds__(256) ada_init_rows_kernel(AdaArgs a, const int32_t *slots, const float *deltas,
                                                           int32_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t r = w0; r < n; r += nw) {
    const int64_t s = slots[r];
    float *row = a.table + s * a.cap;
    const float *d = deltas + r * a.cap;
    double p = 0.0;
    for (int64_t e = lane; e < a.cap; e += 64) {
      const float x = row[e], u = d[e];
      if (a.imp) p += imp_term<float>(x, u);
      row[e] = x + u;
    }
    if (a.imp) {
      const double tot = a.imp[s] + wave_sum_f64(p);
      if (lane == 0) a.imp[s] = tot;
    }
    if (lane == 0) {
      if (a.ver) a.ver[s] += 1;
      a.flags[s] = 3;   // exists | dirty
    }
  }
}

__device__ __forceinline__ uint64_t ld_u64(const uint8_t *p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

// State check (all-or-nothing error contract): before anything of the call is applied,
// replay every touched row's snapshot bookkeeping in message order — each versioned
// record must name a live (row, version) snapshot (old_accum_gradients_.find, :114-116),
// and an end_of_version record releases one client of it (:165-170), which can retire the
// snapshot for the records after it.  A miss sets kStState; ada_apply then skips the call.
// Reads the inverse index without restoring it (ada_apply does that).
__global__ void __launch_bounds__(256) ada_check_kernel(AdaArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  if (!ada_go(a)) return;
  const int S = a.S;
  const int64_t ntiles = (a.max_rows + 63) / 64;
  for (int64_t tile = wave_g; tile < ntiles; tile += nwaves) {
    const int64_t my = tile * 64 + lane;
    const bool mine = my < a.max_rows;
    int32_t idx[kMaxFused];
    bool touched = false;
#pragma unroll
    for (int b = 0; b < kMaxFused; ++b) {
      idx[b] = (b < a.B && mine) ? a.inv[my * a.inv_ss + b * a.inv_sb] : -1;
      touched = touched || idx[b] >= 0;
    }
    uint64_t live = __ballot(touched);
    while (live) {
      const int k = __builtin_ctzll(live);
      live &= live - 1;
      const int64_t s = tile * 64 + k;
      const bool qlane = lane < S;
      const uint64_t sv = qlane ? a.snap_ver[s * S + lane] : 0;
      uint64_t sc = qlane ? a.snap_cnt[s * S + lane] : 0;
#pragma unroll
      for (int b = 0; b < kMaxFused; ++b) {
        const int32_t i = __builtin_amdgcn_readlane(idx[b], k);
        if (b >= a.B || i < 0) continue;
        const Seg sg = a.segs[b * kMaxTables + a.t];
        const uint8_t *rec = a.ss.data[b] + sg.rec0 + 4 + (int64_t)i * a.stride;
        const uint64_t rv = ld_u64(rec + a.cap * 4);
        if (!rv) continue;
        const uint64_t hit = __ballot(qlane && sc != 0 && sv == rv);
        if (!hit) {
          if (lane == 0) atomicOr(a.call_status, kStState);
          break;
        }
        if (rec[a.cap * 4 + 8] != 0 && lane == (int)__builtin_ctzll(hit)) sc -= 1;
      }
    }
  }
}

// ApplyRowOpLog for every record of the call, with the row and its AdaRevisionRow state
// held in registers across the call's records: per touched row, a scalar pre-pass
// resolves each record (payload, snapshot, end_of_version release) in message order into
// a per-wave LDS list; then per chunk of 64*EPL elements the row, accum, z, z_max are
// loaded once, every listed record's step runs in message order, and the four arrays are
// stored once.  VEC: EPL = 4 contiguous elements per lane through 16-B accesses
// (row_capacity % 4 == 0; records are only byte-aligned behind version trailers: gfx950
// runs with unaligned access enabled).
template <bool IMP, int EPL, int OCC = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC))) ada_apply_v2_kernel(AdaArgs a) {
  constexpr int UNR = (OCC > 5 || EPL != 4 || IMP) ? 1 : 2;   // records in flight per element chunk
  __shared__ int32_t s_idx[4][kMaxFused][64];   // the tile's inverse-index entries
  __shared__ const uint8_t *s_rec[4][kMaxFused];
  __shared__ const float *s_old[4][kMaxFused];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + w;
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const bool skip = !ada_go(a);
  const int S = a.S;
  const float step = a.step;
  const int64_t ntiles = (a.max_rows + 63) / 64;
  for (int64_t tile = wave_g; tile < ntiles; tile += nwaves) {
    const int64_t my = tile * 64 + lane;
    const bool mine = my < a.max_rows;
    bool touched = false;
    uint64_t nrec = 0;
    for (int b = 0; b < a.B; ++b) {
      int32_t v = -1;
      if (mine) {
        int32_t *p = a.inv + my * a.inv_ss + b * a.inv_sb;
        v = *p;
        if (v >= 0) {
          touched = true;
          ++nrec;
          *p = -1;
        }
      }
      s_idx[w][b][lane] = v;
    }
    if (skip) continue;
    if (touched) {
      a.flags[my] = 3;
      if (a.ver) a.ver[my] += nrec;
    }
    uint64_t live = __ballot(touched);
    while (live) {
      const int k = __builtin_ctzll(live);
      live &= live - 1;
      const int64_t s = tile * 64 + k;
      bool snap_dirty = false;
      // the row's snapshot slots, slot q in lane q
      const bool qlane = lane < S;
      const uint64_t sv = qlane ? a.snap_ver[s * S + lane] : 0;
      uint64_t sc = qlane ? a.snap_cnt[s * S + lane] : 0;
      int nb = 0;
      for (int b = 0; b < a.B; ++b) {
        const int32_t i = __builtin_amdgcn_readfirstlane(s_idx[w][b][k]);
        if (i < 0) continue;
        const Seg sg = a.segs[b * kMaxTables + a.t];
        const uint8_t *rec = a.ss.data[b] + sg.rec0 + 4 + (int64_t)i * a.stride;
        const float *old = nullptr;
        if (a.version_records) {
          const uint64_t rv = ld_u64(rec + a.cap * 4);
          const bool eov = rec[a.cap * 4 + 8] != 0;
          if (rv) {
            const uint64_t hit = __ballot(qlane && sc != 0 && sv == rv);
            if (!hit) {
              if (lane == 0) atomicOr(a.call_status, kStState);
              continue;
            }
            const int q0 = __builtin_ctzll(hit);
            old = a.snap_acc + (s * S + q0) * a.cap;
            if (eov) {
              if (lane == q0) {
                sc -= 1;
                if (sc == 0) atomicSub(a.words, 1u);
              }
              snap_dirty = true;
            }
          }
        }
        s_rec[w][nb] = rec;   // every lane stores the same (wave-uniform) entry
        s_old[w][nb] = old;
        ++nb;
      }
      float *row = a.table + s * a.cap;
      float *acc = a.acc + s * a.cap, *z = a.z + s * a.cap, *zmax = a.zmax + s * a.cap;
      double impt = IMP ? a.imp[s] : 0.0;
      for (int64_t e = (int64_t)lane * EPL; e < a.cap; e += 64 * EPL) {
        float x[EPL], ac[EPL], zz[EPL], zm[EPL], eta[EPL];
        __builtin_memcpy(x, row + e, 4 * EPL);
        __builtin_memcpy(ac, acc + e, 4 * EPL);
        __builtin_memcpy(zz, z + e, 4 * EPL);
        __builtin_memcpy(zm, zmax + e, 4 * EPL);
        // step/sqrt(z_max) of the current z_max: a record's eta_old is the previous
        // record's eta (same operands, same correctly rounded result)
#pragma unroll
        for (int j = 0; j < EPL; ++j) eta[j] = step / sqrtf(zm[j]);
#pragma unroll UNR
        for (int r = 0; r < nb; ++r) {
          const uint8_t *rec = s_rec[w][r];
          const float *op = s_old[w][r];
          float u[EPL], old[EPL];
          __builtin_memcpy(u, rec + e * 4, 4 * EPL);
          if (op) {
            __builtin_memcpy(old, op + e, 4 * EPL);
          } else {
#pragma unroll
            for (int j = 0; j < EPL; ++j) old[j] = 0.0f;
          }
          double p = 0.0;   // NSSumImpCalc terms of this record's chunk
#pragma unroll
          for (int j = 0; j < EPL; ++j) {
            const float g_bck = ac[j] - old[j];
            const float eta_old = eta[j];
            zz[j] = zz[j] + u[j] * (u[j] + 2.0f * g_bck);
            if (!(zz[j] < zm[j])) {   // z_max grows: a new step size
              zm[j] = zz[j];
              eta[j] = step / sqrtf(zm[j]);
            }
            const float d = -(eta[j] * u[j]) + (eta_old - eta[j]) * g_bck;
            ac[j] = ac[j] + u[j];
            if constexpr (IMP) p += imp_term<float>(x[j], d);
            x[j] = x[j] + d;
          }
          if constexpr (IMP) impt += wave_sum_f64(p);
        }
        __builtin_memcpy(row + e, x, 4 * EPL);
        __builtin_memcpy(acc + e, ac, 4 * EPL);
        __builtin_memcpy(z + e, zz, 4 * EPL);
        __builtin_memcpy(zmax + e, zm, 4 * EPL);
      }
      if (IMP && lane == 0) a.imp[s] = impt;
      if (snap_dirty && qlane) a.snap_cnt[s * S + lane] = sc;
    }
  }
}

// ServerRowSent (:177-190) for the rows in `list` (n entries) or, with list == nullptr,
// for every slot s < n whose serve-back size is non-zero (the rows a push just sent).
// check_only: report (words[2] |= kStCapacity) a row that would need a snapshot slot and
// has none, writing nothing — the push runs this before it clears any dirty bit.
// subs (optional): ServerRowSent's num_clients is the row's subscriber count
// (server_table.cpp:252-255 via CallBackSubs::AppendRowToBuffs).
__global__ void __launch_bounds__(256) ada_sent_kernel(AdaArgs a, const int32_t *list, const int64_t *sizes,
                                                      int64_t n, uint64_t clients, const uint64_t *subs,
                                                      int check_only) {
  const int lane = threadIdx.x & 63;
  const int64_t wave_g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  const int S = a.S;
  for (int64_t base = wave_g * 64; base < n; base += nwaves * 64) {
    const int64_t i = base + lane;
    int64_t mys = -1;
    if (i < n) mys = list ? (int64_t)list[i] : ((sizes[i] != 0) ? i : -1);
    uint64_t live = __ballot(mys >= 0);
    while (live) {
      const int k = __builtin_ctzll(live);
      live &= live - 1;
      const int64_t s = (int64_t)__builtin_amdgcn_readlane((int32_t)mys, k);
      const uint64_t v = a.ver ? a.ver[s] : 0;   // row->get_version() (abstract_server_row.hpp:71)
      int hit = -1, fr = -1;
      for (int q = 0; q < S; ++q) {
        const uint64_t c = a.snap_cnt[s * S + q];
        if (c && a.snap_ver[s * S + q] == v) hit = q;
        if (!c && fr < 0) fr = q;
      }
      if (hit >= 0) continue;   // std::map::insert keeps the live entry
      if (fr < 0) {
        if (lane == 0) atomicOr(a.words + 2, kStCapacity);
        continue;
      }
      if (check_only) continue;
      const uint64_t nc = subs ? (uint64_t)__builtin_popcountll(subs[s]) : clients;
      float *dst = a.snap_acc + (s * S + fr) * a.cap;
      const float *src = a.acc + s * a.cap;
      for (int64_t e = lane; e < a.cap; e += 64) dst[e] = src[e];
      if (lane == 0) {
        a.snap_ver[s * S + fr] = v;
        a.snap_cnt[s * S + fr] = nc;
        atomicAdd(a.words, 1u);
      }
    }
  }
}

__global__ void fill_f32_kernel(float *p, int64_t n, float v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

hipError_t launch_fill_f32(float *p, int64_t n, float v, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(fill_f32_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, n, v);
  return hipGetLastError();
}

hipError_t launch_ada_new_rows(const AdaArgs &a, hipStream_t st) {
  int64_t blocks = (a.max_rows + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(ada_new_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_ada_sort(void *tmp, size_t *bytes, const uint64_t *kin, uint64_t *kout, const int32_t *vin,
                           int32_t *vout, int n, hipStream_t st) {
  return hipcub::DeviceRadixSort::SortPairs(tmp, *bytes, kin, kout, vin, vout, n, 0, 64, st);
}

hipError_t launch_ada_init_rows(const AdaArgs &a, const int32_t *slots, const float *deltas, int32_t n,
                                hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = ((int64_t)n + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ada_init_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, slots, deltas, n);
  return hipGetLastError();
}

// Register-resident state kernel: held to 6 waves/SIMD with one record in flight for f32
// rows of row_capacity % 4 == 0 without importance (4.25-4.34 -> 3.93 ms on C2,
// profiles/r01/exp_ada_variants.txt).
hipError_t launch_ada_apply(const AdaArgs &a, hipStream_t st) {
  const int64_t tiles = (a.max_rows + 63) / 64;
  int64_t blocks = (tiles + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  const bool vec = a.cap % 4 == 0;
  if (vec && !a.imp)
    hipLaunchKernelGGL((ada_apply_v2_kernel<false, 4, 6>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (a.imp && vec)
    hipLaunchKernelGGL((ada_apply_v2_kernel<true, 4>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else if (a.imp)
    hipLaunchKernelGGL((ada_apply_v2_kernel<true, 1>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((ada_apply_v2_kernel<false, 1>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_ada_check(const AdaArgs &a, hipStream_t st) {
  const int64_t tiles = (a.max_rows + 63) / 64;
  int64_t blocks = (tiles + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(ada_check_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_ada_sent(const AdaArgs &a, const int32_t *list, const int64_t *sizes, int64_t n,
                           uint64_t clients, const uint64_t *subs, int check_only, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(ada_sent_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a, list, sizes, n, clients, subs,
                     check_only);
  return hipGetLastError();
}

}  // namespace psx
