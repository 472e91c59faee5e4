// Register-resident fused gaussian: ALL repetitions of a single-band frame in
// ONE launch, every tile held in registers from the first step to the last.
//
// The tile kernel (stencil_swar.hip) relaunches every K steps: each launch
// reloads its whole trapezoid from the frame and stores its kept rows (the
// "memory phase", ~7 us of a ~27 us launch on the headline frame) and pays a
// dispatch + drain (~3 us).  Here a tile loads once, then after every K-step
// phase exchanges only its halo RING with the eight neighbouring tiles through
// memory and keeps going (the reference relaunches per repetition and copies
// the whole image back and forth: cuda/cuda_convolution.cu:66-87).
//
// Per phase p (K steps, the last one possibly fewer):
//   * compute K steps of swar_step (same arithmetic as the tile kernel);
//   * publish: the tile's owned rows within K of its top / bottom (all owned
//     lanes) and its owned lanes within hl of its sides (all owned rows) are
//     stored WRITE-THROUGH (sc1) at their frame positions in frame F(p)
//     (p odd: f1, even: f0 — f0 is the input; a tile writes f0 only after its
//     neighbours finished their initial loads, see the flags), every storing
//     wave drains (vmcnt 0), a barrier, then ONE lane stores the tile's flag
//     = epoch + p (sc1);
//   * consume: one wave polls the neighbours' flags (relaxed sc1 loads,
//     s_sleep, bounded by a wall-clock timeout), ONE agent-scope acquire, a
//     barrier, then every wave reloads its halo lanes / rows from F(p).
//   This is the write-through publish / acquire-consume hand-off of
//   cdna_hip_programming.md Guideline 16 (valid for any workgroup-to-XCD
//   placement).  Double buffering by phase parity: a tile overwrites F(p)
//   positions again only at phase p+2, after its neighbours' p+1 flags, which
//   they set after reading phase p's ring.
//   The last phase stores the whole owned region to F(P) with plain stores.
//
// Co-residency: every tile waits on its neighbours, so the grid must be fully
// resident: the host sizes the tile so that the grid has at most one
// workgroup per CU and uses this kernel only on an otherwise idle device
// (single-image loops).  Every wait is bounded: on timeout the kernel sets
// the error word (host pinned memory) and all waves exit; the host throws.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "pconv/device.hpp"
#include "swar.hpp"
#include "swar_device.hpp"

namespace pconv {
namespace {

using gu32 = __attribute__((address_space(1))) uint32_t;

__device__ __forceinline__ void store_wt(uint8_t* p, u32 v) {
  __hip_atomic_store((gu32*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 load_wt(const uint8_t* p) {
  return __hip_atomic_load((const gu32*)(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int CH, int M, int NW>
__global__ __launch_bounds__(64 * NW) void k_resident(uint8_t* f0, uint8_t* f1, int64_t pitch, int row_bytes,
                                                      int height, int reps, int K, ResidentGeom g, uint32_t* flags,
                                                      uint32_t epoch, uint32_t* err, long long timeout_ticks,
                                                      int acquire) {
  constexpr int NP = 4;  // 4-byte lanes
  __shared__ uint4 lds[2][NW][2][NP / 4][64];
  __shared__ int abort_flag;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = g.hl, vrows = g.vrows;
  const int tile = static_cast<int>(blockIdx.x);
  const int col = tile / g.row_tiles, rtile = tile - col * g.row_tiles;
  const int sA = col, sB = col + g.pair_stride;
  const bool hasB = sB < g.nstrips;
  const int baseA = sA * g.vbytes - hl * 4, baseB = sB * g.vbytes - hl * 4;
  const int xA = baseA + lane * 4, xB = baseB + lane * 4;
  // row_bytes % 4 == 0 (host check): a lane's 4-byte chunk is whole or absent
  const bool okA = xA >= 0 && xA + 4 <= row_bytes;
  const bool okB = hasB && xB >= 0 && xB + 4 <= row_bytes;
  const bool needs_mask = baseA < 0 || baseA + 256 > row_bytes || !hasB || baseB + 256 > row_bytes;
  u32 cm[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) cm[k] = (okA ? 0xffffu : 0u) | (okB ? 0xffff0000u : 0u);

  const int tile_r0 = rtile * vrows;
  const int row_base = tile_r0 - K + w * M;
  const int own_hi = min(tile_r0 + vrows, height);
  const int out_top = min(max(-row_base, 0), M);
  const int out_bot = min(max(height - row_base, 0), M);
  const bool lane_in = lane >= hl && lane < 64 - hl;
  const bool side = lane_in && (lane < 2 * hl || lane >= 64 - 2 * hl);

  u32 D[M][NP];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    const bool rok = fr >= 0 && fr < height;
    const uint8_t* rowp = f0 + static_cast<int64_t>(fr) * pitch;
    const u32 a = rok && okA ? *reinterpret_cast<const u32*>(rowp + xA) : 0u;
    const u32 b = rok && okB ? *reinterpret_cast<const u32*>(rowp + xB) : 0u;
    unpack<NP>(a, b, D[i]);
  }

  // Wave 0, lanes 0..11: the neighbour tile each lane watches (columns
  // col-1, col, col+1 and the strip-pair wrap partner x rows rtile-1..+1).
  int nb = -1;
  if (w == 0 && lane < 12) {
    const int dc = lane / 3, r = rtile + lane % 3 - 1;
    const int c = dc == 0   ? col - 1
                  : dc == 1 ? col
                  : dc == 2 ? col + 1
                            : (col == 0 ? g.pair_stride - 1 : (col == g.pair_stride - 1 ? 0 : -1));
    if (c >= 0 && c < g.pair_stride && r >= 0 && r < g.row_tiles && !(c == col && r == rtile)) nb = c * g.row_tiles + r;
  }
  if (threadIdx.x == 0) abort_flag = 0;  // read only after later barriers

  const int phases = (reps + K - 1) / K;
  for (int p = 1; p <= phases; ++p) {
    const int steps = min(K, reps - (p - 1) * K);
    int t = 0;
    for (; t + 2 <= steps; t += 2) {
      swar_step<CH, NP, M, NW, 1>(D, lds, 0, w, lane, needs_mask, cm, out_top, out_bot);
      swar_step<CH, NP, M, NW, 2>(D, lds, 1, w, lane, needs_mask, cm, out_top, out_bot);
    }
    if (t < steps) swar_step<CH, NP, M, NW, 0>(D, lds, 0, w, lane, needs_mask, cm, out_top, out_bot);

    uint8_t* G = (p & 1) ? f1 : f0;
    // Re-materialise the row geometry here: without the barrier the compiler
    // hoists the per-row ring / reload predicates out of the phase loop and
    // keeps them live through the steps (hundreds of spilled SGPRs).
    int rbase = row_base, t0r = tile_r0, ohi = own_hi, kk = K, vr = vrows;
    asm volatile("" : "+s"(rbase), "+s"(t0r), "+s"(ohi), "+s"(kk), "+s"(vr));
    if (p == phases) {  // the result: every owned byte, plain stores
#pragma unroll
      for (int i = 0; i < M; ++i) {
        const int fr = rbase + i;
        if (fr >= t0r && fr < ohi && lane_in) {
          u32 a, b;
          pack<NP>(D[i], a, b);
          uint8_t* rowq = G + static_cast<int64_t>(fr) * pitch;
          if (okA) *reinterpret_cast<u32*>(rowq + xA) = a;
          if (okB) *reinterpret_cast<u32*>(rowq + xB) = b;
        }
      }
      break;
    }
    // publish the ring, write-through
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int fr = rbase + i;
      const bool vring = fr < t0r + kk || fr >= t0r + vr - kk;
      if (fr >= t0r && fr < ohi && (vring ? lane_in : side)) {
        u32 a, b;
        pack<NP>(D[i], a, b);
        uint8_t* rowq = G + static_cast<int64_t>(fr) * pitch;
        if (okA) store_wt(rowq + xA, a);
        if (okB) store_wt(rowq + xB, b);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
    __syncthreads();
    const uint32_t target = epoch + static_cast<uint32_t>(p);
    if (threadIdx.x == 0) __hip_atomic_store((gu32*)(flags + tile), target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (w == 0) {
      const long long t0 = static_cast<long long>(wall_clock64());
      while (true) {
        const bool ok = nb < 0 || static_cast<int>(__hip_atomic_load((const gu32*)(flags + nb), __ATOMIC_RELAXED,
                                                                     __HIP_MEMORY_SCOPE_AGENT) -
                                                   target) >= 0;
        if (__all(ok)) break;
        if (static_cast<long long>(wall_clock64()) - t0 > timeout_ticks) {
          if (lane == 0) {
            abort_flag = 1;
            __hip_atomic_store(err, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      // With one workgroup per CU every load of the ring is an sc1 load of
      // sc1-stored, drained, flag-published bytes: the acquire can go
      // (MI355X_MICROARCH.md, hand-off table, first row); otherwise keep it.
      if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (abort_flag) return;  // uniform: every wave read it after the barrier
    // reload the halo: rows outside the owned range (all lanes), halo lanes
    // of owned rows; rows outside the image stay zero (re-zeroed every step)
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const int fr = rbase + i;
      const bool rok = fr >= 0 && fr < height;
      const bool hrow = fr < t0r || fr >= ohi;
      if (rok && (hrow || !lane_in)) {
        const uint8_t* rowp = G + static_cast<int64_t>(fr) * pitch;
        const u32 a = okA ? load_wt(rowp + xA) : 0u;
        const u32 b = okB ? load_wt(rowp + xB) : 0u;
        unpack<NP>(a, b, D[i]);
      }
    }
  }
}

// Instantiated wave heights (8 waves per workgroup): the host takes the
// smallest M whose grid fits one workgroup per CU.
constexpr int kResidentM[] = {8, 12, 16, 20};

template <int CH, int M>
const void* resident_fn() {
  return reinterpret_cast<const void*>(&k_resident<CH, M, 8>);
}

const void* resident_kernel(int ch, int m) {
#define PCONV_RES(C_, M_) \
  if (ch == C_ && m == M_) return resident_fn<C_, M_>();
  PCONV_RES(1, 8) PCONV_RES(1, 12) PCONV_RES(1, 16) PCONV_RES(1, 20)
  PCONV_RES(3, 8) PCONV_RES(3, 12) PCONV_RES(3, 16) PCONV_RES(3, 20)
  PCONV_RES(4, 8) PCONV_RES(4, 12) PCONV_RES(4, 16) PCONV_RES(4, 20)
#undef PCONV_RES
  return nullptr;
}

int device_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

}  // namespace

ResidentPlan plan_resident(Channels ch, int64_t rows, int64_t row_bytes, int steps_per_phase) {
  ResidentPlan r;
  const int c = channel_count(ch);
  const int K = steps_per_phase;
  if (K < 1 || rows < 1 || row_bytes % 4 != 0 || (c != 1 && c != 3 && c != 4)) return r;
  const int cus = device_cus();
  if (cus <= 0) return r;
  const int hl = (K * c + 3) / 4;
  const int vbytes = (64 - 2 * hl) * 4;
  if (vbytes <= 0) return r;
  const int nstrips = static_cast<int>(ceil_div<int64_t>(row_bytes, vbytes));
  const int pair_stride = (nstrips + 1) / 2;
  for (int m : kResidentM) {
    const int vrows = 8 * m - 2 * K;
    if (vrows < K) continue;  // a phase must not reach past the neighbouring tile
    const int64_t row_tiles = ceil_div<int64_t>(rows, vrows);
    if (row_tiles * pair_stride > cus) continue;
    r.ok = true;
    r.m = m;
    r.grid = static_cast<int>(row_tiles * pair_stride);
    r.geom = ResidentGeom{hl, vbytes, vrows, nstrips, pair_stride, static_cast<int>(row_tiles)};
    return r;
  }
  return r;
}

void launch_resident(const ResidentLaunch& a, Channels ch, const ResidentPlan& plan, hipStream_t stream) {
  const int c = channel_count(ch);
  PCONV_CHECK(plan.ok && a.reps >= 1 && a.row_bytes % 4 == 0, "resident kernel: unsupported launch");
  PCONV_CHECK(plan.grid <= device_cus(), "resident kernel: grid larger than the CU count");
  const void* fn = resident_kernel(c, plan.m);
  PCONV_CHECK(fn != nullptr, "resident kernel: no instantiation for this shape");
  int per_cu = 0;
  PCONV_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 512, 0));
  PCONV_CHECK(per_cu >= 1, "resident kernel: a workgroup does not fit a CU");
  const int acquire = (per_cu > 1 || a.force_acquire) ? 1 : 0;
  const int rb = static_cast<int>(a.row_bytes), h = static_cast<int>(a.height);
  const long long timeout = static_cast<long long>(a.timeout_s * 1e8);  // wall_clock64: 100 MHz
#define PCONV_RES(C_, M_)                                                                                       \
  if (c == C_ && plan.m == M_) {                                                                                \
    k_resident<C_, M_, 8><<<dim3(plan.grid), dim3(512), 0, stream>>>(a.f0, a.f1, a.pitch, rb, h, a.reps, a.K,     \
                                                                      plan.geom, a.flags, a.epoch, a.err, timeout,   \
                                                                      acquire);                                 \
    PCONV_HIP_CHECK(hipGetLastError());                                                                         \
    return;                                                                                                     \
  }
  PCONV_RES(1, 8) PCONV_RES(1, 12) PCONV_RES(1, 16) PCONV_RES(1, 20)
  PCONV_RES(3, 8) PCONV_RES(3, 12) PCONV_RES(3, 16) PCONV_RES(3, 20)
  PCONV_RES(4, 8) PCONV_RES(4, 12) PCONV_RES(4, 16) PCONV_RES(4, 20)
#undef PCONV_RES
  PCONV_FAIL("resident kernel: no instantiation for this shape");
}

}  // namespace pconv
