// Row-streaming form of the SWAR-32 gaussian: a candidate of the launch tuner
// next to the tile kernels of stencil_swar.hip (same byte-pair layout, same
// horizontal pass and truncations: swar_device.hpp).
//
// A tile kernel holds NW x M rows of a tile in registers, recomputes a
// 2 x steps-row vertical halo per tile (15 % of the work for the 32768^2 grey
// tile {4,20,8} at 12 steps) and meets its waves at an LDS barrier every step.
// Here ONE wave walks down a column strip pair through a segment of rows and
// keeps, for every repetition level s = 1..S, the rolling state of the level
// below it: the horizontal sum of that level's newest row and the pair sum of
// its two newest rows (2 x 4 VGPRs per level).  Each row read from the frame
// advances every level by one row, so level S emits one finished row per row
// read: no LDS, no barrier, and the only vertical redundancy is an S-row ramp
// at each end of a segment (a few % for segments of several hundred rows).
// The cone argument: with the state zero-initialised, level s is exact for
// rows >= (first row read) + s, so reading from y0 - S makes level S exact
// from y0 on; rows outside the image are forced to zero at every level (the
// zero padding of mpi/mpi_convolution.c:111-118, as in the tile kernels).
//
// Two orders of the levels within one row:
//   chained (SKEW = false): level s consumes the row level s-1 produced from
//     this same input row — the S levels form one dependent chain per row,
//     ILP = the 4 pairs of a lane;
//   skewed (SKEW = true): levels run from S down to 1 and level s consumes the
//     row level s-1 produced one input row EARLIER (kept in 4 more VGPRs per
//     level), so the S levels of one row are independent of each other.
// Loads run PF rows ahead through raw buffer ops (rows outside the readable
// frame range and lanes outside the row read as zero, stores outside the
// destination range are dropped, as in k_swar_pf).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <type_traits>

#include "pconv/device.hpp"
#include "swar.hpp"
#include "swar_device.hpp"

namespace pconv {
namespace {

// Truncation of level s (1-based) of S in the paired form: odd levels keep
// 16 x floor(S/16), even levels divide the scaled sum by 256, an odd last
// level truncates plainly.
constexpr int level_mode(int s, int S) { return (s & 1) ? (s == S ? 0 : 1) : 2; }

constexpr int kWavesPerGroup = 4;

template <int CH, int S, bool SKEW>
__global__ __launch_bounds__(64 * kWavesPerGroup) void k_swar_stream(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, int pitch, int row_bytes, int r0, int r1, int g_row0,
    int height, int nstrips, int pair_stride, int nseg, int seg_rows, int ntasks, int xcd_swizzle) {
  constexpr int LW = 4, NP = 4, PF = 4;
  constexpr int HL = (S * CH + LW - 1) / LW;  // halo lanes per side
  constexpr int VB = (64 - 2 * HL) * LW;      // valid bytes per strip
  constexpr int LAG = SKEW ? 2 * S - 1 : S;   // level S emits row (read row - LAG)
  constexpr u32 kOut = 0x80000000u;           // offset past every descriptor's range
  static_assert(2 * HL < 64, "halo wider than the wave");
  const int lane = threadIdx.x & 63;
  int blk = static_cast<int>(blockIdx.x);
  if (xcd_swizzle) {  // each XCD gets one contiguous run of groups (as k_swar)
    const int nwg = static_cast<int>(gridDim.x);
    const int q = nwg >> 3, rem = nwg & 7, xcd = blk & 7, local = blk >> 3;
    blk = xcd * q + min(xcd, rem) + local;
  }
  // consecutive tasks: consecutive segments of one column strip pair
  const int task = blk * kWavesPerGroup + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (task >= ntasks) return;
  const int col = task / nseg, seg = task - col * nseg;
  const int sB = col + pair_stride;
  const int baseA = col * VB - HL * LW, baseB = sB * VB - HL * LW;
  const int pa0 = baseA + lane * LW, pb0 = baseB + lane * LW;
  const int xA = (pa0 >= 0 && pa0 < row_bytes) ? pa0 : -1;
  const int xB = (sB < nstrips && pb0 >= 0 && pb0 < row_bytes) ? pb0 : -1;
  const bool needs_mask = baseA < 0 || baseA + 64 * LW > row_bytes || sB >= nstrips || baseB + 64 * LW > row_bytes;
  u32 cm[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k)
    cm[k] = (xA >= 0 && xA + k < row_bytes ? 0xffffu : 0u) | (xB >= 0 && xB + k < row_bytes ? 0xffff0000u : 0u);
  const bool lane_in = lane >= HL && lane < 64 - HL;
  const int y0 = r0 + seg * seg_rows, y1 = min(y0 + seg_rows, r1);
  // readable source rows [lo_ok, hi_ok); destination rows [r0, st_end)
  const int lo_ok = max(r0 - S, -g_row0), hi_ok = min(r1 + S, height - g_row0);
  const int st_end = min(r1, height - g_row0);
  const int img_lo = -g_row0, img_hi = height - g_row0;
  const int st_hi = min(y1, st_end);
  const auto srsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(src) + static_cast<int64_t>(lo_ok) * pitch, 0, max(hi_ok - lo_ok, 0) * pitch, 0x00020000);
  const auto drsrc = __builtin_amdgcn_make_buffer_rsrc(dst + static_cast<int64_t>(r0) * pitch, 0,
                                                       max(st_end - r0, 0) * pitch, 0x00020000);

  u32 Hp[S][NP], Sp[S][NP];            // level s-1's newest H and newest pair sum (index s-1)
  u32 Pd[SKEW ? S : 1][NP];            // SKEW: level s's row from the previous read row (index s-1)
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      Hp[s][k] = 0;
      Sp[s][k] = 0;
      if constexpr (SKEW) Pd[s][k] = 0;
    }

  auto load = [&](int fr, u32& a, u32& b) {
    const bool rok = fr >= lo_ok && fr < hi_ok;
    const u32 ro = static_cast<u32>(fr - lo_ok) * static_cast<u32>(pitch);
    a = __builtin_amdgcn_raw_buffer_load_b32(srsrc, (rok && xA >= 0) ? ro + static_cast<u32>(xA) : kOut, 0, 0);
    b = __builtin_amdgcn_raw_buffer_load_b32(srsrc, (rok && xB >= 0) ? ro + static_cast<u32>(xB) : kOut, 0, 0);
  };
  // store offsets: lane part, kOut for lanes that store nothing (a row offset
  // < 2^31 added to kOut stays past the range without wrapping)
  const u32 sA = (lane_in && xA >= 0) ? static_cast<u32>(xA) : kOut;
  const u32 sB_ = (lane_in && xB >= 0) ? static_cast<u32>(xB) : kOut;

  // The row loop in four versions, picked once per wave: MASK (a strip pair
  // reaching past the row's ends: columns outside re-zeroed every level) x
  // EDGE (a segment whose levels reach rows outside the image: those rows
  // re-zeroed every level).  Interior waves run neither — written as
  // per-level selects the compiler spent 12 extra VALU per level on both.
  auto run = [&](auto mask_c, auto edge_c) {
    constexpr bool MASK = decltype(mask_c)::value, EDGE = decltype(edge_c)::value;
    // One level s (1-based; a compile-time constant once the level loops are
    // unrolled): X (level s-1's newest row) in, level s row `r` out in X.
    auto level = [&](int s, u32 (&X)[NP], int r) {
      u32 Hn[NP];
      horiz<CH, NP>(X, Hn);
      const int mode = level_mode(s, S);
#pragma unroll
      for (int k = 0; k < NP; ++k) {
        const u32 Sn = keep(Hp[s - 1][k] + Hn[k]);
        const u32 t = Sp[s - 1][k] + Sn;
        X[k] = mode == 0 ? trunc_sum<0>(t) : mode == 1 ? trunc_sum<1>(t) : trunc_sum<2>(t);
        Sp[s - 1][k] = Sn;
        Hp[s - 1][k] = Hn[k];
      }
      if constexpr (MASK) {
#pragma unroll
        for (int k = 0; k < NP; ++k) X[k] &= cm[k];
      }
      if constexpr (EDGE) {
        const u32 rm = (r >= img_lo && r < img_hi) ? ~0u : 0u;  // uniform
#pragma unroll
        for (int k = 0; k < NP; ++k) X[k] &= rm;
      }
    };
    const int ys = y0 - S, ye = y1 + LAG;  // rows read: [ys, ye)
    u32 qa[PF], qb[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) load(ys + u, qa[u], qb[u]);
    for (int y = ys; y < ye; y += PF) {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const int yr = y + u;
        u32 X[NP];
        unpack<NP>(qa[u], qb[u], X);
        load(yr + PF, qa[u], qb[u]);
        if constexpr (SKEW) {
          // levels S..2 from level s-1's row of the previous read row (level
          // s emits row yr - (2s - 1)); each overwrites its own pending row
          // only after level s+1 has consumed it; level 1 from the row read
          u32 T[NP];
#pragma unroll
          for (int k = 0; k < NP; ++k) T[k] = Pd[S - 2][k];
          level(S, T, yr - (2 * S - 1));
#pragma unroll
          for (int s = S - 1; s >= 2; --s) {
#pragma unroll
            for (int k = 0; k < NP; ++k) Pd[s - 1][k] = Pd[s - 2][k];
            level(s, Pd[s - 1], yr - (2 * s - 1));
          }
          level(1, X, yr - 1);
#pragma unroll
          for (int k = 0; k < NP; ++k) {
            Pd[0][k] = X[k];
            X[k] = T[k];  // level S's row, stored below
          }
        } else {
#pragma unroll
          for (int s = 1; s <= S; ++s) level(s, X, yr - s);
        }
        const int ro = yr - LAG;
        if (ro >= y0 && ro < st_hi) {
          u32 a, b;
          pack<NP>(X, a, b);
          const u32 off = static_cast<u32>(ro - r0) * static_cast<u32>(pitch);
          __builtin_amdgcn_raw_buffer_store_b32(a, drsrc, off + sA, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b32(b, drsrc, off + sB_, 0, 0);
        }
      }
    }
  };
  // every level's rows within the image: no re-zeroing of rows
  const bool edge = !(y0 - 3 * S >= img_lo && y1 + LAG <= img_hi);
  using T_ = std::true_type;
  using F_ = std::false_type;
  if (needs_mask) {
    if (edge) run(T_{}, T_{});
    else run(T_{}, F_{});
  } else {
    if (edge) run(F_{}, T_{});
    else run(F_{}, F_{});
  }
}

// Compute units of the current device (the launch's wave target), once.
int cu_count() {
  static const int n = [] {
    int d = 0, c = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess ||
        c <= 0) {
      (void)hipGetLastError();
      return 256;
    }
    return c;
  }();
  return n;
}

// Waves per SIMD the compiled kernel can keep resident (its VGPRs), once.
template <int CH, int S, bool SKEW>
int waves_per_simd() {
  static const int w = [] {
    hipFuncAttributes at{};
    if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_swar_stream<CH, S, SKEW>)) != hipSuccess ||
        at.numRegs <= 0) {
      (void)hipGetLastError();
      return 2;
    }
    return std::max(1, std::min(8, 512 / round_up(at.numRegs, 8)));
  }();
  return w;
}

// One wave per (column strip pair, row segment); segments sized so the
// launch is one round of resident waves (the kernel's occupancy on every
// CU), each at least 4 S rows long.
template <int CH, int S, bool SKEW>
void launch_stream(const StencilLaunch& a, bool xcd_swizzle, hipStream_t st) {
  constexpr int HL = (S * CH + 3) / 4, VB = (64 - 2 * HL) * 4;
  const int64_t rows = a.r1 - a.r0;
  const int64_t nstrips = ceil_div<int64_t>(a.row_bytes, VB);
  const int64_t pair_stride = (nstrips + 1) / 2;
  const int64_t target = int64_t(cu_count()) * 4 * waves_per_simd<CH, S, SKEW>();
  int64_t nseg = std::max<int64_t>(1, std::min<int64_t>(ceil_div<int64_t>(target, pair_stride),
                                                        std::max<int64_t>(1, rows / (4 * S))));
  const int64_t seg_rows = ceil_div<int64_t>(rows, nseg);
  nseg = ceil_div<int64_t>(rows, seg_rows);
  const int64_t ntasks = pair_stride * nseg;
  PCONV_CHECK(ntasks < (int64_t(1) << 31) - kWavesPerGroup, "swar stream kernel: too many tasks");
  const int grid = static_cast<int>(ceil_div<int64_t>(ntasks, kWavesPerGroup));
  const int hmax = static_cast<int>(std::min<int64_t>(a.height, int64_t(1) << 30));
  k_swar_stream<CH, S, SKEW><<<dim3(grid), dim3(64 * kWavesPerGroup), 0, st>>>(
      a.src, a.dst, static_cast<int>(a.pitch), static_cast<int>(a.row_bytes), static_cast<int>(a.r0),
      static_cast<int>(a.r1), static_cast<int>(a.g_row0), hmax, static_cast<int>(nstrips),
      static_cast<int>(pair_stride), static_cast<int>(nseg), static_cast<int>(seg_rows), static_cast<int>(ntasks),
      xcd_swizzle ? 1 : 0);
}

template <int CH, bool SKEW>
void launch_stream_ch(const StencilLaunch& a, bool xs, hipStream_t st) {
  switch (a.steps) {
    case 4: launch_stream<CH, 4, SKEW>(a, xs, st); return;
    case 8: launch_stream<CH, 8, SKEW>(a, xs, st); return;
    case 12: launch_stream<CH, 12, SKEW>(a, xs, st); return;
    default: PCONV_FAIL("swar stream kernel: steps not instantiated");
  }
}

}  // namespace

bool swar_stream_ok(const StencilLaunch& a, int ch) {
  const int64_t src_rows = (a.r1 + a.steps) - (a.r0 - a.steps);
  return (a.steps == 4 || a.steps == 8 || a.steps == 12) && (ch == 1 || ch == 3 || ch == 4) && a.r1 > a.r0 &&
         a.row_bytes % 4 == 0 && src_rows * a.pitch < (int64_t(1) << 31) &&
         (a.r1 - a.r0) * a.pitch < (int64_t(1) << 31);
}

void launch_swar_stream(const StencilLaunch& a, int ch, bool skew, bool xcd_swizzle, hipStream_t st) {
  PCONV_CHECK(swar_stream_ok(a, ch), "swar stream kernel: launch outside its contract");
  if (ch == 1) skew ? launch_stream_ch<1, true>(a, xcd_swizzle, st) : launch_stream_ch<1, false>(a, xcd_swizzle, st);
  else if (ch == 3) skew ? launch_stream_ch<3, true>(a, xcd_swizzle, st) : launch_stream_ch<3, false>(a, xcd_swizzle, st);
  else skew ? launch_stream_ch<4, true>(a, xcd_swizzle, st) : launch_stream_ch<4, false>(a, xcd_swizzle, st);
}

}  // namespace pconv
