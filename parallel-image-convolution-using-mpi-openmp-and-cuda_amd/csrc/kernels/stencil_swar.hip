// Temporal-blocked gaussian, SWAR-32 form — the production fused kernel.
//
// What it replaces: the reference launches one kernel per repetition with one
// thread per pixel, lanes walking down rows (uncoalesced), FP64 math
// (cuda/cuda_convolution.cu:9-47, 66-87).  Here one launch advances `steps`
// repetitions of a whole tile held in registers.
//
// Why SWAR-32: measured on gfx950 (tools/ubench/valu_issue.hip, exact
// encodings in inline asm), VOP1/VOP2 ops (v_add_u32, v_lshrrev_b32,
// v_and_b32 with a literal) issue one wave-instruction per ~2.5 cycles per
// SIMD, every VOP3 encoding (v_add3_u32, v_lshl_add_u32, v_perm_b32, ...) and
// every DPP op ~1.8x that, and packed 16-bit VOP3P ops (v_pk_add_u16,
// v_pk_lshrrev_b16) are slower still (tools/ubench/isa_rates.hip).  Two
// 16-bit fields in a u32 never carry into each other here (every sum stays
// below 4080 < 2^16), so plain 32-bit adds do the packed work at full rate.
//
// Layout: per row a lane holds LW u32 "pairs" P_k = (A_k, B_k): A_k is byte k
// of the lane's LW-byte chunk in column strip A, B_k the same byte of strip
// B (two strips of 64*LW bytes per wave).  The horizontal neighbour of P_k at
// distance CH is P_{k+-CH}, or — across the lane boundary — the neighbouring
// lane's register, read as the DPP source (wave_shr/wave_shl) of the add that
// consumes it.  Per pair per step (swar_device.hpp): 2 v_add_u32 horizontal
// (pair sums X_j + X_{j+CH}, then P_{k-CH} + P_k), 2 vertical (rolling pair
// sums), 2 truncation (v_lshrrev, v_and; 1.5 on average in form 1) —
// no VOP3 in the step, 2*CH of the horizontal adds per row with a DPP
// operand; the byte shuffles (v_perm) happen only when a tile is loaded and
// stored (profiles/r03/valu/).
//
// Tile: NW waves stacked vertically, wave w keeps rows [w*M, (w+1)*M); each
// step the waves swap their boundary rows through LDS (double-buffered by step
// parity: one s_barrier per step).  Garbage enters the tile from outside at
// one row / CH bytes per step and is absorbed by a `steps`-row / ceil(steps*
// CH/LW)-lane halo; rows and columns outside the image are forced to zero
// after every step (zero-padding semantics of mpi/mpi_convolution.c:111-118).
// Tile shape (LW, M, NW) comes from a latency model of one launch (see
// swar_launch_cycles) — big images get the least redundant tile, small bands
// (the 8-GPU split of a small image) get small tiles spread over all CUs.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>

#include "pconv/device.hpp"
#include "swar.hpp"
#include "swar_device.hpp"

namespace pconv {
namespace {

// The `steps` repetitions of a tile in one of two step forms (the tuner
// times both per launch geometry):
//   0: one swar_step per repetition, truncating every step;
//   1: steps in pairs keeping 16 x the truncated value in between (one AND
//      instead of shift + AND every other step), one barrier per step.
// Form 1 costs registers (up to +40 VGPRs on grey tiles).  A third form with
// ONE barrier per pair of steps (two boundary rows per side exchanged, one
// ghost row per side recomputed) never won a tuning and forced it measured
// 0-8 % slower than form 1 (round 5: headline 3.645 vs 3.377 us/rep,
// 32768^2 grey 113.8 vs 109.2; profiles/r05/d/form_ab.jsonl): removed.
template <int CH, int NP, int M, int NW, int FORM>
__device__ __forceinline__ void run_steps(u32 (&D)[M][NP], uint4 (&lds)[2][NW][2][NP / 4][64], int steps, int w,
                                          int lane, bool needs_mask, const u32 (&cm)[NP], int out_top, int out_bot) {
  if constexpr (FORM == 1) {
    int s = 0;
    for (; s + 2 <= steps; s += 2) {
      swar_step<CH, NP, M, NW, 1>(D, lds, 0, w, lane, needs_mask, cm, out_top, out_bot);
      swar_step<CH, NP, M, NW, 2>(D, lds, 1, w, lane, needs_mask, cm, out_top, out_bot);
    }
    if (s < steps) swar_step<CH, NP, M, NW, 0>(D, lds, 0, w, lane, needs_mask, cm, out_top, out_bot);
  } else {
    for (int s = 0; s < steps; ++s)
      swar_step<CH, NP, M, NW, 0>(D, lds, s & 1, w, lane, needs_mask, cm, out_top, out_bot);
  }
}

template <int CH, int LW, int M, int NW, int FORM>
__global__ __launch_bounds__(64 * NW) void k_swar(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  int64_t pitch, int row_bytes, int r0, int r1,
                                                  int steps, int g_row0, int height, int nstrips, int pair_stride,
                                                  int row_tiles, int xcd_swizzle) {
  constexpr int NP = LW;       // pairs per row per lane
  constexpr int NQ = NP / 4;   // uint4 per row per lane
  using CT = typename Chunk<NP>::T;
  // [parity][wave][boundary rows: top, bottom][quad][lane]
  __shared__ uint4 lds[2][NW][2][NQ][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = (steps * CH + LW - 1) / LW;  // halo lanes per side
  const int vbytes = (64 - 2 * hl) * LW;      // valid output bytes per strip
  // 1-D grid of pair_stride x row_tiles workgroups.  The dispatcher deals
  // consecutive workgroup ids round-robin to the 8 XCDs; with xcd_swizzle the
  // ids are remapped (bijectively) so that each XCD receives one contiguous
  // run of tiles, walked down a column strip: vertically adjacent tiles,
  // which read each other's halo rows, share an L2.
  int tile = static_cast<int>(blockIdx.x);
  if (xcd_swizzle) {
    const int nwg = static_cast<int>(gridDim.x);
    const int q = nwg >> 3, rem = nwg & 7, xcd = tile & 7, local = tile >> 3;
    tile = xcd * q + min(xcd, rem) + local;
  }
  const int col = tile / row_tiles, rtile = tile - col * row_tiles;
  const int sA = col, sB = col + pair_stride;
  const bool hasB = sB < nstrips;
  const int baseA = sA * vbytes - hl * LW, baseB = sB * vbytes - hl * LW;
  const int xA = baseA + lane * LW, xB = baseB + lane * LW;
  const int validA = (xA >= 0) ? min(max(row_bytes - xA, 0), LW) : 0;
  const int validB = (hasB && xB >= 0) ? min(max(row_bytes - xB, 0), LW) : 0;
  const bool needs_mask = baseA < 0 || baseA + 64 * LW > row_bytes || !hasB || baseB + 64 * LW > row_bytes;
  u32 cm[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) cm[k] = (k < validA ? 0xffffu : 0u) | (k < validB ? 0xffff0000u : 0u);

  const int vrows = NW * M - 2 * steps;
  const int tile_r0 = r0 + rtile * vrows;
  const int row_base = tile_r0 - steps + w * M;
  const int lo_ok = max(r0 - steps, -g_row0), hi_ok = min(r1 + steps, height - g_row0);

  u32 D[M][NP];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    const bool rok = fr >= lo_ok && fr < hi_ok;
    CT a = Chunk<NP>::zero(), b = Chunk<NP>::zero();
    const uint8_t* rowp = src + static_cast<int64_t>(fr) * pitch;
    if (rok && validA > 0) a = *reinterpret_cast<const CT*>(rowp + xA);
    if (rok && validB > 0) b = *reinterpret_cast<const CT*>(rowp + xB);
    unpack<NP>(a, b, D[i]);
  }
  const int out_top = min(max(-g_row0 - row_base, 0), M);
  const int out_bot = min(max(height - g_row0 - row_base, 0), M);

  run_steps<CH, NP, M, NW, FORM>(D, lds, steps, w, lane, needs_mask, cm, out_top, out_bot);

  const bool lane_in = lane >= hl && lane < 64 - hl;
  const bool stA = lane_in && validA > 0, stB = lane_in && validB > 0;
  const int st_lo = max(tile_r0, r0), st_hi = min(min(tile_r0 + vrows, r1), height - g_row0);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    if (fr >= st_lo && fr < st_hi) {
      CT a, b;
      pack<NP>(D[i], a, b);
      uint8_t* rowq = dst + static_cast<int64_t>(fr) * pitch;
      // Whole chunks as one store; the row's last partial chunk byte by byte
      // (dst may be a packed host buffer with no pad after the row).
      if (stA) {
        if (validA == LW)
          *reinterpret_cast<CT*>(rowq + xA) = a;
        else
          store_bytes<NP>(rowq + xA, a, validA);
      }
      if (stB) {
        if (validB == LW)
          *reinterpret_cast<CT*>(rowq + xB) = b;
        else
          store_bytes<NP>(rowq + xB, b, validB);
      }
    }
  }
}

// Buffer-op form of k_swar (4-byte lanes), one workgroup per tile.
//   Every row load and store is a raw buffer op; rows and lanes outside the
// frame get an offset past the descriptor's range, so the hardware returns
// zeros / drops the store instead of the branches k_swar takes around each
// chunk, and every wave issues exactly 2M loads and 2M stores per tile.  The
// tuner times it against k_swar (4-8 % faster on RGB frames, e.g. the
// headline 3.47 -> 3.19 us/rep; slower on grey ones, where its ALT form needs
// far more VGPRs: profiles/r02/prefetch_kernel.md).  A persistent form that
// walked several tiles per workgroup with the next tile's loads in flight
// measured 10-40 % slower on 32768^2 grey and was removed (round 5; numbers
// in docs/PERFORMANCE.md).
//   Contract (checked at launch): row_bytes % 4 == 0, source and destination
// ranges under 2 GiB.
template <int CH, int M, int NW, int FORM>
__global__ __launch_bounds__(64 * NW) void k_swar_pf(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                     int pitch, int row_bytes, int r0, int r1,
                                                     int steps, int g_row0, int height, int nstrips, int pair_stride,
                                                     int row_tiles, int xcd_swizzle) {
  constexpr int LW = 4, NP = 4, NQ = 1;
  constexpr u32 kOut = 0x80000000u;  // offset past every descriptor's range
  __shared__ uint4 lds[2][NW][2][NQ][64];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = (steps * CH + LW - 1) / LW;
  const int vbytes = (64 - 2 * hl) * LW;
  const int vrows = NW * M - 2 * steps;
  // Source rows [lo_ok, hi_ok) are readable; destination rows [r0, st_end).
  const int lo_ok = max(r0 - steps, -g_row0), hi_ok = min(r1 + steps, height - g_row0);
  const int st_end = min(r1, height - g_row0);
  const auto srsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(src) + static_cast<int64_t>(lo_ok) * pitch, 0, max(hi_ok - lo_ok, 0) * pitch, 0x00020000);
  const auto drsrc = __builtin_amdgcn_make_buffer_rsrc(dst + static_cast<int64_t>(r0) * pitch, 0,
                                                       max(st_end - r0, 0) * pitch, 0x00020000);
  // XCD-aware tile order (as k_swar): each XCD gets one contiguous run of
  // tiles walked down a column strip, so vertically adjacent tiles (which
  // read each other's halo rows) share an L2.
  int tile = static_cast<int>(blockIdx.x);
  if (xcd_swizzle) {
    const int nwg = static_cast<int>(gridDim.x);
    const int q = nwg >> 3, rem = nwg & 7, xcd = tile & 7, local = tile >> 3;
    tile = xcd * q + min(xcd, rem) + local;
  }
  const int col = tile / row_tiles, rtile = tile - col * row_tiles;
  const int sB = col + pair_stride;
  const int baseA = col * vbytes - hl * LW, baseB = sB * vbytes - hl * LW;
  const int pa0 = baseA + lane * LW, pb0 = baseB + lane * LW;
  const int xA = (pa0 >= 0 && pa0 < row_bytes) ? pa0 : -1;
  const int xB = (sB < nstrips && pb0 >= 0 && pb0 < row_bytes) ? pb0 : -1;
  const bool needs_mask = baseA < 0 || baseA + 64 * LW > row_bytes || sB >= nstrips || baseB + 64 * LW > row_bytes;
  const int row_base = r0 + rtile * vrows - steps + w * M;
  u32 D[M][NP];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    const bool rok = fr >= lo_ok && fr < hi_ok;
    const u32 ro = static_cast<u32>(fr - lo_ok) * static_cast<u32>(pitch);
    const u32 a = __builtin_amdgcn_raw_buffer_load_b32(srsrc, (rok && xA >= 0) ? ro + xA : kOut, 0, 0);
    const u32 b = __builtin_amdgcn_raw_buffer_load_b32(srsrc, (rok && xB >= 0) ? ro + xB : kOut, 0, 0);
    unpack<NP>(a, b, D[i]);
  }
  u32 cm[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k)
    cm[k] = (xA >= 0 && xA + k < row_bytes ? 0xffffu : 0u) | (xB >= 0 && xB + k < row_bytes ? 0xffff0000u : 0u);
  const int out_top = min(max(-g_row0 - row_base, 0), M);
  const int out_bot = min(max(height - g_row0 - row_base, 0), M);
  run_steps<CH, NP, M, NW, FORM>(D, lds, steps, w, lane, needs_mask, cm, out_top, out_bot);
  const bool lane_in = lane >= hl && lane < 64 - hl;
  const int tile_r0 = row_base + steps - w * M;
  const int st_lo = max(tile_r0, r0), st_hi = min(tile_r0 + vrows, st_end);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    const bool rst = fr >= st_lo && fr < st_hi;
    const u32 ro = static_cast<u32>(fr - r0) * static_cast<u32>(pitch);
    u32 a, bb;
    pack<NP>(D[i], a, bb);
    __builtin_amdgcn_raw_buffer_store_b32(a, drsrc, (rst && lane_in && xA >= 0) ? ro + xA : kOut, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b32(bb, drsrc, (rst && lane_in && xB >= 0) ? ro + xB : kOut, 0, 0);
  }
}

// Instantiated tile shapes (LW, M, NW).  Taller tiles for large frames
// (fewer ghost rows per tile) were built and timed on 32768^2 grey at fuse 12
// in round 6 and all lost to {4,20,8} (105.4 us/rep): {4,24,8} 110.4-141.6
// (3 waves/SIMD), {4,16,16} 133-137, {4,20,16} 126.6-135.8 (one 16-wave
// workgroup per CU: barrier across 16 waves); profiles/r06/b/shape_sweep.jsonl.
constexpr SwarShape kShapes[] = {
    {8, 8, 8}, {8, 8, 4}, {8, 16, 4}, {8, 4, 8},              // 8-byte lanes: large images
    {4, 8, 8}, {4, 6, 8}, {4, 5, 8}, {4, 4, 8}, {4, 3, 8}, {4, 4, 16},  // 4-byte lanes: small bands
    {4, 2, 16}, {4, 3, 16}, {8, 2, 16}, {8, 4, 16},                     // 16 waves: latency-bound bands
    {4, 16, 4}, {4, 12, 4}, {4, 16, 8}, {4, 12, 8},                     // tall waves: fewer halo rows per tile
    {4, 20, 8},
};

// Process-wide kernel settings (set_xcd_swizzle / set_swar_alt /
// set_prefetch_mode / set_swar_shape / set_autotune / set_tune_candidates;
// no environment variables).
std::atomic<int> g_xcd_swizzle{1};  // XCD-aware tile order (neutral +-2 %, kept on)

bool xcd_swizzle_enabled() { return g_xcd_swizzle.load(std::memory_order_relaxed) != 0; }

std::atomic<int> g_alt_mode{-1};  // step form: -1 tuned, else forced 0 / 1 (run_steps)

int alt_mode() { return g_alt_mode.load(std::memory_order_relaxed); }

// Step form when nothing was tuned (graph capture, autotune off): the paired
// form is faster in most measured geometries.
int default_form() { return alt_mode() >= 0 ? alt_mode() : 1; }

// Kernel of one step form.
template <int CH, int LW, int M, int NW>
auto swar_kernel(int form) {
  using F = decltype(&k_swar<CH, LW, M, NW, 0>);
  return form >= 1 ? static_cast<F>(&k_swar<CH, LW, M, NW, 1>) : static_cast<F>(&k_swar<CH, LW, M, NW, 0>);
}

template <int CH, int M, int NW>
auto swar_pf_kernel(int form) {
  using F = decltype(&k_swar_pf<CH, M, NW, 0>);
  return form >= 1 ? static_cast<F>(&k_swar_pf<CH, M, NW, 1>) : static_cast<F>(&k_swar_pf<CH, M, NW, 0>);
}

template <int CH, int LW, int M, int NW>
void launch_one(const StencilLaunch& a, hipStream_t s, int form) {
  const int steps = a.steps;
  const int hl = (steps * CH + LW - 1) / LW;
  const int vbytes = (64 - 2 * hl) * LW;
  const int vrows = M * NW - 2 * steps;
  PCONV_CHECK(vbytes > 0 && vrows > 0, "swar temporal kernel: steps too large for the tile");
  const int nstrips = static_cast<int>(ceil_div<int64_t>(a.row_bytes, vbytes));
  const int pair_stride = (nstrips + 1) / 2;
  const int row_tiles = ceil_div(static_cast<int>(a.r1 - a.r0), vrows);
  const dim3 grid(pair_stride * row_tiles);
  const int64_t hmax = std::min<int64_t>(a.height, int64_t(1) << 30);
  swar_kernel<CH, LW, M, NW>(form)<<<grid, dim3(64 * NW), 0, s>>>(
      a.src, a.dst, a.pitch, static_cast<int>(a.row_bytes),
      static_cast<int>(a.r0), static_cast<int>(a.r1), steps, static_cast<int>(a.g_row0), static_cast<int>(hmax), nstrips,
      pair_stride, row_tiles, xcd_swizzle_enabled() ? 1 : 0);
}

template <int CH>
void launch_ch(const StencilLaunch& a, hipStream_t s, SwarShape sh, int form) {
#define PCONV_SWAR(LW_, M_, NW_)                            \
  if (sh.lw == LW_ && sh.m == M_ && sh.nw == NW_) {         \
    launch_one<CH, LW_, M_, NW_>(a, s, form);               \
    return;                                                 \
  }
  PCONV_SWAR(8, 8, 8)
  PCONV_SWAR(8, 8, 4)
  PCONV_SWAR(8, 16, 4)
  PCONV_SWAR(8, 4, 8)
  PCONV_SWAR(4, 8, 8)
  PCONV_SWAR(4, 6, 8)
  PCONV_SWAR(4, 5, 8)
  PCONV_SWAR(4, 4, 8)
  PCONV_SWAR(4, 3, 8)
  PCONV_SWAR(4, 4, 16)
  PCONV_SWAR(4, 2, 16)
  PCONV_SWAR(4, 3, 16)
  PCONV_SWAR(8, 2, 16)
  PCONV_SWAR(8, 4, 16)
  PCONV_SWAR(4, 16, 4)
  PCONV_SWAR(4, 12, 4)
  PCONV_SWAR(4, 16, 8)
  PCONV_SWAR(4, 12, 8)
  PCONV_SWAR(4, 20, 8)
#undef PCONV_SWAR
  PCONV_FAIL("swar temporal kernel: unsupported tile shape");
}

// Buffer-op tile kernel (k_swar_pf): shapes instantiated.
constexpr SwarShape kPfShapes[] = {
    {4, 8, 8}, {4, 12, 4}, {4, 16, 4}, {4, 12, 8}, {4, 16, 8}, {4, 20, 8},
};

bool known_pf_shape(const SwarShape& s) {
  for (const auto& k : kPfShapes)
    if (k.lw == s.lw && k.m == s.m && k.nw == s.nw) return true;
  return false;
}

std::atomic<int> g_pf_mode{-1};  // -1 tune, 0 off, 1 forced


int pf_mode() { return g_pf_mode.load(std::memory_order_relaxed); }

// Launches the prefetch kernel can take: 4-byte lanes, whole dwords per row,
// source and destination ranges under 2 GiB (32-bit buffer offsets).
bool pf_launch_ok(const StencilLaunch& a, int steps) {
  const int64_t src_rows = (a.r1 + steps) - (a.r0 - steps), dp = a.pitch;
  return a.row_bytes % 4 == 0 && src_rows * a.pitch < (int64_t(1) << 31) && (a.r1 - a.r0) * dp < (int64_t(1) << 31);
}

template <int CH, int M, int NW>
void launch_pf_one(const StencilLaunch& a, hipStream_t s, int form) {
  const int steps = a.steps;
  const int hl = (steps * CH + 3) / 4;
  const int vbytes = (64 - 2 * hl) * 4;
  const int vrows = M * NW - 2 * steps;
  PCONV_CHECK(vbytes > 0 && vrows > 0, "swar prefetch kernel: steps too large for the tile");
  PCONV_CHECK(pf_launch_ok(a, steps), "swar prefetch kernel: needs whole dwords per row and < 2 GiB ranges");
  const int nstrips = static_cast<int>(ceil_div<int64_t>(a.row_bytes, vbytes));
  const int pair_stride = (nstrips + 1) / 2;
  const int row_tiles = ceil_div(static_cast<int>(a.r1 - a.r0), vrows);
  const int64_t ntiles = int64_t(pair_stride) * row_tiles;
  PCONV_CHECK(ntiles < (int64_t(1) << 31), "swar prefetch kernel: too many tiles");
  const int grid = static_cast<int>(ntiles);
  const int xs = xcd_swizzle_enabled() ? 1 : 0;
  const int hmax = static_cast<int>(std::min<int64_t>(a.height, int64_t(1) << 30));
  swar_pf_kernel<CH, M, NW>(form)<<<dim3(grid), dim3(64 * NW), 0, s>>>(
      a.src, a.dst, static_cast<int>(a.pitch), static_cast<int>(a.row_bytes), static_cast<int>(a.r0),
      static_cast<int>(a.r1), steps, static_cast<int>(a.g_row0), hmax, nstrips, pair_stride, row_tiles, xs);
}

// Tiles of a launch and the workgroups the prefetch kernel keeps resident.
int64_t pf_tiles(SwarShape sh, int ch, int steps, int64_t rows, int64_t row_bytes) {
  const int hl = (steps * ch + sh.lw - 1) / sh.lw;
  const int vbytes = (64 - 2 * hl) * sh.lw;
  const int vrows = sh.m * sh.nw - 2 * steps;
  if (vbytes <= 0 || vrows <= 0 || sh.lw < ch || rows <= 0) return 0;
  return ((ceil_div<int64_t>(row_bytes, vbytes) + 1) / 2) * ceil_div<int64_t>(rows, vrows);
}

template <int CH>
void launch_pf_ch(const StencilLaunch& a, hipStream_t s, SwarShape sh, int form) {
#define PCONV_PF(LW_, M_, NW_)                       \
  if (sh.lw == LW_ && sh.m == M_ && sh.nw == NW_) {  \
    launch_pf_one<CH, M_, NW_>(a, s, form);          \
    return;                                          \
  }
  PCONV_PF(4, 8, 8) PCONV_PF(4, 12, 4) PCONV_PF(4, 16, 4) PCONV_PF(4, 12, 8) PCONV_PF(4, 16, 8) PCONV_PF(4, 20, 8)
#undef PCONV_PF
  PCONV_FAIL("swar prefetch kernel: unsupported tile shape");
}

bool known_shape(const SwarShape& s) {
  for (const auto& k : kShapes)
    if (k.lw == s.lw && k.m == s.m && k.nw == s.nw) return true;
  return false;
}

// Shape override (tuning / tests): set_swar_shape().
std::mutex g_shape_mu;
bool g_have_shape = false;
SwarShape g_shape;

bool override_shape(SwarShape& out) {
  std::lock_guard<std::mutex> lk(g_shape_mu);
  if (g_have_shape) out = g_shape;
  return g_have_shape;
}

}  // namespace

void set_swar_shape(int lw, int m, int nw) {
  std::lock_guard<std::mutex> lk(g_shape_mu);
  if (lw == 0) {
    g_have_shape = false;
    return;
  }
  const SwarShape s{lw, m, nw};
  PCONV_CHECK(known_shape(s), "set_swar_shape: shape not instantiated");
  g_shape = s;
  g_have_shape = true;
}

std::vector<SwarShape> swar_shapes() { return std::vector<SwarShape>(std::begin(kShapes), std::end(kShapes)); }

namespace {

// Resources of one instantiation (VGPRs per lane, LDS bytes per workgroup)
// as the compiler built it, from the runtime (hipFuncGetAttributes), cached.
struct KernelRes {
  int vgpr = 0;
  int lds = 0;
  bool measured = false;
};

template <int CH>
KernelRes query_res(SwarShape sh, int form) {
  hipFuncAttributes at{};
  hipError_t e = hipErrorInvalidValue;
#define PCONV_SWAR(LW_, M_, NW_)                                                                     \
  if (sh.lw == LW_ && sh.m == M_ && sh.nw == NW_)                                                   \
    e = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(swar_kernel<CH, LW_, M_, NW_>(form)));
  PCONV_SWAR(8, 8, 8)
  PCONV_SWAR(8, 8, 4)
  PCONV_SWAR(8, 16, 4)
  PCONV_SWAR(8, 4, 8)
  PCONV_SWAR(4, 8, 8)
  PCONV_SWAR(4, 6, 8)
  PCONV_SWAR(4, 5, 8)
  PCONV_SWAR(4, 4, 8)
  PCONV_SWAR(4, 3, 8)
  PCONV_SWAR(4, 4, 16)
  PCONV_SWAR(4, 2, 16)
  PCONV_SWAR(4, 3, 16)
  PCONV_SWAR(8, 2, 16)
  PCONV_SWAR(8, 4, 16)
  PCONV_SWAR(4, 16, 4)
  PCONV_SWAR(4, 12, 4)
  PCONV_SWAR(4, 16, 8)
  PCONV_SWAR(4, 12, 8)
  PCONV_SWAR(4, 20, 8)
#undef PCONV_SWAR
  KernelRes r;
  if (e == hipSuccess && at.numRegs > 0) {
    r.vgpr = at.numRegs;
    r.lds = static_cast<int>(at.sharedSizeBytes);
    r.measured = true;
  } else {  // no device yet: estimate (register tile + temporaries; LDS = boundary rows)
    (void)hipGetLastError();
    r.vgpr = round_up(sh.m * sh.lw + 3 * sh.lw + 40, 8);
    r.lds = sh.nw * sh.lw * 1024;
  }
  return r;
}

KernelRes kernel_res(SwarShape sh, int ch, int form) {
  static std::mutex mu;
  static std::map<std::tuple<int, int, int, int, int>, KernelRes> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_tuple(ch, sh.lw, sh.m, sh.nw, form);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  const KernelRes r = ch == 1 ? query_res<1>(sh, form) : ch == 3 ? query_res<3>(sh, form) : query_res<4>(sh, form);
  if (r.measured) cache.emplace(key, r);  // estimates (no device) are not cached
  return r;
}

}  // namespace

// Latency model of one launch on 256 CUs x 4 SIMDs, in gfx950 cycles.
//   * VALU instructions per wave: steps x per-step row work + load/pack/store
//     (matches SQ_INSTS_VALU within ~10 %, profiles/r01/pmc_sq_*).
//   * A SIMD with k resident waves retires one wave-instruction per
//     max(k x 2.88, 5.86) / k cycles: 5.86 with one wave (issue latency),
//     2.88 once two or more overlap (tools/ubench/isa_rates.hip).
//   * Per step ~550 cycles of LDS exchange + barrier latency, ~570 cycles of
//     load latency per register row, ~17.8k cycles per launch (dispatch,
//     first loads, drain).
//   * Workgroups per CU limited by the kernel's real VGPRs and LDS
//     (hipFuncGetAttributes) and 32 waves per CU; the busiest CU sets the time.
// Constants fitted (median error 9 %) to 228 measured launches over 14 shapes,
// 4 image sizes, grey/RGB and 1-8-way bands (profiles/r01/band_shape_sweep.txt;
// tools/fit_swar_data.py + tools/fit_swar_model.py); they pick the measured
// best shape in 6 of 6 configurations of the current kernel.
void set_xcd_swizzle(bool on) { g_xcd_swizzle.store(on ? 1 : 0, std::memory_order_relaxed); }
void set_swar_alt(int mode) { g_alt_mode.store(mode < 0 ? -1 : std::min(mode, 1), std::memory_order_relaxed); }
void set_prefetch_mode(int mode) { g_pf_mode.store(mode < 0 ? -1 : mode > 0 ? 1 : 0, std::memory_order_relaxed); }
std::vector<SwarShape> swar_prefetch_shapes() { return std::vector<SwarShape>(std::begin(kPfShapes), std::end(kPfShapes)); }

SwarResources swar_resources(SwarShape s, int ch) {
  const KernelRes r = kernel_res(s, ch, default_form());
  return SwarResources{r.vgpr, r.lds, r.measured};
}

double swar_launch_cycles(SwarShape s, int steps, int ch, int64_t rows, int64_t row_bytes) {
  constexpr double kCyclesMin = 2.88, kCyclesOneWave = 5.86, kStep = 549.0, kRowLoad = 568.0, kLaunch = 17813.0;
  const int np = s.lw;
  const int hl = (steps * ch + s.lw - 1) / s.lw;
  if (2 * hl >= 64) return 1e300;
  const int64_t vbytes = (64 - 2 * hl) * s.lw;
  const int64_t pairs = (ceil_div<int64_t>(row_bytes, vbytes) + 1) / 2;
  const int vrows = s.m * s.nw - 2 * steps;
  if (vrows <= 0 || np < ch) return 1e300;
  const double g = static_cast<double>(pairs * ceil_div<int64_t>(rows, vrows));
  const KernelRes res = kernel_res(s, ch, default_form());
  const int vgpr_waves = std::max(1, std::min(8, 512 / round_up(std::max(res.vgpr, 1), 8)));
  const int lds_wgs = res.lds > 0 ? (160 * 1024) / res.lds : 8;
  const int L = std::max(1, std::min({lds_wgs, vgpr_waves * 4 / s.nw, 32 / s.nw}));
  const double per_cu = std::ceil(g / 256.0);
  const double rounds = std::ceil(per_cu / L);
  const double k = std::min<double>(per_cu, L) * s.nw / 4.0;  // waves per SIMD
  // lane-crossing operands per row: 2 x ch pair sums take a DPP source (CH of
  // the P_j, CH of the H_k, swar_device.hpp horiz); a DPP add issues at ~1.8x
  // a plain v_add_u32 (tools/ubench/valu_issue.hip), so each costs 0.8 extra
  const double cross = 1.6 * ch;
  const double stage = (s.m + 2) * (2.0 * np + cross) + s.m * 4.0 * np + 24.0;
  const double instr = steps * stage + 40.0 + 3.0 * s.m * np;
  const double round_cycles = instr * std::max(k * kCyclesMin, kCyclesOneWave) + steps * kStep + kRowLoad * s.m;
  return rounds * round_cycles + kLaunch;
}

SwarShape pick_swar_shape(int steps, int ch, int64_t rows, int64_t row_bytes) {
  SwarShape best{0, 0, 0};
  if (override_shape(best) && best.m * best.nw > 2 * steps && best.lw >= ch &&
      2 * ((steps * ch + best.lw - 1) / best.lw) < 64)
    return best;
  double best_cost = 1e300;
  for (const auto& c : kShapes) {
    const double cost = swar_launch_cycles(c, steps, ch, rows, row_bytes);
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  PCONV_CHECK(best.m > 0, "swar temporal kernel: steps too large for every tile shape");
  return best;
}

namespace {

struct SwarChoice {
  SwarShape shape;
  int form = 1;  // step form of run_steps
  int kern = 0;  // 0 tile kernel k_swar, 1 buffer-op tile kernel k_swar_pf
};

void launch_choice(const StencilLaunch& a, Channels ch, hipStream_t stream, SwarChoice c) {
  if (c.kern == 1) {
    switch (ch) {
      case Channels::Grey: launch_pf_ch<1>(a, stream, c.shape, c.form); break;
      case Channels::Rgb: launch_pf_ch<3>(a, stream, c.shape, c.form); break;
      case Channels::Rgba: launch_pf_ch<4>(a, stream, c.shape, c.form); break;
    }
    return;
  }
  switch (ch) {
    case Channels::Grey: launch_ch<1>(a, stream, c.shape, c.form); break;
    case Channels::Rgb: launch_ch<3>(a, stream, c.shape, c.form); break;
    case Channels::Rgba: launch_ch<4>(a, stream, c.shape, c.form); break;
  }
}

// Empirical tuning: the model ranks the shapes, the best few are timed in both
// step forms on the actual launch (same src -> dst, so the repeats are
// harmless: every run writes the same bytes) and the fastest (shape, form) is
// cached per (channels, steps, rows, row bytes).  Never while the stream is
// being captured into a graph (the engine tunes a step's launches first).
struct TuneKey {
  int ch, steps;
  int64_t rows, row_bytes;
  bool operator<(const TuneKey& o) const {
    return std::tie(ch, steps, rows, row_bytes) < std::tie(o.ch, o.steps, o.rows, o.row_bytes);
  }
};
std::mutex g_tune_mu;
std::map<TuneKey, SwarChoice> g_tuned;
std::atomic<int> g_autotune{1};
std::atomic<int> g_tune_candidates{6};  // model-ranked shapes timed per launch geometry

bool autotune_enabled() { return g_autotune.load(std::memory_order_relaxed) != 0; }

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

constexpr int kTuneRepeats = 3;
constexpr int kTunePasses = 2;

SwarChoice tuned_choice(const StencilLaunch& a, Channels ch, hipStream_t stream, bool may_measure) {
  const int c = channel_count(ch);
  const int64_t rows = a.r1 - a.r0;
  const int mode = alt_mode();
  SwarChoice fallback;
  fallback.form = default_form();
  if (pf_mode() == 1 && pf_launch_ok(a, a.steps) && (override_shape(fallback.shape) || !autotune_enabled())) {
    // forced prefetch kernel, untuned: the overridden shape if it has a
    // prefetch instantiation, else the first prefetch shape that runs
    if (!override_shape(fallback.shape) || !known_pf_shape(fallback.shape) ||
        pf_tiles(fallback.shape, c, a.steps, rows, a.row_bytes) == 0) {
      fallback.shape = SwarShape{0, 0, 0};
      for (const auto& p : kPfShapes)
        if (pf_tiles(p, c, a.steps, rows, a.row_bytes) > 0) {
          fallback.shape = p;
          break;
        }
    }
    if (fallback.shape.m > 0) {
      fallback.kern = 1;
      return fallback;
    }
    fallback.shape = pick_swar_shape(a.steps, c, rows, a.row_bytes);
    return fallback;
  }
  if (override_shape(fallback.shape) || !autotune_enabled()) {
    if (!override_shape(fallback.shape)) fallback.shape = pick_swar_shape(a.steps, c, rows, a.row_bytes);
    return fallback;
  }
  const TuneKey key{c, a.steps, rows, a.row_bytes};
  {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    auto it = g_tuned.find(key);
    if (it != g_tuned.end()) {
      SwarChoice r = it->second;
      if (mode >= 0) r.form = mode;  // forced form (the shape stays tuned)
      return r;
    }
  }
  fallback.shape = pick_swar_shape(a.steps, c, rows, a.row_bytes);
  if (!may_measure || capturing(stream)) return fallback;
  std::vector<std::pair<double, SwarShape>> ranked;
  for (const auto& sh : kShapes) {
    const double cost = swar_launch_cycles(sh, a.steps, c, rows, a.row_bytes);
    if (cost < 1e299) ranked.emplace_back(cost, sh);
  }
  PCONV_CHECK(!ranked.empty(), "swar temporal kernel: steps too large for every tile shape");
  std::sort(ranked.begin(), ranked.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
  // set_tune_candidates widens the timed set (A/B of the model's ranking)
  const size_t keep = static_cast<size_t>(std::max(1, g_tune_candidates.load(std::memory_order_relaxed)));
  if (ranked.size() > keep) ranked.resize(keep);
  std::vector<SwarChoice> cands;
  for (const auto& r : ranked)
    for (int form = 0; form <= 1; ++form)
      if (mode < 0 || mode == form)
        cands.push_back(SwarChoice{r.second, form, 0});
  // Buffer-op tile kernel (k_swar_pf, one workgroup per tile) for the
  // model's candidate shapes it instantiates: hardware zero-fill of rows and
  // lanes outside the frame instead of branches (measured 2-6 % faster on RGB
  // frames, slower on grey ones: profiles/r02/prefetch_kernel.md).
  if (pf_mode() != 0 && pf_launch_ok(a, a.steps)) {
    std::vector<SwarChoice> pfs;
    for (const auto& r : ranked)
      if (known_pf_shape(r.second))
        for (int form = 0; form <= 1; ++form)
          if (mode < 0 || mode == form)
            pfs.push_back(SwarChoice{r.second, form, 1});
    if (pf_mode() == 1 && !pfs.empty()) cands.clear();  // forced: only these candidates
    cands.insert(cands.end(), pfs.begin(), pfs.end());
  }
  SwarChoice best = cands.front();
  if (cands.size() > 1) {
    // Two interleaved passes, each candidate's best kept: a single pass in a
    // fixed order mis-ranked large launches (the first candidates ran while
    // clocks and caches were still settling; 32768^2 grey picked a shape 7 %
    // slower than the best).
    Event e0 = Event::create(true), e1 = Event::create(true);
    std::vector<float> t(cands.size(), 1e30f);
    for (int pass = 0; pass < kTunePasses; ++pass) {
      for (size_t i = 0; i < cands.size(); ++i) {
        if (pass == 0) launch_choice(a, ch, stream, cands[i]);  // warm (code object, caches)
        e0.record(stream);
        for (int r = 0; r < kTuneRepeats; ++r) launch_choice(a, ch, stream, cands[i]);
        e1.record(stream);
        PCONV_HIP_CHECK(hipEventSynchronize(e1.get()));
        t[i] = std::min(t[i], Event::elapsed_ms(e0, e1));
      }
    }
    best = cands[std::min_element(t.begin(), t.end()) - t.begin()];
  }
  std::lock_guard<std::mutex> lk(g_tune_mu);
  g_tuned.emplace(key, best);
  return best;
}

}  // namespace

void set_autotune(bool on) { g_autotune.store(on ? 1 : 0, std::memory_order_relaxed); }
void set_tune_candidates(int n) { g_tune_candidates.store(std::max(1, n), std::memory_order_relaxed); }
bool set_shape_tuning(bool on) {
  const bool prev = autotune_enabled();
  set_autotune(on);
  return prev;
}

bool shape_tuning_enabled() { return autotune_enabled(); }

void clear_swar_tuning() {
  {
    std::lock_guard<std::mutex> lk(g_tune_mu);
    g_tuned.clear();
  }
  clear_float_tuning();
}

std::vector<std::pair<std::vector<int64_t>, SwarShape>> swar_tuned() {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  std::vector<std::pair<std::vector<int64_t>, SwarShape>> out;
  for (const auto& kv : g_tuned)
    out.push_back({{kv.first.ch, kv.first.steps, kv.first.rows, kv.first.row_bytes, kv.second.form,
                    kv.second.kern},
                   kv.second.shape});
  return out;
}

namespace {

// 16 bytes per lane, grid-stride over (row, 16-byte chunk); rows whose start
// is not 16-byte aligned on either side fall back to dwords or bytes.
__global__ __launch_bounds__(256) void k_copy_rows(const uint8_t* __restrict__ src, int64_t sp,
                                                   uint8_t* __restrict__ dst, int64_t dp, int64_t row_bytes,
                                                   int64_t chunks_per_row, int64_t total) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int64_t y = i / chunks_per_row, x = (i - y * chunks_per_row) * 16;
    const uint8_t* s = src + y * sp + x;
    uint8_t* d = dst + y * dp + x;
    const int n = static_cast<int>(min<int64_t>(16, row_bytes - x));
    const uintptr_t al = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d);
    if (n == 16 && (al & 15) == 0) {
      *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
    } else if (n == 16 && (al & 3) == 0) {
#pragma unroll
      for (int k = 0; k < 4; ++k) reinterpret_cast<u32*>(d)[k] = reinterpret_cast<const u32*>(s)[k];
    } else {
      for (int k = 0; k < n; ++k) d[k] = s[k];
    }
  }
}

__global__ __launch_bounds__(256) void k_fill_zero(uint4* __restrict__ p, int64_t n16) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride)
    p[i] = make_uint4(0, 0, 0, 0);
}

unsigned copy_blocks(int64_t work) {
  // enough waves to keep PCIe / HBM busy (256 CUs x 8), never more than the work
  return static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(ceil_div<int64_t>(work, 256), 2048)));
}

}  // namespace

void launch_copy_rows(const uint8_t* src, int64_t sp, uint8_t* dst, int64_t dp, int64_t row_bytes, int64_t rows,
                      hipStream_t stream, int max_blocks) {
  PCONV_CHECK(row_bytes >= 0 && rows >= 0 && sp >= row_bytes && dp >= row_bytes, "copy_rows: bad geometry");
  if (row_bytes == 0 || rows == 0) return;
  const int64_t cpr = ceil_div<int64_t>(row_bytes, 16), total = cpr * rows;
  unsigned blocks = copy_blocks(total);
  if (max_blocks > 0) blocks = std::min<unsigned>(blocks, static_cast<unsigned>(max_blocks));
  k_copy_rows<<<dim3(blocks), dim3(256), 0, stream>>>(src, sp, dst, dp, row_bytes, cpr, total);
  PCONV_HIP_CHECK(hipGetLastError());
}

void launch_fill_zero(uint8_t* p, int64_t bytes, hipStream_t stream) {
  PCONV_CHECK(bytes % 16 == 0 && reinterpret_cast<uintptr_t>(p) % 16 == 0, "fill_zero: needs 16-byte granules");
  if (bytes == 0) return;
  k_fill_zero<<<dim3(copy_blocks(bytes / 16)), dim3(256), 0, stream>>>(reinterpret_cast<uint4*>(p), bytes / 16);
  PCONV_HIP_CHECK(hipGetLastError());
}

void preload_kernel_module() {
  // Any attribute query of a kernel makes the runtime load the code object of
  // its translation unit (all of this file's kernels); no GPU work is issued.
  hipFuncAttributes at{};
  if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&k_fill_zero)) != hipSuccess) (void)hipGetLastError();
}

void prepare_swar(const StencilLaunch& a, Channels ch, hipStream_t stream) { (void)tuned_choice(a, ch, stream, true); }

void launch_swar(const StencilLaunch& a, Channels ch, hipStream_t stream) {
  launch_choice(a, ch, stream, tuned_choice(a, ch, stream, true));
}

}  // namespace pconv
