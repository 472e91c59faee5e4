// CDNA4 (gfx950) stencil kernels.  See include/pconv/kernels.hpp for the
// design summary and the reference kernels they replace.
//
// Packed-pair layout used by the gaussian kernels
// -----------------------------------------------
// A lane owns 16 consecutive row bytes b0..b15 (one dwordx4).  They are held
// as eight u16x2 "pairs"  P_k = (b_k, b_{k+8}), k = 0..7, so a horizontal tap
// at distance CH bytes is simply pair P_{k±CH}: no byte shuffles inside the
// arithmetic.  The CH pairs on each side (k = -CH..-1 and 8..7+CH) come from
// the neighbouring dwords.  One v_perm_b32 builds a pair, one v_pk_add_u16 +
// one v_pk_mad_u16 apply a [1,2,1] pass to two values at once.  Sums stay
// below 4080 < 2^16, the >>4 is one 32-bit shift (bytes 0 and 2 of each
// dword hold the results) and four v_perm_b32 + four v_perm_b32 repack 16
// bytes.  ~3.9 VALU ops per output byte for RGB, ~3.6 for grey.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "pconv/kernels.hpp"
#include "pconv/device.hpp"
#include "swar.hpp"

namespace pconv {
namespace {

using u32 = uint32_t;

__device__ __forceinline__ u32 perm(u32 hi, u32 lo, u32 sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

// Selector building the pair (lo.byte j, hi.byte j) zero-extended to u16x2.
__device__ __forceinline__ constexpr u32 pair_sel(int j) {
  return 0x0c000c00u | ((4u + static_cast<u32>(j)) << 16) | static_cast<u32>(j);
}

__device__ __forceinline__ u32 pk_add(u32 a, u32 b) {
  u32 r;
  asm("v_pk_add_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// 2*b + ac on both u16 halves.
__device__ __forceinline__ u32 pk_mad2(u32 b, u32 ac) {
  u32 r;
  asm("v_pk_mad_u16 %0, %1, 2, %2 op_sel_hi:[1,0,1]" : "=v"(r) : "v"(b), "v"(ac));
  return r;
}

struct Row16 {
  u32 L, d0, d1, d2, d3, R;  // bytes [-4,0) , [0,16) , [16,20)
};

// A row outside the global image reads as zeros whatever the frame holds
// there (zero-padding semantics, mpi/mpi_convolution.c:111-118): the frame
// invariant "ghost rows beyond the image edge stay zero" is then not needed
// for correctness (e.g. a band whose ghost rows a transport filled).
__device__ __forceinline__ Row16 load_row_in(const uint8_t* __restrict__ p, bool in_image) {
  Row16 r{0, 0, 0, 0, 0, 0};
  if (!in_image) return r;
  const uint4 v = *reinterpret_cast<const uint4*>(p);
  r.L = *reinterpret_cast<const u32*>(p - 4);
  r.R = *reinterpret_cast<const u32*>(p + 16);
  r.d0 = v.x;
  r.d1 = v.y;
  r.d2 = v.z;
  r.d3 = v.w;
  return r;
}

// Horizontal [1,2,1] pass at tap distance CH over the 16 owned bytes.
template <int CH>
__device__ __forceinline__ void horiz(const Row16& b, u32 (&H)[8]) {
  u32 P[8 + 2 * CH];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    P[CH + k] = perm(b.d2, b.d0, pair_sel(k));
    P[CH + 4 + k] = perm(b.d3, b.d1, pair_sel(k));
  }
#pragma unroll
  for (int j = 1; j <= CH; ++j) P[CH - j] = perm(b.d1, b.L, pair_sel(4 - j));  // (b_{-j}, b_{8-j})
#pragma unroll
  for (int j = 0; j < CH; ++j) P[CH + 8 + j] = perm(b.R, b.d2, pair_sel(j));   // (b_{8+j}, b_{16+j})
#pragma unroll
  for (int k = 0; k < 8; ++k) H[k] = pk_mad2(P[CH + k], pk_add(P[k], P[2 * CH + k]));
}

// (V >> 4) for eight pairs -> 16 bytes in natural order.
__device__ __forceinline__ uint4 pack16(const u32 (&V)[8]) {
  u32 S[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) S[k] = V[k] >> 4;  // bytes 0 and 2 hold (lo>>4, hi>>4)
  const u32 t0 = perm(S[1], S[0], 0x06020400u);  // out0 out1 out8  out9
  const u32 t1 = perm(S[3], S[2], 0x06020400u);  // out2 out3 out10 out11
  const u32 t2 = perm(S[5], S[4], 0x06020400u);  // out4 out5 out12 out13
  const u32 t3 = perm(S[7], S[6], 0x06020400u);  // out6 out7 out14 out15
  uint4 o;
  o.x = perm(t1, t0, 0x05040100u);
  o.y = perm(t3, t2, 0x05040100u);
  o.z = perm(t1, t0, 0x07060302u);
  o.w = perm(t3, t2, 0x07060302u);
  return o;
}

// Zero bytes at and beyond `valid` (1..15) of a 16-byte vector.
__device__ __forceinline__ uint4 mask_tail(uint4 o, int valid) {
  u32 w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int keep = min(max(valid - 4 * i, 0), 4);
    const u32 m = keep >= 4 ? 0xffffffffu : ((1u << (8 * keep)) - 1u);
    w[i] &= m;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------------------
// Gaussian, one repetition.  Block = 64 lanes along the row x 4 row groups;
// each lane produces 16 bytes x RPT consecutive rows.
// ---------------------------------------------------------------------------
template <int CH, int RPT>
__global__ __launch_bounds__(256) void k_binomial(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  int64_t pitch, int row_bytes, int r0, int r1, int img_lo,
                                                  int img_hi) {
  const int x = (blockIdx.x * 64 + threadIdx.x) * 16;
  const int rs = r0 + (blockIdx.y * 4 + threadIdx.y) * RPT;
  if (x >= row_bytes || rs >= r1) return;
  const int n = min(RPT, r1 - rs);
  const uint8_t* p = src + static_cast<int64_t>(rs - 1) * pitch + x;
  uint8_t* q = dst + static_cast<int64_t>(rs) * pitch + x;
  const int valid = row_bytes - x;
  auto inside = [&](int r) { return r >= img_lo && r < img_hi; };

  u32 Ha[8], Hb[8];
  horiz<CH>(load_row_in(p, inside(rs - 1)), Ha);
  horiz<CH>(load_row_in(p + pitch, inside(rs)), Hb);
  p += 2 * pitch;
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    if (i >= n) break;
    u32 Hc[8];
    horiz<CH>(load_row_in(p, inside(rs + i + 1)), Hc);
    p += pitch;
    u32 V[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) V[k] = pk_mad2(Hb[k], pk_add(Ha[k], Hc[k]));
    uint4 o = pack16(V);
    if (valid < 16) o = mask_tail(o, valid);
    *reinterpret_cast<uint4*>(q) = o;
    q += pitch;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      Ha[k] = Hb[k];
      Hb[k] = Hc[k];
    }
  }
}

// ---------------------------------------------------------------------------
// Generic 9-tap (integer-exact or float32) — one row x 16 bytes per lane.
// ---------------------------------------------------------------------------
struct Taps9 {
  int t[9];
  float w[9];
  int shift;
};

__device__ __forceinline__ u32 byte_at(const u32 (&w)[6], int b) {  // b in [-4, 20)
  return (w[(b + 4) >> 2] >> (8 * ((b + 4) & 3))) & 0xffu;
}

template <int CH, bool FLOAT>
__global__ __launch_bounds__(256) void k_generic9(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                  int64_t pitch, int row_bytes, int r0, int r1, Taps9 tp,
                                                  int img_lo, int img_hi) {
  const int x = (blockIdx.x * 64 + threadIdx.x) * 16;
  const int r = r0 + blockIdx.y * 4 + threadIdx.y;
  if (x >= row_bytes || r >= r1) return;
  u32 rows[3][6];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const int rr = r - 1 + k;
    const Row16 b = load_row_in(src + static_cast<int64_t>(rr) * pitch + x, rr >= img_lo && rr < img_hi);
    rows[k][0] = b.L;
    rows[k][1] = b.d0;
    rows[k][2] = b.d1;
    rows[k][3] = b.d2;
    rows[k][4] = b.d3;
    rows[k][5] = b.R;
  }
  u32 out[4] = {0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    u32 v;
    if constexpr (FLOAT) {
#pragma clang fp contract(off)  // multiply-then-add, one rounding each (reference x86 semantics)
      float acc = 0.0f;
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int l = 0; l < 3; ++l) {
          const float pv = static_cast<float>(byte_at(rows[k], j + (l - 1) * CH));
          acc = __fadd_rn(acc, __fmul_rn(pv, tp.w[k * 3 + l]));  // reference order, no FMA
        }
      v = acc > 0.0f ? (acc >= 255.0f ? 255u : static_cast<u32>(acc)) : 0u;
    } else {
      int acc = 0;
#pragma unroll
      for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int l = 0; l < 3; ++l) acc += tp.t[k * 3 + l] * static_cast<int>(byte_at(rows[k], j + (l - 1) * CH));
      v = static_cast<u32>(min(acc >> tp.shift, 255));
    }
    out[j >> 2] |= v << (8 * (j & 3));
  }
  uint4 o = make_uint4(out[0], out[1], out[2], out[3]);
  const int valid = row_bytes - x;
  if (valid < 16) o = mask_tail(o, valid);
  *reinterpret_cast<uint4*>(dst + static_cast<int64_t>(r) * pitch + x) = o;
}

constexpr int kRowsPerLane = 4;

template <int CH>
void launch_ch(const Filter& f, const StencilLaunch& a, hipStream_t s, KernelVariant v) {
  const int rows = static_cast<int>(a.r1 - a.r0);
  // frame rows inside the global image (clamped to the frame; 32-bit indices checked by the caller)
  const int lo = static_cast<int>(std::max<int64_t>(-a.g_row0, a.frame_lo));
  const int hi = static_cast<int>(std::min<int64_t>(a.height - a.g_row0, a.frame_hi));
  const int chunks = static_cast<int>(ceil_div<int64_t>(a.row_bytes, 16));
  const dim3 block(64, 4);
  if (v == KernelVariant::Binomial) {
    const dim3 grid(ceil_div(chunks, 64), ceil_div(rows, 4 * kRowsPerLane));
    k_binomial<CH, kRowsPerLane><<<grid, block, 0, s>>>(a.src, a.dst, a.pitch, static_cast<int>(a.row_bytes),
                                                         static_cast<int>(a.r0), static_cast<int>(a.r1), lo, hi);
  } else {
    Taps9 tp;
    for (int i = 0; i < 9; ++i) {
      tp.t[i] = f.taps[i];
      tp.w[i] = f.weights[i];
    }
    tp.shift = f.shift;
    const dim3 grid(ceil_div(chunks, 64), ceil_div(rows, 4));
    if (v == KernelVariant::Float9)
      k_generic9<CH, true><<<grid, block, 0, s>>>(a.src, a.dst, a.pitch, static_cast<int>(a.row_bytes),
                                                  static_cast<int>(a.r0), static_cast<int>(a.r1), tp, lo, hi);
    else
      k_generic9<CH, false><<<grid, block, 0, s>>>(a.src, a.dst, a.pitch, static_cast<int>(a.row_bytes),
                                                   static_cast<int>(a.r0), static_cast<int>(a.r1), tp, lo, hi);
  }
}

}  // namespace

const char* kernel_variant_name(KernelVariant v) {
  switch (v) {
    case KernelVariant::Auto: return "auto";
    case KernelVariant::Binomial: return "binomial";
    case KernelVariant::Temporal: return "temporal";
    case KernelVariant::Int9: return "int9";
    case KernelVariant::Float9: return "float9";
    case KernelVariant::FloatTemporal: return "float_temporal";
  }
  return "?";
}

bool supports_fusion(const Filter& f, KernelVariant v) {
  if (f.binomial121)
    return v == KernelVariant::Auto || v == KernelVariant::Temporal;
  // any other filter: the float temporal kernel (reference float32 semantics)
  return v == KernelVariant::Auto || v == KernelVariant::FloatTemporal;
}

int auto_fuse(const Filter& f, KernelVariant v, int64_t frame_bytes, int channels) {
  if (!supports_fusion(f, v)) return 1;
  // float temporal kernel (gpurun_out/r03/g/float_sweep.jsonl, tuned shapes):
  // grey 1920x2520 box 3.5 us/rep at 8 vs 3.9 at 4; RGB 8.0 at 4 vs 9.5 at 8
  if (!f.binomial121) return channels == 1 ? 8 : 4;
  // Grey frames far beyond the Infinity Cache: 12 repetitions per launch
  // measured 2-6 % faster than 8 in every run (32768^2: 113.2-116.2 vs
  // 116.9-121.1 us/rep over four boxes; 16384^2: 30.6 vs 32.2;
  // profiles/r02/tile_shapes.md, prefetch_kernel.md).  RGB's horizontal halo
  // is 3x wider and deeper fusion makes it slower: 8 everywhere else.
  if (channels == 1 && frame_bytes >= (int64_t(256) << 20)) return 12;
  return 8;
}


void prepare_stencil(const Filter& f, Channels ch, const StencilLaunch& a_in, hipStream_t stream, KernelVariant v) {
  StencilLaunch a = a_in;
  a.r0 = std::max(a.r0, -a.g_row0);
  a.r1 = std::min(a.r1, a.height - a.g_row0);
  if (a.r1 <= a.r0) return;
  if (v == KernelVariant::Auto && f.binomial121 && a.steps > 1) v = KernelVariant::Temporal;
  if (v == KernelVariant::Auto && !f.binomial121 && a.steps > 1) v = KernelVariant::FloatTemporal;
  if (v == KernelVariant::Temporal && f.binomial121 && a.steps <= kMaxFusedSteps) prepare_swar(a, ch, stream);
  if (v == KernelVariant::FloatTemporal && a.steps <= kMaxFusedSteps) prepare_float_temporal(f, ch, a, stream);
}

void launch_stencil(const Filter& f, Channels ch, const StencilLaunch& a_in, hipStream_t stream, KernelVariant v) {
  // Rows outside the global image stay zero: clip the output region to it.
  StencilLaunch a = a_in;
  a.r0 = std::max(a.r0, -a.g_row0);
  a.r1 = std::min(a.r1, a.height - a.g_row0);
  if (a.r1 <= a.r0) return;
  // Geometry guards: every access of the launch must stay inside the frame.
  PCONV_CHECK(a.src && a.dst && a.src != a.dst, "launch_stencil: bad buffers");
  PCONV_CHECK(a.steps >= 1, "launch_stencil: steps must be >= 1");
  PCONV_CHECK(a.r0 - a.steps >= a.frame_lo && a.r1 + a.steps <= a.frame_hi,
              "launch_stencil: rows [" + std::to_string(a.r0) + "," + std::to_string(a.r1) + ") +/- " +
                  std::to_string(a.steps) + " exceed frame [" + std::to_string(a.frame_lo) + "," +
                  std::to_string(a.frame_hi) + ")");
  PCONV_CHECK(a.pitch % 16 == 0 && a.pitch >= kPadLeft + round_up<int64_t>(a.row_bytes, 16) + 16,
              "launch_stencil: pitch too small for 16-byte vector access");
  PCONV_CHECK(a.row_bytes < (int64_t(1) << 31) && a.r1 - a.frame_lo < (int64_t(1) << 31),
              "launch_stencil: geometry exceeds 32-bit kernel indices");
  if (v == KernelVariant::Auto)
    v = f.binomial121 ? (a.steps > 1 ? KernelVariant::Temporal : KernelVariant::Binomial)
                      : (a.steps > 1 ? KernelVariant::FloatTemporal
                                     : (f.int_exact ? KernelVariant::Int9 : KernelVariant::Float9));
  if (v == KernelVariant::FloatTemporal) {
    launch_float_temporal(f, ch, a, stream);
    PCONV_HIP_CHECK(hipGetLastError());
    return;
  }
  PCONV_CHECK(a.steps == 1 || v == KernelVariant::Temporal,
              "launch_stencil: fused steps not supported by kernel '" + std::string(kernel_variant_name(v)) + "'");
  if (v == KernelVariant::Temporal) {
    PCONV_CHECK(f.binomial121, "temporal kernel requires the gaussian filter");
    PCONV_CHECK(a.steps <= kMaxFusedSteps, "temporal kernel: too many fused steps");
    PCONV_CHECK(a.height < (int64_t(1) << 30) && a.g_row0 < (int64_t(1) << 30), "temporal kernel: rows exceed 2^30");
    launch_swar(a, ch, stream);
    PCONV_HIP_CHECK(hipGetLastError());
    return;
  }
  if (v == KernelVariant::Binomial)
    PCONV_CHECK(f.binomial121, "binomial kernel requires the gaussian filter");
  if (v == KernelVariant::Int9)
    PCONV_CHECK(f.int_exact && f.abs_sum() * 255 < (1 << 30), "int9 kernel requires an int-exact filter");
  switch (ch) {
    case Channels::Grey: launch_ch<1>(f, a, stream, v); break;
    case Channels::Rgb: launch_ch<3>(f, a, stream, v); break;
    case Channels::Rgba: launch_ch<4>(f, a, stream, v); break;
  }
  PCONV_HIP_CHECK(hipGetLastError());
}

}  // namespace pconv
