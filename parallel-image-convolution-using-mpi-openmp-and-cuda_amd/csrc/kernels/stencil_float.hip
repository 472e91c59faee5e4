// Temporal-blocked kernel for ANY 3x3 filter in the reference's float32
// semantics (box/9 and "edge_detection"/28 of mpi/mpi_convolution.c:90-100,
// custom filters): `steps` repetitions per launch, the tile resident in
// registers between steps — one HBM/Infinity-Cache round trip per launch
// instead of per repetition (k_generic9 in stencil.hip, one launch per rep).
//
// Numerics, per output byte and step, exactly the reference's
// (mpi/mpi_convolution.c:303-307):
//   acc = 0; for k in 0..2, l in 0..2: acc = fl(acc + fl(p[k][l] * w[k*3+l]))
//   out = trunc(acc) clamped to [0, 255]
// separate multiply and add (no contraction: the TU is built with
// -ffp-contract=off; products and sums are packed f32 ops, one rounding each),
// row-major tap order, truncation after EVERY step, zero outside the image at
// every step.  UNIFORM filters (all nine weights equal, e.g. box) compute each
// input byte's product once per row instead of once per tap: fl(p * w) does
// not depend on the tap, so the chain of additions is unchanged.
//
// Tile: NW waves stacked vertically, wave w keeps M rows x 8 bytes per lane
// (a 512-byte strip per wave row) as packed bytes.  Horizontal neighbours at
// distance CH (<= 4) come from the adjacent lanes by DPP wave_shr / wave_shl;
// vertical neighbours across waves through LDS (double-buffered by step
// parity, one barrier per step).  The tile's halo (`steps` rows, ceil(steps *
// CH / 8) lanes per side) absorbs what enters from outside the tile.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "pconv/device.hpp"
#include "pconv/kernels.hpp"

namespace pconv {
namespace {

using u32 = uint32_t;

struct FloatTaps {
  float w[9];
};

__device__ __forceinline__ float ub(u32 x, int k) { return static_cast<float>((x >> (8 * k)) & 0xffu); }

// Pairs of floats (bytes j and j + 4 of a lane's 8): every operation on a pair
// is one packed f32 instruction (v_pk_mul_f32 / v_pk_add_f32), each half
// rounded exactly like its scalar twin.  The TU is built with
// -ffp-contract=off, so a product never fuses into the following add.
typedef float f2 __attribute__((ext_vector_type(2)));

// Row (8 bytes per lane) -> pairs E[j] = (byte j - CH, byte j + 4 - CH) for
// j in [0, 4 + 2 CH): bytes [-CH, 8 + CH) of the row (times w when UNIFORM).
template <int CH, bool UNIFORM>
__device__ __forceinline__ void expand(const u32 (&X)[2], float w, f2 (&E)[4 + 2 * CH]) {
  const u32 l = __builtin_amdgcn_mov_dpp(X[1], 0x138, 0xf, 0xf, true);  // wave_shr:1 -> left lane's bytes 4..7
  const u32 r = __builtin_amdgcn_mov_dpp(X[0], 0x130, 0xf, 0xf, true);  // wave_shl:1 -> right lane's bytes 0..3
  float e[8 + 2 * CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) e[j] = ub(l, 4 - CH + j);
#pragma unroll
  for (int j = 0; j < 8; ++j) e[CH + j] = ub(X[j >> 2], j & 3);
#pragma unroll
  for (int j = 0; j < CH; ++j) e[CH + 8 + j] = ub(r, j);
#pragma unroll
  for (int j = 0; j < 4 + 2 * CH; ++j) E[j] = (f2){e[j], e[j + 4]};
  if constexpr (UNIFORM) {
    const f2 ww = (f2){w, w};
#pragma unroll
    for (int j = 0; j < 4 + 2 * CH; ++j) E[j] = E[j] * ww;
  }
}

// Output bytes j and j + 4 (j < 4) as floats holding trunc(acc): integers, so
// v_cvt_pk_u8_f32 packs them exactly whatever its rounding mode, saturating
// the ones outside [0, 255].  Reference order: row k (a: above, b: this row, c: below),
// then column l.
template <int CH, bool UNIFORM>
__device__ __forceinline__ f2 out_pair(const f2 (&a)[4 + 2 * CH], const f2 (&b)[4 + 2 * CH],
                                       const f2 (&c)[4 + 2 * CH], int j, const f2 (&w)[9]) {
  f2 acc;
  if constexpr (UNIFORM) {
    acc = a[j];  // 0 + fl(p*w) is exact
    acc = acc + a[j + CH];
    acc = acc + a[j + 2 * CH];
    acc = acc + b[j];
    acc = acc + b[j + CH];
    acc = acc + b[j + 2 * CH];
    acc = acc + c[j];
    acc = acc + c[j + CH];
    acc = acc + c[j + 2 * CH];
  } else {
    acc = a[j] * w[0];
    acc = acc + a[j + CH] * w[1];
    acc = acc + a[j + 2 * CH] * w[2];
    acc = acc + b[j] * w[3];
    acc = acc + b[j + CH] * w[4];
    acc = acc + b[j + 2 * CH] * w[5];
    acc = acc + c[j] * w[6];
    acc = acc + c[j + CH] * w[7];
    acc = acc + c[j + 2 * CH] * w[8];
  }
  // reference store: float -> uint8 truncation, clamped like the CPU oracle.
  // The clamp is the packer's: v_cvt_pk_u8_f32 saturates to [0, 255]
  // (measured: -1e9, -5, -0.5 -> 0; 256, 300, 1e9 -> 255;
  // tools/ubench/cvt_pk_u8.hip, profiles/r03/float/cvt_pk_u8.txt), and
  // cvt(trunc(x)) == trunc(clamp(x, 0, 255)) for every finite x, so no
  // v_med3_f32 (a VOP3, ~1.8 issue slots) per output.
  return (f2){__builtin_truncf(acc.x), __builtin_truncf(acc.y)};
}

template <int CH, bool UNIFORM, int M, int NW>
__global__ __launch_bounds__(64 * NW) void k_float_temporal(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                            int64_t pitch, int row_bytes, int r0, int r1, int steps,
                                                            int g_row0, int height, FloatTaps tp) {
  __shared__ uint2 lds[2][NW][2][64];  // [parity][wave][top/bottom][lane]
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = (steps * CH + 7) >> 3;  // halo lanes per side
  const int vlanes = 64 - 2 * hl;
  const int chunk = static_cast<int>(blockIdx.x) * vlanes - hl + lane;  // 8-byte column chunk of this lane
  const int x = chunk * 8;
  const int nchunks = (row_bytes + 7) >> 3;
  const bool col_in = chunk >= 0 && chunk < nchunks;
  const int vrows = NW * M - 2 * steps;
  const int tile_r0 = r0 + static_cast<int>(blockIdx.y) * vrows;
  const int row_base = tile_r0 - steps + w * M;
  const float w0 = tp.w[0];
  f2 wv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) wv[k] = (f2){tp.w[k], tp.w[k]};

  // bytes of this lane inside the image row (0..8)
  const int valid = col_in ? min(row_bytes - x, 8) : 0;
  const u32 m0 = valid >= 4 ? 0xffffffffu : (valid <= 0 ? 0u : ((1u << (8 * valid)) - 1u));
  const u32 m1 = valid >= 8 ? 0xffffffffu : (valid <= 4 ? 0u : ((1u << (8 * (valid - 4))) - 1u));
  const bool edge_strip = blockIdx.x == 0 || static_cast<int>(blockIdx.x) * vlanes - hl + 64 >= nchunks;

  u32 D[M][2];
  const int lo_ok = max(r0 - steps, -g_row0), hi_ok = min(r1 + steps, height - g_row0);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    uint2 v = make_uint2(0, 0);
    if (col_in && fr >= lo_ok && fr < hi_ok) {
      // 8-byte aligned (pitch % 16 == 0, data column 0 is 16-byte aligned); the
      // partial last chunk reads into the zero pad columns of the frame row
      v = *reinterpret_cast<const uint2*>(src + static_cast<int64_t>(fr) * pitch + x);
    }
    D[i][0] = v.x & m0;
    D[i][1] = v.y & m1;
  }
  const int out_top = min(max(-g_row0 - row_base, 0), M);
  const int out_bot = min(max(height - g_row0 - row_base, 0), M);

  for (int s = 0; s < steps; ++s) {
    const int par = s & 1;
    lds[par][w][0][lane] = make_uint2(D[0][0], D[0][1]);
    lds[par][w][1][lane] = make_uint2(D[M - 1][0], D[M - 1][1]);
    __syncthreads();
    u32 A[2], B[2];
    {
      const int wa = w > 0 ? w - 1 : 0;
      const int wb = w < NW - 1 ? w + 1 : w;
      const uint2 a = lds[par][wa][1][lane], b = lds[par][wb][0][lane];
      A[0] = a.x;
      A[1] = a.y;
      B[0] = b.x;
      B[1] = b.y;
    }
    f2 ea[4 + 2 * CH], eb[4 + 2 * CH], ec[4 + 2 * CH];
    expand<CH, UNIFORM>(A, w0, ea);
    expand<CH, UNIFORM>(D[0], w0, eb);
#pragma unroll
    for (int i = 0; i < M; ++i) {
      if (i + 1 < M)
        expand<CH, UNIFORM>(D[i + 1], w0, ec);
      else
        expand<CH, UNIFORM>(B, w0, ec);
      u32 o0 = 0, o1 = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f2 v = out_pair<CH, UNIFORM>(ea, eb, ec, j, wv);
        o0 = __builtin_amdgcn_cvt_pk_u8_f32(v.x, j, o0);
        o1 = __builtin_amdgcn_cvt_pk_u8_f32(v.y, j, o1);
      }
      D[i][0] = o0;
      D[i][1] = o1;
#pragma unroll
      for (int j = 0; j < 4 + 2 * CH; ++j) {
        ea[j] = eb[j];
        eb[j] = ec[j];
      }
    }
    if (edge_strip) {
#pragma unroll
      for (int i = 0; i < M; ++i) {
        D[i][0] &= m0;
        D[i][1] &= m1;
      }
    }
    if (out_top > 0 || out_bot < M) {
#pragma unroll
      for (int i = 0; i < M; ++i)
        if (i < out_top || i >= out_bot) {
          D[i][0] = 0;
          D[i][1] = 0;
        }
    }
  }

  const bool lane_ok = col_in && lane >= hl && lane < 64 - hl;
  const int st_lo = max(tile_r0, r0), st_hi = min(min(tile_r0 + vrows, r1), height - g_row0);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    if (lane_ok && fr >= st_lo && fr < st_hi) {
      uint8_t* q = dst + static_cast<int64_t>(fr) * pitch + x;
      if (valid == 8) {
        *reinterpret_cast<uint2*>(q) = make_uint2(D[i][0], D[i][1]);
      } else {  // partial last chunk: never write past the row's last byte
        const u32 lo = D[i][0], hi = D[i][1];
        for (int b = 0; b < valid; ++b) q[b] = static_cast<uint8_t>((b < 4 ? lo : hi) >> (8 * (b & 3)));
      }
    }
  }
}

struct FtShape {
  int m, nw;
};

// Tile shape when nothing is tuned (one-shot CLI, a capture before tuning):
// the largest tile (least halo) whose grid fills the chip — at least 3/4 of
// a workgroup per CU — and whose last round of workgroups is at least 3/4
// full.  Fits the sweep (gpurun_out/r03/g/float_sweep.jsonl): 1920x2520 RGB
// at 4 steps -> 16x8 (252 workgroups: 8.0 us/rep, best), at 8 steps -> 16x4
// (9.5, best 9.5); grey at 8 steps -> 16x4 (3.6, best 3.5); 8192^2 RGB ->
// 16x8 (best).  set_float_shape(M, NW) forces one.
std::atomic<int> g_ft_force_m{0}, g_ft_force_nw{0};

FtShape pick_ft_shape(int steps, int ch, int64_t rows, int64_t row_bytes) {
  static const FtShape cands[] = {{16, 8}, {16, 4}, {8, 8}, {8, 4}, {4, 8}};  // largest tiles first
  if (const int fm = g_ft_force_m.load(std::memory_order_relaxed)) {
    const int fnw = g_ft_force_nw.load(std::memory_order_relaxed);
    for (const auto& c : cands)
      if (c.m == fm && c.nw == fnw) return c;
  }
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess)
      n = 256;
    return std::max(1, n);
  }();
  const int hl = (steps * ch + 7) / 8;
  const int64_t ctiles = ceil_div<int64_t>(ceil_div<int64_t>(row_bytes, 8), std::max(1, 64 - 2 * hl));
  FtShape most{4, 8};
  int64_t most_wgs = -1;
  for (const auto& c : cands) {
    const int vrows = c.m * c.nw - 2 * steps;
    if (vrows <= 0) continue;
    const int64_t wgs = ctiles * ceil_div<int64_t>(rows, vrows);
    const int64_t rounds = ceil_div<int64_t>(wgs, cus);
    if (4 * wgs >= 3 * static_cast<int64_t>(cus) && 4 * wgs >= 3 * rounds * cus) return c;
    if (wgs > most_wgs) {
      most_wgs = wgs;
      most = c;
    }
  }
  return most;  // a small frame: the shape with the most workgroups
}

template <int CH, bool UNIFORM, int M, int NW>
void launch_ft_shape(const StencilLaunch& a, const FloatTaps& tp, hipStream_t s) {
  const int steps = a.steps;
  const int hl = (steps * CH + 7) / 8;
  const int vlanes = 64 - 2 * hl;
  const int vrows = M * NW - 2 * steps;
  PCONV_CHECK(vlanes > 0 && vrows > 0, "float temporal kernel: steps too large for the tile");
  const int nchunks = static_cast<int>(ceil_div<int64_t>(a.row_bytes, 8));
  const dim3 grid(ceil_div(nchunks, vlanes), ceil_div(static_cast<int>(a.r1 - a.r0), vrows));
  k_float_temporal<CH, UNIFORM, M, NW><<<grid, dim3(64 * NW), 0, s>>>(
      a.src, a.dst, a.pitch, static_cast<int>(a.row_bytes), static_cast<int>(a.r0), static_cast<int>(a.r1), steps,
      static_cast<int>(a.g_row0), static_cast<int>(std::min<int64_t>(a.height, int64_t(1) << 30)), tp);
}

template <int CH, bool UNIFORM>
void launch_ft_with(const StencilLaunch& a, const FloatTaps& tp, hipStream_t s, FtShape sh) {
#define PCONV_FT(M_, NW_)                                  \
  if (sh.m == M_ && sh.nw == NW_) {                        \
    launch_ft_shape<CH, UNIFORM, M_, NW_>(a, tp, s);       \
    return;                                                \
  }
  PCONV_FT(16, 8)
  PCONV_FT(8, 8)
  PCONV_FT(16, 4)
  PCONV_FT(8, 4)
  PCONV_FT(4, 8)
#undef PCONV_FT
  PCONV_FAIL("float temporal kernel: unsupported tile shape");
}

// Empirical shape tuning, as for the SWAR kernel (stencil_swar.hip): on the
// first launch of a geometry every candidate runs the REAL launch (same src
// -> dst, so repeats write the same bytes) in two interleaved timed passes and
// the fastest is cached per (channels, uniform, steps, rows, row bytes).  The
// shape is a large lever on these small frames and not monotonic in the
// model (1920x2520 RGB box, 4 steps: 8.0 us/rep with 16x8 tiles, 9.2-10.4
// with the others; gpurun_out/r03/g/float_sweep.jsonl).  Never while the
// stream is being captured: the engine tunes a step's launches first.
struct FtKey {
  int ch;
  bool uniform;
  int steps;
  int64_t rows, row_bytes;
  bool operator<(const FtKey& o) const {
    return std::tie(ch, uniform, steps, rows, row_bytes) < std::tie(o.ch, o.uniform, o.steps, o.rows, o.row_bytes);
  }
};
std::mutex g_ft_mu;
std::map<FtKey, FtShape> g_ft_tuned;

bool capturing_ft(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

template <int CH, bool UNIFORM>
FtShape tuned_ft_shape(const StencilLaunch& a, const FloatTaps& tp, hipStream_t s) {
  const FtShape model = pick_ft_shape(a.steps, CH, a.r1 - a.r0, a.row_bytes);
  if (g_ft_force_m.load(std::memory_order_relaxed) || !shape_tuning_enabled()) return model;
  const FtKey key{CH, UNIFORM, a.steps, a.r1 - a.r0, a.row_bytes};
  {
    std::lock_guard<std::mutex> lk(g_ft_mu);
    auto it = g_ft_tuned.find(key);
    if (it != g_ft_tuned.end()) return it->second;
  }
  if (capturing_ft(s)) return model;
  static const FtShape cands[] = {{16, 8}, {8, 8}, {16, 4}, {8, 4}, {4, 8}};
  std::vector<FtShape> ok;
  for (const auto& c : cands)
    if (c.m * c.nw - 2 * a.steps > 0) ok.push_back(c);
  PCONV_CHECK(!ok.empty(), "float temporal kernel: steps too large for every tile shape");
  FtShape best = ok.front();
  if (ok.size() > 1) {
    Event e0 = Event::create(true), e1 = Event::create(true);
    std::vector<float> t(ok.size(), 1e30f);
    for (int pass = 0; pass < 2; ++pass)
      for (size_t i = 0; i < ok.size(); ++i) {
        if (pass == 0) launch_ft_with<CH, UNIFORM>(a, tp, s, ok[i]);  // warm
        e0.record(s);
        for (int r = 0; r < 3; ++r) launch_ft_with<CH, UNIFORM>(a, tp, s, ok[i]);
        e1.record(s);
        PCONV_HIP_CHECK(hipEventSynchronize(e1.get()));
        t[i] = std::min(t[i], Event::elapsed_ms(e0, e1));
      }
    best = ok[std::min_element(t.begin(), t.end()) - t.begin()];
  }
  std::lock_guard<std::mutex> lk(g_ft_mu);
  g_ft_tuned.emplace(key, best);
  return best;
}

template <int CH, bool UNIFORM>
void launch_ft(const StencilLaunch& a, const FloatTaps& tp, hipStream_t s, bool launch) {
  const FtShape sh = tuned_ft_shape<CH, UNIFORM>(a, tp, s);
  if (launch) launch_ft_with<CH, UNIFORM>(a, tp, s, sh);
}

template <int CH>
void launch_ft_ch(const Filter& f, const StencilLaunch& a, hipStream_t s, bool launch) {
  FloatTaps tp;
  bool uniform = true;
  for (int i = 0; i < 9; ++i) {
    tp.w[i] = f.weights[i];
    uniform = uniform && f.weights[i] == f.weights[0];
  }
  if (uniform)
    launch_ft<CH, true>(a, tp, s, launch);
  else
    launch_ft<CH, false>(a, tp, s, launch);
}

}  // namespace

namespace {

void float_temporal(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream, bool launch) {
  PCONV_CHECK(a.steps >= 1 && a.steps <= kMaxFusedSteps, "float temporal kernel: steps out of range");
  PCONV_CHECK(a.height < (int64_t(1) << 30) && a.g_row0 < (int64_t(1) << 30), "float temporal kernel: rows exceed 2^30");
  PCONV_CHECK(a.row_bytes > 0 && a.row_bytes < (int64_t(1) << 30), "float temporal kernel: row bytes out of range");
  switch (ch) {
    case Channels::Grey: launch_ft_ch<1>(f, a, stream, launch); break;
    case Channels::Rgb: launch_ft_ch<3>(f, a, stream, launch); break;
    case Channels::Rgba: launch_ft_ch<4>(f, a, stream, launch); break;
  }
}

}  // namespace

void launch_float_temporal(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream) {
  float_temporal(f, ch, a, stream, true);
}

void prepare_float_temporal(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream) {
  float_temporal(f, ch, a, stream, false);
}

void set_float_shape(int m, int nw) {
  g_ft_force_m.store(m > 0 ? m : 0, std::memory_order_relaxed);
  g_ft_force_nw.store(m > 0 ? nw : 0, std::memory_order_relaxed);
}

void clear_float_tuning() {
  std::lock_guard<std::mutex> lk(g_ft_mu);
  g_ft_tuned.clear();
}

}  // namespace pconv
