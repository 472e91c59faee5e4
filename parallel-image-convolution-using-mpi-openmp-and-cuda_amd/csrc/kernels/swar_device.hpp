// Device helpers of the SWAR-32 gaussian shared by the tile kernel
// (stencil_swar.hip) and the register-resident kernel (stencil_resident.hip):
// the byte-pair layout, the horizontal [1,2,1] with DPP lane crossing, and one
// interior-first repetition of a wave's register rows.  See stencil_swar.hip
// for the layout and the measurements behind these forms.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace pconv {
namespace {

using u32 = uint32_t;

__device__ __forceinline__ u32 perm(u32 hi, u32 lo, u32 sel) { return __builtin_amdgcn_perm(hi, lo, sel); }

// Selector building the pair (lo.byte j, hi.byte j) zero-extended to u16x2.
__device__ __forceinline__ constexpr u32 pair_sel(int j) {
  return 0x0c000c00u | ((4u + static_cast<u32>(j)) << 16) | static_cast<u32>(j);
}

// Keeps `v` in a register as computed: stops instruction selection from
// merging the next add into a 3-input v_add3 (VOP3 cannot take a DPP source
// on gfx950), so the lane-crossing tap folds into v_add_u32_dpp.
__device__ __forceinline__ u32 opaque(u32 v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Horizontal [1,2,1] at tap distance CH over NP pairs; taps in the
// neighbouring lane come through DPP (wave_shr:1 / wave_shl:1, bound_ctrl: 0
// past the wave edge).
//   NP = 4: most taps cross lanes (RGB: 6 of 8 per row), so each one is the
//     DPP source of its add (v_add_u32_dpp) — 2 VALU ops per pair instead of
//     up to 4 with separate v_mov_b32_dpp;
//   NP = 8: few taps cross lanes and the register budget is tight (the big
//     tiles sit at 2 waves/SIMD); the plain form keeps the compiler free to
//     schedule (folding costs these tiles ~20 VGPRs = one wave per SIMD).
template <int CH, int NP>
__device__ __forceinline__ void horiz(const u32 (&X)[NP], u32 (&H)[NP]) {
  static_assert(CH <= NP, "tap distance must not exceed the pairs per lane");
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int l = k - CH, r = k + CH;
    if constexpr (NP == 4) {
      u32 t = X[k] << 1;
      if (l >= 0) t += X[l];
      if (r < NP) t += X[r];
      if (l < 0) t = __builtin_amdgcn_mov_dpp(X[NP + l], 0x138, 0xf, 0xf, true) + opaque(t);
      if (r >= NP) t = __builtin_amdgcn_mov_dpp(X[r - NP], 0x130, 0xf, 0xf, true) + opaque(t);
      H[k] = t;
    } else {
      const u32 lv = l >= 0 ? X[l] : __builtin_amdgcn_mov_dpp(X[NP + l], 0x138, 0xf, 0xf, true);
      const u32 rv = r < NP ? X[r] : __builtin_amdgcn_mov_dpp(X[r - NP], 0x130, 0xf, 0xf, true);
      H[k] = (X[k] << 1) + (lv + rv);
    }
  }
}

template <int NP>
struct Chunk;  // raw bytes of one lane's chunk in one strip
template <>
struct Chunk<8> {
  using T = uint2;
  __device__ static T zero() { return make_uint2(0, 0); }
};
template <>
struct Chunk<4> {
  using T = u32;
  __device__ static T zero() { return 0u; }
};

template <int NP>
__device__ __forceinline__ void unpack(const typename Chunk<NP>::T& a, const typename Chunk<NP>::T& b, u32 (&D)[NP]) {
  if constexpr (NP == 8) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      D[k] = perm(b.x, a.x, pair_sel(k));
      D[4 + k] = perm(b.y, a.y, pair_sel(k));
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) D[k] = perm(b, a, pair_sel(k));
  }
}

template <int NP>
__device__ __forceinline__ void pack(const u32 (&D)[NP], typename Chunk<NP>::T& a, typename Chunk<NP>::T& b) {
  if constexpr (NP == 8) {
    const u32 t0 = perm(D[1], D[0], 0x06020400u);  // A0 A1 B0 B1
    const u32 t1 = perm(D[3], D[2], 0x06020400u);  // A2 A3 B2 B3
    const u32 t2 = perm(D[5], D[4], 0x06020400u);
    const u32 t3 = perm(D[7], D[6], 0x06020400u);
    a = make_uint2(perm(t1, t0, 0x05040100u), perm(t3, t2, 0x05040100u));
    b = make_uint2(perm(t1, t0, 0x07060302u), perm(t3, t2, 0x07060302u));
  } else {
    const u32 t0 = perm(D[1], D[0], 0x06020400u);
    const u32 t1 = perm(D[3], D[2], 0x06020400u);
    a = perm(t1, t0, 0x05040100u);
    b = perm(t1, t0, 0x07060302u);
  }
}

template <int NP>
__device__ __forceinline__ void store_bytes(uint8_t* p, const typename Chunk<NP>::T& v, int n) {
  u32 w[2];
  if constexpr (NP == 8) {
    w[0] = v.x;
    w[1] = v.y;
  } else {
    w[0] = v;
    w[1] = 0;
  }
  for (int k = 0; k < n; ++k) p[k] = static_cast<uint8_t>(w[k >> 2] >> (8 * (k & 3)));
}

// One repetition of a wave's M register rows, interior first: the wave
// publishes its two boundary rows to LDS, computes its interior rows 1..M-2
// (they need only its own registers) while the other waves catch up, and only
// then meets them at the barrier to finish rows 0 and M-1 with the
// neighbours' rows — the LDS round trip and the barrier wait hide behind M-2
// rows of arithmetic (measured 2-13 % over exchanging first).  MODE picks the
// truncation: 0 floor(S/16); 1 keeps 16 x floor(S/16) (one AND; the next step
// then sums values < 2^12 into fields < 2^16); 2 floor(S/256) of such a step.
// Out-of-image rows and columns are re-zeroed after every step.
template <int MODE>
__device__ __forceinline__ u32 trunc_sum(u32 S) {
  if constexpr (MODE == 0) return (S >> 4) & 0x00ff00ffu;
  else if constexpr (MODE == 1) return S & 0x0ff00ff0u;
  else return (S >> 8) & 0x00ff00ffu;
}

template <int CH, int NP, int M, int NW, int MODE = 0>
__device__ __forceinline__ void swar_step(u32 (&D)[M][NP], uint4 (&lds)[2][NW][2][NP / 4][64], int par, int w,
                                             int lane, bool needs_mask, const u32 (&cm)[NP], int out_top,
                                             int out_bot) {
  static_assert(M >= 2, "interior-first step needs two register rows per wave");
  constexpr int NQ = NP / 4;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    lds[par][w][0][q][lane] = make_uint4(D[0][4 * q], D[0][4 * q + 1], D[0][4 * q + 2], D[0][4 * q + 3]);
    lds[par][w][1][q][lane] = make_uint4(D[M - 1][4 * q], D[M - 1][4 * q + 1], D[M - 1][4 * q + 2], D[M - 1][4 * q + 3]);
  }
  u32 H0[NP], H1[NP], Hp[NP], Hc[NP];
  horiz<CH, NP>(D[0], H0);
  horiz<CH, NP>(D[1], H1);
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    Hp[k] = H0[k];
    Hc[k] = H1[k];
  }
  u32 Sc[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) Sc[k] = Hp[k] + Hc[k];
#pragma unroll
  for (int i = 1; i + 1 < M; ++i) {
    u32 Hn[NP];
    horiz<CH, NP>(D[i + 1], Hn);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const u32 Sn = Hc[k] + Hn[k];
      D[i][k] = trunc_sum<MODE>(Sc[k] + Sn);
      Sc[k] = Sn;
      Hp[k] = Hc[k];
      Hc[k] = Hn[k];
    }
  }
  // Hp = H[M-2], Hc = H[M-1] (old rows); H0, H1 = H[0], H[1].
  __syncthreads();
  {
    const int wa = w > 0 ? w - 1 : 0;       // wave 0: tile top halo, value irrelevant
    const int wb = w < NW - 1 ? w + 1 : w;  // last wave: tile bottom halo
    u32 A[NP], B[NP];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const uint4 av = lds[par][wa][1][q][lane], bv = lds[par][wb][0][q][lane];
      A[4 * q] = av.x; A[4 * q + 1] = av.y; A[4 * q + 2] = av.z; A[4 * q + 3] = av.w;
      B[4 * q] = bv.x; B[4 * q + 1] = bv.y; B[4 * q + 2] = bv.z; B[4 * q + 3] = bv.w;
    }
    u32 Ha[NP], Hb[NP];
    horiz<CH, NP>(A, Ha);
    horiz<CH, NP>(B, Hb);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      D[0][k] = trunc_sum<MODE>((Ha[k] + H0[k]) + (H0[k] + H1[k]));
      D[M - 1][k] = trunc_sum<MODE>((Hp[k] + Hc[k]) + (Hc[k] + Hb[k]));
    }
  }
  if (needs_mask) {
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
      for (int k = 0; k < NP; ++k) D[i][k] &= cm[k];
  }
  if (out_top > 0 || out_bot < M) {
#pragma unroll
    for (int i = 0; i < M; ++i)
      if (i < out_top || i >= out_bot)
#pragma unroll
        for (int k = 0; k < NP; ++k) D[i][k] = 0;
  }
}

}  // namespace
}  // namespace pconv
