// Device helpers of the SWAR-32 gaussian tile kernels (stencil_swar.hip):
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

// Hides `v` from instruction combining only (non-volatile: free to
// schedule).  On gfx950 every VOP3 encoding (v_add3_u32, v_lshl_add_u32,
// v_perm_b32, v_bfe_u32, ...) and every DPP op issues at ~half the rate of a
// VOP2 v_add_u32 / v_lshrrev_b32 / v_and_b32 (4.3-4.7 vs 2.4-2.7 cycles per
// wave-instruction at 4 waves/SIMD, tools/ubench/valu_issue.hip,
// profiles/r03/valu/README.md).  keep() stops two dependent adds from fusing
// into a v_add3_u32 where the first one is also needed on its own (a fused
// add3 beside the plain add costs 2.8 issue slots for what two adds do in 2),
// and stops a lane-crossing add from becoming v_mov_b32_dpp + v_add3_u32 (VOP3
// cannot take a DPP source on gfx950) instead of one v_add_u32_dpp.
__device__ __forceinline__ u32 keep(u32 v) {
  asm("" : "+v"(v));
  return v;
}

// Horizontal [1,2,1] at tap distance CH over NP pairs, as two pair sums:
//   P_j = X_j + X_{j+CH},   H_k = P_{k-CH} + P_k  (= X_{k-CH} + 2 X_k + X_{k+CH}).
// Two v_add_u32 per pair and no shift (the direct form needs v_lshlrev or a
// VOP3 v_lshl_add_u32 for 2 X_k, then two adds); the operands that live in the
// neighbouring lane are the DPP source of their add: X_{j+CH} past the lane's
// last pair from lane+1 (wave_shl:1), P_{k-CH} before its first pair from
// lane-1 (wave_shr:1); bound_ctrl gives 0 past the wave edge.  Edge lanes:
// lane 63 sees X = 0 beyond it (as the direct form does); lane 0 misses both
// terms of P_{k-CH} for k < CH instead of one — those bytes are halo garbage
// either way (the tile's halo is sized for the CH bytes per step that enter
// at a strip edge, whatever their values), and columns outside the image are
// real zeros inside the strip, where the two forms agree exactly.
// The neighbouring lane's value (DIR +1: lane + 1, -1: lane - 1) as the DPP
// source of the add that consumes it.  Read with an LDS permute instead
// (ds_bpermute, off the VALU, the add a plain VOP2): bit-exact but slower —
// us per repetition, headline 4.78 vs 3.32, 8-way band 2.17 vs 1.47, 32768^2
// grey 105.7-108.2 vs 105.0-108.7 (the permute's latency waits;
// profiles/r06/w/).
template <int DIR>
__device__ __forceinline__ u32 xlane(u32 v) {
  return __builtin_amdgcn_mov_dpp(v, DIR > 0 ? 0x130 : 0x138, 0xf, 0xf, true);
}

template <int CH, int NP>
__device__ __forceinline__ void horiz(const u32 (&X)[NP], u32 (&H)[NP]) {
  static_assert(CH <= NP, "tap distance must not exceed the pairs per lane");
  u32 P[NP];
#pragma unroll
  for (int j = 0; j < NP; ++j)
    P[j] = keep(j + CH < NP ? X[j] + X[j + CH] : xlane<1>(X[j + CH - NP]) + X[j]);
#pragma unroll
  for (int k = 0; k < NP; ++k) H[k] = keep(k >= CH ? P[k - CH] + P[k] : xlane<-1>(P[k - CH + NP]) + P[k]);
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

// lds[parity][wave][2][quad][lane]: slot 0 = the wave's top row, slot 1 its
// bottom row.
template <int CH, int NP, int M, int NW, int MODE = 0>
__device__ __forceinline__ void swar_step(u32 (&D)[M][NP], uint4 (&lds)[2][NW][2][NP / 4][64], int par, int w,
                                             int lane, bool needs_mask, const u32 (&cm)[NP], int out_top,
                                             int out_bot) {
  static_assert(M >= 2, "interior-first step needs two register rows per wave");
  constexpr int NQ = NP / 4;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    lds[par][w][0][q][lane] = make_uint4(D[0][4 * q], D[0][4 * q + 1], D[0][4 * q + 2], D[0][4 * q + 3]);
    lds[par][w][1][q][lane] =
        make_uint4(D[M - 1][4 * q], D[M - 1][4 * q + 1], D[M - 1][4 * q + 2], D[M - 1][4 * q + 3]);
  }
  // Vertical [1,2,1] as rolling pair sums S_i = H_i + H_{i+1}; row i is
  // S_{i-1} + S_i: two v_add_u32 per pair (keep(): no v_add3_u32 that would
  // redo an add the next row needs anyway).
  u32 H0[NP], Hc[NP], S01[NP], Sc[NP];
  horiz<CH, NP>(D[0], H0);
  horiz<CH, NP>(D[1], Hc);
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    S01[k] = keep(H0[k] + Hc[k]);
    Sc[k] = S01[k];
  }
#pragma unroll
  for (int i = 1; i + 1 < M; ++i) {
    u32 Hn[NP];
    horiz<CH, NP>(D[i + 1], Hn);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const u32 Sn = keep(Hc[k] + Hn[k]);
      D[i][k] = trunc_sum<MODE>(Sc[k] + Sn);
      Sc[k] = Sn;
      Hc[k] = Hn[k];
    }
  }
  // Sc = S_{M-2} = H[M-2] + H[M-1], Hc = H[M-1] (old rows); S01 = H[0] + H[1].
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
      D[0][k] = trunc_sum<MODE>(keep(Ha[k] + H0[k]) + S01[k]);
      D[M - 1][k] = trunc_sum<MODE>(Sc[k] + keep(Hc[k] + Hb[k]));
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
