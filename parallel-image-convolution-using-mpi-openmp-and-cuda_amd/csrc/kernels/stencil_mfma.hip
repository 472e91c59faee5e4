// MFMA prototype of one gaussian step on a grey frame (VERDICT r02 item 4:
// "prototype MFMA for the VALU-limited large frames").  Opt-in only
// (KernelVariant::Mfma, `--kernel mfma`); the tuner never picks it — see
// docs/PERFORMANCE.md §4 for the measured comparison with the SWAR kernels.
//
// The separable [1,2,1] x [1,2,1] step as two banded 16x16x16 f16 matrix
// products per 16x16 input tile, exact in integers:
//   pass 1 (horizontal): D1 = P * Bh + C1   P = input tile as the A operand
//       (lane l: row l%16, four consecutive columns 4*(l/16)..+3), each byte b
//       encoded as the f16 1024 + b (one v_perm per two bytes: exponent byte
//       0x64 beside the pixel byte), Bh banded, C1 = -4 * 1024 removes the
//       encoding offset: D1 = exact horizontal sums (<= 1020) for columns 1..14.
//   pass 2 (vertical): D2 = Bv * f16(D1)   D1's accumulator layout (lane l:
//       rows 4*(l/16)..+3 of column l%16) IS the B operand layout, so no
//       shuffle between the passes; D1 <= 1020 is exact in f16, D2 <= 4080
//       exact in f32.  Rows 1..14 valid.
//   out = (u32)D2 >> 4  — the reference's truncating store of sum/16
//       (mpi/mpi_convolution.c:303-307).
// Each 16x16 tile yields a 14x14 output block (the band's edges need the
// neighbouring input rows/columns), i.e. 196 of 256 products are kept.
// Zero padding: pixels outside the image are encoded as value 0.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pconv/kernels.hpp"

namespace pconv {
namespace {

using u32 = uint32_t;
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kBlk = 14;  // output rows / columns per 16x16 tile
constexpr int kNB = 8;    // tiles per wave along the row

__device__ __forceinline__ h4 as_h4(u32 lo, u32 hi) {
  typedef u32 u2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(h4, (u2){lo, hi});
}

// Banded [1,2,1] entry: 1 at |d| == 1, 2 at d == 0.
__device__ __forceinline__ _Float16 band(int d) {
  return d == 0 ? static_cast<_Float16>(2.0f) : ((d == 1 || d == -1) ? static_cast<_Float16>(1.0f)
                                                                    : static_cast<_Float16>(0.0f));
}

__global__ __launch_bounds__(256) void k_mfma_grey_step(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                        int64_t pitch, int row_bytes, int r0, int r1, int g_row0,
                                                        int height) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;  // 0..3: k-group (A/B operands) or row group (accumulators)
  const int c16 = lane & 15;
  const int R0 = r0 + (static_cast<int>(blockIdx.y) * 4 + wave) * kBlk;  // first output row of the strip
  if (R0 >= r1) return;
  // constant operands: Bh[k][n] = band(k - n), B layout (k = 4q + j, n = c16);
  // Bv[m][k] = band(k - m), A layout (m = c16, k = 4q + j)
  h4 bh, bv;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    bh[j] = band(4 * q + j - c16);
    bv[j] = band(4 * q + j - c16);
  }
  const f4 c1 = (f4){-4096.0f, -4096.0f, -4096.0f, -4096.0f};
  const f4 zero = (f4){0.0f, 0.0f, 0.0f, 0.0f};
  // input row of this lane for the A operand: tile row c16 = frame row R0 - 1 + c16
  const int in_row = R0 - 1 + c16;
  const bool row_in = in_row + g_row0 >= 0 && in_row + g_row0 < height;
  const uint8_t* prow = src + static_cast<int64_t>(in_row) * pitch;
  const int cx0 = static_cast<int>(blockIdx.x) * kBlk * kNB;
  for (int t = 0; t < kNB; ++t) {
    const int C0 = cx0 + t * kBlk;  // first output column of the tile
    if (C0 >= row_bytes) break;
    // four consecutive input columns C0 - 1 + 4q .. +3 of row in_row
    u32 b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = C0 - 1 + 4 * q + j;
      b[j] = (row_in && col >= 0 && col < row_bytes) ? prow[col] : 0u;
    }
    const u32 lo = b[0] | (b[1] << 16) | 0x64006400u;  // f16 1024 + b0, 1024 + b1
    const u32 hi = b[2] | (b[3] << 16) | 0x64006400u;
    const f4 d1 = __builtin_amdgcn_mfma_f32_16x16x16f16(as_h4(lo, hi), bh, c1, 0, 0, 0);
    // D1 (rows 4q..4q+3 of column c16) -> f16 B operand (exact: |D1| <= 1020)
    h4 hb;
#pragma unroll
    for (int j = 0; j < 4; ++j) hb[j] = static_cast<_Float16>(d1[j]);
    const f4 d2 = __builtin_amdgcn_mfma_f32_16x16x16f16(bv, hb, zero, 0, 0, 0);
    // outputs: rows R0 - 1 + 4q + j (tile rows 1..14), column C0 - 1 + c16 (tile columns 1..14)
    const int col = C0 - 1 + c16;
    if (c16 >= 1 && c16 <= kBlk && col < row_bytes) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = 4 * q + j;
        const int row = R0 - 1 + m;
        if (m >= 1 && m <= kBlk && row < r1)
          dst[static_cast<int64_t>(row) * pitch + col] = static_cast<uint8_t>(static_cast<u32>(d2[j]) >> 4);
      }
    }
  }
}

}  // namespace

void launch_mfma_grey_step(const StencilLaunch& a, hipStream_t stream) {
  PCONV_CHECK(a.steps == 1, "mfma prototype: one step per launch");
  PCONV_CHECK(a.dst_pitch == 0 || a.dst_pitch == a.pitch, "mfma prototype: no separate destination pitch");
  PCONV_CHECK(a.height < (int64_t(1) << 30) && a.g_row0 < (int64_t(1) << 30), "mfma prototype: rows exceed 2^30");
  PCONV_CHECK(a.row_bytes > 0 && a.row_bytes < (int64_t(1) << 30), "mfma prototype: row bytes out of range");
  const int rows = static_cast<int>(a.r1 - a.r0);
  const dim3 grid(static_cast<unsigned>(ceil_div<int64_t>(a.row_bytes, kBlk * kNB)),
                  static_cast<unsigned>(ceil_div(ceil_div(rows, kBlk), 4)));
  k_mfma_grey_step<<<grid, dim3(256), 0, stream>>>(a.src, a.dst, a.pitch, static_cast<int>(a.row_bytes),
                                                   static_cast<int>(a.r0), static_cast<int>(a.r1),
                                                   static_cast<int>(a.g_row0), static_cast<int>(a.height));
}

}  // namespace pconv
