// 3x3 filter value type.
//
// The reference builds a `float**` 3x3 from integer taps divided by a double
// constant (mpi/mpi_convolution.c:88-102): gaussian/16 is active, box/9 and
// "edge_detection"/28 are commented-out alternatives.  The CUDA path hard-codes
// the gaussian (cuda/cuda_convolution.cu:12,29).
//
// Semantics: out = trunc( sum_{k,l} w[k][l] * in[y+k-1][x+l-1] ),
// evaluated in float32 in row-major tap order with separate multiply and add
// (x86 gcc, no FMA contraction), w = (float)(tap / (double)divisor), zero
// outside the image.  When the divisor is a power of two and the taps are
// non-negative every partial sum is exact in float32, so the integer formula
// (sum tap*p) >> log2(divisor) is bit-identical — that is the fast path.
#pragma once

#include <array>
#include <string>

namespace pconv {

struct Filter {
  std::string name;
  std::array<int, 9> taps{};     // row-major
  int divisor = 1;
  std::array<float, 9> weights{};  // (float)(taps[i] / (double)divisor)
  bool int_exact = false;        // integer formula == float32 reference semantics
  int shift = 0;                 // log2(divisor) when int_exact
  bool binomial121 = false;      // taps == [1,2,1] (x) [1,2,1]: separable fast path

  static Filter gaussian();  // [[1,2,1],[2,4,2],[1,2,1]] / 16 (active in the reference)
  static Filter box();       // all ones / 9
  static Filter edge();      // [[1,4,1],[4,8,4],[1,4,1]] / 28 (reference name "edge_detection")
  static Filter custom(const std::array<int, 9>& taps, int divisor, const std::string& name = "custom");
  static Filter by_name(const std::string& name);  // "gaussian" | "box" | "edge"

  // Sum of |taps|; used for u16 overflow checks in the packed-integer kernels.
  int abs_sum() const;
};

}  // namespace pconv
