// CPU stencil oracle + OpenMP backend (see cpu_stencil.hpp).
//
// Compiled with -ffp-contract=off: the float path must be multiply-then-add
// with one rounding each, in row-major tap order, like the x86 gcc reference
// (mpi/mpi_convolution.c:303-307, :313-318).
#include "pconv/cpu_stencil.hpp"

#include <omp.h>
#include <sched.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace pconv {

namespace {

inline uint8_t sat_trunc(float v) {
  // float -> uint8_t truncation; out-of-range values (only possible for custom
  // filters with negative taps) saturate instead of the reference's UB.
  if (!(v > 0.0f)) return 0;
  if (v >= 255.0f) return 255;
  return static_cast<uint8_t>(static_cast<int>(v));
}

// (Σ tap·p) >> 4 with taps [1,2,1]⊗[1,2,1]: the vertical sums of the row once
// into a 16-bit scratch row (every sum <= 1020; the full sum <= 4080 < 2^16),
// then the horizontal pass — two passes of 16-bit lanes the compiler
// vectorises.  Built twice: the x86-64 baseline and an AVX2 clone picked at
// run time (the GPU boxes' and this container's CPUs have AVX2; no -march
// flag, so the binary still runs anywhere).
#define PCONV_ROW_BINOMIAL_BODY                                                               \
  for (int64_t x = -CH; x < n + CH; ++x) v[x + CH] = static_cast<uint16_t>(a[x] + 2 * b[x] + c[x]); \
  for (int64_t x = 0; x < n; ++x)                                                             \
    o[x] = static_cast<uint8_t>(static_cast<uint16_t>(v[x] + 2 * v[x + CH] + v[x + 2 * CH]) >> 4);

template <int CH>
void row_binomial_base(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* o, int64_t n, uint16_t* v) {
  PCONV_ROW_BINOMIAL_BODY
}

template <int CH>
__attribute__((target("avx2"))) void row_binomial_avx2(const uint8_t* a, const uint8_t* b, const uint8_t* c,
                                                       uint8_t* o, int64_t n, uint16_t* v) {
  PCONV_ROW_BINOMIAL_BODY
}
#undef PCONV_ROW_BINOMIAL_BODY

template <int CH>
void row_binomial(const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* o, int64_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  thread_local std::vector<uint16_t> scratch;
  if (scratch.size() < static_cast<size_t>(n + 2 * CH)) scratch.resize(static_cast<size_t>(n + 2 * CH));
  if (avx2)
    row_binomial_avx2<CH>(a, b, c, o, n, scratch.data());
  else
    row_binomial_base<CH>(a, b, c, o, n, scratch.data());
}

// Integer-exact custom filters (non-negative taps, power-of-two divisor).
#define PCONV_ROW_INT_BODY                                                                          \
  const int t0 = t[0], t1 = t[1], t2 = t[2], t3 = t[3], t4 = t[4], t5 = t[5], t6 = t[6], t7 = t[7], \
            t8 = t[8];                                                                              \
  for (int64_t x = 0; x < n; ++x) {                                                                 \
    const int acc = t0 * a[x - CH] + t1 * a[x] + t2 * a[x + CH] + t3 * b[x - CH] + t4 * b[x] +       \
                    t5 * b[x + CH] + t6 * c[x - CH] + t7 * c[x] + t8 * c[x + CH];                   \
    o[x] = static_cast<uint8_t>(std::min(acc >> s, 255));                                            \
  }

template <int CH>
void row_int_base(const int* t, int s, const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* o, int64_t n) {
  PCONV_ROW_INT_BODY
}

template <int CH>
__attribute__((target("avx2"))) void row_int_avx2(const int* t, int s, const uint8_t* a, const uint8_t* b,
                                                  const uint8_t* c, uint8_t* o, int64_t n) {
  PCONV_ROW_INT_BODY
}
#undef PCONV_ROW_INT_BODY

template <int CH>
void row_int(const Filter& f, const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* o, int64_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2)
    row_int_avx2<CH>(f.taps.data(), f.shift, a, b, c, o, n);
  else
    row_int_base<CH>(f.taps.data(), f.shift, a, b, c, o, n);
}

// Float filters: per output, acc = 0; acc += fl(p * w) over the nine taps in
// row-major order (the reference's sequence, one rounding per op, no FMA:
// -ffp-contract=off, and the AVX2 clone does not enable FMA).  Outputs are
// independent, so vectorising across x keeps every output's order.
#define PCONV_ROW_FLOAT_BODY                                                                  \
  const float w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4], w5 = w[5], w6 = w[6], w7 = w[7], \
              w8 = w[8];                                                                      \
  for (int64_t x = 0; x < n; ++x) {                                                           \
    float acc = 0.0f;                                                                         \
    acc = acc + static_cast<float>(a[x - CH]) * w0;                                           \
    acc = acc + static_cast<float>(a[x]) * w1;                                                \
    acc = acc + static_cast<float>(a[x + CH]) * w2;                                           \
    acc = acc + static_cast<float>(b[x - CH]) * w3;                                           \
    acc = acc + static_cast<float>(b[x]) * w4;                                                \
    acc = acc + static_cast<float>(b[x + CH]) * w5;                                           \
    acc = acc + static_cast<float>(c[x - CH]) * w6;                                           \
    acc = acc + static_cast<float>(c[x]) * w7;                                                \
    acc = acc + static_cast<float>(c[x + CH]) * w8;                                           \
    o[x] = sat_trunc(acc);                                                                    \
  }

template <int CH>
void row_float_base(const float* w, const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* o, int64_t n) {
  PCONV_ROW_FLOAT_BODY
}

template <int CH>
__attribute__((target("avx2"))) void row_float_avx2(const float* w, const uint8_t* a, const uint8_t* b,
                                                    const uint8_t* c, uint8_t* o, int64_t n) {
  PCONV_ROW_FLOAT_BODY
}
#undef PCONV_ROW_FLOAT_BODY

template <int CH>
void row_float(const Filter& f, const uint8_t* a, const uint8_t* b, const uint8_t* c, uint8_t* o, int64_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2)
    row_float_avx2<CH>(f.weights.data(), a, b, c, o, n);
  else
    row_float_base<CH>(f.weights.data(), a, b, c, o, n);
}

template <int CH>
void step_rows(const Filter& f, const FrameLayout& lay, const uint8_t* src, uint8_t* dst, int64_t r0, int64_t r1,
               CpuBackend be) {
  const int64_t n = lay.row_bytes;
  auto body = [&](int64_t r) {
    const uint8_t* a = src + lay.offset(r - 1);
    const uint8_t* b = src + lay.offset(r);
    const uint8_t* c = src + lay.offset(r + 1);
    uint8_t* o = dst + lay.offset(r);
    if (f.binomial121)
      row_binomial<CH>(a, b, c, o, n);
    else if (f.int_exact)
      row_int<CH>(f, a, b, c, o, n);
    else
      row_float<CH>(f, a, b, c, o, n);
  };
  if (be == CpuBackend::OpenMP) {
    // Below ~32 KiB of output a step is a few microseconds on one core: the
    // team's fork/join costs as much, and on a loaded host a preempted team
    // member stalls the barrier for a whole scheduler slice.
    const bool team = (r1 - r0) * n >= (int64_t{32} << 10);
#pragma omp parallel for schedule(static) if (team)
    for (int64_t r = r0; r < r1; ++r) body(r);
  } else {
    for (int64_t r = r0; r < r1; ++r) body(r);
  }
}

}  // namespace

void cpu_step(const Filter& f, Channels ch, const FrameLayout& lay, const uint8_t* src_frame, uint8_t* dst_frame,
              int64_t r0, int64_t r1, CpuBackend be) {
  PCONV_CHECK(r0 >= -lay.halo + 1 && r1 <= lay.rows + lay.halo - 1 && r0 <= r1, "cpu_step: rows out of frame");
  switch (ch) {
    case Channels::Grey: step_rows<1>(f, lay, src_frame, dst_frame, r0, r1, be); break;
    case Channels::Rgb: step_rows<3>(f, lay, src_frame, dst_frame, r0, r1, be); break;
    case Channels::Rgba: step_rows<4>(f, lay, src_frame, dst_frame, r0, r1, be); break;
  }
}

void cpu_fused_launch(const Filter& f, Channels ch, const FrameLayout& lay, const uint8_t* src_frame,
                      uint8_t* dst_frame, int64_t lo, int64_t hi, int steps, int64_t g_row0, int64_t height,
                      CpuBackend be) {
  PCONV_CHECK(steps >= 1 && lo <= hi, "cpu_fused_launch: bad arguments");
  PCONV_CHECK(lo - steps >= -lay.halo && hi + steps <= lay.rows + lay.halo, "cpu_fused_launch: rows exceed frame");
  if (lo == hi) return;
  if (steps == 1) {
    // Single step never writes rows outside the image: clip like the kernels' caller.
    const int64_t a = std::max(lo, -g_row0), b = std::min(hi, height - g_row0);
    if (a < b) cpu_step(f, ch, lay, src_frame, dst_frame, a, b, be);
    return;
  }
  const size_t n = static_cast<size_t>(lay.bytes());
  std::vector<uint8_t> A(src_frame, src_frame + n), B(src_frame, src_frame + n);
  uint8_t* cur = A.data();
  uint8_t* nxt = B.data();
  for (int j = 1; j <= steps; ++j) {
    const int64_t ext = steps - j;
    const int64_t a = std::max(lo - ext, -g_row0), b = std::min(hi + ext, height - g_row0);
    if (a < b) cpu_step(f, ch, lay, cur, nxt, a, b, be);
    std::swap(cur, nxt);
  }
  for (int64_t r = lo; r < hi; ++r) {
    const bool inside = g_row0 + r >= 0 && g_row0 + r < height;
    if (inside)
      std::memcpy(dst_frame + lay.offset(r), cur + lay.offset(r), lay.row_bytes);
    else
      std::memset(dst_frame + lay.offset(r), 0, lay.row_bytes);
  }
}

namespace {

int cgroup_cpu_quota() {
  // cgroup v2: "max 100000" or "<quota> <period>"; v1: cfs_quota_us / cfs_period_us.
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long long period = 0;
    const int n = std::fscanf(f, "%31s %lld", q, &period);
    std::fclose(f);
    if (n == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const long long quota = std::atoll(q);
      if (quota > 0) return static_cast<int>((quota + period - 1) / period);
    }
    return 0;
  }
  long long quota = -1, period = 0;
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    if (std::fscanf(f, "%lld", &quota) != 1) quota = -1;
    std::fclose(f);
  }
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
    if (std::fscanf(f, "%lld", &period) != 1) period = 0;
    std::fclose(f);
  }
  return quota > 0 && period > 0 ? static_cast<int>((quota + period - 1) / period) : 0;
}

}  // namespace

int default_cpu_threads() {
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : omp_get_num_procs();
  const int q = cgroup_cpu_quota();
  if (q > 0) n = std::min(n, q);
  if (n > 2) n -= 1;
  return std::max(1, n);
}

int configure_cpu_threads(int share) {
  if (std::getenv("OMP_NUM_THREADS")) return omp_get_max_threads();
  const int n = std::max(1, default_cpu_threads() / std::max(1, share));
  omp_set_num_threads(n);
  return n;
}

void cpu_convolve(const Filter& f, const ImageGeom& geom, const uint8_t* in, uint8_t* out, int reps, CpuBackend be,
                  int threads) {
  geom.validate();
  PCONV_CHECK(reps >= 0, "repetitions must be >= 0");
  const int64_t rb = geom.row_bytes();
  const FrameLayout lay = FrameLayout::make(rb, geom.height, 1);
  std::vector<uint8_t> fa(static_cast<size_t>(lay.bytes()), 0), fb(static_cast<size_t>(lay.bytes()), 0);
  for (int64_t r = 0; r < geom.height; ++r) std::memcpy(fa.data() + lay.offset(r), in + r * rb, rb);
  const int saved = omp_get_max_threads();
  if (be == CpuBackend::OpenMP && threads <= 0 && !std::getenv("OMP_NUM_THREADS")) threads = default_cpu_threads();
  if (be == CpuBackend::OpenMP && threads > 0) omp_set_num_threads(threads);
  uint8_t* src = fa.data();
  uint8_t* dst = fb.data();
  for (int t = 0; t < reps; ++t) {
    cpu_step(f, geom.channels, lay, src, dst, 0, geom.height, be);
    std::swap(src, dst);  // newest result is always in `src` (fixes SURVEY §A3)
  }
  if (be == CpuBackend::OpenMP && threads > 0) omp_set_num_threads(saved);
  for (int64_t r = 0; r < geom.height; ++r) std::memcpy(out + r * rb, src + lay.offset(r), rb);
}

}  // namespace pconv
