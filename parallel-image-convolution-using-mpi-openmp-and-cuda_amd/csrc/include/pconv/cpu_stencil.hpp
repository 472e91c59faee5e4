// CPU stencil: the serial oracle and the OpenMP backend.
//
// Reference: Convolution() loops a rectangular region of the padded local block
// (mpi/mpi_convolution.c:288-299) and calls ConvolutionforGrey/RGB per pixel
// (:301-322), a float MAC over a `float**` filter.  The OpenMP build adds
// `#pragma omp parallel for ... collapse(3)` on a 2-deep nest
// (open-mp/omp_convolution.c:292,297), which does not compile.
//
// Here the CPU path works on the same FrameLayout as the GPU (zero pad ring),
// computes any row range of a frame, and has two arithmetic modes:
//   * integer  (Σ tap·p) >> shift   when filter.int_exact   (bit-exact, §0.1)
//   * float32  mul-then-add in reference tap order, truncating store.
// The OpenMP variant parallelises the row loop (correct `collapse`-free form).
#pragma once

#include <cstdint>

#include "pconv/filter.hpp"
#include "pconv/image.hpp"

namespace pconv {

enum class CpuBackend { Serial, OpenMP };

// Frame pointers here are the frame BASE (row -halo, column -kPadLeft).
// One step: for owned rows [r0, r1) of the frame, dst = conv(src).  Pixels whose
// global row lies outside [0, image_height) are treated as zero by the caller's
// frame (ghost rows hold zeros at the global image edges).
void cpu_step(const Filter& f, Channels ch, const FrameLayout& lay, const uint8_t* src_frame,
              uint8_t* dst_frame, int64_t r0, int64_t r1, CpuBackend be);

// Reference semantics of one fused launch (what the temporal GPU kernel
// computes): `steps` repetitions starting from src rows [lo-steps, hi+steps),
// rows outside the global image [0, height) held at zero after every step;
// writes rows [lo, hi) of dst only.  g_row0 = global row of frame row 0.
void cpu_fused_launch(const Filter& f, Channels ch, const FrameLayout& lay, const uint8_t* src_frame,
                      uint8_t* dst_frame, int64_t lo, int64_t hi, int steps, int64_t g_row0, int64_t height,
                      CpuBackend be);

// reps steps on a contiguous image (pitch == row_bytes), zero-padded semantics.
// Ping-pongs internally; result written to `out` (may alias `in`).
void cpu_convolve(const Filter& f, const ImageGeom& geom, const uint8_t* in, uint8_t* out,
                  int reps, CpuBackend be, int threads = 0);

// OpenMP team size when the user set none (OMP_NUM_THREADS unset, no
// --threads): the CPUs this process may run on (affinity mask), capped by the
// cgroup CPU quota (a container or GPU-box slice sees every CPU of the
// machine but may use only its quota), minus one when more than two remain —
// a fork/join team that claims EVERY available CPU while anything else runs
// spins into the scheduler (measured 10 ms per parallel region with 8
// threads on 8 busy vCPUs vs 5 us with 7).
int default_cpu_threads();
// Apply default_cpu_threads() unless OMP_NUM_THREADS is set; `share` divides
// the CPUs between that many processes (ranks on one node).  Returns the team size.
int configure_cpu_threads(int share = 1);

}  // namespace pconv
