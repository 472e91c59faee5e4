// Device stencil kernels (CDNA4 / gfx950) — host-side launch interface.
//
// Reference kernels: kernelConvolutionforGrey / kernelConvolutionforRGB
// (cuda/cuda_convolution.cu:9-47): one thread per pixel with lanes walking
// down ROWS (uncoalesced), FP64 /16.0, border ring never written, RGB grid 3x
// too wide with out-of-bounds accesses.
//
// pconv kernels treat a row as a byte vector (RGB = 3W bytes, horizontal tap
// stride = CH bytes), so one template serves grey/RGB/RGBA:
//   * lanes walk along a row, 16 bytes per lane (dwordx4 loads/stores);
//   * the gaussian runs in packed 16-bit integer SIMD (v_perm_b32 byte
//     unpack, v_pk_add_u16 / v_pk_mad_u16, shift, v_perm_b32 repack), exactly
//     reproducing the float32 reference;
//   * each lane marches down RPT rows keeping the horizontal sums of the last
//     two rows in registers (every input row is loaded and unpacked once);
//   * the temporal-blocked SWAR kernel fuses `steps` repetitions in one
//     launch (kernels/stencil_swar.hip).
// The frame's zero pad (image.hpp) provides the boundary; no edge branches.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "pconv/filter.hpp"
#include "pconv/image.hpp"

namespace pconv {

struct StencilLaunch {
  const uint8_t* src = nullptr;  // frame: owned row 0, data column 0
  uint8_t* dst = nullptr;        // same layout as src
  int64_t pitch = 0;
  int64_t row_bytes = 0;
  int64_t r0 = 0, r1 = 0;        // output rows [r0, r1) in frame-local numbering
  int64_t frame_lo = 0;          // first readable frame row (= -halo)
  int64_t frame_hi = 0;          // one past the last readable frame row (= rows + halo)
  int steps = 1;                 // fused repetitions (temporal blocking) in this launch
  int64_t g_row0 = 0;            // global image row of frame row 0
  int64_t height = 0;            // global image height (rows outside are zero each step)
};

enum class KernelVariant : int {
  Auto = 0,      // pick by filter / steps
  Binomial = 1,  // packed-u16 gaussian, 1 step per launch
  Temporal = 2,  // SWAR-32 gaussian, `steps` fused in registers (production)
  Int9 = 3,      // generic int-exact 9-tap
  Float9 = 4,    // generic float32 9-tap (reference rounding)
  FloatTemporal = 6,  // any 3x3 filter, float32 reference rounding, `steps` fused in registers
};

const char* kernel_variant_name(KernelVariant v);

// Largest `steps` the temporal kernel accepts.
constexpr int kMaxFusedSteps = 16;

// Enqueue one stencil launch on `stream`.  Validates the geometry against the
// frame before launching (no out-of-frame access is possible).
void launch_stencil(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream,
                    KernelVariant v = KernelVariant::Auto);
// Settle per-launch choices (SWAR tile-shape tuning) for a launch that will be
// enqueued later — e.g. inside a graph capture, where nothing may be timed.
void prepare_stencil(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream,
                     KernelVariant v = KernelVariant::Auto);

// `steps` repetitions of ANY 3x3 filter in the reference's float32 semantics
// in one launch (kernels/stencil_float.hip): box/9, edge/28, custom filters.
void launch_float_temporal(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream);
// Tune the float kernel's tile shape for this launch geometry now (before a
// graph capture); clear the cache of tuned shapes.
void prepare_float_temporal(const Filter& f, Channels ch, const StencilLaunch& a, hipStream_t stream);
void clear_float_tuning();
// Force the float kernel's tile (m rows per wave, nw waves; m = 0: the model
// / tuner again).  An unknown shape is ignored.
void set_float_shape(int m, int nw);

// Whether `v` (or Auto) can fuse `steps` > 1 for this filter.
bool supports_fusion(const Filter& f, KernelVariant v);

// Default repetitions per launch for a band frame of `frame_bytes`: 1 without
// fusion; 12 for grey frames of 256 MiB and more (far beyond the Infinity
// Cache: 32768^2 grey 113.2-116.2 us/rep at 12 vs 116.9-121.1 at 8 over four
// boxes, 16384^2 30.6 vs 32.2; profiles/r02/tile_shapes.md,
// prefetch_kernel.md); 8 everywhere else (RGB's 3x wider horizontal halo makes
// deeper fusion slower; 1920x2520 RGB 3.5 us/rep at 8 vs 4.0 at 6, 8192^2 RGB
// within 2 % either way).  Other filters (float temporal kernel): 4.
int auto_fuse(const Filter& f, KernelVariant v, int64_t frame_bytes, int channels = 0);

// Row copy by the CUs: `rows` rows of `row_bytes` from src (row pitch sp) to
// dst (row pitch dp); either side may be pinned host memory (the CUs move the
// bytes over PCIe) or device memory.  No SDMA engine and no runtime blit
// program is involved — a one-shot process saves their first-use set-up
// (~8 ms per SDMA direction and the blit code object, profiles/r02/), at
// 44-53 GB/s instead of SDMA's 54 (tools/ubench/copy_bw.hip).
// max_blocks > 0 caps the grid (a copy beside stencil launches leaves them CUs).
void launch_copy_rows(const uint8_t* src, int64_t sp, uint8_t* dst, int64_t dp, int64_t row_bytes, int64_t rows,
                      hipStream_t stream, int max_blocks = 0);
// Zero `bytes` (a multiple of 16, 16-byte aligned) with a kernel of this module.
void launch_fill_zero(uint8_t* p, int64_t bytes, hipStream_t stream);
// Load the code object of the temporal / copy kernels now (a one-shot process
// calls it from a helper thread while it creates its first hardware queue).
void preload_kernel_module();

// Empirical tile-shape tuning on / off (off: the latency model's pick);
// returns the previous setting.  A one-shot process turns it off: timing a
// dozen candidates costs more than the loop they would speed up.
bool set_shape_tuning(bool on);
bool shape_tuning_enabled();

}  // namespace pconv
