// Internal interface of the SWAR-32 temporal kernel (kernels/stencil_swar.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <utility>
#include <vector>

#include "pconv/kernels.hpp"

namespace pconv {

// Tile of the SWAR kernel: lw bytes per lane per strip (4 or 8), m rows per
// wave, nw waves stacked vertically per workgroup.
struct SwarShape {
  int lw = 8, m = 8, nw = 8;
};

// Latency model of one launch (cycles) and the shape it picks.
double swar_launch_cycles(SwarShape s, int steps, int ch, int64_t rows, int64_t row_bytes);
SwarShape pick_swar_shape(int steps, int ch, int64_t rows, int64_t row_bytes);

// Enqueue the fused gaussian for `a.steps` repetitions.  Shape: forced
// (set_swar_shape), else tuned on first use (the model's best candidates
// timed on this launch; set_autotune(false): model only), else the model's
// pick while a graph is being captured.
void launch_swar(const StencilLaunch& a, Channels ch, hipStream_t stream);
// Tune (if needed) without enqueueing the launch — before a graph capture.
void prepare_swar(const StencilLaunch& a, Channels ch, hipStream_t stream);
void set_autotune(bool on);
// How many of the model's best shapes the tuner times (default 6).
void set_tune_candidates(int n);
void clear_swar_tuning();
// Tuned entries: ({channels, steps, rows, row_bytes, step_form, kernel}, shape); kernel 0: the tile
// kernel k_swar, 1: the buffer-op tile kernel k_swar_pf.
std::vector<std::pair<std::vector<int64_t>, SwarShape>> swar_tuned();

// Force a tile shape (lw = 0 restores the model) and list the instantiated ones.
void set_swar_shape(int lw, int m, int nw);
std::vector<SwarShape> swar_shapes();
// VGPRs per lane and LDS bytes of one instantiation as the runtime reports
// them (measured = false: no device, model estimate).
struct SwarResources {
  int vgpr = 0;
  int lds = 0;
  bool measured = false;
};
SwarResources swar_resources(SwarShape s, int ch);
// XCD-aware tile order of the SWAR kernels (default on).
void set_xcd_swizzle(bool on);
// Step form: -1 tuned per launch geometry (default), 0 truncate every step,
// 1 steps in pairs with a scale-16 intermediate (larger modes clamp to 1).
void set_swar_alt(int mode);
// Buffer-op tile kernel (k_swar_pf): -1 among the tuned candidates
// (default), 0 never, 1 forced; with the mode forced, a shape set by
// set_swar_shape that it instantiates is used as is (tests).
void set_prefetch_mode(int mode);
std::vector<SwarShape> swar_prefetch_shapes();

}  // namespace pconv
