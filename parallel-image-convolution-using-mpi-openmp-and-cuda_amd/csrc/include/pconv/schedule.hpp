// Rep-loop schedule for one row band: when to exchange halos, which rows each
// launch computes, and which launches may overlap the exchange.
//
// Reference loop (mpi/mpi_convolution.c:156-240), per rep: post Isend/Irecv of
// depth-1 halos to <=4 neighbours, compute the WHOLE block (reading halo cells
// whose Irecv is still pending — undefined behaviour), then per neighbour wait
// and recompute that edge strip, recompute corners, wait sends, swap.
//
// pconv generalises it to deep halos + temporal fusion:
//   * exchange `halo_depth` (D) ghost rows at once, every D reps at most;
//   * between exchanges each launch advances `steps` (<= fuse T) reps and
//     computes a region that shrinks by `steps` rows into the ghost zone, so
//     no rep needs fresh neighbour data until the ghost rows are used up
//     (communication-avoiding "ghost zone expansion");
//   * in an exchange phase the interior launch (reads owned rows only) is
//     marked `after_halo = false` and runs concurrently with the exchange; the
//     two boundary launches wait for it.  Interior/boundary are disjoint by
//     construction, so nothing reads a row that is still being received.
// The same plan drives the GPU engine (HIP + RCCL), the one-device N-band
// emulator and the CPU/gloo emulator, so the CPU tests check the exact
// schedule the GPUs run.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "pconv/partition.hpp"

namespace pconv {

struct LaunchSpec {
  int steps = 1;          // reps advanced by this launch
  int64_t lo = 0, hi = 0; // output rows [lo, hi), frame-local (may reach into ghost rows)
  bool after_halo = false;
};

struct Phase {
  int64_t exchange_depth = 0;  // > 0: exchange this many ghost rows before computing
  int steps = 1;               // every launch of a phase advances the same reps
  std::vector<LaunchSpec> launches;
};

struct PlanConfig {
  int halo_depth = 1;          // D: ghost rows exchanged at once (>= fuse)
  int fuse = 1;                // T: max reps per launch
  bool overlap = true;         // split interior/boundary around exchanges
  bool halo_preloaded = false; // ghost rows already valid before the first phase
};

std::vector<Phase> plan_band(const Band& band, int reps, const PlanConfig& cfg);

// Human-readable dump (tests / --explain).
std::string describe_plan(const std::vector<Phase>& plan);

// Clamp a requested halo depth / fuse to what the band layout allows.
PlanConfig normalize_plan_config(PlanConfig cfg, int64_t min_band_rows, int max_fuse);

}  // namespace pconv
