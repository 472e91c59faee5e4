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

// ---------------------------------------------------------------------------
// Row streaming WITHIN one image.
//
// The reference's GPU_convolution() (cuda/cuda_convolution.cu:60-97) is a
// serial chain: H2D of the whole image, every repetition, D2H of the whole
// image.  Here the input rows arrive in C chunks (top to bottom) and every
// level of an exchange-free plan (level j = the output of plan launch j) is
// advanced as far as the rows uploaded so far allow, so the H2D of chunk c+1,
// the launches of chunk c and the D2H of the rows finished by chunk c-1 run
// at the same time on three streams.  No row is uploaded twice: a level's
// launch near a chunk boundary reads the rows of the previous chunk that are
// already resident on the device.
//
// Fronts: W_0(c) = u_c (rows uploaded after chunk c) and, for level j with
// s_j steps (s_0 = 0), W_j(c) = W_{j-1}(c) - max(s_j, s_{j-1}) clipped to
// the level's region [lo_j, hi_j); after the last chunk (or once level j-1
// is complete) W_j = hi_j.  Chunk c's launch of level j computes
// [W_j(c-1), W_j(c)).  Why it is race-free with only two frames (level j is
// written into frame j % 2, over level j-2):
//   * reads of level j-1 stop at W_j(c) + s_j <= W_{j-1}(c): rows already
//     computed (or outside the image after the last chunk);
//   * level j overwrites level j-2 only below W_{j-1}(c) - s_{j-1}, the first
//     level-(j-2) row the next chunk's level-(j-1) launch still reads;
//   * uploads write frame 0 at rows >= u_c, above every row any launch of
//     chunks <= c reads or writes; downloads read final rows below W_L(c),
//     which no later launch writes.
// tests/test_stream_plan.py checks these read/write sets exhaustively and
// replays plans on the CPU against the oracle.
struct StreamChunk {
  int64_t up_lo = 0, up_hi = 0;      // input rows uploaded by this chunk (frame-local, may be empty)
  std::vector<LaunchSpec> launches;  // in stream order
  std::vector<int> levels;           // 1-based level of each launch (reads frame (level-1)%2, writes level%2)
  int64_t down_lo = 0, down_hi = 0;  // owned rows final after this chunk's launches (may be empty)
};

struct StreamPlan {
  int levels = 0;  // L = launches of the underlying plan; the result ends in frame L % 2
  std::vector<StreamChunk> chunks;
};

// True when `plan` can be streamed: >= 1 phase, no exchange, one launch each.
bool streamable(const std::vector<Phase>& plan);

// Upload boundaries for `chunks` chunks of input rows [in_lo, in_hi): even
// chunks, the last one 6/5 as tall (weights 5, ..., 5, 6).  A chunk's
// launches cost about the same whatever its rows (the kernel's per-step
// latency on a small grid), so small chunks only lengthen the compute chain:
// one headline image 0.5325-0.5376 ms with 3,3,3,4 / 4,4,4,5 / 5,5,5,6 /
// 4,5,5,5 against 0.5480-0.5517 with the former 1, 2, 2, 1 (half-size first
// and last chunks), window ms/step unchanged (profiles/r06/o, p).
std::vector<int64_t> stream_cuts(int64_t in_lo, int64_t in_hi, int chunks);
// Upload boundaries for chunks of rows in proportion to `weights` (one
// chunk per weight, each > 0); chunks that would be empty are merged.
std::vector<int64_t> stream_cuts_weighted(int64_t in_lo, int64_t in_hi, const std::vector<int>& weights);

// cuts: strictly increasing interior boundaries (in_lo < cut < in_hi).
StreamPlan plan_streamed(const std::vector<Phase>& plan, int64_t in_lo, int64_t in_hi, int64_t owned_rows,
                         const std::vector<int64_t>& cuts);

// Clamp a requested halo depth / fuse to what the band layout allows.
PlanConfig normalize_plan_config(PlanConfig cfg, int64_t min_band_rows, int max_fuse);

}  // namespace pconv
