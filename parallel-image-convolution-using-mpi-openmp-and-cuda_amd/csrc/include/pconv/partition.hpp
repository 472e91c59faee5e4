// Domain decomposition.
//
// The reference picks a 2-D process grid with RowsDivision()
// (mpi/mpi_convolution.c:350-364): rows_to | n, rows_to | H, (n/rows_to) | W,
// minimising H/rows_to + W/cols_to, ties -> smallest rows_to; it aborts
// "Cannot divide to processes" otherwise (:53-58).  Its 2-D blocks miss the
// diagonal halo corners.
//
// pconv decomposes into contiguous ROW BANDS: any H >= n, remainder rows go to
// the first H % n ranks.  Halos are then whole contiguous rows (one RCCL
// message per neighbour, no derived datatypes, no corners).  The reference's
// grid chooser is kept (`reference_rows_division`) for parity tests and for
// the 2-D block mode of the CPU emulator.
#pragma once

#include <cstdint>
#include <vector>

namespace pconv {

struct Band {
  int rank = 0;
  int world = 1;
  int64_t y0 = 0;     // first owned global row
  int64_t rows = 0;   // owned rows
  int up = -1;        // rank owning rows above (y0-1), -1 at the image top
  int down = -1;      // rank owning rows below, -1 at the image bottom
};

// Row-band partition of `height` rows over `world` ranks.  Throws if height < world.
Band row_band(int64_t height, int world, int rank);
std::vector<Band> row_bands(int64_t height, int world);

// Exact reimplementation of the reference's grid chooser (returns 0 on failure).
int reference_rows_division(int n_processes, int rows, int columns);

}  // namespace pconv
