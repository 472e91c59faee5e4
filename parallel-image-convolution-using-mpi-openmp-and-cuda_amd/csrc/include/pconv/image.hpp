// Image geometry and the padded "frame" layout shared by the CPU oracle and
// the device buffers.
//
// The reference keeps a calloc'd (R+2) x (C+2) (grey) or (R+2) x (3C+6) (RGB)
// block whose zero ring doubles as the zero boundary (mpi/mpi_convolution.c:
// 104-124) and indexes it with offset(a,i,j,pitch) (:324-326).  pconv keeps the
// same idea but sizes it for 16-byte vector access:
//
//   * a row holds `row_bytes = width * channels` interleaved bytes;
//   * every frame row is `pitch` bytes: kPadLeft zero bytes, the row, then at
//     least kPadRight zero bytes (pitch rounded up to kPitchAlign);
//   * `halo` zero/ghost rows sit above and below the owned rows.
// Kernels never branch on the left/right/top/bottom image edge: they read the
// zero pad.  All offsets are 64-bit (the reference used int).
#pragma once

#include <cstddef>
#include <cstdint>

#include "pconv/common.hpp"

namespace pconv {

constexpr int kPadLeft = 16;     // keeps data rows 16-byte aligned
constexpr int kPadRight = 32;    // covers the +ch taps and one 16-B over-read
constexpr int kPitchAlign = 128;

struct ImageGeom {
  int64_t width = 0;   // pixels per row
  int64_t height = 0;  // rows
  Channels channels = Channels::Grey;

  int ch() const { return channel_count(channels); }
  int64_t row_bytes() const { return width * ch(); }
  int64_t bytes() const { return row_bytes() * height; }
  int64_t pixels() const { return width * height; }
  void validate() const;
};

// Frame = rows [-halo, rows + halo) x bytes [-kPadLeft, pitch - kPadLeft).
struct FrameLayout {
  int64_t row_bytes = 0;
  int64_t rows = 0;   // owned rows
  int64_t halo = 0;   // ghost rows on each side
  int64_t pitch = 0;

  static FrameLayout make(int64_t row_bytes, int64_t rows, int64_t halo);
  int64_t total_rows() const { return rows + 2 * halo; }
  int64_t bytes() const { return total_rows() * pitch; }
  // Byte offset of (owned row r, data column 0); r may be in [-halo, rows+halo).
  int64_t offset(int64_t r) const { return (r + halo) * pitch + kPadLeft; }
};

}  // namespace pconv
