// Raw (headerless) 8-bit image I/O.
//
// Reference: MPI-IO per-row seek+read of the owned block (mpi/mpi_convolution.c:
// 126-140) and seek+write into "blur_"+argv[1] (:244-262); POSIX
// read_info/write_info loops (cuda/functions.c:31-45) used by cuda/main.c:23-44.
// Fixed here: return codes are checked, a short file is an
// error (read_info spun forever at EOF), the output is truncated (O_TRUNC), and
// every size/offset is 64-bit.  Bands are read with pread at their own offsets
// so N ranks read disjoint parts of one file in parallel (the MPI-IO analogue).
#pragma once

#include <cstdint>
#include <string>

#include "pconv/image.hpp"

namespace pconv {

// "dir/x.raw" -> "dir/blur_x.raw" (reference: "blur_" + argv[1], which breaks
// for paths with a directory component; identical for bare file names).
std::string output_path_for(const std::string& input_path, const std::string& prefix = "blur_");

int64_t file_size(const std::string& path);

// Check that the file holds exactly geom.bytes() (or at least, if !exact).
void validate_input_file(const std::string& path, const ImageGeom& geom, bool exact = false);

// Read global rows [y0, y0+rows) into dst with the given destination pitch
// (dst points at the first byte of row y0).
void read_rows(const std::string& path, const ImageGeom& geom, int64_t y0, int64_t rows,
               uint8_t* dst, int64_t dst_pitch);

// Create/truncate the output file to geom.bytes() (done once, by one rank).
void create_output(const std::string& path, const ImageGeom& geom);

// Write global rows [y0, y0+rows) from src (pitch src_pitch) into an existing file.
void write_rows(const std::string& path, const ImageGeom& geom, int64_t y0, int64_t rows,
                const uint8_t* src, int64_t src_pitch);

// Whole-image convenience wrappers (contiguous, pitch == row_bytes).
void read_image(const std::string& path, const ImageGeom& geom, uint8_t* dst);
void write_image(const std::string& path, const ImageGeom& geom, const uint8_t* src);

// Deterministic synthetic random-byte image (splitmix64 stream), used by the
// bench and by `--synthetic SEED`; fills rows [y0, y0+rows) exactly as the
// whole-image generator would, so ranks can synthesise their band locally.
void synth_rows(const ImageGeom& geom, uint64_t seed, int64_t y0, int64_t rows,
                uint8_t* dst, int64_t dst_pitch);

}  // namespace pconv
