// pconv — MI355X-native 2-D image-convolution stencil engine.
//
// Common types, error handling and small utilities shared by every layer.
//
// Reference parity notes
//   * `color_t {GREY, RGB}` (mpi/mpi_convolution.c:8) and the *reversed* enum in
//     cuda/functions.h:20 are replaced by `Channels`, whose value is the byte
//     stride of one pixel.  The kernels are templated on it.
//   * `CUDA_SAFE_CALL` (cuda/functions.h:10-16) becomes PCONV_HIP_CHECK /
//     PCONV_RCCL_CHECK, which throw a rank-tagged pconv::Error instead of
//     calling exit() so the Python layer and the CLI can report failures.
//   * `FRACTION_CEILING` (cuda/functions.h:18) becomes ceil_div().
#pragma once

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace pconv {

// Pixel layout: value == bytes per pixel (interleaved), so row_bytes = W * ch.
enum class Channels : int { Grey = 1, Rgb = 3, Rgba = 4 };

inline int channel_count(Channels c) { return static_cast<int>(c); }
const char* channels_name(Channels c);
Channels parse_channels(const std::string& s);  // "grey" | "rgb" | "rgba"

// Thrown by every layer.  `what()` carries "[rank R] where: message".
class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& msg) : std::runtime_error(msg) {}
};

// Process-wide rank tag used in error messages (set by the distributed layer).
void set_error_rank(int rank);
int error_rank();
[[noreturn]] void raise_error(const char* file, int line, const std::string& msg);

template <typename T>
constexpr T ceil_div(T a, T b) { return (a + b - 1) / b; }
template <typename T>
constexpr T round_up(T a, T b) { return ceil_div(a, b) * b; }

// Monotonic wall clock in seconds (replaces micro_time(), cuda/functions.c:47-51,
// whose gettimeofday call sat inside assert() and vanished under NDEBUG).
double wall_seconds();

// Escape a free-form string (paths, error text) for a JSON string literal.
std::string json_escape(const std::string& s);

}  // namespace pconv

#define PCONV_FAIL(msg) ::pconv::raise_error(__FILE__, __LINE__, (msg))
#define PCONV_CHECK(cond, msg)                 \
  do {                                         \
    if (!(cond)) ::pconv::raise_error(__FILE__, __LINE__, (msg)); \
  } while (0)
