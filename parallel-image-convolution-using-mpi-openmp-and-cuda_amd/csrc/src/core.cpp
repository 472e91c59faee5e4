// Core value types: errors, channels, filters, geometry, partitioning.
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <sstream>

#include "pconv/common.hpp"
#include "pconv/filter.hpp"
#include "pconv/image.hpp"
#include "pconv/partition.hpp"

namespace pconv {

// ---------------------------------------------------------------- errors
namespace {
std::atomic<int> g_rank{-1};
}

void set_error_rank(int rank) { g_rank.store(rank); }
int error_rank() { return g_rank.load(); }

void raise_error(const char* file, int line, const std::string& msg) {
  std::ostringstream os;
  const int r = g_rank.load();
  if (r >= 0) os << "[rank " << r << "] ";
  const char* base = file;
  for (const char* p = file; *p; ++p)
    if (*p == '/') base = p + 1;
  os << base << ":" << line << ": " << msg;
  throw Error(os.str());
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (char ch : s) {
    if (ch == '"' || ch == '\\') o += '\\';
    if (static_cast<unsigned char>(ch) < 0x20) {
      o += ' ';
      continue;
    }
    o += ch;
  }
  return o;
}

double wall_seconds() {
  using clk = std::chrono::steady_clock;
  return std::chrono::duration<double>(clk::now().time_since_epoch()).count();
}

// ---------------------------------------------------------------- channels
const char* channels_name(Channels c) {
  switch (c) {
    case Channels::Grey: return "grey";
    case Channels::Rgb: return "rgb";
    case Channels::Rgba: return "rgba";
  }
  return "?";
}

Channels parse_channels(const std::string& s) {
  if (s == "grey") return Channels::Grey;
  if (s == "rgb") return Channels::Rgb;
  if (s == "rgba") return Channels::Rgba;
  PCONV_FAIL("unknown image type '" + s + "' (expected grey|rgb|rgba)");
}

// ---------------------------------------------------------------- filters
Filter Filter::custom(const std::array<int, 9>& taps, int divisor, const std::string& name) {
  PCONV_CHECK(divisor > 0, "filter divisor must be positive");
  Filter f;
  f.name = name;
  f.taps = taps;
  f.divisor = divisor;
  bool nonneg = true;
  long sum = 0;
  for (int i = 0; i < 9; ++i) {
    // Reference: myFilter[i][j] = tap / 16.0 -> double division, stored as float.
    f.weights[i] = static_cast<float>(taps[i] / static_cast<double>(divisor));
    nonneg = nonneg && taps[i] >= 0;
    sum += std::abs(taps[i]);
  }
  const bool pow2 = (divisor & (divisor - 1)) == 0;
  // Exactness: every product p*tap/div and every partial sum is a multiple of
  // 1/div below 2^24/div, hence exactly representable; truncation of a
  // non-negative value == floor == arithmetic shift.
  f.int_exact = nonneg && pow2 && sum * 255L < (1L << 24);
  f.shift = 0;
  if (pow2)
    while ((1 << f.shift) < divisor) ++f.shift;
  const std::array<int, 9> b121{1, 2, 1, 2, 4, 2, 1, 2, 1};
  f.binomial121 = f.int_exact && taps == b121 && divisor == 16;
  return f;
}

Filter Filter::gaussian() { return custom({1, 2, 1, 2, 4, 2, 1, 2, 1}, 16, "gaussian"); }
Filter Filter::box() { return custom({1, 1, 1, 1, 1, 1, 1, 1, 1}, 9, "box"); }
Filter Filter::edge() { return custom({1, 4, 1, 4, 8, 4, 1, 4, 1}, 28, "edge"); }

Filter Filter::by_name(const std::string& name) {
  if (name == "gaussian") return gaussian();
  if (name == "box") return box();
  if (name == "edge" || name == "edge_detection") return edge();
  PCONV_FAIL("unknown filter '" + name + "' (expected gaussian|box|edge)");
}

int Filter::abs_sum() const {
  int s = 0;
  for (int t : taps) s += std::abs(t);
  return s;
}

// ---------------------------------------------------------------- geometry
void ImageGeom::validate() const {
  PCONV_CHECK(width > 0 && height > 0, "image width and height must be positive");
  PCONV_CHECK(width <= (int64_t(1) << 30) && height <= (int64_t(1) << 30), "image dimension too large");
}

FrameLayout FrameLayout::make(int64_t row_bytes, int64_t rows, int64_t halo) {
  PCONV_CHECK(row_bytes > 0 && rows >= 0 && halo >= 0, "bad frame layout");
  FrameLayout l;
  l.row_bytes = row_bytes;
  l.rows = rows;
  l.halo = halo;
  l.pitch = round_up<int64_t>(kPadLeft + round_up<int64_t>(row_bytes, 16) + kPadRight, kPitchAlign);
  return l;
}

// ---------------------------------------------------------------- partition
Band row_band(int64_t height, int world, int rank) {
  PCONV_CHECK(world >= 1 && rank >= 0 && rank < world, "bad rank/world");
  PCONV_CHECK(height >= world, "cannot divide " + std::to_string(height) + " rows over " +
                                   std::to_string(world) + " ranks");
  Band b;
  b.rank = rank;
  b.world = world;
  const int64_t base = height / world, rem = height % world;
  b.rows = base + (rank < rem ? 1 : 0);
  b.y0 = rank * base + std::min<int64_t>(rank, rem);
  b.up = rank > 0 ? rank - 1 : -1;
  b.down = rank + 1 < world ? rank + 1 : -1;
  return b;
}

std::vector<Band> row_bands(int64_t height, int world) {
  std::vector<Band> v;
  for (int r = 0; r < world; ++r) v.push_back(row_band(height, world, r));
  return v;
}

int reference_rows_division(int n_processes, int rows, int columns) {
  int best = 0;
  int perimeter_min = rows + columns + 1;
  for (int rows_to = 1; rows_to <= n_processes; ++rows_to) {
    if (n_processes % rows_to || rows % rows_to) continue;
    const int columns_to = n_processes / rows_to;
    if (columns % columns_to) continue;
    const int perimeter = rows / rows_to + columns / columns_to;
    if (perimeter < perimeter_min) {
      perimeter_min = perimeter;
      best = rows_to;
    }
  }
  return best;
}

}  // namespace pconv
