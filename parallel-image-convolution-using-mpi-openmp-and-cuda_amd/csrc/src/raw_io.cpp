// Raw image I/O with pread/pwrite at 64-bit offsets (see raw_io.hpp).
#include "pconv/raw_io.hpp"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <vector>

namespace pconv {

namespace {

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) ::close(fd);
  }
};

std::string errno_str() { return std::strerror(errno); }

void pread_all(int fd, uint8_t* dst, int64_t n, int64_t off, const std::string& path) {
  int64_t done = 0;
  while (done < n) {
    const ssize_t r = ::pread(fd, dst + done, static_cast<size_t>(n - done), off + done);
    if (r < 0) {
      if (errno == EINTR) continue;
      PCONV_FAIL("read " + path + ": " + errno_str());
    }
    if (r == 0) PCONV_FAIL("read " + path + ": unexpected end of file at byte " + std::to_string(off + done));
    done += r;
  }
}

void pwrite_all(int fd, const uint8_t* src, int64_t n, int64_t off, const std::string& path) {
  int64_t done = 0;
  while (done < n) {
    const ssize_t r = ::pwrite(fd, src + done, static_cast<size_t>(n - done), off + done);
    if (r < 0) {
      if (errno == EINTR) continue;
      PCONV_FAIL("write " + path + ": " + errno_str());
    }
    if (r == 0) PCONV_FAIL("write " + path + ": no progress at byte " + std::to_string(off + done));
    done += r;
  }
}

}  // namespace

std::string output_path_for(const std::string& input_path, const std::string& prefix) {
  const auto slash = input_path.find_last_of('/');
  if (slash == std::string::npos) return prefix + input_path;
  return input_path.substr(0, slash + 1) + prefix + input_path.substr(slash + 1);
}

int64_t file_size(const std::string& path) {
  struct stat st;
  if (::stat(path.c_str(), &st) != 0) PCONV_FAIL("cannot open " + path + ": " + errno_str());
  return static_cast<int64_t>(st.st_size);
}

void validate_input_file(const std::string& path, const ImageGeom& geom, bool exact) {
  geom.validate();
  const int64_t sz = file_size(path);
  const int64_t need = geom.bytes();
  if (sz < need || (exact && sz != need))
    PCONV_FAIL(path + " holds " + std::to_string(sz) + " bytes, a " + std::to_string(geom.width) + "x" +
               std::to_string(geom.height) + " " + channels_name(geom.channels) + " image needs " +
               std::to_string(need));
}

void read_rows(const std::string& path, const ImageGeom& geom, int64_t y0, int64_t rows, uint8_t* dst,
               int64_t dst_pitch) {
  PCONV_CHECK(y0 >= 0 && rows >= 0 && y0 + rows <= geom.height, "read_rows: row range out of image");
  if (rows == 0) return;
  Fd f;
  f.fd = ::open(path.c_str(), O_RDONLY);
  if (f.fd < 0) PCONV_FAIL("cannot open " + path + ": " + errno_str());
  const int64_t rb = geom.row_bytes();
  if (dst_pitch == rb) {
    pread_all(f.fd, dst, rb * rows, rb * y0, path);
    return;
  }
  // Strided destination (a padded frame): read in large contiguous chunks
  // through a bounce buffer instead of one syscall per row.
  const int64_t chunk_rows = std::max<int64_t>(1, (int64_t(8) << 20) / rb);
  std::vector<uint8_t> tmp(static_cast<size_t>(std::min(rows, chunk_rows) * rb));
  for (int64_t r = 0; r < rows; r += chunk_rows) {
    const int64_t n = std::min(chunk_rows, rows - r);
    pread_all(f.fd, tmp.data(), n * rb, rb * (y0 + r), path);
    for (int64_t i = 0; i < n; ++i) std::memcpy(dst + (r + i) * dst_pitch, tmp.data() + i * rb, rb);
  }
}

void create_output(const std::string& path, const ImageGeom& geom) {
  Fd f;
  f.fd = ::open(path.c_str(), O_CREAT | O_WRONLY | O_TRUNC, 0644);
  if (f.fd < 0) PCONV_FAIL("cannot open-create " + path + ": " + errno_str());
  if (::ftruncate(f.fd, geom.bytes()) != 0) PCONV_FAIL("truncate " + path + ": " + errno_str());
}

void write_rows(const std::string& path, const ImageGeom& geom, int64_t y0, int64_t rows, const uint8_t* src,
                int64_t src_pitch) {
  PCONV_CHECK(y0 >= 0 && rows >= 0 && y0 + rows <= geom.height, "write_rows: row range out of image");
  if (rows == 0) return;
  Fd f;
  f.fd = ::open(path.c_str(), O_WRONLY);
  if (f.fd < 0) PCONV_FAIL("cannot open " + path + " for writing: " + errno_str());
  const int64_t rb = geom.row_bytes();
  if (src_pitch == rb) {
    pwrite_all(f.fd, src, rb * rows, rb * y0, path);
    return;
  }
  const int64_t chunk_rows = std::max<int64_t>(1, (int64_t(8) << 20) / rb);
  std::vector<uint8_t> tmp(static_cast<size_t>(std::min(rows, chunk_rows) * rb));
  for (int64_t r = 0; r < rows; r += chunk_rows) {
    const int64_t n = std::min(chunk_rows, rows - r);
    for (int64_t i = 0; i < n; ++i) std::memcpy(tmp.data() + i * rb, src + (r + i) * src_pitch, rb);
    pwrite_all(f.fd, tmp.data(), n * rb, rb * (y0 + r), path);
  }
}

void read_image(const std::string& path, const ImageGeom& geom, uint8_t* dst) {
  validate_input_file(path, geom);
  read_rows(path, geom, 0, geom.height, dst, geom.row_bytes());
}

void write_image(const std::string& path, const ImageGeom& geom, const uint8_t* src) {
  create_output(path, geom);
  write_rows(path, geom, 0, geom.height, src, geom.row_bytes());
}

namespace {
inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
}  // namespace

void synth_rows(const ImageGeom& geom, uint64_t seed, int64_t y0, int64_t rows, uint8_t* dst, int64_t dst_pitch) {
  // Byte i of the image is byte (i % 8) of splitmix64(seed * 2^40 + i / 8):
  // random-access, so any band is generated independently and identically.
  const int64_t rb = geom.row_bytes();
  const uint64_t base = seed << 40;
#pragma omp parallel for schedule(static) if (rows * rb > (int64_t(1) << 22))
  for (int64_t r = 0; r < rows; ++r) {
    uint8_t* out = dst + r * dst_pitch;
    const int64_t g0 = (y0 + r) * rb;
    uint64_t w = splitmix64(base + static_cast<uint64_t>(g0 >> 3));
    for (int64_t x = 0; x < rb; ++x) {
      const int64_t g = g0 + x;
      if ((g & 7) == 0) w = splitmix64(base + static_cast<uint64_t>(g >> 3));
      out[x] = static_cast<uint8_t>(w >> (8 * (g & 7)));
    }
  }
}

}  // namespace pconv
