// Native unit tests for the host-side runtime (no GPU, no HIP calls):
// partitioner, filters, CPU oracle, distributed schedule, raw I/O, CLI,
// synthetic images.  Built by `make -C <pkg>/csrc test-native` with
// AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5 "race detection /
// sanitizers": ASan/UBSan on CPU code) and run by tests/test_native_cpp.py.
//
// The oracle here is deliberately naive and independent of cpu_stencil.cpp:
// double loops over a zero-padded copy, integer or float32 sequential MAC.
#include <unistd.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "pconv/cli.hpp"
#include "pconv/cpu_stencil.hpp"
#include "pconv/filter.hpp"
#include "pconv/image.hpp"
#include "pconv/partition.hpp"
#include "pconv/raw_io.hpp"
#include "pconv/schedule.hpp"

using namespace pconv;

namespace {

int g_failures = 0, g_checks = 0;

#define EXPECT(cond)                                                         \
  do {                                                                       \
    ++g_checks;                                                              \
    if (!(cond)) {                                                           \
      ++g_failures;                                                          \
      std::fprintf(stderr, "%s:%d: EXPECT failed: %s\n", __FILE__, __LINE__, #cond); \
    }                                                                        \
  } while (0)

bool throws(const std::function<void()>& f) {
  try {
    f();
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

// ---------------------------------------------------------------- oracle
std::vector<uint8_t> naive_step(const Filter& f, const std::vector<uint8_t>& in, int64_t w, int64_t h, int ch) {
  std::vector<uint8_t> out(in.size());
  for (int64_t y = 0; y < h; ++y)
    for (int64_t x = 0; x < w; ++x)
      for (int c = 0; c < ch; ++c) {
        auto px = [&](int64_t yy, int64_t xx) -> int {
          if (yy < 0 || yy >= h || xx < 0 || xx >= w) return 0;
          return in[(yy * w + xx) * ch + c];
        };
        int v;
        if (f.int_exact) {
          int acc = 0;
          for (int k = 0; k < 3; ++k)
            for (int l = 0; l < 3; ++l) acc += f.taps[k * 3 + l] * px(y + k - 1, x + l - 1);
          v = acc >> f.shift;
        } else {
          float acc = 0.0f;
          for (int k = 0; k < 3; ++k)
            for (int l = 0; l < 3; ++l) {
              volatile float prod = static_cast<float>(px(y + k - 1, x + l - 1)) * f.weights[k * 3 + l];
              acc = acc + prod;
            }
          v = static_cast<int>(acc);
        }
        out[(y * w + x) * ch + c] = static_cast<uint8_t>(v < 0 ? 0 : v > 255 ? 255 : v);
      }
  return out;
}

std::vector<uint8_t> naive(const Filter& f, std::vector<uint8_t> img, int64_t w, int64_t h, int ch, int reps) {
  for (int r = 0; r < reps; ++r) img = naive_step(f, img, w, h, ch);
  return img;
}

std::vector<uint8_t> random_bytes(size_t n, uint32_t seed) {
  std::mt19937 g(seed);
  std::vector<uint8_t> v(n);
  for (auto& b : v) b = static_cast<uint8_t>(g() & 0xff);
  return v;
}

Channels chan(int c) { return c == 1 ? Channels::Grey : c == 3 ? Channels::Rgb : Channels::Rgba; }

// ---------------------------------------------------------------- tests
void test_partition() {
  for (int64_t h = 1; h <= 41; ++h)
    for (int n = 1; n <= 8 && n <= h; ++n) {
      const auto bs = row_bands(h, n);
      EXPECT(static_cast<int>(bs.size()) == n);
      int64_t y = 0;
      for (int r = 0; r < n; ++r) {
        const Band& b = bs[r];
        EXPECT(b.y0 == y && b.rows >= 1);
        EXPECT(b.rows == h / n + (r < h % n ? 1 : 0));  // remainder to the first ranks
        EXPECT(b.up == (r > 0 ? r - 1 : -1) && b.down == (r < n - 1 ? r + 1 : -1));
        const Band one = row_band(h, n, r);
        EXPECT(one.y0 == b.y0 && one.rows == b.rows);
        y += b.rows;
      }
      EXPECT(y == h);
    }
  EXPECT(throws([] { row_band(3, 4, 0); }));
  // The reference grid choice (mpi/mpi_convolution.c:350-364) for 1920x2520.
  EXPECT(reference_rows_division(4, 2520, 1920) == 2);
  EXPECT(reference_rows_division(16, 2520, 1920) == 4);
}

void test_filters() {
  const Filter g = Filter::gaussian(), b = Filter::box(), e = Filter::edge();
  EXPECT(g.int_exact && g.binomial121 && g.shift == 4);
  EXPECT(!b.int_exact && !e.int_exact);
  EXPECT(Filter::by_name("edge").divisor == 28 && throws([] { Filter::by_name("sobel"); }));
  // gaussian: float32 reference semantics == integer formula.
  std::mt19937 rng(7);
  int bad = 0;
  for (int t = 0; t < 200000; ++t) {
    int p[9], acc = 0;
    float facc = 0.0f;
    for (int i = 0; i < 9; ++i) {
      p[i] = static_cast<int>(rng() & 0xff);
      acc += g.taps[i] * p[i];
      volatile float prod = static_cast<float>(p[i]) * g.weights[i];
      facc = facc + prod;
    }
    bad += (acc >> 4) != static_cast<int>(facc);
  }
  EXPECT(bad == 0);
}

void test_cpu_oracle() {
  for (const char* fname : {"gaussian", "box", "edge"})
    for (int ch : {1, 3, 4})
      for (auto wh : {std::pair<int, int>{1, 1}, {1, 7}, {9, 1}, {3, 3}, {17, 11}, {33, 20}})
        for (int reps : {0, 1, 2, 5}) {
          const Filter f = Filter::by_name(fname);
          const int64_t w = wh.first, h = wh.second;
          const auto img = random_bytes(static_cast<size_t>(w * h * ch), static_cast<uint32_t>(w * 131 + h + ch));
          const auto ref = naive(f, img, w, h, ch, reps);
          ImageGeom geo{w, h, chan(ch)};
          std::vector<uint8_t> a(img.size()), o(img.size());
          cpu_convolve(f, geo, img.data(), a.data(), reps, CpuBackend::Serial);
          cpu_convolve(f, geo, img.data(), o.data(), reps, CpuBackend::OpenMP, 3);
          EXPECT(a == ref);
          EXPECT(o == ref);
        }
}

// The distributed schedule on CPU frames: bands, deep halos, fused launches,
// interior/boundary split; ghost rows copied between neighbours' frames.
void test_distributed_schedule() {
  const Filter f = Filter::gaussian();
  const int64_t w = 23, h = 37;
  const int ch = 3;
  const auto img = random_bytes(static_cast<size_t>(w * h * ch), 99);
  for (int world : {1, 2, 3, 5})
    for (int D : {1, 2, 4, 7})
      for (int T : {1, 2, 4})
        for (bool overlap : {false, true})
          for (bool preload : {false, true})
            for (int reps : {0, 1, 6, 13}) {
              if (T > D) continue;
              const ImageGeom geo{w, h, Channels::Rgb};
              const int64_t rb = geo.row_bytes();
              struct B {
                Band band;
                FrameLayout lay;
                std::vector<uint8_t> fr[2];
                int cur = 0;
              };
              std::vector<B> bs(world);
              PlanConfig cfg;
              cfg.halo_depth = D;
              cfg.fuse = T;
              cfg.overlap = overlap;
              cfg = normalize_plan_config(cfg, world > 1 ? h / world : 0, 16);
              for (int r = 0; r < world; ++r) {
                B& x = bs[r];
                x.band = row_band(h, world, r);
                x.lay = FrameLayout::make(rb, x.band.rows, cfg.halo_depth);
                for (auto& v : x.fr) v.assign(static_cast<size_t>(x.lay.bytes()), 0);
                int64_t a = 0, e = x.band.rows;
                if (preload && world > 1) {
                  a = -std::min<int64_t>(cfg.halo_depth, x.band.y0);
                  e = x.band.rows + std::min<int64_t>(cfg.halo_depth, h - x.band.y0 - x.band.rows);
                }
                for (int64_t row = a; row < e; ++row)
                  std::memcpy(x.fr[0].data() + x.lay.offset(row), img.data() + (x.band.y0 + row) * rb, rb);
              }
              std::vector<std::vector<Phase>> plans;
              for (auto& x : bs) {
                PlanConfig c = cfg;
                c.halo_preloaded = preload && world > 1;
                plans.push_back(plan_band(x.band, reps, c));
              }
              for (size_t i = 0; i < plans[0].size(); ++i) {
                for (int r = 0; r < world; ++r) {
                  const int64_t d = plans[r][i].exchange_depth;
                  if (!d) continue;
                  B& x = bs[r];
                  if (x.band.up >= 0) {
                    B& p = bs[x.band.up];
                    std::memcpy(x.fr[x.cur].data() + x.lay.offset(-d) - kPadLeft,
                                p.fr[p.cur].data() + p.lay.offset(p.band.rows - d) - kPadLeft, d * x.lay.pitch);
                  }
                  if (x.band.down >= 0) {
                    B& p = bs[x.band.down];
                    std::memcpy(x.fr[x.cur].data() + x.lay.offset(x.band.rows) - kPadLeft,
                                p.fr[p.cur].data() + p.lay.offset(0) - kPadLeft, d * x.lay.pitch);
                  }
                }
                for (int r = 0; r < world; ++r) {
                  B& x = bs[r];
                  for (const auto& l : plans[r][i].launches)
                    cpu_fused_launch(f, geo.channels, x.lay, x.fr[x.cur].data(), x.fr[x.cur ^ 1].data(), l.lo, l.hi,
                                     l.steps, x.band.y0, h, CpuBackend::Serial);
                  x.cur ^= 1;
                }
              }
              std::vector<uint8_t> got(img.size());
              for (auto& x : bs)
                for (int64_t row = 0; row < x.band.rows; ++row)
                  std::memcpy(got.data() + (x.band.y0 + row) * rb, x.fr[x.cur].data() + x.lay.offset(row), rb);
              const bool ok = got == naive(f, img, w, h, ch, reps);
              if (!ok)
                std::fprintf(stderr, "schedule mismatch: world=%d D=%d T=%d overlap=%d preload=%d reps=%d\n", world, D,
                             T, overlap, preload, reps);
              EXPECT(ok);
            }
}

void test_raw_io() {
  char tmpl[] = "/tmp/pconv_native_XXXXXX";
  const char* dir = mkdtemp(tmpl);
  EXPECT(dir != nullptr);
  const std::string d(dir ? dir : "/tmp");
  const ImageGeom geo{13, 9, Channels::Rgb};
  const auto img = random_bytes(static_cast<size_t>(geo.bytes()), 5);
  const std::string p = d + "/img.raw";
  write_image(p, geo, img.data());
  EXPECT(file_size(p) == geo.bytes());
  std::vector<uint8_t> back(img.size());
  read_image(p, geo, back.data());
  EXPECT(back == img);
  // rows [3, 7) into a pitched buffer
  const int64_t pitch = geo.row_bytes() + 5;
  std::vector<uint8_t> rows(static_cast<size_t>(4 * pitch), 0xCD);
  read_rows(p, geo, 3, 4, rows.data(), pitch);
  bool rows_ok = true;
  for (int r = 0; r < 4; ++r) {
    rows_ok &= std::memcmp(rows.data() + r * pitch, img.data() + (3 + r) * geo.row_bytes(), geo.row_bytes()) == 0;
    rows_ok &= rows[r * pitch + geo.row_bytes()] == 0xCD;  // pad untouched
  }
  EXPECT(rows_ok);
  // short and missing files are errors (the reference spun forever / read zeros)
  const ImageGeom big{13, 10, Channels::Rgb};
  EXPECT(throws([&] { validate_input_file(p, big); }));
  EXPECT(throws([&] { validate_input_file(d + "/missing.raw", geo); }));
  // create_output truncates a longer stale file (the reference kept its tail)
  const std::string o = d + "/out.raw";
  const ImageGeom huge{100, 100, Channels::Grey};
  std::vector<uint8_t> junk(static_cast<size_t>(huge.bytes()), 7);
  write_image(o, huge, junk.data());
  create_output(o, geo);
  EXPECT(file_size(o) == geo.bytes());
  write_rows(o, geo, 0, geo.height, img.data(), geo.row_bytes());
  read_image(o, geo, back.data());
  EXPECT(back == img);
  EXPECT(output_path_for("img.raw") == "blur_img.raw");
  EXPECT(output_path_for("a/b/img.raw") == "a/b/blur_img.raw");
  std::remove(p.c_str());
  std::remove(o.c_str());
  rmdir(d.c_str());
}

void test_synthetic() {
  const ImageGeom geo{31, 29, Channels::Rgb};
  std::vector<uint8_t> whole(static_cast<size_t>(geo.bytes())), parts(whole.size());
  synth_rows(geo, 42, 0, geo.height, whole.data(), geo.row_bytes());
  int64_t y = 0;
  for (int64_t n : {5, 1, 13, 10}) {
    synth_rows(geo, 42, y, n, parts.data() + y * geo.row_bytes(), geo.row_bytes());
    y += n;
  }
  EXPECT(whole == parts);
  std::vector<uint8_t> other(whole.size());
  synth_rows(geo, 43, 0, geo.height, other.data(), geo.row_bytes());
  EXPECT(other != whole);
}

void test_cli() {
  const auto c = parse_cli({"conv", "img.raw", "1920", "2520", "40", "rgb", "--gpus", "4", "--filter", "box",
                            "--halo", "8", "--fuse", "4", "--transport", "shm", "--exchange-halo", "--json"});
  EXPECT(c.width == 1920 && c.height == 2520 && c.reps == 40 && c.channels == Channels::Rgb);
  EXPECT(c.gpus == 4 && c.filter == "box" && c.halo == 8 && c.fuse == 4 && c.transport == "shm");
  EXPECT(!c.preload_halo && c.json);
  EXPECT(throws([] { parse_cli({"conv", "img.raw", "10", "10", "1"}); }));                 // 4 positionals
  EXPECT(throws([] { parse_cli({"conv", "img.raw", "10", "10", "1", "purple"}); }));       // bad type
  EXPECT(throws([] { parse_cli({"conv", "img.raw", "-3", "10", "1", "grey"}); }));         // width
  EXPECT(throws([] { parse_cli({"conv", "img.raw", "10", "10x", "1", "grey"}); }));        // not a number
  EXPECT(throws([] { parse_cli({"conv", "img.raw", "10", "10", "1", "grey", "--fuse", "99"}); }));
  EXPECT(throws([] { parse_cli({"conv", "img.raw", "10", "10", "1", "grey", "--bogus"}); }));
  EXPECT(usage_text("conv").rfind("Error Input!", 0) == 0);
}

// Round-5 flags: every pipeline / kernel policy is a flag (no environment
// variable changes behaviour), with its range checked.
void test_cli_policy_flags() {
  const auto d = parse_cli({"conv", "img.raw", "64", "48", "5", "grey"});
  EXPECT(d.tune == -1 && d.ring_chunk_bytes == (int64_t(32) << 20) && d.auto_gpu_min_s == 0.1);
  EXPECT(d.cu_mask_queues && d.head_on_slot_streams && d.ipc_pull == "grid" && d.numa_bind);
  const auto c = parse_cli({"conv", "img.raw", "64", "48", "5", "grey", "--tune", "off", "--ring-chunk-bytes", "0",
                            "--auto-gpu-min", "0.5", "--pool-queues", "--head-pool-streams", "--ipc-pull", "sdma",
                            "--no-numa-bind", "--stream-chunks", "6", "--transport", "ipc"});
  EXPECT(c.tune == 0 && c.ring_chunk_bytes == 0 && c.auto_gpu_min_s == 0.5);
  EXPECT(!c.cu_mask_queues && !c.head_on_slot_streams && c.ipc_pull == "sdma" && !c.numa_bind);
  EXPECT(c.stream_chunks == 6 && c.transport == "ipc");
  EXPECT(parse_cli({"conv", "i", "8", "8", "1", "grey", "--tune", "on"}).tune == 1);
  EXPECT(throws([] { parse_cli({"conv", "i", "8", "8", "1", "grey", "--ipc-pull", "warp"}); }));
  EXPECT(throws([] { parse_cli({"conv", "i", "8", "8", "1", "grey", "--tune", "maybe"}); }));
  EXPECT(throws([] { parse_cli({"conv", "i", "8", "8", "1", "grey", "--stream-chunks", "-1"}); }));  // wave mode removed
  EXPECT(throws([] { parse_cli({"conv", "i", "8", "8", "1", "grey", "--ring-chunk-bytes", "-5"}); }));
}

// The streamed plan on CPU frames: uploads in chunks, every level advanced as
// far as the uploaded rows allow (plan_streamed), the result equal to the
// whole-image oracle — the schedule the GPU's head streaming runs.
void test_streamed_plan_cpu() {
  const Filter f = Filter::gaussian();
  const int64_t w = 19, h = 53;
  const int ch = 3;
  const ImageGeom geo{w, h, Channels::Rgb};
  const int64_t rb = geo.row_bytes();
  const auto img = random_bytes(static_cast<size_t>(w * h * ch), 7);
  for (int chunks : {2, 3, 4, 7})
    for (int T : {1, 4, 8})
      for (int reps : {1, 9, 20}) {
        PlanConfig cfg;
        cfg.halo_depth = T;
        cfg.fuse = T;
        cfg.overlap = false;
        cfg = normalize_plan_config(cfg, 0, 16);
        const Band band = row_band(h, 1, 0);
        const auto ph = plan_band(band, reps, cfg);
        const StreamPlan sp = plan_streamed(ph, 0, h, h, stream_cuts(0, h, chunks));
        const FrameLayout lay = FrameLayout::make(rb, h, cfg.halo_depth);
        std::vector<uint8_t> fr[2] = {std::vector<uint8_t>(static_cast<size_t>(lay.bytes()), 0),
                                      std::vector<uint8_t>(static_cast<size_t>(lay.bytes()), 0)};
        // rows are taken from the result frame right after the chunk that
        // declares them final (down_lo/down_hi), as the GPU's downloads are
        std::vector<uint8_t> got(img.size(), 0xEE);
        const auto& out = fr[sp.levels & 1];
        for (const auto& c : sp.chunks) {
          for (int64_t row = c.up_lo; row < c.up_hi; ++row)
            std::memcpy(fr[0].data() + lay.offset(row), img.data() + row * rb, rb);
          for (size_t i = 0; i < c.launches.size(); ++i) {
            const int src = (c.levels[i] - 1) & 1;
            const auto& l = c.launches[i];
            cpu_fused_launch(f, geo.channels, lay, fr[src].data(), fr[src ^ 1].data(), l.lo, l.hi, l.steps, 0, h,
                             CpuBackend::Serial);
          }
          for (int64_t row = c.down_lo; row < c.down_hi; ++row)
            std::memcpy(got.data() + row * rb, out.data() + lay.offset(row), rb);
        }
        const bool ok = got == naive(f, img, w, h, ch, reps);
        if (!ok) std::fprintf(stderr, "streamed plan mismatch: chunks=%d T=%d reps=%d\n", chunks, T, reps);
        EXPECT(ok);
      }
}

}  // namespace

int main() {
  test_partition();
  test_filters();
  test_cpu_oracle();
  test_distributed_schedule();
  test_raw_io();
  test_synthetic();
  test_cli();
  test_cli_policy_flags();
  test_streamed_plan_cpu();
  std::printf("native tests: %d checks, %d failures\n", g_checks, g_failures);
  return g_failures ? 1 : 0;
}
