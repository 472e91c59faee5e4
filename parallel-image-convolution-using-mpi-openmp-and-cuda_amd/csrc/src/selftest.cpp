// RCCL self-tests and the crash reporter (see selftest.hpp).
#include "pconv/selftest.hpp"

#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <sstream>

#include "pconv/cpu_stencil.hpp"
#include "pconv/device.hpp"
#include "pconv/engine.hpp"
#include "pconv/rccl_comm.hpp"

namespace pconv {

// ------------------------------------------------------------ crash reporter

namespace {

constexpr int kCrashSignals[] = {SIGSEGV, SIGBUS, SIGILL, SIGFPE, SIGABRT};
struct sigaction g_prev[sizeof(kCrashSignals) / sizeof(int)];
bool g_installed = false;
int g_fds[2] = {2, -1};  // stderr, and PCONV_CRASH_LOG when set (test runners capture fd 2)
// PCONV_CRASH_LOG's path, copied at install time: the file is opened only
// when a signal arrives (open(2) is async-signal-safe), so a process that
// never crashes leaves no empty log behind.
char g_log_path[1024] = {0};

void write_str(const char* s) {
  for (int fd : g_fds)
    if (fd >= 0) (void)!::write(fd, s, std::strlen(s));
}

void write_hex(uintptr_t v) {
  char buf[2 + 16 + 1];
  buf[0] = '0';
  buf[1] = 'x';
  for (int i = 0; i < 16; ++i) buf[2 + i] = "0123456789abcdef"[(v >> (60 - 4 * i)) & 0xf];
  buf[18] = '\0';
  write_str(buf);
}

// Signal names from a fixed table: strsignal() is not async-signal-safe.
const char* signal_name(int sig) {
  switch (sig) {
    case SIGSEGV: return "Segmentation fault";
    case SIGBUS: return "Bus error";
    case SIGILL: return "Illegal instruction";
    case SIGFPE: return "Floating point exception";
    case SIGABRT: return "Aborted";
    default: return "signal";
  }
}

void on_fatal(int sig, siginfo_t* info, void* uctx) {
  // Only async-signal-safe calls up to backtrace (backtrace() itself may
  // allocate on first use: it is primed in install_crash_handler).
  if (g_log_path[0] && g_fds[1] < 0) g_fds[1] = ::open(g_log_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  write_str("\n[pconv] fatal signal ");
  char num[8];
  int k = 0, v = sig;
  do {
    num[k++] = static_cast<char>('0' + v % 10);
    v /= 10;
  } while (v && k < 7);
  while (k) {
    char c[2] = {num[--k], 0};
    write_str(c);
  }
  write_str(" (");
  write_str(signal_name(sig));
  write_str(") at address ");
  write_hex(reinterpret_cast<uintptr_t>(info ? info->si_addr : nullptr));
  write_str("\n[pconv] native backtrace (library(+offset) -> llvm-addr2line -e library offset):\n");
  void* frames[64];
  const int n = backtrace(frames, 64);
  for (int fd : g_fds)
    if (fd >= 0) backtrace_symbols_fd(frames, n, fd);
  // Hand over to the previous handler (faulthandler: Python frames), else
  // the default action (core / termination with the signal's status).
  size_t i = 0;
  while (kCrashSignals[i] != sig) ++i;
  const struct sigaction& p = g_prev[i];
  sigaction(sig, &p, nullptr);
  if ((p.sa_flags & SA_SIGINFO) && p.sa_sigaction) {
    p.sa_sigaction(sig, info, uctx);
  } else if (p.sa_handler != SIG_DFL && p.sa_handler != SIG_IGN && p.sa_handler) {
    p.sa_handler(sig);
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

}  // namespace

void install_crash_handler() {
  if (g_installed) return;
  // A copy of the report to a file: a test runner that captures fd 2 drops
  // what a dying process wrote there (faulthandler writes to a saved fd).
  if (const char* p = std::getenv("PCONV_CRASH_LOG")) {
    std::strncpy(g_log_path, p, sizeof(g_log_path) - 1);
    g_log_path[sizeof(g_log_path) - 1] = '\0';
  }
  void* prime[2];
  (void)backtrace(prime, 2);  // loads libgcc's unwinder outside the handler
  // An alternate stack: a stack overflow must still be reported.
  static char altstack[64 * 1024];
  stack_t ss{};
  ss.ss_sp = altstack;
  ss.ss_size = sizeof(altstack);
  (void)sigaltstack(&ss, nullptr);
  for (size_t i = 0; i < sizeof(kCrashSignals) / sizeof(int); ++i) {
    struct sigaction sa {};
    sa.sa_sigaction = on_fatal;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigaction(kCrashSignals[i], &sa, &g_prev[i]);
  }
  g_installed = true;
}

// ------------------------------------------------------------ CPU oracle

std::vector<uint8_t> reflected_band_oracle(const Filter& f, Channels ch, int64_t row_bytes, int64_t rows, int64_t halo,
                                           const std::vector<Phase>& plan, const uint8_t* owned, int64_t y0,
                                           int64_t height, int64_t pre_exchange) {
  const FrameLayout lay = FrameLayout::make(row_bytes, rows, halo);
  std::vector<uint8_t> fr[2] = {std::vector<uint8_t>(static_cast<size_t>(lay.bytes()), 0),
                                std::vector<uint8_t>(static_cast<size_t>(lay.bytes()), 0)};
  for (int64_t r = 0; r < rows; ++r) std::memcpy(fr[0].data() + lay.offset(r), owned + r * row_bytes, row_bytes);
  auto refresh = [&](std::vector<uint8_t>& f8, int64_t d) {
    PCONV_CHECK(d >= 1 && d <= halo && d <= rows, "oracle: bad exchange depth");
    uint8_t* b = f8.data();
    for (int64_t i = 0; i < d; ++i) {
      std::memcpy(b + lay.offset(-d + i), b + lay.offset(i), row_bytes);            // above <- my top rows
      std::memcpy(b + lay.offset(rows + i), b + lay.offset(rows - d + i), row_bytes);  // below <- my bottom rows
    }
    for (int64_t r = -d; r < rows + d; ++r)  // outside the global image: the kernels read zeros
      if (y0 + r < 0 || y0 + r >= height) std::memset(b + lay.offset(r), 0, row_bytes);
  };
  int cur = 0;
  if (pre_exchange > 0) refresh(fr[0], pre_exchange);
  for (const auto& ph : plan) {
    if (ph.exchange_depth > 0) refresh(fr[cur], ph.exchange_depth);
    for (const auto& l : ph.launches)
      cpu_fused_launch(f, ch, lay, fr[cur].data(), fr[cur ^ 1].data(), l.lo, l.hi, l.steps, y0, height,
                       CpuBackend::Serial);
    cur ^= 1;
  }
  std::vector<uint8_t> out(static_cast<size_t>(rows * row_bytes));
  for (int64_t r = 0; r < rows; ++r) std::memcpy(out.data() + r * row_bytes, fr[cur].data() + lay.offset(r), row_bytes);
  return out;
}

// ------------------------------------------------------------ self-tests

namespace {

std::vector<uint8_t> random_bytes(size_t n, uint64_t seed) {
  std::vector<uint8_t> v(n);
  uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
  for (auto& b : v) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    b = static_cast<uint8_t>(x >> 24);
  }
  return v;
}

Band self_band(int64_t y0, int64_t rows) {
  Band b;
  b.rank = 0;
  b.world = 1;
  b.y0 = y0;
  b.rows = rows;
  b.up = 0;  // the 1-rank communicator's only rank: send/recv to self
  b.down = 0;
  return b;
}

int64_t count_diff(const uint8_t* a, const uint8_t* b, size_t n) {
  int64_t bad = 0;
  for (size_t i = 0; i < n; ++i) bad += a[i] != b[i];
  return bad;
}

}  // namespace

std::string rccl_selftest_exchange(int device) {
  set_device(device);
  auto comm = std::make_shared<RcclComm>(rccl_unique_id(), 0, 1, device);
  auto tr = std::make_shared<RcclTransport>(comm);
  struct Case {
    Channels ch;
    int64_t w;
    int reps, halo, fuse;
    bool overlap;
  };
  const Case cases[] = {{Channels::Rgb, 57, 13, 4, 4, true},     {Channels::Rgb, 57, 13, 4, 4, false},
                        {Channels::Grey, 1920, 20, 8, 8, true},  {Channels::Grey, 1920, 17, 6, 3, true},
                        {Channels::Rgb, 333, 40, 40, 8, true},   {Channels::Grey, 64, 5, 1, 1, true},
                        {Channels::Rgba, 45, 24, 12, 8, false}};
  const int64_t y0 = 37, rows = 48, height = 130;
  const Filter f = Filter::gaussian();
  int checked = 0, exchanges = 0;
  for (const Case& c : cases) {
    ImageGeom g;
    g.width = c.w;
    g.height = height;
    g.channels = c.ch;
    EngineOptions o;
    o.device = device;
    o.halo_depth = c.halo;
    o.fuse = c.fuse;
    o.overlap = c.overlap;
    BandEngine e(g, self_band(y0, rows), f, o);
    e.set_transport(tr);
    const int64_t rb = e.layout().row_bytes;
    const auto owned = random_bytes(static_cast<size_t>(rows * rb), 7 + checked);
    const auto plan = e.plan(c.reps);
    const auto ref = reflected_band_oracle(f, c.ch, rb, rows, e.layout().halo, plan, owned.data(), y0, height);
    std::vector<uint8_t> got(owned.size());
    for (int pass = 0; pass < 2; ++pass) {  // the second pass starts from the other frame parity
      e.upload_rows(owned.data(), rb, 0, rows);
      e.run(c.reps);
      comm->wait(e.comm_stream(), 60.0);
      comm->wait(e.compute_stream(), 60.0);
      e.synchronize();
      e.download_rows(got.data(), rb, 0, rows);
      e.synchronize();
      const int64_t bad = count_diff(got.data(), ref.data(), got.size());
      PCONV_CHECK(bad == 0, "rccl_selftest_exchange: " + std::to_string(bad) + " bytes differ (case " +
                                std::to_string(checked) + ", pass " + std::to_string(pass) + ")");
      exchanges += e.last_stats().exchanges;
    }
    ++checked;
  }
  std::ostringstream os;
  os << "{\"selftest\": \"rccl_exchange\", \"cases\": " << checked << ", \"exchanges\": " << exchanges
     << ", \"status\": \"ok\", \"rccl_version\": \"" << rccl_version() << "\", \"rccl_path\": \""
     << json_escape(rccl_library_path()) << "\"}";
  return os.str();
}

std::string rccl_selftest_multicomm(int device, int slots, int images, double timeout_s) {
  PCONV_CHECK(slots >= 1 && slots <= 8 && images >= 1, "rccl_selftest_multicomm: bad slots/images");
  set_device(device);
  const int64_t y0 = 211, rows = 96, height = 520, w = 301;
  ImageGeom g;
  g.width = w;
  g.height = height;
  g.channels = Channels::Rgb;
  const Filter f = Filter::gaussian();
  struct Case {
    int reps, halo, fuse;
  };
  // halo >= reps: one whole-zone exchange per image, then a cached rep-loop
  // graph; halo < reps: exchange phases inside the run (stream-ordered).
  const Case cases[] = {{40, 40, 8}, {20, 8, 4}, {24, 8, 8}};
  int checked = 0;
  // directly issued images, then images captured as ONE graph each (upload,
  // RCCL exchange(s), launches, download: BandEngine::process_graph)
  // slot_comm: the exchange phases split (interior || exchange on the slot's
  // comm stream, edges after the halo event), captured with a fork/join
  for (const bool slot_comm : {false, true})
  for (const bool captured : {false, true})
  for (const Case& c : cases) {
    EngineOptions o;
    o.device = device;
    o.halo_depth = c.halo;
    o.fuse = c.fuse;
    BandPipeline pipe(g, self_band(y0, rows), f, o, slots, -1, /*slot_streams=*/true, /*step_graphs=*/captured,
                      slot_comm);
    std::vector<std::shared_ptr<RcclComm>> comms;
    for (int k = 0; k < slots; ++k) {
      comms.push_back(std::make_shared<RcclComm>(rccl_unique_id(), 0, 1, device));
      pipe.set_slot_transport(k, std::make_shared<RcclTransport>(comms.back()));
    }
    BandEngine& e0 = pipe.slot(0);
    const int64_t rb = e0.layout().row_bytes;
    const int64_t D = e0.layout().halo;
    const bool whole_zone = e0.exchange_free(c.reps, true);
    e0.set_halo_valid(whole_zone);
    const auto plan = e0.plan(c.reps);
    e0.set_halo_valid(false);
    std::vector<PinnedBuffer> in, out;
    std::vector<std::vector<uint8_t>> refs;
    for (int k = 0; k < slots; ++k) {
      in.emplace_back(static_cast<size_t>(rows * rb));
      out.emplace_back(static_cast<size_t>(rows * rb));
      const auto owned = random_bytes(static_cast<size_t>(rows * rb), 100 + k + 10 * checked);
      std::memcpy(in.back().data(), owned.data(), owned.size());
      refs.push_back(reflected_band_oracle(f, g.channels, rb, rows, D, plan, owned.data(), y0, height,
                                           whole_zone ? D : 0));
    }
    for (int i = 0; i < images; ++i) {
      const int k = i % slots;
      pipe.submit(in[k].data(), 0, rows, out[k].data(), c.reps);
      if (k == slots - 1 || i == images - 1) {
        // one round of images in flight on `slots` communicators at once
        for (int s = 0; s < slots; ++s) comms[s]->wait(pipe.slot(s).compute_stream(), timeout_s);
        pipe.drain();
        for (int s = 0; s <= k; ++s) {
          const int64_t bad = count_diff(out[s].data(), refs[s].data(), refs[s].size());
          PCONV_CHECK(bad == 0, "rccl_selftest_multicomm: image " + std::to_string(i - k + s) + " (slot " +
                                    std::to_string(s) + "): " + std::to_string(bad) + " bytes differ");
          std::memset(out[s].data(), 0, refs[s].size());
        }
      }
    }
    ++checked;
  }
  std::ostringstream os;
  os << "{\"selftest\": \"rccl_multicomm\", \"communicators\": " << slots << ", \"images_per_case\": " << images
     << ", \"cases\": " << checked << ", \"captured_cases\": " << checked / 2 << ", \"split_cases\": " << checked / 2
     << ", \"status\": \"ok\", \"rccl_version\": \"" << rccl_version() << "\", \"rccl_path\": \""
     << json_escape(rccl_library_path()) << "\"}";
  return os.str();
}

int selftest_main(const std::vector<std::string>& args) {
  // args: conv --selftest NAME [--device D] [--op OP] [--mode MODE] [--bytes N] [--slots S] [--images N]
  install_crash_handler();
  PCONV_CHECK(args.size() >= 3, "usage: conv --selftest {rccl-capture|rccl-exchange|rccl-multicomm|all} [options]");
  const std::string name = args[2];
  int device = 0, slots = 3, images = 60;
  int64_t bytes = 4096;
  std::string op = "sendrecv", mode = "relaxed";
  for (size_t i = 3; i < args.size(); i += 2) {
    const std::string& k = args[i];
    PCONV_CHECK(i + 1 < args.size(), "selftest: option " + k + " needs a value");
    const std::string& v = args[i + 1];
    if (k == "--device")
      device = std::stoi(v);
    else if (k == "--op")
      op = v;
    else if (k == "--mode")
      mode = v;
    else if (k == "--bytes")
      bytes = std::stoll(v);
    else if (k == "--slots")
      slots = std::stoi(v);
    else if (k == "--images")
      images = std::stoi(v);
    else
      PCONV_FAIL("selftest: unknown option " + k);
  }
  try {
    if (name == "rccl-capture" || name == "all") std::printf("%s\n", rccl_capture_probe(op, mode, bytes, device).c_str());
    if (name == "rccl-exchange" || name == "all") std::printf("%s\n", rccl_selftest_exchange(device).c_str());
    if (name == "rccl-multicomm" || name == "all")
      std::printf("%s\n", rccl_selftest_multicomm(device, slots, images, 60.0).c_str());
    if (name != "rccl-capture" && name != "rccl-exchange" && name != "rccl-multicomm" && name != "all")
      PCONV_FAIL("selftest: unknown test " + name);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "selftest %s failed: %s\n", name.c_str(), e.what());
    return 1;
  }
  const HipRuntimeInfo h = hip_runtime_info();
  std::printf("{\"selftest\": \"%s\", \"status\": \"ok\", \"hip_runtime_version\": %d, \"hip_runtime_path\": \"%s\"}\n",
              name.c_str(), h.runtime_version, json_escape(h.runtime_path).c_str());
  std::fflush(stdout);
  return 0;
}

}  // namespace pconv
