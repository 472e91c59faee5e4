// `conv` application (see app.hpp).
#include "pconv/app.hpp"

#include <omp.h>
#include <sys/mman.h>
#include <sys/wait.h>
#include <unistd.h>

#include <climits>

#include <algorithm>
#include <atomic>
#include <list>
#include <tuple>
#include <cinttypes>
#include <cstdio>
#include <cstring>
#include <sstream>
#include <thread>

#include "pconv/cpu_stencil.hpp"
#include "pconv/device.hpp"
#include "pconv/engine.hpp"
#include "pconv/ipc_halo.hpp"
#include "pconv/kernels.hpp"
#include "pconv/raw_io.hpp"
#include "pconv/rccl_comm.hpp"
#include "pconv/selftest.hpp"
#include "pconv/service.hpp"
#include "pconv/trace.hpp"

namespace pconv {

namespace {

constexpr int kMaxRanks = 64;
constexpr int kAutoHaloCap = 64;

ImageGeom geom_of(const CliConfig& c) {
  ImageGeom g;
  g.width = c.width;
  g.height = c.height;
  g.channels = c.channels;
  g.validate();
  return g;
}

std::string out_path(const CliConfig& c) { return c.out.empty() ? output_path_for(c.image) : c.out; }

void load_rows(const CliConfig& c, const ImageGeom& g, int64_t y0, int64_t rows, uint8_t* dst, int64_t pitch) {
  if (c.synthetic)
    synth_rows(g, c.seed, y0, rows, dst, pitch);
  else
    read_rows(c.image, g, y0, rows, dst, pitch);
}

EngineOptions engine_options(const CliConfig& c, const ImageGeom& g, int world, int device) {
  const Filter f = Filter::by_name(c.filter);
  EngineOptions o;
  o.device = device;
  o.variant = c.variant;
  o.overlap = c.overlap;
  o.use_graph = c.graph && world == 1;
  const bool fusable = supports_fusion(f, c.variant);
  o.fuse = c.fuse > 0 ? c.fuse : auto_fuse(f, c.variant, g.row_bytes() * (g.height / std::max(1, world)), g.ch());
  if (!fusable) o.fuse = 1;
  o.fuse = std::max(1, std::min(o.fuse, std::max(1, c.reps)));
  if (c.halo > 0) {
    o.halo_depth = c.halo;
  } else if (world > 1) {
    // Deep ghost zone: fewest exchanges, bounded redundant compute.
    const int64_t min_rows = g.height / world;
    o.halo_depth = static_cast<int>(std::min<int64_t>({std::max(1, c.reps), kAutoHaloCap, min_rows}));
  } else {
    o.halo_depth = o.fuse;
  }
  o.halo_depth = std::max(o.halo_depth, o.fuse);
  return o;
}

int64_t compare_with_oracle(const CliConfig& c, const ImageGeom& g, const uint8_t* result) {
  std::vector<uint8_t> in(static_cast<size_t>(g.bytes())), ref(static_cast<size_t>(g.bytes()));
  load_rows(c, g, 0, g.height, in.data(), g.row_bytes());
  cpu_convolve(Filter::by_name(c.filter), g, in.data(), ref.data(), c.reps, CpuBackend::OpenMP, c.threads);
  int64_t bad = 0;
  for (size_t i = 0; i < ref.size(); ++i) bad += ref[i] != result[i];
  return bad;
}

// ------------------------------------------------------------------ CPU
AppReport run_cpu(const CliConfig& c) {
  const double t0 = wall_seconds();
  const ImageGeom g = geom_of(c);
  if (!c.synthetic) validate_input_file(c.image, g);
  std::vector<uint8_t> img(static_cast<size_t>(g.bytes()));
  load_rows(c, g, 0, g.height, img.data(), g.row_bytes());
  const Filter f = Filter::by_name(c.filter);
  const CpuBackend be = c.backend == Backend::Omp ? CpuBackend::OpenMP : CpuBackend::Serial;
  AppReport r;
  r.kernel = be == CpuBackend::OpenMP ? "cpu-omp" : "cpu-serial";
  // Zero-padded ping-pong frames (the reference's calloc'd buffers,
  // mpi/mpi_convolution.c:104-124) set up outside the timed loop, like its
  // MPI_Wtime bracket (:151-154,242); the OpenMP team is started first.
  const int64_t rb = g.row_bytes();
  const FrameLayout lay = FrameLayout::make(rb, g.height, 1);
  std::vector<uint8_t> fa(static_cast<size_t>(lay.bytes()), 0), fb(static_cast<size_t>(lay.bytes()), 0);
  for (int64_t y = 0; y < g.height; ++y) std::memcpy(fa.data() + lay.offset(y), img.data() + y * rb, rb);
  if (be == CpuBackend::OpenMP) {
    if (c.threads > 0)
      omp_set_num_threads(c.threads);
    else
      (void)configure_cpu_threads();
#pragma omp parallel
    { (void)omp_get_thread_num(); }
  }
  uint8_t* src = fa.data();
  uint8_t* dst = fb.data();
  auto copy_out = [&] {
    for (int64_t y = 0; y < g.height; ++y) std::memcpy(img.data() + y * rb, src + lay.offset(y), rb);
  };
  const double l0 = wall_seconds();
  for (int done = 0; done < c.reps;) {
    cpu_step(f, g.channels, lay, src, dst, 0, g.height, be);
    std::swap(src, dst);  // newest result is always `src`
    ++done;
    if (c.checkpoint_every > 0 && done % c.checkpoint_every == 0 && done < c.reps) {
      copy_out();
      write_image(out_path(c) + ".rep" + std::to_string(done), g, img.data());
    }
  }
  r.loop_s = wall_seconds() - l0;
  copy_out();
  r.output = out_path(c);
  write_image(r.output, g, img.data());
  if (c.check) r.mismatches = compare_with_oracle(c, g, img.data());
  r.e2e_s = wall_seconds() - t0;
  return r;
}

// Phase clock for the end-to-end breakdown.
struct PhaseClock {
  std::vector<std::pair<std::string, double>>* out;
  double t;
  explicit PhaseClock(std::vector<std::pair<std::string, double>>* o) : out(o), t(wall_seconds()) {}
  void mark(const char* name) {
    const double now = wall_seconds();
    out->emplace_back(name, now - t);
    t = now;
  }
};

// Seconds since this process was exec'ed (/proc/self/stat field 22, in clock
// ticks since boot, against CLOCK_BOOTTIME): covers the dynamic loader and
// static initialisers that no in-process timer sees.  10 ms resolution.
double seconds_since_exec() {
  FILE* f = std::fopen("/proc/self/stat", "r");
  if (!f) return 0;
  char buf[1024];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');  // comm may contain spaces
  if (!p) return 0;
  unsigned long long start = 0;
  int field = 2;
  for (const char* q = p + 1; *q && field < 22; ++q)
    if (*q == ' ' && ++field == 22) start = std::strtoull(q + 1, nullptr, 10);
  timespec ts{};
  clock_gettime(CLOCK_BOOTTIME, &ts);
  const double hz = static_cast<double>(sysconf(_SC_CLK_TCK));
  return (ts.tv_sec + ts.tv_nsec * 1e-9) - static_cast<double>(start) / hz;
}

// ------------------------------------------------------------------ 1 GPU
}  // namespace

// Resources a resident server keeps between jobs (service.hpp): engines per
// (geometry, filter, launch options), least recently used first out, and one
// pinned staging buffer grown on demand.
struct JobCache {
  using Key = std::tuple<int64_t, int64_t, int, std::string, int, int, int, bool, bool, bool>;
  std::list<std::pair<Key, std::unique_ptr<BandEngine>>> engines;
  PinnedBuffer host;
  int max_engines = 8;
  int device = 0;

  BandEngine& engine(const ImageGeom& g, const Filter& f, const EngineOptions& o, const std::string& fname,
                     bool* fresh) {
    const Key k{g.width, g.height, channel_count(g.channels), fname, o.fuse, o.halo_depth,
                static_cast<int>(o.variant), o.overlap, o.use_graph, o.kernel_copies};
    for (auto it = engines.begin(); it != engines.end(); ++it)
      if (it->first == k) {
        engines.splice(engines.begin(), engines, it);
        *fresh = false;
        return *engines.front().second;
      }
    while (static_cast<int>(engines.size()) >= max_engines) engines.pop_back();
    engines.emplace_front(k, std::make_unique<BandEngine>(g, row_band(g.height, 1, 0), f, o));
    *fresh = true;
    return *engines.front().second;
  }
  uint8_t* staging(size_t bytes) {
    if (host.size() < bytes) {
      host = PinnedBuffer();  // free first: never hold both
      host = PinnedBuffer(bytes);
    }
    return host.data();
  }
};

JobCache* new_job_cache(int device, int max_engines) {
  auto* c = new JobCache();
  c->device = device;
  c->max_engines = std::max(1, max_engines);
  return c;
}
void delete_job_cache(JobCache* c) { delete c; }

namespace {

// Ring staging of large one-shot images (run_gpu1): kRingSlots pinned
// chunks of CliConfig::ring_chunk_bytes (--ring-chunk-bytes; 0 = one pinned
// copy of the whole image).
constexpr int kRingSlots = 3;

AppReport run_gpu1(const CliConfig& c, JobCache* cache) {
  AppReport r;
  const double t0 = wall_seconds();
  PhaseClock pc(&r.phases);
  const ImageGeom g = geom_of(c);
  if (!c.synthetic) validate_input_file(c.image, g);
  const Filter f = Filter::by_name(c.filter);
  const int device = cache ? cache->device : 0;
  set_device(device);
  std::thread preload;  // joined before the engine's first kernel
  if (!cache) {
    PCONV_HIP_CHECK(hipFree(nullptr));  // the runtime + device context (cudaMalloc's hidden cost in the reference)
    pc.mark("hip_init");
    // The kernels' code object (~6 ms to load on first use) loads on a helper
    // thread while this one allocates staging, reads the image and creates
    // the first hardware queue (~20 ms).
    preload = std::thread([device] {
      if (hipSetDevice(device) == hipSuccess) preload_kernel_module();
    });
  }
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } join_preload{preload};
  // One-shot process: the model's tile shape, no timing of candidates (2-4 ms
  // of tuning launches against a 0.03-0.7 ms loop; profiles/r02/raw/startup/
  // cli_modes.jsonl) unless --tune on; a resident server tunes unless
  // --tune off.
  struct TuneScope {
    bool active = false, prev = true;
    ~TuneScope() {
      if (active) (void)set_shape_tuning(prev);
    }
  } tune_scope;
  const bool tune = c.tune < 0 ? cache != nullptr : c.tune == 1;
  tune_scope.active = true;
  tune_scope.prev = set_shape_tuning(tune);
  // Large one-shot images go through a small ring of pinned chunks instead
  // of one pinned copy of the whole image: pinning costs ~0.24 ms per MB
  // (32768^2 grey: 0.244 s of a 0.69 s run, profiles/r04/trace20/), and the
  // ring overlaps reading chunk k+1 with the upload of chunk k, and the
  // download of chunk k+1 with writing chunk k (one writer: writes of
  // several threads into one file measured slower, 0.20 vs 0.13 s for 1 GB).  The full buffer stays for
  // --check / checkpoints (they need the whole result in host memory) and for
  // the resident server (its staging is allocated once).
  const int64_t rb = g.row_bytes();
  const int64_t ring_rows = std::max<int64_t>(1, c.ring_chunk_bytes / rb);
  const bool ring = !cache && !c.check && c.checkpoint_every == 0 && c.ring_chunk_bytes > 0 &&
                    g.height > (kRingSlots - 1) * ring_rows;  // >= kRingSlots chunks
  PinnedBuffer own_host;
  uint8_t* host = nullptr;
  if (cache) {
    host = cache->staging(static_cast<size_t>(g.bytes()));
  } else {
    own_host = PinnedBuffer(static_cast<size_t>(ring ? kRingSlots * ring_rows * rb : g.bytes()));
    host = own_host.data();
  }
  pc.mark("pinned_alloc");
  if (!ring) {
    load_rows(c, g, 0, g.height, host, rb);
    pc.mark(c.synthetic ? "synthesize" : "read");
  }
  EngineOptions o = engine_options(c, g, 1, device);
  // One-shot process: CU copies skip the SDMA / blit first-use set-up; a
  // resident server has paid it once and keeps SDMA.
  o.kernel_copies = c.copies < 0 ? cache == nullptr : c.copies == 1;
  Stream own_stream;  // declared before the engine: outlives it
  std::unique_ptr<BandEngine> own_eng;
  bool fresh = true;
  if (cache) {
    (void)cache->engine(g, f, o, c.filter, &fresh);
  } else {
    // The process's first stream = its first hardware queue (~20 ms of
    // runtime set-up), timed apart from the frames and the first kernel.
    own_stream = Stream::create(0);
    o.compute_stream = own_stream.get();
    pc.mark("queue");
    if (preload.joinable()) preload.join();
    own_eng = std::make_unique<BandEngine>(g, row_band(g.height, 1, 0), f, o);
  }
  BandEngine& eng = cache ? *cache->engines.front().second : *own_eng;
  pc.mark("device_alloc");
  if (c.explain) std::fprintf(stderr, "%s", describe_plan(eng.plan(c.reps)).c_str());
  const int warmup = fresh ? c.warmup : 0;  // a cached engine is warm (code objects, tuning, graphs)
  // Every launch shape of the job's plan, once: a full fused launch plus the
  // remainder launch (a 32768^2 x200 warm-up of all 200 reps cost 23 ms).
  const int fz = std::max(1, eng.options().fuse);
  const int warm_reps = c.reps <= 2 * fz ? c.reps : fz + c.reps % fz;
  for (int i = 0; i < warmup; ++i) eng.run(warm_reps);  // zero frames stay zero
  if (warmup > 0) {
    eng.synchronize();
    pc.mark("warmup");
  }
  std::vector<Event> ring_ev;
  if (ring) {
    for (int i = 0; i < kRingSlots; ++i) ring_ev.push_back(Event::create());
    for (int64_t r = 0, k = 0; r < g.height; r += ring_rows, ++k) {
      const int64_t n = std::min(ring_rows, g.height - r);
      const int slot = static_cast<int>(k % kRingSlots);
      uint8_t* buf = host + slot * ring_rows * rb;
      if (k >= kRingSlots) ring_ev[slot].sync();  // this slot's previous upload is done
      load_rows(c, g, r, n, buf, rb);
      eng.upload_rows(buf, rb, r, r + n);
      ring_ev[slot].record(eng.compute_stream());
    }
  } else {
    eng.upload_rows(host, rb, 0, g.height);
  }
  eng.synchronize();
  pc.mark(ring ? "read_and_h2d" : "h2d");
  r.output = out_path(c);
  const double l0 = wall_seconds();
  int done = 0;
  const int chunk = c.checkpoint_every > 0 ? c.checkpoint_every : std::max(1, c.reps);
  while (done < c.reps) {
    const int k = std::min(chunk, c.reps - done);
    eng.run(k);
    eng.synchronize();
    r.launches += eng.last_stats().launches;
    done += k;
    if (c.checkpoint_every > 0 && done < c.reps) {
      eng.download_rows(host, g.row_bytes(), 0, g.height);
      eng.synchronize();
      write_image(r.output + ".rep" + std::to_string(done), g, host);
    }
  }
  r.loop_s = wall_seconds() - l0;
  pc.mark("loop");
  if (ring) {
    create_output(r.output, g);
    const int64_t nchunks = (g.height + ring_rows - 1) / ring_rows;
    auto issue = [&](int64_t k) {
      const int64_t r0 = k * ring_rows, n = std::min(ring_rows, g.height - r0);
      const int slot = static_cast<int>(k % kRingSlots);
      eng.download_rows(host + slot * ring_rows * rb, rb, r0, r0 + n);
      ring_ev[slot].record(eng.compute_stream());
    };
    for (int64_t k = 0; k < std::min<int64_t>(kRingSlots, nchunks); ++k) issue(k);
    for (int64_t k = 0; k < nchunks; ++k) {
      const int slot = static_cast<int>(k % kRingSlots);
      ring_ev[slot].sync();
      const int64_t r0 = k * ring_rows, n = std::min(ring_rows, g.height - r0);
      write_rows(r.output, g, r0, n, host + slot * ring_rows * rb, rb);
      if (k + kRingSlots < nchunks) issue(k + kRingSlots);
    }
    pc.mark("d2h_and_write");
  } else {
    eng.download_rows(host, rb, 0, g.height);
    eng.synchronize();
    pc.mark("d2h");
    write_image(r.output, g, host);
    pc.mark("write");
  }
  r.e2e_s = wall_seconds() - t0;
  r.halo = eng.options().halo_depth;
  r.fuse = eng.options().fuse;
  r.kernel = kernel_variant_name(eng.options().variant);
  r.copies = eng.options().kernel_copies ? "kernel" : "sdma";
  if (c.check) r.mismatches = compare_with_oracle(c, g, host);
  r.since_exec_s = seconds_since_exec();
  return r;
}

// ------------------------------------------------------- CPU or GPU, priced
// `--backend auto`, the one-shot form of the reference's cuda/main.c:20-49
// run.  A cold process spends 50-190 ms bringing the GPU up (runtime,
// context, first queue; BASELINE.md phase tables) before its first kernel,
// while one repetition of a 1920x2520 RGB frame takes ~0.5 ms on the
// node's CPUs.  So the job is priced on the CPU first:
//   * stage 1, a <= 256-row sample: above CliConfig::auto_gpu_min_s
//     (--auto-gpu-min, default 0.1 s) the GPU path runs the job alone (the
//     host never holds the image twice);
//   * stage 2, the whole frame on the host: the first repetition is real
//     work and re-prices the job at memory speed; if the rest is still worth
//     a GPU it goes there, otherwise the CPU finishes without any HIP call
//     (no driver open, no teardown wait for the next process).
// A failed GPU bring-up leaves the job on the CPU (auto_choice says why).
// Measured and removed (round 5): a CPU head start handing the newest frame
// to a GPU brought up on a helper thread — bit-exact, but slower whenever the
// job is worth a GPU (8192^2 RGB x100 0.31 vs 0.23 s, 32768^2 grey x200 1.43
// vs 0.74 s: the CPU team and the bring-up compete for the host).
AppReport run_auto(const CliConfig& c) {
  AppReport r;
  const double t0 = wall_seconds();
  PhaseClock pc(&r.phases);
  const ImageGeom g = geom_of(c);
  if (!c.synthetic) validate_input_file(c.image, g);
  const Filter f = Filter::by_name(c.filter);
  const int64_t rb = g.row_bytes();
  const FrameLayout lay = FrameLayout::make(rb, g.height, 1);
  if (c.threads > 0)
    omp_set_num_threads(c.threads);
  else
    (void)configure_cpu_threads();
#pragma omp parallel
  { (void)omp_get_thread_num(); }  // the team starts here, not inside a timed step
  r.output = out_path(c);
  r.kernel = "cpu-omp";
  const double thr = c.auto_gpu_min_s;
  char est[128];

  // Stage 1: price from the first rows only (a frame of <= 256 rows), so a
  // job bound for the GPU never reads or allocates the whole image on the
  // host twice.  The fastest of up to 3 trials (stopping once 3 ms are
  // spent): one trial on a loaded host can be a barrier's scheduling delay.
  // The sample stays in the CPU's caches, so it can only under-price a large
  // frame: above the threshold the job is the GPU's for sure.
  if (c.reps > 0) {
    const int64_t sample = std::min<int64_t>(g.height, 256);
    const FrameLayout sl = FrameLayout::make(rb, sample, 1);
    std::vector<uint8_t> sa(static_cast<size_t>(sl.bytes()), 0), sb(static_cast<size_t>(sl.bytes()), 0);
    load_rows(c, g, 0, sample, sa.data() + sl.offset(0), sl.pitch);
    double best = 1e30, spent = 0;
    for (int t = 0; t < 3 && spent < 3e-3; ++t) {
      const double s0 = wall_seconds();
      cpu_step(f, g.channels, sl, sa.data(), sb.data(), 0, sample, CpuBackend::OpenMP);
      const double dt = wall_seconds() - s0;
      best = std::min(best, dt);
      spent += dt;
    }
    r.cpu_rep_s = best * static_cast<double>(g.height) / static_cast<double>(sample);
  }
  pc.mark("auto_price");
  double cpu_s = r.cpu_rep_s * c.reps;
  std::snprintf(est, sizeof(est), "cpu estimate %.4f s", cpu_s);

  // The GPU path on its own; false (auto_choice says why) if the GPU cannot
  // run the job.
  AppReport gr;
  auto gpu_alone = [&]() -> bool {
    try {
      const double pre = wall_seconds() - t0;
      gr = run_gpu1(c, nullptr);
      gr.e2e_s += pre;  // pricing the job counts too
      gr.cpu_reps = 0;
      gr.gpu_reps = c.reps;
      gr.cpu_rep_s = r.cpu_rep_s;
      gr.gpus = 1;
      gr.auto_choice = std::string("gpu (") + est + ")";
      gr.phases.insert(gr.phases.begin(), {"auto_price", pre});
      return true;
    } catch (const std::exception& e) {
      r.auto_choice = std::string("gpu failed (") + e.what() + "); cpu, " + est;
      return false;
    }
  };
  bool gpu_failed = false;
  if (c.reps > 0 && cpu_s >= thr) {
    if (gpu_alone()) return gr;
    gpu_failed = true;
  }

  // Stage 2: the whole image on the host; the first repetition is timed on
  // the full frame and re-prices the job.
  std::vector<uint8_t> fa(static_cast<size_t>(lay.bytes()), 0), fb(static_cast<size_t>(lay.bytes()), 0);
  load_rows(c, g, 0, g.height, fa.data() + lay.offset(0), lay.pitch);
  pc.mark(c.synthetic ? "synthesize" : "read");
  uint8_t* src = fa.data();
  uint8_t* dst = fb.data();
  int done = 0;
  auto cpu_rep = [&] {
    cpu_step(f, g.channels, lay, src, dst, 0, g.height, CpuBackend::OpenMP);
    std::swap(src, dst);  // newest result is always `src`
    ++done;
  };
  double l0 = wall_seconds();
  if (c.reps > 0) cpu_rep();
  if (c.reps > 0 && !gpu_failed) {
    const double first = wall_seconds() - l0;
    // Only up: a full frame past the caches runs at memory speed, which the
    // sample does not see (8192^2 RGB: sample 1.0 ms a repetition, the frame
    // 3.7 ms).
    if (first > r.cpu_rep_s) {
      r.cpu_rep_s = first;
      cpu_s = first * c.reps;
      std::snprintf(est, sizeof(est), "cpu estimate %.4f s from the first full repetition", cpu_s);
    }
    if (first * (c.reps - 1) >= thr) {
      std::vector<uint8_t>().swap(fa);  // the GPU path stages the image itself
      std::vector<uint8_t>().swap(fb);
      if (gpu_alone()) return gr;
      gpu_failed = true;
      fa.assign(static_cast<size_t>(lay.bytes()), 0);  // back to the CPU: the frames again
      fb.assign(static_cast<size_t>(lay.bytes()), 0);
      load_rows(c, g, 0, g.height, fa.data() + lay.offset(0), lay.pitch);
      src = fa.data();
      dst = fb.data();
      done = 0;
      l0 = wall_seconds();
      cpu_rep();
    }
  }
  if (!gpu_failed) r.auto_choice = std::string("cpu only (job shorter than gpu start-up: ") + est + ")";
  while (done < c.reps) cpu_rep();
  r.cpu_reps = done;
  r.gpu_reps = 0;
  r.loop_s = wall_seconds() - l0;
  pc.mark("cpu_loop");
  std::vector<uint8_t> img(static_cast<size_t>(g.bytes()));
  for (int64_t y = 0; y < g.height; ++y) std::memcpy(img.data() + y * rb, src + lay.offset(y), static_cast<size_t>(rb));
  write_image(r.output, g, img.data());
  pc.mark("write");
  r.e2e_s = wall_seconds() - t0;
  if (c.check) r.mismatches = compare_with_oracle(c, g, img.data());
  r.gpus = 0;
  r.since_exec_s = seconds_since_exec();
  return r;
}

// ------------------------------------------------------------------ N GPUs
struct SharedState {
  std::atomic<int> id_ready;
  uint8_t id[kUniqueIdBytes];
  std::atomic<int> arrived;
  std::atomic<int> generation;
  std::atomic<int> failed;
  double loop_s[kMaxRanks];
  int launches[kMaxRanks];
  int exchanges[kMaxRanks];
  char error[512];
  // --transport ipc: every rank's frame handles (hipIpcMemHandle_t x 2) and
  // the flag segment's name
  uint8_t ipc_handles[kMaxRanks][kIpcHandleBytes];
  char ipc_segment[64];
};

void shm_barrier(SharedState* s, int world, double timeout_s) {
  const int gen = s->generation.load();
  if (s->arrived.fetch_add(1) + 1 == world) {
    s->arrived.store(0);
    s->generation.fetch_add(1);
    return;
  }
  const double t0 = wall_seconds();
  while (s->generation.load() == gen) {
    if (s->failed.load()) PCONV_FAIL("peer rank failed");
    if (wall_seconds() - t0 > timeout_s) PCONV_FAIL("barrier timed out");
    std::this_thread::yield();
  }
}

// Host-staged halo transport through the launcher's shared memory (the
// shared-memory path of an MPI library): each rank stages its boundary rows
// into its own slots, all ranks meet at a barrier, each copies its
// neighbours' slots into its ghost rows, and a second barrier frees the slots.
// Synchronous; needs no RCCL, so several ranks may share one GPU.
class ShmTransport : public HaloTransport {
 public:
  ShmTransport(SharedState* sh, uint8_t* slots, int64_t slot_bytes, int rank, int world, double timeout_s)
      : sh_(sh), slots_(slots), slot_bytes_(slot_bytes), rank_(rank), world_(world), timeout_s_(timeout_s) {}

  void exchange(BandEngine& e, int64_t depth, hipStream_t stream) override {
    TraceRange tr("pconv.halo.shm");
    const Band& b = e.band();
    const int64_t pitch = e.layout().pitch;
    const int64_t n = depth * pitch;
    PCONV_CHECK(n <= slot_bytes_, "shm halo: slot too small");
    uint8_t* row0 = e.src_frame() - kPadLeft;
    if (b.up >= 0) PCONV_HIP_CHECK(hipMemcpyAsync(slot(rank_, 0), row0, n, hipMemcpyDeviceToHost, stream));
    if (b.down >= 0)
      PCONV_HIP_CHECK(hipMemcpyAsync(slot(rank_, 1), row0 + (b.rows - depth) * pitch, n, hipMemcpyDeviceToHost, stream));
    PCONV_HIP_CHECK(hipStreamSynchronize(stream));
    shm_barrier(sh_, world_, timeout_s_);
    if (b.up >= 0) PCONV_HIP_CHECK(hipMemcpyAsync(row0 - n, slot(b.up, 1), n, hipMemcpyHostToDevice, stream));
    if (b.down >= 0)
      PCONV_HIP_CHECK(hipMemcpyAsync(row0 + b.rows * pitch, slot(b.down, 0), n, hipMemcpyHostToDevice, stream));
    PCONV_HIP_CHECK(hipStreamSynchronize(stream));
    shm_barrier(sh_, world_, timeout_s_);
  }
  const char* name() const override { return "shm"; }

 private:
  uint8_t* slot(int r, int which) const { return slots_ + (static_cast<int64_t>(r) * 2 + which) * slot_bytes_; }
  SharedState* sh_;
  uint8_t* slots_;
  int64_t slot_bytes_;
  int rank_, world_;
  double timeout_s_;
};

void run_rank(const CliConfig& c, SharedState* sh, uint8_t* halo_slots, int64_t slot_bytes, int rank) {
  set_error_rank(rank);
  const ImageGeom g = geom_of(c);
  const int world = c.gpus;
  const int ndev = device_count();
  const bool shm = c.transport == "shm", ipc = c.transport == "ipc";
  // RCCL needs one GPU per rank; the shared-memory and IPC transports may
  // oversubscribe (several ranks on one GPU).
  PCONV_CHECK(shm || ipc || ndev >= world,
              "need " + std::to_string(world) + " GPUs, " + std::to_string(ndev) + " visible (try --transport shm)");
  const int device = rank % ndev;
  set_device(device);
  if (world > 1 && c.numa_bind) (void)bind_to_device_numa(device);  // this rank's host work on its GPU's socket
  const Filter f = Filter::by_name(c.filter);
  const Band b = row_band(g.height, world, rank);
  const EngineOptions o = engine_options(c, g, world, device);
  BandEngine eng(g, b, f, o);
  if (c.explain && rank == 0) std::fprintf(stderr, "%s", describe_plan(eng.plan(c.reps)).c_str());
  const int64_t d = eng.layout().halo;
  // Ghost rows straight from the file (free here) unless --exchange-halo:
  // then the first phase exchanges them like every later one.
  const int64_t above = c.preload_halo ? std::min<int64_t>(d, b.y0) : 0;
  const int64_t below = c.preload_halo ? std::min<int64_t>(d, g.height - (b.y0 + b.rows)) : 0;
  const int64_t rb = g.row_bytes();
  PinnedBuffer host(static_cast<size_t>((b.rows + above + below) * rb));
  {
    TraceRange tr("pconv.io.read_band");
    load_rows(c, g, b.y0 - above, b.rows + above + below, host.data(), rb);
  }

  std::shared_ptr<RcclComm> comm;
  std::shared_ptr<IpcHaloTransport> ipct;
  if (shm) {
    eng.set_transport(std::make_shared<ShmTransport>(sh, halo_slots, slot_bytes, rank, world, c.timeout_s));
  } else if (ipc) {
    // Device-side pulls of the neighbours' rows (ipc_halo.hpp): export this
    // rank's frames, meet, open the neighbours' frames, meet.
    ipct = std::make_shared<IpcHaloTransport>(eng, sh->ipc_segment, 0, 1, c.timeout_s, parse_ipc_pull(c.ipc_pull));
    const auto h = ipct->local_handles();
    std::memcpy(sh->ipc_handles[rank], h.data(), h.size());
    shm_barrier(sh, world, c.timeout_s);
    auto blob = [&](int r) {
      return r < 0 ? std::vector<uint8_t>() : std::vector<uint8_t>(sh->ipc_handles[r], sh->ipc_handles[r] + h.size());
    };
    ipct->connect(blob(b.up), blob(b.down));
    eng.set_transport(ipct);
    shm_barrier(sh, world, c.timeout_s);
    ipct->self_test(std::min(5.0, c.timeout_s));  // fails fast, named, on a visibility gap
    if (rank == 0) ipc_unlink_segment(sh->ipc_segment);  // every rank has it mapped
  } else {
    if (rank == 0) {
      const auto id = rccl_unique_id();
      std::memcpy(sh->id, id.data(), kUniqueIdBytes);
      sh->id_ready.store(1);
    } else {
      const double t0 = wall_seconds();
      while (!sh->id_ready.load()) {
        if (sh->failed.load()) PCONV_FAIL("peer rank failed");
        if (wall_seconds() - t0 > c.timeout_s) PCONV_FAIL("timed out waiting for the RCCL unique id");
        std::this_thread::yield();
      }
    }
    std::vector<uint8_t> id(sh->id, sh->id + kUniqueIdBytes);
    comm = std::make_shared<RcclComm>(id, rank, world, device);
    eng.set_transport(std::make_shared<RcclTransport>(comm));
  }

  for (int i = 0; i < c.warmup; ++i) {  // zero frames stay zero; every rank runs the same phases
    eng.run(c.reps);
    if (comm) comm->wait(eng.comm_stream(), c.timeout_s);
    eng.synchronize();
    if (ipct) ipct->check();
  }
  eng.upload_rows(host.data(), rb, -above, b.rows + below);
  eng.set_halo_valid(c.preload_halo);
  eng.synchronize();
  shm_barrier(sh, world, c.timeout_s);  // MPI_Barrier before the timer (mpi_convolution.c:151)
  const double l0 = wall_seconds();
  // --checkpoint-every K: the run in chunks of K repetitions; after each
  // chunk but the last every rank pwrites its band into <out>.rep<done>
  // (pre-sized by the launcher).  A later chunk exchanges its ghost rows
  // (run() invalidates the pre-loaded ones).
  const int chunk = c.checkpoint_every > 0 ? c.checkpoint_every : std::max(1, c.reps);
  int done = 0, launches = 0, exchanges = 0;
  do {
    const int k = std::min(chunk, c.reps - done);
    eng.run(k);
    if (comm) {
      comm->wait(eng.compute_stream(), c.timeout_s);
      comm->wait(eng.comm_stream(), c.timeout_s);
    }
    eng.synchronize();
    if (ipct) ipct->check();
    launches += eng.last_stats().launches;
    exchanges += eng.last_stats().exchanges;
    done += k;
    if (c.checkpoint_every > 0 && done < c.reps) {
      eng.download_rows(host.data(), rb, 0, b.rows);
      eng.synchronize();
      write_rows(out_path(c) + ".rep" + std::to_string(done), g, b.y0, b.rows, host.data(), rb);
    }
  } while (done < c.reps);
  sh->loop_s[rank] = wall_seconds() - l0;
  sh->launches[rank] = launches;
  sh->exchanges[rank] = exchanges;
  eng.download_rows(host.data(), rb, 0, b.rows);
  eng.synchronize();
  {
    TraceRange tr("pconv.io.write_band");
    write_rows(out_path(c), g, b.y0, b.rows, host.data(), rb);
  }
  shm_barrier(sh, world, c.timeout_s);
}

AppReport run_multi(const CliConfig& c) {
  const double t0 = wall_seconds();
  const ImageGeom g = geom_of(c);
  PCONV_CHECK(c.gpus <= kMaxRanks, "too many ranks");
  PCONV_CHECK(g.height >= c.gpus, "image has fewer rows than ranks");
  if (!c.synthetic) validate_input_file(c.image, g);
  // One node by construction: RCCL's bootstrap sockets over loopback (the
  // halo data itself goes over xGMI), unless the user chose an interface.
  if (c.transport == "rccl") ::setenv("NCCL_SOCKET_IFNAME", "lo", 0);
  create_output(out_path(c), g);  // sized + truncated once, ranks pwrite their bands
  if (c.checkpoint_every > 0)
    for (int d = c.checkpoint_every; d < c.reps; d += c.checkpoint_every)
      create_output(out_path(c) + ".rep" + std::to_string(d), g);
  void* mem = mmap(nullptr, sizeof(SharedState), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  PCONV_CHECK(mem != MAP_FAILED, "mmap shared state failed");
  auto* sh = new (mem) SharedState();
  sh->id_ready = 0;
  sh->arrived = 0;
  sh->generation = 0;
  sh->failed = 0;
  if (c.transport == "ipc") {
    std::snprintf(sh->ipc_segment, sizeof(sh->ipc_segment), "/pconv_conv_%d", static_cast<int>(getpid()));
    ipc_create_segment(sh->ipc_segment, c.gpus, 1);
  }
  // Halo staging slots for --transport shm: [rank][top|bottom][depth * pitch].
  uint8_t* slots = nullptr;
  int64_t slot_bytes = 0, slots_total = 0;
  if (c.transport == "shm") {
    const EngineOptions o = engine_options(c, g, c.gpus, 0);
    slot_bytes = static_cast<int64_t>(o.halo_depth) * FrameLayout::make(g.row_bytes(), 1, o.halo_depth).pitch;
    slots_total = slot_bytes * 2 * c.gpus;
    void* sm = mmap(nullptr, static_cast<size_t>(slots_total), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    PCONV_CHECK(sm != MAP_FAILED, "mmap halo slots failed");
    slots = static_cast<uint8_t*>(sm);
  }
  std::fflush(stdout);
  std::fflush(stderr);
  std::vector<pid_t> kids;
  for (int r = 0; r < c.gpus; ++r) {
    const pid_t pid = fork();
    PCONV_CHECK(pid >= 0, "fork failed");
    if (pid == 0) {
      int code = 0;
      try {
        run_rank(c, sh, slots, slot_bytes, r);
      } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        if (!sh->failed.exchange(1)) std::snprintf(sh->error, sizeof(sh->error), "%s", e.what());
        code = 1;
      }
      std::fflush(stdout);
      std::fflush(stderr);
      _exit(code);
    }
    kids.push_back(pid);
  }
  bool ok = true;
  for (pid_t p : kids) {
    int st = 0;
    waitpid(p, &st, 0);
    ok = ok && WIFEXITED(st) && WEXITSTATUS(st) == 0;
  }
  if (c.transport == "ipc") ipc_unlink_segment(sh->ipc_segment);  // (no-op when rank 0 already did)
  if (slots) munmap(slots, static_cast<size_t>(slots_total));
  AppReport r;
  r.gpus = c.gpus;
  r.output = out_path(c);
  if (!ok) {
    std::string msg = sh->error[0] ? sh->error : "a worker process died";
    munmap(mem, sizeof(SharedState));
    PCONV_FAIL("multi-GPU run failed: " + msg);
  }
  for (int i = 0; i < c.gpus; ++i) {
    r.loop_s = std::max(r.loop_s, sh->loop_s[i]);  // max over ranks, like the reference
    r.launches = std::max(r.launches, sh->launches[i]);
    r.exchanges = std::max(r.exchanges, sh->exchanges[i]);
  }
  munmap(mem, sizeof(SharedState));
  const EngineOptions o = engine_options(c, g, c.gpus, 0);
  r.halo = o.halo_depth;
  r.fuse = o.fuse;
  r.kernel = kernel_variant_name(o.variant);
  if (c.check) {
    std::vector<uint8_t> out(static_cast<size_t>(g.bytes()));
    read_image(r.output, g, out.data());
    r.mismatches = compare_with_oracle(c, g, out.data());
  }
  r.e2e_s = wall_seconds() - t0;
  return r;
}


// ------------------------------------------------------------------ bench
// `conv ... --bench K`: bench.py's serving step (H2D + reps + D2H per image,
// `slots` images in flight, one BandPipeline per rank, pre-loaded ghost
// rows) on the NATIVE stack — the HIP runtime this binary links (ROCm), no
// torch, no Python — with the same K-step timing between barriers, the max
// over ranks, the single-image latency, the box's PCIe pair floor and an
// oracle check of every rank's newest image.  Ranks are forked before any
// HIP call (like run_multi); N = 1 runs in this process.
struct BenchShared {
  SharedState st;            // barrier + error reporting (run_multi's)
  double sec[kMaxRanks];     // timed region per rank
  double lat_ms[kMaxRanks];  // median single-image latency per rank
  double pair_ms[kMaxRanks];
  int64_t h2d_bytes[kMaxRanks];  // per image: band + pre-loaded ghost rows
  int64_t d2h_bytes[kMaxRanks];  // per image: owned rows
  int launches, halo, fuse, hip_version;
  char hip_path[512];
};

constexpr double kBaselineMpix = 190.3;  // CUDA 1920x2520 RGB 40 reps end to end, GTX 970

void bench_rank(const CliConfig& c, BenchShared* sh, uint8_t* image, int rank) {
  set_error_rank(rank);
  const ImageGeom g = geom_of(c);
  const bool emu = c.emulate_world > 0;
  const int world = emu ? c.emulate_world : c.gpus;
  const int ndev_ranks = emu ? 1 : world;  // processes sharing the node's GPUs
  if (emu) rank = c.emulate_rank;
  const int ndev = device_count();
  PCONV_CHECK(c.transport == "shm" || ndev >= ndev_ranks,
              "need " + std::to_string(world) + " GPUs, " + std::to_string(ndev) + " visible (--transport shm lets "
              "bench ranks share one GPU)");
  const int device = emu ? 0 : rank % ndev;
  set_device(device);
  if (world > 1 && c.numa_bind) (void)bind_to_device_numa(device);
  const Filter f = Filter::by_name(c.filter);
  const Band b = row_band(g.height, world, rank);
  EngineOptions o = engine_options(c, g, world, device);
  o.cu_mask_queues = c.cu_mask_queues;
  o.head_on_slot_streams = c.head_on_slot_streams;
  // Pre-loaded ghost zone deep enough for every repetition (exchange-free
  // images, like bench.py's headline): rows of the band's dependency cone.
  if (world > 1 && c.halo == 0 && c.reps <= g.height / world) o.halo_depth = std::max(c.reps, o.fuse);
  o.stream_chunks = c.stream_chunks;
  BandPipeline pipe(g, b, f, o, c.slots, -1, /*slot_streams=*/true, /*step_graphs=*/true, /*slot_comm=*/false);
  BandEngine& e0 = pipe.slot(0);
  const int64_t d = e0.layout().halo;
  const int64_t above = world > 1 ? std::min<int64_t>(d, b.y0) : 0;
  const int64_t below = world > 1 ? std::min<int64_t>(d, g.height - (b.y0 + b.rows)) : 0;
  PCONV_CHECK(e0.exchange_free(c.reps, world > 1),
              "--bench needs exchange-free images: " + std::to_string(c.reps) + " repetitions with a " +
                  std::to_string(d) + "-row ghost zone");
  const int64_t rb = g.row_bytes(), in_rows = b.rows + above + below;
  std::vector<PinnedBuffer> ins, outs;
  for (int k = 0; k < c.slots; ++k) {
    ins.emplace_back(static_cast<size_t>(in_rows * rb));
    outs.emplace_back(static_cast<size_t>(b.rows * rb));
  }
  // set-up: a slow pinned buffer would pace the whole pipeline (docs/ROUND6.md §1)
  if (c.qualify_staging) (void)qualify_staging(device, ins, outs, rb, in_rows, b.rows);
  load_rows(c, g, b.y0 - above, in_rows, ins[0].data(), rb);
  for (int k = 1; k < c.slots; ++k) std::memcpy(ins[k].data(), ins[0].data(), ins[0].size());
  // rows the CPU just wrote out of every CPU cache: the copy engines' reads
  // then never fetch dirty lines from the cores that wrote them
  if (c.flush_staging)
    for (auto& x : ins) flush_host_cache(x.data(), x.size());
  int64_t n = 0;
  auto submit = [&]() {
    const int k = static_cast<int>(n++ % c.slots);
    pipe.submit(ins[k].data(), -above, b.rows + below, outs[k].data(), c.reps);
    return k;
  };
  for (int i = 0; i < c.warmup; ++i) submit();
  pipe.drain();
  shm_barrier(&sh->st, ndev_ranks, c.timeout_s);
  const double t0 = wall_seconds();
  for (int i = 0; i < c.bench_steps; ++i) submit();
  pipe.drain();
  const double t1 = wall_seconds();
  shm_barrier(&sh->st, ndev_ranks, c.timeout_s);
  const int slot = emu ? 0 : rank;  // shared-state index of this process
  sh->sec[slot] = t1 - t0;
  sh->h2d_bytes[slot] = in_rows * rb;
  sh->d2h_bytes[slot] = b.rows * rb;
  // one image alone (nothing else queued): the reference GPU_convolution() scope
  std::vector<double> lat;
  int last = 0;
  for (int i = 0; i < 7; ++i) {
    const double a = wall_seconds();
    last = submit();
    pipe.drain();
    lat.push_back((wall_seconds() - a) * 1e3);
  }
  std::sort(lat.begin(), lat.end());
  sh->lat_ms[slot] = lat[lat.size() / 2];
  std::memcpy(image + b.y0 * rb, outs[last].data(), static_cast<size_t>(b.rows * rb));
  sh->pair_ms[slot] = copy_pair_floor_ms(device, rb, in_rows, b.rows, 8);
  if (slot == 0) {
    sh->launches = e0.last_stats().launches;
    sh->halo = static_cast<int>(d);
    sh->fuse = e0.options().fuse;
    const HipRuntimeInfo h = hip_runtime_info();
    sh->hip_version = h.runtime_version;
    std::snprintf(sh->hip_path, sizeof(sh->hip_path), "%s", h.runtime_path.c_str());
  }
  shm_barrier(&sh->st, ndev_ranks, c.timeout_s);
}

std::string bench_metric(const CliConfig& c) {
  const bool head = c.width == 1920 && c.height == 2520 && c.channels == Channels::Rgb && c.reps == 40 &&
                    c.filter == "gaussian";
  if (head) return "Mpixels/sec (and wall-time) for 1920x2520 RGB, 40 reps at 1/2/4/8 MI355X";
  std::string ch = channels_name(c.channels);
  for (auto& x : ch) x = static_cast<char>(std::toupper(static_cast<unsigned char>(x)));
  return "Mpixels/sec (and wall-time) for " + std::to_string(c.width) + "x" + std::to_string(c.height) + " " + ch +
         ", " + std::to_string(c.reps) + " reps" + (c.filter == "gaussian" ? "" : " " + c.filter) +
         " at 1/2/4/8 MI355X";
}

std::string run_bench_impl(const CliConfig& c) {
  const ImageGeom g = geom_of(c);
  PCONV_CHECK(c.backend == Backend::Hip, "--bench needs --backend hip");
  PCONV_CHECK(c.gpus >= 1 && c.gpus <= kMaxRanks && g.height >= c.gpus, "--bench: bad rank count");
  if (!c.synthetic) validate_input_file(c.image, g);
  void* mem = mmap(nullptr, sizeof(BenchShared), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  PCONV_CHECK(mem != MAP_FAILED, "mmap bench state failed");
  auto* sh = new (mem) BenchShared();
  sh->st.arrived = 0;
  sh->st.generation = 0;
  sh->st.failed = 0;
  void* im = mmap(nullptr, static_cast<size_t>(g.bytes()), PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
  PCONV_CHECK(im != MAP_FAILED, "mmap bench image failed");
  auto* image = static_cast<uint8_t*>(im);
  bool ok = true;
  std::string err;
  if (c.gpus == 1) {
    try {
      bench_rank(c, sh, image, 0);
    } catch (const std::exception& e) {
      ok = false;
      err = e.what();
    }
  } else {
    std::fflush(stdout);
    std::fflush(stderr);
    std::vector<pid_t> kids;
    for (int r = 0; r < c.gpus; ++r) {
      const pid_t pid = fork();
      PCONV_CHECK(pid >= 0, "fork failed");
      if (pid == 0) {
        int code = 0;
        try {
          bench_rank(c, sh, image, r);
        } catch (const std::exception& e) {
          std::fprintf(stderr, "%s\n", e.what());
          if (!sh->st.failed.exchange(1)) std::snprintf(sh->st.error, sizeof(sh->st.error), "%s", e.what());
          code = 1;
        }
        std::fflush(stdout);
        std::fflush(stderr);
        _exit(code);
      }
      kids.push_back(pid);
    }
    for (pid_t p : kids) {
      int st = 0;
      waitpid(p, &st, 0);
      ok = ok && WIFEXITED(st) && WEXITSTATUS(st) == 0;
    }
    if (!ok) err = sh->st.error[0] ? sh->st.error : "a bench rank died";
  }
  if (!ok) {
    munmap(im, static_cast<size_t>(g.bytes()));
    munmap(mem, sizeof(BenchShared));
    PCONV_FAIL("bench failed: " + err);
  }
  double sec = 0, lat = 0, pair = 0;
  std::ostringstream per, h2d, d2h;
  for (int r = 0; r < c.gpus; ++r) {
    sec = std::max(sec, sh->sec[r]);
    lat = std::max(lat, sh->lat_ms[r]);
    pair = std::max(pair, sh->pair_ms[r]);
    per << (r ? ", " : "") << sh->sec[r] / c.bench_steps * 1e3;
    h2d << (r ? ", " : "") << sh->h2d_bytes[r];
    d2h << (r ? ", " : "") << sh->d2h_bytes[r];
  }
  int64_t mism = -1;
  if (c.check && c.emulate_world > 0) {
    // the emulated rank's rows only (the rest of the image was never computed)
    const Band b = row_band(g.height, c.emulate_world, c.emulate_rank);
    std::vector<uint8_t> in(static_cast<size_t>(g.bytes())), ref(static_cast<size_t>(g.bytes()));
    load_rows(c, g, 0, g.height, in.data(), g.row_bytes());
    cpu_convolve(Filter::by_name(c.filter), g, in.data(), ref.data(), c.reps, CpuBackend::OpenMP, c.threads);
    mism = 0;
    for (int64_t i = b.y0 * g.row_bytes(); i < (b.y0 + b.rows) * g.row_bytes(); ++i) mism += ref[i] != image[i];
  } else if (c.check) {
    mism = compare_with_oracle(c, g, image);
  }
  const double px = static_cast<double>(c.width) * static_cast<double>(c.height) * c.reps;
  const double value = px * c.bench_steps / sec / 1e6;
  const bool head = c.width == 1920 && c.height == 2520 && c.channels == Channels::Rgb && c.reps == 40 &&
                    c.filter == "gaussian";
  std::ostringstream os;
  os.setf(std::ios::fixed);
  os.precision(4);
  os << "{\"metric\": \"" << bench_metric(c) << "\", \"value\": " << value << ", \"unit\": \"Mpix/s\", \"n_gpus\": "
     << c.gpus << ", \"steps\": " << c.bench_steps << ", \"warmup\": " << c.warmup
     << ", \"ms_per_step\": " << sec / c.bench_steps * 1e3 << ", \"higher_is_better\": true, \"scaling\": \"strong\""
     << ", \"vs_baseline\": ";
  if (head)
    os << value / kBaselineMpix;
  else
    os << "null";
  os << ", \"vs_baseline_basis\": \"pipelined throughput vs reference single-run end-to-end (CUDA, GTX 970)\""
     << ", \"dtype\": \"fp32-exact (packed 16-bit integer, bit-identical to the reference float32)\""
     << ", \"data\": \"" << (c.synthetic ? "synthetic random bytes" : "file") << "\", \"config\": {\"model\": \"3x3 "
     << c.filter << " convolution, " << c.width << "x" << c.height << " " << channels_name(c.channels) << ", "
     << c.reps << " reps\", \"global_batch\": 1, \"seq_len\": " << c.height << ", \"parallelism\": \"rowband"
     << c.gpus << "\", \"step\": \"H2D + reps + D2H per image (reference GPU_convolution scope)\", \"halo_mode\": \""
     << (c.gpus > 1 || c.emulate_world > 1 ? "preload" : "none") << "\", \"images_in_flight\": " << c.slots
     << ", \"stream_chunks\": " << c.stream_chunks
     << ", \"cu_mask_queues\": " << (c.cu_mask_queues ? "true" : "false")
     << ", \"head_on_slot_streams\": " << (c.head_on_slot_streams ? "true" : "false")
     << ", \"numa_bind\": " << (c.numa_bind ? "true" : "false") << ", \"halo_depth\": " << sh->halo << ", \"fuse\": " << sh->fuse
     << ", \"launches_per_step\": " << sh->launches << "}, \"latency_ms\": " << lat
     << ", \"copy_floor\": {\"pair_ms\": " << pair << "}";
  if (mism >= 0)
    os << ", \"mismatches\": " << mism
       << ", \"check\": \"newest image of every rank vs the CPU oracle (OpenMP), after the timed region\"";
  if (c.emulate_world > 0)
    os << ", \"emulated\": \"rank " << c.emulate_rank << " of a " << c.emulate_world
       << "-way split on one GPU; value = this rank's step rate x full-image pixels (proxy, not a multi-GPU "
          "measurement)\"";
  os << ", \"runtime\": {\"stack\": \"native conv (no torch)\", \"hip_runtime_version\": " << sh->hip_version
     << ", \"hip_runtime_path\": \"" << json_escape(sh->hip_path) << "\", \"rccl_version\": null}"
     << ", \"per_rank_ms_per_step\": [" << per.str() << "]"
     << ", \"h2d_bytes_per_step\": [" << h2d.str() << "], \"d2h_bytes_per_step\": [" << d2h.str() << "]}";
  munmap(im, static_cast<size_t>(g.bytes()));
  munmap(mem, sizeof(BenchShared));
  return os.str();
}

}  // namespace

std::string run_bench(const CliConfig& c) { return run_bench_impl(c); }

AppReport run_app(const CliConfig& c, JobCache* cache) {
  AppReport r;
  if (c.backend == Backend::Auto && cache == nullptr && c.checkpoint_every == 0) {
    r = run_auto(c);  // sets r.gpus (0 when the GPU was not used)
  } else if (c.backend == Backend::Cpu || c.backend == Backend::Omp) {
    r = run_cpu(c);
    r.gpus = 0;
  } else if (c.gpus > 1) {
    // (--backend auto in a resident server or with checkpoints: the GPU path)
    PCONV_CHECK(cache == nullptr, "the resident service runs one GPU per server (--gpus 1)");
    r = run_multi(c);
    r.gpus = c.gpus;
  } else {
    r = run_gpu1(c, cache);
    r.gpus = c.gpus;
  }
  const double px = static_cast<double>(c.width) * static_cast<double>(c.height) * c.reps;
  r.mpix_per_s = r.loop_s > 0 ? px / r.loop_s / 1e6 : 0.0;
  return r;
}

std::string report_json(const CliConfig& c, const AppReport& r) {
  std::ostringstream os;
  const double px = static_cast<double>(c.width) * static_cast<double>(c.height) * c.reps;
  os << "{\"width\": " << c.width << ", \"height\": " << c.height << ", \"channels\": \""
     << channels_name(c.channels) << "\", \"reps\": " << c.reps << ", \"filter\": \"" << c.filter
     << "\", \"backend\": \""
     << (c.backend == Backend::Hip ? "hip" : c.backend == Backend::Omp ? "omp" : c.backend == Backend::Auto ? "auto" : "cpu")
     << "\", \"gpus\": " << r.gpus << ", \"kernel\": \"" << r.kernel << "\", \"halo\": " << r.halo
     << ", \"fuse\": " << r.fuse << ", \"launches\": " << r.launches << ", \"exchanges\": " << r.exchanges
     << ", \"loop_s\": " << r.loop_s << ", \"e2e_s\": " << r.e2e_s << ", \"loop_mpix_per_s\": " << r.mpix_per_s
     << ", \"e2e_mpix_per_s\": " << (r.e2e_s > 0 ? px / r.e2e_s / 1e6 : 0.0)
     << ", \"mismatches\": " << r.mismatches << ", \"output\": \"" << json_escape(r.output) << "\""
     << ", \"rccl_loaded\": " << (rccl_loaded() ? "true" : "false");
  if (rccl_loaded()) os << ", \"rccl_version\": \"" << rccl_version() << "\", \"rccl_path\": \""
                        << json_escape(rccl_library_path()) << "\"";
  if (r.cpu_reps >= 0)
    os << ", \"cpu_reps\": " << r.cpu_reps << ", \"gpu_reps\": " << r.gpu_reps << ", \"cpu_rep_s\": " << r.cpu_rep_s
       << ", \"auto_choice\": \"" << json_escape(r.auto_choice) << "\"";
  if ((c.backend == Backend::Hip && c.gpus <= 1) || r.gpu_reps > 0) {  // (the --gpus N launcher never touches HIP)
    const HipRuntimeInfo h = hip_runtime_info();
    os << ", \"hip_runtime_version\": " << h.runtime_version << ", \"hip_runtime_path\": \""
       << json_escape(h.runtime_path) << "\"";
  }
  if (!r.copies.empty()) os << ", \"copies\": \"" << r.copies << "\"";
  if (!r.phases.empty()) {
    os << ", \"phases_s\": {";
    for (size_t i = 0; i < r.phases.size(); ++i)
      os << (i ? ", " : "") << "\"" << r.phases[i].first << "\": " << r.phases[i].second;
    os << "}, \"since_exec_s\": " << r.since_exec_s;
  }
  os << "}";
  return os.str();
}

namespace {

double json_number(const std::string& js, const std::string& key, double dflt) {
  const std::string k = "\"" + key + "\": ";
  const size_t p = js.find(k);
  if (p == std::string::npos) return dflt;
  return std::strtod(js.c_str() + p + k.size(), nullptr);
}

std::string absolute_path(const std::string& p) {
  if (p.empty() || p[0] == '/') return p;
  char buf[PATH_MAX];
  PCONV_CHECK(::getcwd(buf, sizeof(buf)) != nullptr, "getcwd failed");
  return std::string(buf) + "/" + p;
}

// Client half of the resident service: the job runs in the server's warm
// context; this process times it from after argument parsing to the answer
// (the reference's bracket, cuda/main.c:20-49) and prints the same lines.
int run_client(const std::string& prog, const std::vector<std::string>& args, const CliConfig& c) {
  const double t0 = wall_seconds();
  std::vector<std::string> job{prog};
  for (size_t i = 1; i < args.size(); ++i) {
    if (args[i] == "--server") {
      ++i;
      continue;
    }
    if (i == 1 && !c.synthetic) {
      job.push_back(absolute_path(args[i]));
      continue;
    }
    job.push_back(args[i]);
    if (args[i] == "--out" && i + 1 < args.size()) job.push_back(absolute_path(args[++i]));
  }
  // The default output lands next to the input as seen from THIS process.
  if (c.out.empty()) {
    job.push_back("--out");
    job.push_back(absolute_path(output_path_for(args[1])));
  }
  const std::string reply = service_request(c.server, job, c.timeout_s);
  const double e2e = wall_seconds() - t0;
  if (reply.find("\"error\"") != std::string::npos) {
    std::fprintf(stderr, "%s: server: %s\n", prog.c_str(), reply.c_str());
    return EXIT_FAILURE;
  }
  const double loop_s = json_number(reply, "loop_s", 0.0);
  const int64_t bad = static_cast<int64_t>(json_number(reply, "mismatches", -1.0));
  if (!c.quiet) {
    TimeFormat fmt = c.format;
    if (fmt == TimeFormat::Auto) fmt = c.backend == Backend::Hip ? TimeFormat::Cuda : TimeFormat::Mpi;
    if (fmt == TimeFormat::Mpi || fmt == TimeFormat::Both) std::printf("%f\n", loop_s);
    if (fmt == TimeFormat::Cuda || fmt == TimeFormat::Both) std::printf("Execution time: %.3f sec\n", e2e);
  }
  if (c.json) {
    std::string js = reply;
    const size_t close = js.rfind('}');
    if (close != std::string::npos)
      js.insert(close, ", \"served\": true, \"server\": \"" + c.server + "\", \"client_e2e_s\": " +
                           std::to_string(e2e) + ", \"client_since_exec_s\": " + std::to_string(seconds_since_exec()));
    std::printf("%s\n", js.c_str());
  }
  if (c.check) {
    std::fprintf(stderr, "check: %" PRId64 " mismatching bytes vs CPU oracle\n", bad);
    if (bad != 0) return 2;
  }
  return EXIT_SUCCESS;
}

}  // namespace

int conv_main(int argc, char** argv) {
  std::vector<std::string> args(argv, argv + argc);
  const std::string prog = argc > 0 ? argv[0] : "conv";
  for (const auto& a : args)
    if (a == "-h" || a == "--help") {
      std::fputs(help_text(prog).c_str(), stdout);
      return 0;
    }
  if (args.size() >= 2 && args[1] == "--selftest") {
    try {
      return selftest_main(args);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s: %s\n", prog.c_str(), e.what());
      return EXIT_FAILURE;
    }
  }
  if (args.size() >= 2 && args[1] == "--serve") {
    try {
      return serve_main(parse_serve_args(args));
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s: %s\n", prog.c_str(), e.what());
      return EXIT_FAILURE;
    }
  }
  CliConfig c;
  try {
    c = parse_cli(args);
  } catch (const Error& e) {
    const std::string m = e.what();
    if (m.size() >= 5 && m.compare(m.size() - 5, 5, "usage") == 0)
      std::fputs(usage_text(prog).c_str(), stderr);
    else
      std::fprintf(stderr, "%s: %s\n%s", prog.c_str(), m.c_str(), usage_text(prog).c_str());
    return EXIT_FAILURE;
  }
  if (!c.server.empty()) {
    try {
      return run_client(prog, args, c);
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s: %s\n", prog.c_str(), e.what());
      return EXIT_FAILURE;
    }
  }
  if (c.bench_steps > 0) {
    try {
      std::printf("%s\n", run_bench(c).c_str());
      return EXIT_SUCCESS;
    } catch (const std::exception& e) {
      std::fprintf(stderr, "%s: %s\n", prog.c_str(), e.what());
      return EXIT_FAILURE;
    }
  }
  try {
    const AppReport r = run_app(c);
    if (!c.quiet) {
      TimeFormat fmt = c.format;
      if (fmt == TimeFormat::Auto)
        fmt = ((c.backend == Backend::Hip || c.backend == Backend::Auto) && c.gpus == 1) ? TimeFormat::Cuda : TimeFormat::Mpi;
      if (fmt == TimeFormat::Mpi || fmt == TimeFormat::Both) std::printf("%f\n", r.loop_s);
      if (fmt == TimeFormat::Cuda || fmt == TimeFormat::Both) std::printf("Execution time: %.3f sec\n", r.e2e_s);
    }
    if (c.json) std::printf("%s\n", report_json(c, r).c_str());
    if (c.check) {
      std::fprintf(stderr, "check: %" PRId64 " mismatching bytes vs CPU oracle\n", r.mismatches);
      if (r.mismatches != 0) return 2;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s: %s\n", prog.c_str(), e.what());
    return EXIT_FAILURE;
  }
  return EXIT_SUCCESS;
}

}  // namespace pconv
