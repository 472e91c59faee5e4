// CLI parsing (see cli.hpp).
#include "pconv/cli.hpp"

#include <cerrno>
#include <climits>
#include <cstdlib>

namespace pconv {

namespace {

int64_t parse_int(const std::string& s, const char* what, int64_t lo, int64_t hi) {
  if (s.empty()) PCONV_FAIL(std::string("invalid ") + what + ": empty");
  errno = 0;
  char* end = nullptr;
  const long long v = std::strtoll(s.c_str(), &end, 10);
  if (errno != 0 || end == s.c_str() || *end != '\0')
    PCONV_FAIL(std::string("invalid ") + what + " '" + s + "': not an integer");
  if (v < lo || v > hi)
    PCONV_FAIL(std::string("invalid ") + what + " '" + s + "': must be in [" + std::to_string(lo) + ", " +
               std::to_string(hi) + "]");
  return v;
}

}  // namespace

std::string usage_text(const std::string& prog) {
  return "Error Input!\n" + prog + " image_name width height repetitions [rgb/grey].\n";
}

std::string help_text(const std::string& prog) {
  return "usage: " + prog +
         " image.raw width height repetitions {grey,rgb,rgba} [options]\n"
         "  --backend {hip,cpu,omp,auto}  compute backend (default hip; auto: the job is priced on the CPU from\n"
         "                            a row sample, then from its first full repetition; above --auto-gpu-min\n"
         "                            seconds of CPU time the GPU runs it alone, otherwise the CPU runs it and\n"
         "                            the GPU is never touched)\n"
         "  --auto-gpu-min S          --backend auto: CPU seconds above which the GPU runs the job (default 0.1)\n"
         "  --gpus N                  row-band decomposition over N GPUs, one process each (RCCL halos)\n"
         "  --filter {gaussian,box,edge}  3x3 filter (default gaussian)\n"
         "  --halo D                  ghost rows exchanged at once (default: auto)\n"
         "  --fuse T                  repetitions fused per kernel launch (default: auto)\n"
         "  --no-overlap              do not overlap halo exchange with interior compute\n"
         "  --graph                   capture the repetition loop in a hipGraph (1 GPU)\n"
         "  --kernel {auto,binomial,temporal,int9,float9,float_temporal}\n"
         "  --out PATH                output file (default: blur_<image> next to the input)\n"
         "  --synthetic SEED          use a deterministic random image instead of reading the file\n"
         "  --check                   verify the result against the CPU oracle\n"
         "  --json                    print a JSON metrics line\n"
         "  --threads N               OpenMP threads for --backend omp\n"
         "  --format {cuda,mpi,both}  timing line(s) to print (default: cuda for 1 GPU, mpi otherwise)\n"
         "  --checkpoint-every K      write <out>.rep<N> every K repetitions\n"
         "  --explain                 print the halo/launch schedule\n"
         "  --timeout S               RCCL watchdog timeout in seconds (default 600)\n"
         "  --transport {rccl,shm,ipc}  multi-GPU halo transport (shm: host-staged through shared memory;\n"
         "                            ipc: device-side pulls of the neighbours' rows through HIP IPC;\n"
         "                            both let several ranks share one GPU)\n"
         "  --exchange-halo           ranks load only their own rows; ghost rows come from neighbours\n"
         "  --warmup N                untimed runs of the schedule before loading the image (default 1;\n"
         "                            loads the kernels' code objects and sets up RCCL connections)\n"
         "  --quiet                   suppress the timing lines\n"
         "  --server SOCKET           run the job on a resident `conv --serve SOCKET` (warm GPU context)\n"
         "  --copies {auto,sdma,kernel}  1-GPU host<->device copies: SDMA engines or CU kernels (auto:\n"
         "                            kernels in a one-shot process, SDMA in a resident server)\n"
         "  --bench K                 serving bench: K timed images (H2D + reps + D2H each) per rank after\n"
         "                            --warmup untimed ones; prints bench.py's JSON line (native stack)\n"
         "  --slots S                 --bench: images in flight (default 4)\n"
         "  --stream-chunks C         --bench: rows of each image streamed in C chunks (0 = off)\n"
         "  --emulate W:R             --bench: time rank R of a W-way split alone (per-rank proxy)\n"
         "  --pool-queues             --bench: slot streams from the runtime's queue pool (default: each on\n"
         "                            its own CU-masked hardware queue)\n"
         "  --head-pool-streams       --bench: a streamed head image's copies on two pool streams (default:\n"
         "                            the next two slots' streams)\n"
         "  --ipc-pull {grid,single,sdma}  --transport ipc: pull form (default grid: many workgroups)\n"
         "  --tune {auto,on,off}      SWAR tile-shape tuning (auto: off for a one-shot run, on in a server)\n"
         "  --ring-chunk-bytes B      one-shot staging ring chunk (default 32 MiB; 0 = one pinned image)\n"
         "  --no-numa-bind            N > 1: leave each rank's CPU affinity alone\n"
         "  --no-qualify-staging      --bench: keep the first pinned staging buffers (default: time each slot's\n"
         "                            buffers at set-up and replace any >5% slower than the best)\n"
         "  --no-flush-staging        --bench: leave the loaded input rows in the CPU caches (default: clflush)\n"

         "\n"
         "       " + prog + " --serve SOCKET [--device D] [--idle-timeout S] [--max-engines N]\n"
         "                            resident service: initialise the GPU once, then run jobs sent by\n"
         "                            `--server SOCKET` clients one at a time\n";
}

CliConfig parse_cli(const std::vector<std::string>& args) {
  // Reference contract: argc == 6 and argv[5] in {grey, rgb}; anything else
  // prints usage_text and exits with EXIT_FAILURE.
  if (args.size() < 6) PCONV_FAIL("usage");
  CliConfig c;
  c.image = args[1];
  const std::string& type = args[5];
  if (type != "grey" && type != "rgb" && type != "rgba") PCONV_FAIL("usage");
  c.channels = parse_channels(type);
  c.width = parse_int(args[2], "width", 1, int64_t(1) << 30);
  c.height = parse_int(args[3], "height", 1, int64_t(1) << 30);
  c.reps = static_cast<int>(parse_int(args[4], "repetitions", 0, INT_MAX));
  for (size_t i = 6; i < args.size(); ++i) {
    const std::string& a = args[i];
    auto next = [&](const char* what) -> std::string {
      if (i + 1 >= args.size()) PCONV_FAIL(std::string("missing value for ") + what);
      return args[++i];
    };
    if (a == "--backend") {
      const std::string v = next("--backend");
      if (v == "hip") c.backend = Backend::Hip;
      else if (v == "cpu") c.backend = Backend::Cpu;
      else if (v == "omp") c.backend = Backend::Omp;
      else if (v == "auto") c.backend = Backend::Auto;
      else PCONV_FAIL("invalid --backend '" + v + "' (hip|cpu|omp|auto)");
    } else if (a == "--gpus") {
      c.gpus = static_cast<int>(parse_int(next("--gpus"), "--gpus", 1, 64));
    } else if (a == "--filter") {
      c.filter = next("--filter");
      if (c.filter != "gaussian" && c.filter != "box" && c.filter != "edge")
        PCONV_FAIL("invalid --filter '" + c.filter + "' (gaussian|box|edge)");
    } else if (a == "--halo") {
      c.halo = static_cast<int>(parse_int(next("--halo"), "--halo", 1, 1 << 20));
    } else if (a == "--fuse") {
      c.fuse = static_cast<int>(parse_int(next("--fuse"), "--fuse", 1, kMaxFusedSteps));
    } else if (a == "--no-overlap") {
      c.overlap = false;
    } else if (a == "--graph") {
      c.graph = true;
    } else if (a == "--kernel") {
      const std::string v = next("--kernel");
      if (v == "auto") c.variant = KernelVariant::Auto;
      else if (v == "binomial") c.variant = KernelVariant::Binomial;
      else if (v == "temporal") c.variant = KernelVariant::Temporal;
      else if (v == "int9") c.variant = KernelVariant::Int9;
      else if (v == "float9") c.variant = KernelVariant::Float9;
      else if (v == "float_temporal") c.variant = KernelVariant::FloatTemporal;
      else PCONV_FAIL("invalid --kernel '" + v + "'");
    } else if (a == "--out") {
      c.out = next("--out");
    } else if (a == "--synthetic") {
      c.synthetic = true;
      c.seed = static_cast<uint64_t>(parse_int(next("--synthetic"), "--synthetic", 0, INT64_MAX));
    } else if (a == "--check") {
      c.check = true;
    } else if (a == "--json") {
      c.json = true;
    } else if (a == "--threads") {
      c.threads = static_cast<int>(parse_int(next("--threads"), "--threads", 1, 4096));
    } else if (a == "--format") {
      const std::string v = next("--format");
      if (v == "cuda") c.format = TimeFormat::Cuda;
      else if (v == "mpi") c.format = TimeFormat::Mpi;
      else if (v == "both") c.format = TimeFormat::Both;
      else PCONV_FAIL("invalid --format '" + v + "' (cuda|mpi|both)");
    } else if (a == "--checkpoint-every") {
      c.checkpoint_every = static_cast<int>(parse_int(next("--checkpoint-every"), "--checkpoint-every", 1, INT_MAX));
    } else if (a == "--explain") {
      c.explain = true;
    } else if (a == "--timeout") {
      c.timeout_s = static_cast<double>(parse_int(next("--timeout"), "--timeout", 1, 86400));
    } else if (a == "--quiet") {
      c.quiet = true;
    } else if (a == "--transport") {
      c.transport = next("--transport");
      if (c.transport != "rccl" && c.transport != "shm" && c.transport != "ipc")
        PCONV_FAIL("invalid --transport '" + c.transport + "' (rccl|shm|ipc)");
    } else if (a == "--exchange-halo") {
      c.preload_halo = false;
    } else if (a == "--copies") {
      const std::string v = next("--copies");
      if (v == "auto") c.copies = -1;
      else if (v == "sdma") c.copies = 0;
      else if (v == "kernel") c.copies = 1;
      else PCONV_FAIL("invalid --copies '" + v + "' (auto|sdma|kernel)");
    } else if (a == "--server") {
      c.server = next("--server");
    } else if (a == "--bench") {
      c.bench_steps = static_cast<int>(parse_int(next("--bench"), "--bench", 1, 1 << 24));
    } else if (a == "--slots") {
      c.slots = static_cast<int>(parse_int(next("--slots"), "--slots", 1, 8));
    } else if (a == "--emulate") {
      const std::string v = next("--emulate");
      const size_t colon = v.find(':');
      if (colon == std::string::npos) PCONV_FAIL("invalid --emulate '" + v + "' (WORLD:RANK)");
      c.emulate_world = static_cast<int>(parse_int(v.substr(0, colon), "--emulate world", 1, 64));
      c.emulate_rank = static_cast<int>(parse_int(v.substr(colon + 1), "--emulate rank", 0, c.emulate_world - 1));
    } else if (a == "--stream-chunks") {
      c.stream_chunks = static_cast<int>(parse_int(next("--stream-chunks"), "--stream-chunks", 0, 4096));
    } else if (a == "--pool-queues") {
      c.cu_mask_queues = false;
    } else if (a == "--head-pool-streams") {
      c.head_on_slot_streams = false;
    } else if (a == "--ipc-pull") {
      c.ipc_pull = next("--ipc-pull");
      if (c.ipc_pull != "grid" && c.ipc_pull != "single" && c.ipc_pull != "sdma")
        PCONV_FAIL("invalid --ipc-pull '" + c.ipc_pull + "' (grid|single|sdma)");
    } else if (a == "--tune") {
      const std::string v = next("--tune");
      if (v == "auto") c.tune = -1;
      else if (v == "on") c.tune = 1;
      else if (v == "off") c.tune = 0;
      else PCONV_FAIL("invalid --tune '" + v + "' (auto|on|off)");
    } else if (a == "--ring-chunk-bytes") {
      c.ring_chunk_bytes = parse_int(next("--ring-chunk-bytes"), "--ring-chunk-bytes", 0, int64_t(1) << 40);
    } else if (a == "--auto-gpu-min") {
      const std::string v = next("--auto-gpu-min");
      char* end = nullptr;
      c.auto_gpu_min_s = std::strtod(v.c_str(), &end);
      if (v.empty() || *end != '\0' || !(c.auto_gpu_min_s >= 0)) PCONV_FAIL("invalid --auto-gpu-min '" + v + "'");
    } else if (a == "--no-numa-bind") {
      c.numa_bind = false;
    } else if (a == "--no-qualify-staging") {
      c.qualify_staging = false;
    } else if (a == "--no-flush-staging") {
      c.flush_staging = false;
    } else if (a == "--warmup") {
      c.warmup = static_cast<int>(parse_int(next("--warmup"), "--warmup", 0, 100));
    } else {
      PCONV_FAIL("unknown option '" + a + "'");
    }
  }
  if (c.backend != Backend::Hip && c.gpus != 1) PCONV_FAIL("--gpus requires --backend hip");
  if (c.backend == Backend::Auto && c.bench_steps > 0) PCONV_FAIL("--bench runs on the GPU (--backend hip)");
  if (c.emulate_world > 0 && (c.bench_steps == 0 || c.gpus != 1))
    PCONV_FAIL("--emulate needs --bench and --gpus 1 (one process times one rank of the split)");
  return c;
}

}  // namespace pconv
