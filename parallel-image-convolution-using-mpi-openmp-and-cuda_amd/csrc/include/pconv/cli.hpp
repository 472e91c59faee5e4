// Command-line contract.
//
// Reference: `Usage()` (mpi/mpi_convolution.c:328-348) and `Initialization()`
// (cuda/functions.c:10-29): exactly 5 positional arguments
//   image.raw width height repetitions {grey|rgb}
// parsed with atoi (no validation), error text "Error Input!" + usage line and
// exit(EXIT_FAILURE) / MPI_Abort.  pconv keeps the positional contract
// bit-compatible (same order, same type words, same error text) and adds
// optional flags AFTER it.  Numbers are validated strictly.
#pragma once

#include <string>
#include <vector>

#include "pconv/common.hpp"
#include "pconv/kernels.hpp"

namespace pconv {

// Auto (one-shot, 1 GPU): the job is priced on the CPU from a row sample
// (then from its first full repetition); short jobs run on the CPU and never
// touch the GPU, the rest on the GPU path alone (app.cpp run_auto).
enum class Backend { Hip, Cpu, Omp, Auto };
enum class TimeFormat { Auto, Cuda, Mpi, Both };

struct CliConfig {
  std::string image;
  int64_t width = 0, height = 0;
  int reps = 0;
  Channels channels = Channels::Grey;

  Backend backend = Backend::Hip;
  int gpus = 1;
  std::string filter = "gaussian";
  int halo = 0;   // 0 = auto
  int fuse = 0;   // 0 = auto
  bool overlap = true;
  bool graph = false;
  KernelVariant variant = KernelVariant::Auto;
  std::string out;  // "" = blur_<name>
  bool synthetic = false;
  uint64_t seed = 0;
  bool check = false;
  bool json = false;
  int threads = 0;
  TimeFormat format = TimeFormat::Auto;
  int checkpoint_every = 0;
  bool explain = false;
  double timeout_s = 600.0;
  bool quiet = false;
  std::string transport = "rccl";  // multi-GPU halo transport: rccl | shm (host-staged, shared memory)
  bool preload_halo = true;        // ranks read their ghost rows from the input (no exchange at start)
  int warmup = 1;                  // untimed runs of the whole schedule on the zeroed frames first
  std::string server;              // client mode: run the job on the resident server at this socket
  int copies = -1;                 // host<->device copies: -1 auto, 0 SDMA (hipMemcpy2DAsync), 1 CU kernels
  // Serving bench (bench.py's step on the native stack): K timed images, each
  // H2D + reps + D2H, `slots` in flight; 0 = off (a normal run).
  int bench_steps = 0;
  int slots = 4;
  int stream_chunks = 0;  // rows streamed within each image (EngineOptions::stream_chunks)
  // --bench --emulate W:R: time rank R of a W-way split alone in this process
  // (its band + pre-loaded ghost rows): the per-rank proxy of bench.py
  // --emulate, on the native stack.  0 = off.
  int emulate_world = 0, emulate_rank = 0;
  // ---- policy knobs (no environment variables; echoed in the JSON lines)
  int tune = -1;                          // SWAR tile tuning: -1 auto (one-shot off, server on), 0 off, 1 on
  int64_t ring_chunk_bytes = int64_t(32) << 20;  // one-shot ring staging chunk (0: one pinned image)
  double auto_gpu_min_s = 0.1;            // --backend auto: CPU seconds above which the GPU runs the job
  bool cu_mask_queues = true;             // --bench: slot streams on dedicated (CU-masked) queues
  bool head_on_slot_streams = true;       // --bench: streamed head image's copies on the next slots' streams
  std::string ipc_pull = "grid";          // --transport ipc: pull form (grid | single | sdma)
  bool numa_bind = true;                  // N > 1: each rank on its GPU's NUMA node
  bool qualify_staging = true;            // --bench: time every slot's pinned buffers, replace slow ones
  bool flush_staging = true;              // --bench: clflush the CPU-written input rows out of the CPU caches
};

// Parse argv.  Throws pconv::Error with the message to print on bad input.
CliConfig parse_cli(const std::vector<std::string>& args);
// The reference usage text (cuda/functions.c:26 form).
std::string usage_text(const std::string& prog);
// Full option help.
std::string help_text(const std::string& prog);

}  // namespace pconv
