// `conv` application: single-GPU, CPU and multi-GPU (native fork launcher) runs.
//
// Reference drivers: cuda/main.c:10-53 (parse, time, read, GPU_convolution,
// write blur_<name>, print "Execution time: %.3f sec") and
// mpi/mpi_convolution.c:17-286 (mpiexec -n P; MPI-IO band reads; loop timing
// between MPI_Barrier/MPI_Wtime; max over ranks printed as "%f").
//
// Multi-GPU: `conv ... --gpus N` forks N worker processes BEFORE any HIP call
// (one process per GPU, like mpiexec).  Workers share an anonymous mmap used
// to hand out the RCCL unique id, as a barrier, and to collect per-rank loop
// times (the reference's Send/Recv max-gather).  Each worker preads only its
// band (+ ghost rows) and pwrites only its band of the pre-sized output file.
#pragma once

#include <string>
#include <vector>

#include "pconv/cli.hpp"

namespace pconv {

struct AppReport {
  double loop_s = 0;       // max over ranks of the rep-loop time
  double e2e_s = 0;        // end-to-end wall time (incl. I/O and device init)
  double mpix_per_s = 0;   // W*H*reps / loop_s / 1e6
  int gpus = 1;
  int halo = 1, fuse = 1;
  int launches = 0, exchanges = 0;
  int64_t mismatches = -1; // --check result (-1 = not checked)
  std::string kernel;
  std::string copies;  // 1 GPU: "sdma" | "kernel" host<->device copies
  std::string output;
  // End-to-end breakdown (seconds, in order): the reference's timer covers
  // everything after argument parsing (cuda/main.c:20-49), HIP/CUDA context
  // creation included; these phases say where that time goes.
  std::vector<std::pair<std::string, double>> phases;
  double since_exec_s = 0;  // process start (exec) -> report, 10 ms resolution (/proc)
  // --backend auto: repetitions run on the CPU before the handoff / on the
  // GPU after it, the CPU's measured time per repetition, and why the GPU
  // was (not) used.
  int cpu_reps = -1, gpu_reps = -1;
  double cpu_rep_s = 0;
  std::string auto_choice;
};

// Runs the CLI (argv as given).  Returns the process exit code.
int conv_main(int argc, char** argv);

// Engines / staging kept by a resident server between jobs (service.hpp).
struct JobCache;
JobCache* new_job_cache(int device, int max_engines);
void delete_job_cache(JobCache* c);

// Library entry: run a parsed config in this process (1 GPU or CPU), or via
// the fork launcher when cfg.gpus > 1.  With a cache (resident server) the
// device context is already up and engines are reused across jobs.
AppReport run_app(const CliConfig& cfg, JobCache* cache = nullptr);

std::string report_json(const CliConfig& cfg, const AppReport& r);

// `--bench K`: bench.py's serving step on the native stack (fork launcher for
// N > 1); returns bench.py's JSON line.
std::string run_bench(const CliConfig& cfg);

}  // namespace pconv
