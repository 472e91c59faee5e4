// Native self-tests of the RCCL halo paths and a crash reporter.
//
// The same checks run in two processes with two different stacks: the `conv`
// CLI (`conv --selftest NAME`: ROCm 7.2's HIP runtime and librccl, resolved
// through the binary's rpath) and a torch process (the Python tests: torch's
// bundled HIP runtime and librccl, which the extension binds to because torch
// loads them first).  Every check compares the bytes that RCCL delivered and
// the kernels consumed against a CPU model, so "ran without error" never
// counts as a pass.  Reference being replaced: MPI_Isend/Irecv of boundary
// rows, inner compute, MPI_Wait, edges (mpi/mpi_convolution.c:156-240).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "pconv/filter.hpp"
#include "pconv/image.hpp"
#include "pconv/schedule.hpp"

namespace pconv {

// SIGSEGV / SIGBUS / SIGILL / SIGFPE / SIGABRT: print the signal, the faulting
// address and a native backtrace (backtrace_symbols_fd: library + offset,
// resolvable with llvm-addr2line) to stderr, then hand the signal to the
// handler that was installed before (Python's faulthandler prints the Python
// frames) or to the default action.  Idempotent.  With PCONV_CRASH_LOG set,
// the report is also appended to that file (test runners capture fd 2).
void install_crash_handler();

// CPU model of a self-neighbour band's run (1-rank communicator, up = down =
// self): before every exchange the ghost zone is refreshed with the band's own
// rows (above: rows [0, d); below: rows [rows - d, rows)), which is what RCCL
// send/recv-to-self delivers; ghost rows outside the global image read as 0.
// `pre_exchange` > 0 models an exchange_now() of that depth before the plan.
std::vector<uint8_t> reflected_band_oracle(const Filter& f, Channels ch, int64_t row_bytes, int64_t rows, int64_t halo,
                                           const std::vector<Phase>& plan, const uint8_t* owned, int64_t y0,
                                           int64_t height, int64_t pre_exchange = 0);

// Grouped ncclSend/ncclRecv to self (op "sendrecv") or a 1-rank ncclAllReduce
// (op "allreduce"), issued on the capturing stream or (ops "*_fork") on a
// second stream that joined the capture through an event, captured into a
// hipGraph with capture mode "global",
// "thread_local" or "relaxed" (or "none": issued directly, the control), the
// graph launched `launches` times, received bytes checked.  Progress lines go
// to stderr before each step (so a crash names its step).  Returns a JSON
// object; throws on a byte mismatch.
std::string rccl_capture_probe(const std::string& op, const std::string& mode, int64_t bytes, int device,
                               int launches = 3);

// A mid-image self-neighbour band (y0 > 0, y0 + rows < height) run through
// BandEngine + RcclTransport for several (reps, halo, fuse, overlap, channels)
// cases, each compared byte for byte with reflected_band_oracle.  JSON result;
// throws on the first mismatch.
std::string rccl_selftest_exchange(int device);

// `slots` 1-rank communicators, one per slot stream of a slot-exchange
// BandPipeline, drive `images` exchange images (each slot's exchanges in its
// own stream order, several communicators in flight at once); every image
// compared with the oracle; each slot's drain bounded by `timeout_s` with RCCL
// async-error polling.  Every case runs twice: images issued directly, and
// images captured as one hipGraph each (RCCL send/recv inside the capture).
// JSON result; throws on mismatch or timeout.
std::string rccl_selftest_multicomm(int device, int slots, int images, double timeout_s);

// `conv --selftest {rccl-capture|rccl-exchange|rccl-multicomm|all} [options]`.
int selftest_main(const std::vector<std::string>& args);

}  // namespace pconv
