// Trace ranges for rocprofv3 (`--marker-trace`): roctx push/pop around the
// engine's phases, pipeline images, halo exchanges and band I/O.
//
// The reference has wall clocks only (MPI_Wtime, mpi/mpi_convolution.c:154,242;
// gettimeofday inside an assert, cuda/functions.c:47-51).  Enabled with
// PCONV_TRACE=1: the roctx library is dlopen'ed on first use, so builds and
// runs without it (or without the variable) pay one branch per range.
#pragma once

namespace pconv {

bool trace_enabled();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

class TraceRange {
 public:
  explicit TraceRange(const char* name) : on_(trace_enabled()) {
    if (on_) trace_push(name);
  }
  ~TraceRange() {
    if (on_) trace_pop();
  }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;

 private:
  bool on_;
};

}  // namespace pconv
