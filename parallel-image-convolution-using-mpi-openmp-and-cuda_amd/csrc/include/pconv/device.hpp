// HIP runtime layer: RAII device/pinned buffers, streams, events, checks.
//
// Replaces the reference's synchronous pageable copies, cudaMalloc inside the
// timed region and deprecated cudaThreadSynchronize
// (cuda/cuda_convolution.cu:56-101): buffers are allocated once and reused,
// host staging is pinned (hipHostMalloc) so copies are async DMA, and all
// ordering is expressed with streams + events.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "pconv/common.hpp"

#define PCONV_HIP_CHECK(expr)                                                                  \
  do {                                                                                         \
    hipError_t _e = (expr);                                                                    \
    if (_e != hipSuccess)                                                                      \
      ::pconv::raise_error(__FILE__, __LINE__, std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

namespace pconv {

int device_count();
void set_device(int device);
std::string device_name(int device);
// PCI address of a device, lower case ("0000:75:00.0").
std::string device_pci_bus_id(int device);
// The HIP runtime this process runs on (which may differ from the one the
// code was compiled against: torch processes load torch's bundled runtime):
// runtime and driver versions from the API, the runtime library's path, and
// the compile-time HIP version.
struct HipRuntimeInfo {
  int runtime_version = 0;
  int driver_version = 0;
  std::string runtime_path;
  std::string compiled_version;
};
HipRuntimeInfo hip_runtime_info();
// Restrict the calling process to the CPUs local to `device` (sysfs
// local_cpulist of its PCI function, intersected with the current affinity).
// Returns the CPUs kept, 0 if nothing changed.
int bind_to_device_numa(int device);

// PCIe floor of one pipelined step on this box: `iters` pitched (2-D) H2D
// copies of `rows_in` rows and, concurrently on a second stream, `iters`
// pitched D2H copies of `rows_out` rows — the copy shapes the serving
// pipeline issues — timed together; returns ms per (H2D, D2H) pair.  With
// both directions busy the link carries less than the sum of the solo rates
// (~94 GB/s in both directions together on the measured boxes), so this, not
// the slower solo copy, is what a PCIe-bound step converges to.
double copy_pair_floor_ms(int device, int64_t row_bytes, int64_t rows_in, int64_t rows_out, int iters);
// NUMA node of every page of a host range (move_pages(2) query, nothing
// moved): node -> pages; a negative key is -errno for pages the kernel could
// not report, <= -1000 when the query itself failed.  And a GPU's own node
// (sysfs numa_node of its PCI function, -1 if unknown).
std::map<int, int64_t> page_nodes(const void* p, size_t bytes);
int device_numa_node(int device);
// Write back and evict a host range from every CPU cache (clflush per line):
// staging rows the CPU has just written stop being dirty lines that each DMA
// read of the copy engines must fetch from a core's cache.
void flush_host_cache(const void* p, size_t bytes);
struct CopyFloor {
  double h2d_ms = 0, d2h_ms = 0, pair_ms = 0;
};
// The same copies from / into GIVEN pinned host buffers (nullptr: fresh
// ones), each direction alone and both together, ms per copy / pair (the
// best of two runs of `iters`): whether one slot's staging buffers are
// slower than another's.
CopyFloor copy_floor_on(int device, uint8_t* host_in, uint8_t* host_out, int64_t row_bytes, int64_t rows_in,
                        int64_t rows_out, int iters);

class PinnedBuffer;
// Staging qualification (the C++ twin of DistributedBlur._qualify_staging,
// for `conv --bench`): every slot's pinned input / output buffer through the
// copy engines once; a buffer more than `tolerance` slower than the best of
// its direction is replaced by a fresh allocation (rejected ones held until
// the search ends), up to `attempts` rounds.  Measured on MI355X boxes: in
// some processes one pinned buffer uploads at ~42 instead of ~55 GB/s and
// paces a whole pipeline (docs/ROUND6.md §1).
struct StagingReport {
  std::vector<CopyFloor> first, final;
  CopyFloor fresh;  // the same copies through freshly allocated buffers (the reference)
  int replaced = 0;
};
StagingReport qualify_staging(int device, std::vector<PinnedBuffer>& ins, std::vector<PinnedBuffer>& outs,
                              int64_t row_bytes, int64_t rows_in, int64_t rows_out, double tolerance = 1.05,
                              int attempts = 3);

class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  explicit DeviceBuffer(size_t bytes);
  // hipExtMallocWithFlags (hipDeviceMallocFinegrained / hipDeviceMallocUncached):
  // device memory with explicit coherence, e.g. words other GPUs store into.
  DeviceBuffer(size_t bytes, unsigned flags);
  ~DeviceBuffer();
  DeviceBuffer(DeviceBuffer&& o) noexcept { *this = std::move(o); }
  DeviceBuffer& operator=(DeviceBuffer&& o) noexcept;
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  uint8_t* data() const { return ptr_; }
  size_t size() const { return bytes_; }

 private:
  uint8_t* ptr_ = nullptr;
  size_t bytes_ = 0;
};

class PinnedBuffer {
 public:
  PinnedBuffer() = default;
  explicit PinnedBuffer(size_t bytes);
  ~PinnedBuffer();
  PinnedBuffer(PinnedBuffer&& o) noexcept { *this = std::move(o); }
  PinnedBuffer& operator=(PinnedBuffer&& o) noexcept;
  PinnedBuffer(const PinnedBuffer&) = delete;
  PinnedBuffer& operator=(const PinnedBuffer&) = delete;
  uint8_t* data() const { return ptr_; }
  size_t size() const { return bytes_; }

 private:
  uint8_t* ptr_ = nullptr;
  size_t bytes_ = 0;
};

class Stream {
 public:
  Stream() = default;
  static Stream create(int priority = 0);
  // A stream on its own hardware queue restricted to the CUs set in `mask`
  // (bit i of word w = CU 32*w + i); all-ones = every CU.
  static Stream create_cu_masked(const std::vector<uint32_t>& mask);
  ~Stream();
  Stream(Stream&& o) noexcept : s_(o.s_) { o.s_ = nullptr; }
  Stream& operator=(Stream&& o) noexcept {
    std::swap(s_, o.s_);
    return *this;
  }
  hipStream_t get() const { return s_; }
  void sync() const;

 private:
  hipStream_t s_ = nullptr;
};

class Event {
 public:
  Event() = default;
  static Event create(bool timing = false);
  ~Event();
  Event(Event&& o) noexcept : e_(o.e_) { o.e_ = nullptr; }
  Event& operator=(Event&& o) noexcept {
    std::swap(e_, o.e_);
    return *this;
  }
  hipEvent_t get() const { return e_; }
  void record(hipStream_t s) const;
  void wait_on(hipStream_t s) const;  // make stream s wait for this event
  void sync() const;
  // milliseconds between two recorded timing events
  static float elapsed_ms(const Event& a, const Event& b);

 private:
  hipEvent_t e_ = nullptr;
};

// The copies behind the copy floors, set up once (device frames, pinned host
// rows unless given, two streams; first-use costs paid in the constructor),
// then timed on demand: run(n, up, down) issues n pitched H2D copies on one
// stream and / or n pitched D2H copies on another and returns ms per copy
// (pair) over the whole run — no minimum taken, so ranks that run at once
// see each other's traffic (bench.py's concurrent floors).
class CopyProbe {
 public:
  CopyProbe(int device, uint8_t* host_in, uint8_t* host_out, int64_t row_bytes, int64_t rows_in, int64_t rows_out);
  double run(int n, bool up, bool down);

 private:
  int device_;
  int64_t row_bytes_, rows_in_, rows_out_, pitch_;
  DeviceBuffer din_, dout_;
  PinnedBuffer hin_own_, hout_own_;
  uint8_t* host_in_;
  uint8_t* host_out_;
  Stream s1_, s2_;
  Event e0_, a_, b_;
};

}  // namespace pconv
