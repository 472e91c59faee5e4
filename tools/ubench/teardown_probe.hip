// Round 5: what in one GPU process makes the NEXT process's runtime start-up
// slow (the back-to-back CUDA table: hip_init 187 ms median vs 53 ms after an
// idle gap).  A "previous" process does some of a one-shot
// `conv` run's work and exits; the "next" process times its first HIP call.
//
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/teardown_probe.hip -o /tmp/teardown_probe
//   /tmp/teardown_probe <mode> [MB]      (mode: init | stream | pinned | dev | kernel | all | all_free)
//   /tmp/teardown_probe measure          (prints {"hip_init_ms": ...})
//
// all_free: like all, then releases everything (streams, memory) and calls
// hipDeviceReset before exit (is the teardown the process exit's or the
// resources'?).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

__global__ void k_touch(unsigned char* p, size_t n) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i < n) p[i] = static_cast<unsigned char>(p[i] + 1);
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "measure";
  const size_t mb = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 15;
  const size_t bytes = mb << 20;
  const double t0 = now_ms();
  CK(hipFree(nullptr));
  const double t1 = now_ms();
  if (mode == "measure") {
    std::printf("{\"hip_init_ms\": %.2f}\n", t1 - t0);
    return 0;
  }
  hipStream_t s = nullptr;
  void* h = nullptr;
  void* d = nullptr;
  const bool all = mode == "all" || mode == "all_free";
  if (mode == "stream" || mode == "kernel" || all) CK(hipStreamCreate(&s));
  if (mode == "pinned" || all) {
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    std::memset(h, 1, bytes);
  }
  if (mode == "dev" || mode == "kernel" || all) CK(hipMalloc(&d, bytes));
  if (mode == "kernel" || all) {
    k_touch<<<dim3(static_cast<unsigned>((bytes + 255) / 256)), dim3(256), 0, s>>>(static_cast<unsigned char*>(d), bytes);
    if (h) CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));
  }
  const double t2 = now_ms();
  if (mode == "all_free") {
    if (s) CK(hipStreamDestroy(s));
    if (h) CK(hipHostFree(h));
    if (d) CK(hipFree(d));
    CK(hipDeviceReset());
  }
  const double t3 = now_ms();
  std::printf("{\"mode\": \"%s\", \"hip_init_ms\": %.2f, \"work_ms\": %.2f, \"free_ms\": %.2f}\n", mode.c_str(),
              t1 - t0, t2 - t1, t3 - t2);
  return 0;
}
