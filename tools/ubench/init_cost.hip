// Start-up cost of the HIP runtime on this box, step by step (the part of
// the reference's end-to-end timer, cuda/main.c:20-49, that is not
// convolution: context creation, allocation, first copies, code objects).
//
//   hipcc --offload-arch=gfx950 -O2 tools/ubench/init_cost.hip -o /tmp/init_cost
//   /tmp/init_cost [bytes] [streams]
//
// Prints one JSON line of milliseconds per step.  Every step is the FIRST call
// of its kind in the process: run it as a fresh process per measurement.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

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
  const size_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (size_t(1920) * 2520 * 3);
  const int nstreams = argc > 2 ? std::atoi(argv[2]) : 1;
  std::vector<std::pair<std::string, double>> ph;
  double t = now_ms();
  auto mark = [&](const char* name) {
    const double n = now_ms();
    ph.emplace_back(name, n - t);
    t = n;
  };
  CK(hipInit(0));
  mark("hipInit");
  int n = 0;
  CK(hipGetDeviceCount(&n));
  mark("hipGetDeviceCount");
  CK(hipSetDevice(0));
  mark("hipSetDevice");
  CK(hipFree(nullptr));
  mark("hipFree0_context");
  void* host = nullptr;
  CK(hipHostMalloc(&host, bytes, hipHostMallocDefault));
  mark("hipHostMalloc");
  std::memset(host, 1, bytes);
  mark("host_first_touch");
  unsigned char* d0 = nullptr;
  unsigned char* d1 = nullptr;
  CK(hipMalloc(&d0, bytes));
  mark("hipMalloc_1");
  CK(hipMalloc(&d1, bytes));
  mark("hipMalloc_2");
  std::vector<hipStream_t> ss(nstreams);
  for (auto& s : ss) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  mark("hipStreamCreate");
  CK(hipMemsetAsync(d0, 0, bytes, ss[0]));
  CK(hipStreamSynchronize(ss[0]));
  mark("first_memset");
  CK(hipMemcpyAsync(d1, host, bytes, hipMemcpyHostToDevice, ss[0]));
  CK(hipStreamSynchronize(ss[0]));
  mark("first_h2d");
  CK(hipMemcpyAsync(d1, host, bytes, hipMemcpyHostToDevice, ss[0]));
  CK(hipStreamSynchronize(ss[0]));
  mark("second_h2d");
  k_touch<<<dim3((bytes + 255) / 256), dim3(256), 0, ss[0]>>>(d1, bytes);
  CK(hipStreamSynchronize(ss[0]));
  mark("first_kernel");
  k_touch<<<dim3((bytes + 255) / 256), dim3(256), 0, ss[0]>>>(d1, bytes);
  CK(hipStreamSynchronize(ss[0]));
  mark("second_kernel");
  CK(hipMemcpyAsync(host, d1, bytes, hipMemcpyDeviceToHost, ss[0]));
  CK(hipStreamSynchronize(ss[0]));
  mark("first_d2h");
  CK(hipMemcpyAsync(host, d1, bytes, hipMemcpyDeviceToHost, ss[0]));
  CK(hipStreamSynchronize(ss[0]));
  mark("second_d2h");
  std::printf("{\"bytes\": %zu, \"streams\": %d, \"ms\": {", bytes, nstreams);
  double total = 0;
  for (size_t i = 0; i < ph.size(); ++i) {
    std::printf("%s\"%s\": %.3f", i ? ", " : "", ph[i].first.c_str(), ph[i].second);
    total += ph[i].second;
  }
  std::printf("}, \"total_ms\": %.3f}\n", total);
  for (auto& s : ss) CK(hipStreamDestroy(s));
  CK(hipFree(d0));
  CK(hipFree(d1));
  CK(hipHostFree(host));
  return 0;
}
