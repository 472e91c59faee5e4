// Host-side cost of the HIP runtime calls a serving step issues (gfx950,
// ROCm runtime as shipped): async 1-D / 2-D copies from pinned memory, event
// record / stream-wait, kernel launch, graph launch.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/api_cost.hip -o tools/ubench/api_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                           \
    }                                                                     \
  } while (0)

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 12345) p[0] = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t W = 5760, H = 315, P = 5888;
  void *h, *d;
  CHECK(hipHostMalloc(&h, W * H, 0));
  CHECK(hipMalloc(&d, P * (H + 8)));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const int N = 200;
  for (int round = 0; round < 2; ++round) {
    double t0 = now_us();
    for (int i = 0; i < N; ++i) CHECK(hipMemcpyAsync(d, h, W * H, hipMemcpyHostToDevice, s1));
    double t1 = now_us();
    CHECK(hipStreamSynchronize(s1));
    printf("hipMemcpyAsync H2D 1.8MB        %7.2f us/call (host)\n", (t1 - t0) / N);
    t0 = now_us();
    for (int i = 0; i < N; ++i) CHECK(hipMemcpy2DAsync(d, P, h, W, W, H, hipMemcpyHostToDevice, s1));
    t1 = now_us();
    CHECK(hipStreamSynchronize(s1));
    printf("hipMemcpy2DAsync H2D 1.8MB      %7.2f us/call (host)\n", (t1 - t0) / N);
    t0 = now_us();
    for (int i = 0; i < N; ++i) CHECK(hipMemcpy2DAsync(h, W, d, P, W, H, hipMemcpyDeviceToHost, s1));
    t1 = now_us();
    CHECK(hipStreamSynchronize(s1));
    printf("hipMemcpy2DAsync D2H 1.8MB      %7.2f us/call (host)\n", (t1 - t0) / N);
    t0 = now_us();
    for (int i = 0; i < N; ++i) {
      CHECK(hipEventRecord(ev, s1));
      CHECK(hipStreamWaitEvent(s2, ev, 0));
    }
    t1 = now_us();
    CHECK(hipDeviceSynchronize());
    printf("eventRecord+streamWaitEvent     %7.2f us/pair (host)\n", (t1 - t0) / N);
    t0 = now_us();
    for (int i = 0; i < N; ++i) empty_kernel<<<256, 256, 0, s1>>>(nullptr);
    t1 = now_us();
    CHECK(hipStreamSynchronize(s1));
    double t2 = now_us();
    printf("kernel launch (empty, 256 WGs)  %7.2f us/call host, %7.2f us/kernel until drained\n", (t1 - t0) / N,
           (t2 - t0) / N);
    // graph of 5 kernels
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s2, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 5; ++k) empty_kernel<<<256, 256, 0, s2>>>(nullptr);
    CHECK(hipStreamEndCapture(s2, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    t0 = now_us();
    for (int i = 0; i < N; ++i) CHECK(hipGraphLaunch(ge, s2));
    t1 = now_us();
    CHECK(hipStreamSynchronize(s2));
    t2 = now_us();
    printf("graph launch (5 empty kernels)  %7.2f us/call host, %7.2f us/graph until drained\n", (t1 - t0) / N,
           (t2 - t0) / N);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
  }
  return 0;
}
