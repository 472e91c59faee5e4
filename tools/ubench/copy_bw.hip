// PCIe copy bandwidth for the serving pipeline's shapes (pinned host memory):
// contiguous vs pitched (hipMemcpy2DAsync into a padded frame), H2D, D2H and
// both directions at once on two streams.
// build: hipcc --offload-arch=gfx950 -O3 tools/ubench/copy_bw.hip -o tools/ubench/copy_bw
#include <hip/hip_runtime.h>

#include <sys/mman.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                        \
  do {                                                                  \
    hipError_t e = (x);                                                 \
    if (e != hipSuccess) {                                              \
      printf("HIP error %s at line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                         \
    }                                                                   \
  } while (0)

// Zero-copy: the CUs move the bytes over PCIe themselves (pinned host memory
// is mapped into the GPU's address space).  One uint4 per lane, rows pitched.
__global__ void k_copy_rows(const uint8_t* __restrict__ src, size_t sp, uint8_t* __restrict__ dst, size_t dp, int w16,
                            int h) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  const int y = blockIdx.y;
  if (x >= w16 || y >= h) return;
  const uint4 v = reinterpret_cast<const uint4*>(src + y * sp)[x];
  reinterpret_cast<uint4*>(dst + y * dp)[x] = v;
}

int main(int argc, char** argv) {
  // 1920x2520 RGB row bytes, frame pitch; optional argv[1] = rows (e.g. 395:
  // one rank's band + ghost rows of the 8-way split), argv[2] = iterations.
  // argv[4] / argv[5]: row bytes / frame pitch (default: the RGB headline frame)
  const size_t W = argc > 4 ? static_cast<size_t>(atol(argv[4])) : 5760;
  const size_t P = argc > 5 ? static_cast<size_t>(atol(argv[5])) : 5888;
  const size_t H = argc > 1 ? static_cast<size_t>(atol(argv[1])) : 2520;
  const size_t bytes = W * H;
  void *h_in, *h_out, *d_a, *d_b;
  // argv[3] = "thp": host buffers from 2 MB-aligned anonymous memory with
  // transparent huge pages requested, then registered (hipHostRegister) —
  // fewer IOMMU / page-table entries per DMA than hipHostMalloc's pages.
  const bool thp = argc > 3 && std::strcmp(argv[3], "thp") == 0;  // any other word: hipHostMalloc
  if (thp) {
    const size_t span = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    for (void** hp : {&h_in, &h_out}) {
      void* m = mmap(nullptr, span + (size_t(2) << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) return 1;
      void* a = reinterpret_cast<void*>((reinterpret_cast<uintptr_t>(m) + (size_t(2) << 20) - 1) & ~((uintptr_t(2) << 20) - 1));
      (void)madvise(a, span, MADV_HUGEPAGE);
      std::memset(a, 1, span);
      CHECK(hipHostRegister(a, span, hipHostRegisterDefault));
      *hp = a;
    }
  } else {
    CHECK(hipHostMalloc(&h_in, bytes, 0));
    CHECK(hipHostMalloc(&h_out, bytes, 0));
  }
  CHECK(hipMalloc(&d_a, P * (H + 16)));
  CHECK(hipMalloc(&d_b, P * (H + 16)));
  hipStream_t s1, s2;
  CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int iters = argc > 2 ? atoi(argv[2]) : 20;
  printf("rows %zu, %.2f MB per copy, %d iterations, host memory: %s\n", H, W * H / 1e6, iters, thp ? "THP + hipHostRegister" : "hipHostMalloc");
  auto report = [&](const char* name, float ms, double gb) {
    printf("%-34s %8.3f ms/iter  %6.1f GB/s\n", name, ms / iters, gb * iters / (ms * 1e-3));
  };
  for (int round = 0; round < 2; ++round) {
    float ms;
    // H2D contiguous
    CHECK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i) CHECK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1));
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("H2D contiguous", ms, bytes / 1e9);
    // H2D pitched
    CHECK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i)
      CHECK(hipMemcpy2DAsync((char*)d_a + 16, P, h_in, W, W, H, hipMemcpyHostToDevice, s1));
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("H2D pitched (2D)", ms, bytes / 1e9);
    // D2H contiguous
    CHECK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i) CHECK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1));
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("D2H contiguous", ms, bytes / 1e9);
    // D2H pitched
    CHECK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i)
      CHECK(hipMemcpy2DAsync(h_out, W, (char*)d_b + 16, P, W, H, hipMemcpyDeviceToHost, s1));
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("D2H pitched (2D)", ms, bytes / 1e9);
    // both directions concurrently (pitched), two streams; wall by host events
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    for (int i = 0; i < iters; ++i) {
      CHECK(hipMemcpy2DAsync((char*)d_a + 16, P, h_in, W, W, H, hipMemcpyHostToDevice, s1));
      CHECK(hipMemcpy2DAsync(h_out, W, (char*)d_b + 16, P, W, H, hipMemcpyDeviceToHost, s2));
    }
    hipEvent_t ea, eb;
    CHECK(hipEventCreate(&ea));
    CHECK(hipEventCreate(&eb));
    CHECK(hipEventRecord(ea, s1));
    CHECK(hipEventRecord(eb, s2));
    CHECK(hipStreamWaitEvent(0, ea, 0));
    CHECK(hipStreamWaitEvent(0, eb, 0));
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("H2D+D2H concurrent (per pair)", ms, 2 * bytes / 1e9);
    // concurrent contiguous
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    for (int i = 0; i < iters; ++i) {
      CHECK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1));
      CHECK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s2));
    }
    CHECK(hipEventRecord(ea, s1));
    CHECK(hipEventRecord(eb, s2));
    CHECK(hipStreamWaitEvent(0, ea, 0));
    CHECK(hipStreamWaitEvent(0, eb, 0));
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("H2D+D2H concurrent contiguous", ms, 2 * bytes / 1e9);
    // zero-copy kernels (pitched device frame, contiguous host rows)
    const int w16 = static_cast<int>(W / 16);
    const dim3 blk(256), grd((w16 + 255) / 256, H);
    CHECK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i)
      k_copy_rows<<<grd, blk, 0, s1>>>((const uint8_t*)h_in, W, (uint8_t*)d_a + 16 + 0, P, w16, H);
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("H2D zero-copy kernel", ms, bytes / 1e9);
    CHECK(hipEventRecord(e0, s1));
    for (int i = 0; i < iters; ++i)
      k_copy_rows<<<grd, blk, 0, s1>>>((const uint8_t*)d_b + 16, P, (uint8_t*)h_out, W, w16, H);
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("D2H zero-copy kernel", ms, bytes / 1e9);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    for (int i = 0; i < iters; ++i) {
      k_copy_rows<<<grd, blk, 0, s1>>>((const uint8_t*)h_in, W, (uint8_t*)d_a + 16, P, w16, H);
      k_copy_rows<<<grd, blk, 0, s2>>>((const uint8_t*)d_b + 16, P, (uint8_t*)h_out, W, w16, H);
    }
    CHECK(hipEventRecord(ea, s1));
    CHECK(hipEventRecord(eb, s2));
    CHECK(hipStreamWaitEvent(0, ea, 0));
    CHECK(hipStreamWaitEvent(0, eb, 0));
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("H2D+D2H zero-copy concurrent", ms, 2 * bytes / 1e9);
    // mixed: SDMA H2D + zero-copy D2H kernel
    CHECK(hipEventRecord(e0, 0));
    CHECK(hipStreamWaitEvent(s1, e0, 0));
    CHECK(hipStreamWaitEvent(s2, e0, 0));
    for (int i = 0; i < iters; ++i) {
      CHECK(hipMemcpy2DAsync((char*)d_a + 16, P, h_in, W, W, H, hipMemcpyHostToDevice, s1));
      k_copy_rows<<<grd, blk, 0, s2>>>((const uint8_t*)d_b + 16, P, (uint8_t*)h_out, W, w16, H);
    }
    CHECK(hipEventRecord(ea, s1));
    CHECK(hipEventRecord(eb, s2));
    CHECK(hipStreamWaitEvent(0, ea, 0));
    CHECK(hipStreamWaitEvent(0, eb, 0));
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    report("SDMA H2D + zero-copy D2H", ms, 2 * bytes / 1e9);
    // the same copies as hipGraph memcpy nodes (the serving step graphs
    // capture their H2D / D2H this way): 1-D vs 2-D (pitched) D2H node
    for (int two_d = 0; two_d <= 1; ++two_d) {
      hipGraph_t g;
      hipGraphExec_t ge;
      CHECK(hipStreamBeginCapture(s1, hipStreamCaptureModeRelaxed));
      if (two_d)
        CHECK(hipMemcpy2DAsync(h_out, W, (char*)d_b + 16, P, W, H, hipMemcpyDeviceToHost, s1));
      else
        CHECK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1));
      CHECK(hipStreamEndCapture(s1, &g));
      CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      CHECK(hipGraphLaunch(ge, s1));
      CHECK(hipStreamSynchronize(s1));
      CHECK(hipEventRecord(e0, s1));
      for (int i = 0; i < iters; ++i) CHECK(hipGraphLaunch(ge, s1));
      CHECK(hipEventRecord(e1, s1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      report(two_d ? "D2H graph node, pitched (2D)" : "D2H graph node, contiguous", ms, bytes / 1e9);
      CHECK(hipGraphExecDestroy(ge));
      CHECK(hipGraphDestroy(g));
    }
    // each direction split in halves on two streams (4 SDMA queues busy)
    {
      static hipStream_t s3 = nullptr, s4 = nullptr;
      if (!s3) {
        CHECK(hipStreamCreateWithFlags(&s3, hipStreamNonBlocking));
        CHECK(hipStreamCreateWithFlags(&s4, hipStreamNonBlocking));
      }
      const size_t H2 = H / 2;
      hipEvent_t ec, ed;
      CHECK(hipEventCreate(&ec));
      CHECK(hipEventCreate(&ed));
      CHECK(hipEventRecord(e0, 0));
      for (hipStream_t q : {s1, s2, s3, s4}) CHECK(hipStreamWaitEvent(q, e0, 0));
      for (int i = 0; i < iters; ++i) {
        CHECK(hipMemcpy2DAsync((char*)d_a + 16, P, h_in, W, W, H2, hipMemcpyHostToDevice, s1));
        CHECK(hipMemcpy2DAsync((char*)d_a + 16 + H2 * P, P, (char*)h_in + H2 * W, W, W, H - H2, hipMemcpyHostToDevice, s3));
        CHECK(hipMemcpy2DAsync(h_out, W, (char*)d_b + 16, P, W, H2, hipMemcpyDeviceToHost, s2));
        CHECK(hipMemcpy2DAsync((char*)h_out + H2 * W, W, (char*)d_b + 16 + H2 * P, P, W, H - H2, hipMemcpyDeviceToHost, s4));
      }
      CHECK(hipEventRecord(ea, s1));
      CHECK(hipEventRecord(eb, s2));
      CHECK(hipEventRecord(ec, s3));
      CHECK(hipEventRecord(ed, s4));
      for (hipEvent_t x : {ea, eb, ec, ed}) CHECK(hipStreamWaitEvent(0, x, 0));
      CHECK(hipEventRecord(e1, 0));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      report("H2D+D2H halves on 4 streams", ms, 2 * bytes / 1e9);
    }
  }
  return 0;
}
