// What a persistent (single-launch) temporal kernel could save per launch,
// for the headline frame (1920x2520 RGB, 5760-byte rows, 14.5 MB): the cost
// of a launch with the production tile kernel's grid shape (742 workgroups
// x 512 threads, 32 KB LDS) when it does
//   (a) nothing               -> dispatch + wave launch + drain,
//   (b) only its memory phase -> load the tile rows (8 rows x 2 strips x 4 B
//       per lane, the k_swar<3,4,8,8> pattern), store the kept rows,
// back to back on one stream, as in the 5-launch hipGraph of 40 repetitions.
// A persistent kernel keeps (b) once per 8-step phase (tiles must re-read
// what their neighbours wrote) and adds a grid-wide barrier; it removes at
// most (a) per launch.
//
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/launch_cost.hip -o tools/ubench/launch_cost
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e_ = (x);                                                 \
    if (e_ != hipSuccess) {                                              \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      return 1;                                                          \
    }                                                                    \
  } while (0)

constexpr int kRowBytes = 5760, kRows = 2520, kPitch = 5888, kWaves = 8, kM = 8;
constexpr int kHalo = 6;                                // lanes per side (8 steps x 3 B / 4 B)
constexpr int kVbytes = (64 - 2 * kHalo) * 4;           // 208 valid bytes per strip
constexpr int kStrips = (kRowBytes + kVbytes - 1) / kVbytes;  // 28
constexpr int kPairs = (kStrips + 1) / 2;               // 14
constexpr int kVrows = kWaves * kM - 16;                // 48 kept rows per tile
constexpr int kRowTiles = (kRows + kVrows - 1) / kVrows;  // 53

__global__ __launch_bounds__(512) void k_empty(int* sink) {
  __shared__ int lds[8192];  // 32 KB, the tile kernel's footprint
  if (threadIdx.x == 0 && blockIdx.x == 0x7fffffff) sink[0] = lds[0];
}

__global__ __launch_bounds__(512) void k_tile_io(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
  __shared__ int lds[8192];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tile = blockIdx.x, col = tile / kRowTiles, rt = tile - col * kRowTiles;
  const int xA = col * kVbytes - kHalo * 4 + lane * 4, xB = (col + kPairs) * kVbytes - kHalo * 4 + lane * 4;
  const int r0 = rt * kVrows - 8 + w * kM;
  uint32_t a[kM], b[kM];
#pragma unroll
  for (int i = 0; i < kM; ++i) {
    const int r = r0 + i;
    const bool ok = r >= 0 && r < kRows;
    a[i] = ok && xA >= 0 && xA + 4 <= kRowBytes ? *reinterpret_cast<const uint32_t*>(src + r * kPitch + xA) : 0u;
    b[i] = ok && xB >= 0 && xB + 4 <= kRowBytes ? *reinterpret_cast<const uint32_t*>(src + r * kPitch + xB) : 0u;
  }
  if (threadIdx.x == 0) lds[w] = static_cast<int>(a[0]);
  __syncthreads();
  const bool in = lane >= kHalo && lane < 64 - kHalo;
#pragma unroll
  for (int i = 0; i < kM; ++i) {
    const int r = r0 + i;
    if (!in || r < rt * kVrows || r >= (rt + 1) * kVrows || r >= kRows) continue;
    if (xA >= 0 && xA + 4 <= kRowBytes) *reinterpret_cast<uint32_t*>(dst + r * kPitch + xA) = a[i] + lds[0] * 0;
    if (xB >= 0 && xB + 4 <= kRowBytes) *reinterpret_cast<uint32_t*>(dst + r * kPitch + xB) = b[i];
  }
}

// Same bytes as k_tile_io, 16 B per lane: a wave instruction covers two
// tile rows x both strips (4 x 256 B) instead of one row of one strip.
__global__ __launch_bounds__(512) void k_tile_io16(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
  __shared__ int lds[8192];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tile = blockIdx.x, col = tile / kRowTiles, rt = tile - col * kRowTiles;
  const int q = lane >> 4, l16 = lane & 15;  // quarter: (row parity, strip), 16 lanes x 16 B = 256 B
  const int strip = q & 1 ? col + kPairs : col;
  const int x = strip * kVbytes - kHalo * 4 + l16 * 16;
  const int r0 = rt * kVrows - 8 + w * kM;
  uint4 v[kM / 2];
#pragma unroll
  for (int i = 0; i < kM / 2; ++i) {
    const int r = r0 + 2 * i + (q >> 1);
    const bool ok = r >= 0 && r < kRows && x >= 0 && x + 16 <= kRowBytes;
    v[i] = ok ? *reinterpret_cast<const uint4*>(src + r * kPitch + x) : make_uint4(0, 0, 0, 0);
  }
  if (threadIdx.x == 0) lds[w] = static_cast<int>(v[0].x);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kM / 2; ++i) {
    const int r = r0 + 2 * i + (q >> 1);
    if (r < rt * kVrows || r >= (rt + 1) * kVrows || r >= kRows || x < 0 || x + 16 > kRowBytes) continue;
    uint4 o = v[i];
    o.x += lds[0] * 0;
    *reinterpret_cast<uint4*>(dst + r * kPitch + x) = o;
  }
}

int main() {
  const size_t bytes = static_cast<size_t>(kPitch) * (kRows + 16);
  uint8_t *s = nullptr, *d = nullptr;
  int* sink = nullptr;
  CK(hipMalloc(&s, bytes));
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(s, 1, bytes));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid(kPairs * kRowTiles), block(64 * kWaves);
  const int iters = 200;
  float ms = 0;
  for (int round = 0; round < 3; ++round) {
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) k_empty<<<grid, block, 0, st>>>(sink);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const float empty_us = ms * 1e3f / iters;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) k_tile_io<<<grid, block, 0, st>>>(i & 1 ? d + 8 * kPitch : s + 8 * kPitch,
                                                                    i & 1 ? s + 8 * kPitch : d + 8 * kPitch);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const float io_us = ms * 1e3f / iters;
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) k_tile_io16<<<grid, block, 0, st>>>(i & 1 ? d + 8 * kPitch : s + 8 * kPitch,
                                                                      i & 1 ? s + 8 * kPitch : d + 8 * kPitch);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const float io16_us = ms * 1e3f / iters;
    std::printf("{\"round\": %d, \"grid\": %u, \"block\": %u, \"empty_launch_us\": %.2f, \"tile_io_launch_us\": %.2f, "
                "\"tile_io16_launch_us\": %.2f}\n", round, grid.x, block.x, empty_us, io_us, io16_us);
  }
  return 0;
}
