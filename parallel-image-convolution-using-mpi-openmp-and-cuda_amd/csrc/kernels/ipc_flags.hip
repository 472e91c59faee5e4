// Flag kernels of the HIP-IPC halo protocol (include/pconv/ipc_halo.hpp).
//
// One thread each.  The flag words live in host shared memory that every
// rank's GPU maps; they are read and written with system-scope atomics
// through ordinary vector memory instructions (global loads / stores with
// the system-coherence bits), so a rank's GPU sees a neighbour's store
// without any cache maintenance.  Every wait is bounded by a wall-clock
// timeout (wall_clock64, constant rate): on expiry the rank's error word is
// set and the kernel returns, so no wave ever spins without end.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pconv/device.hpp"
#include "pconv/ipc_halo.hpp"

namespace pconv {
namespace {

__device__ __forceinline__ uint32_t load_sys(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void store_sys(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Wait until *p >= target (wrap-safe); false on timeout.
__device__ bool wait_ge(const uint32_t* p, uint32_t target, uint64_t t0, uint64_t timeout) {
  while (static_cast<int32_t>(load_sys(p) - target) < 0) {
    if (static_cast<uint64_t>(wall_clock64()) - t0 > timeout) return false;
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

__global__ __launch_bounds__(64) void k_ipc_signal_wait(IpcFlags* f, int me, int up, int down, uint64_t timeout) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  // Everything earlier on this stream (the launches that produced this
  // rank's boundary rows) is complete when the kernel starts: publish them.
  const uint32_t n = load_sys(&f[me].count) + 1;
  store_sys(&f[me].count, n);
  store_sys(&f[me].level, n);
  bool ok = true;
  if (up >= 0) ok = wait_ge(&f[up].level, n, t0, timeout);
  if (ok && down >= 0) ok = wait_ge(&f[down].level, n, t0, timeout);
  if (!ok) store_sys(&f[me].err, 1u);
}

__global__ __launch_bounds__(64) void k_ipc_ack_wait(IpcFlags* f, int me, int up, int down, uint64_t timeout) {
  if (threadIdx.x != 0) return;
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  const uint32_t n = load_sys(&f[me].count);
  store_sys(&f[me].ack, n);  // this rank's copies of exchange #n are complete
  bool ok = true;
  if (up >= 0) ok = wait_ge(&f[up].ack, n, t0, timeout);
  if (ok && down >= 0) ok = wait_ge(&f[down].ack, n, t0, timeout);
  if (!ok) store_sys(&f[me].err, 2u);
}

// The pull itself: `bytes` (a multiple of 16) from each neighbour's frame into
// this rank's ghost rows, 16 bytes per lane, grid-stride.  Skipped when this
// rank's wait timed out: the neighbour may be gone, its frames unmapped.
__global__ __launch_bounds__(256) void k_ipc_pull(const IpcFlags* f, int me, uint4* __restrict__ dst_up,
                                                  const uint4* __restrict__ src_up, uint4* __restrict__ dst_down,
                                                  const uint4* __restrict__ src_down, int64_t n16) {
  if (__hip_atomic_load(&f[me].err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += stride) {
    if (src_up) dst_up[i] = src_up[i];
    if (src_down) dst_down[i] = src_down[i];
  }
}

// The whole exchange as ONE dispatch (one workgroup): thread 0 publishes and
// waits for the neighbours' rows, the workgroup pulls them, thread 0
// publishes "copied" and waits for the neighbours' copies.  The rows a
// neighbour pulls were produced by an EARLIER kernel of its stream (the
// command processor's end-of-kernel release wrote them back on every XCD);
// this kernel's system-scope acquire (thread 0, before the barrier)
// invalidates this CU's caches before any thread loads them.  Three
// dispatches (signal / pull / ack) cost ~14 us more per exchange on the
// 8-way proxy (profiles/r04/slots_b/).
__global__ __launch_bounds__(1024) void k_ipc_exchange(IpcFlags* f, int me, int up, int down, uint64_t timeout,
                                                       uint4* __restrict__ dst_up, const uint4* __restrict__ src_up,
                                                       uint4* __restrict__ dst_down,
                                                       const uint4* __restrict__ src_down, int64_t n16) {
  __shared__ int ok_s;
  if (threadIdx.x == 0) {
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    const uint32_t n = load_sys(&f[me].count) + 1;
    store_sys(&f[me].count, n);
    store_sys(&f[me].level, n);
    bool ok = true;
    if (up >= 0) ok = wait_ge(&f[up].level, n, t0, timeout);
    if (ok && down >= 0) ok = wait_ge(&f[down].level, n, t0, timeout);
    if (!ok) store_sys(&f[me].err, 1u);
    ok_s = ok;
    // the acquire's cache invalidate completes asynchronously: wait for it
    // before the barrier releases the other waves' loads of the neighbours'
    // rows (CDNA4 guide, Guideline 16)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (!ok_s) return;  // a neighbour may be gone: do not touch its frames
  for (int64_t i = threadIdx.x; i < n16; i += blockDim.x) {
    if (src_up) dst_up[i] = src_up[i];
    if (src_down) dst_down[i] = src_down[i];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    const uint32_t n = load_sys(&f[me].count);
    store_sys(&f[me].ack, n);
    bool ok = true;
    if (up >= 0) ok = wait_ge(&f[up].ack, n, t0, timeout);
    if (ok && down >= 0) ok = wait_ge(&f[down].ack, n, t0, timeout);
    if (!ok) store_sys(&f[me].err, 2u);
  }
}

}  // namespace

void launch_ipc_exchange(IpcFlags* flags, int me, int up, int down, uint64_t timeout_ticks, uint8_t* dst_up,
                         const uint8_t* src_up, uint8_t* dst_down, const uint8_t* src_down, int64_t bytes,
                         hipStream_t s) {
  PCONV_CHECK(bytes % 16 == 0, "ipc exchange: rows must span whole 16-byte granules");
  for (const void* p : {static_cast<const void*>(dst_up), static_cast<const void*>(src_up),
                        static_cast<const void*>(dst_down), static_cast<const void*>(src_down)})
    PCONV_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "ipc exchange: unaligned row pointer");
  k_ipc_exchange<<<dim3(1), dim3(1024), 0, s>>>(flags, me, up, down, timeout_ticks, reinterpret_cast<uint4*>(dst_up),
                                                reinterpret_cast<const uint4*>(src_up),
                                                reinterpret_cast<uint4*>(dst_down),
                                                reinterpret_cast<const uint4*>(src_down), bytes / 16);
  PCONV_HIP_CHECK(hipGetLastError());
}

void launch_ipc_pull(const IpcFlags* flags, int me, uint8_t* dst_up, const uint8_t* src_up, uint8_t* dst_down,
                     const uint8_t* src_down, int64_t bytes, hipStream_t s) {
  PCONV_CHECK(bytes % 16 == 0, "ipc pull: rows must span whole 16-byte granules");
  for (const void* p : {static_cast<const void*>(dst_up), static_cast<const void*>(src_up),
                        static_cast<const void*>(dst_down), static_cast<const void*>(src_down)})
    PCONV_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "ipc pull: unaligned row pointer");
  const int64_t n16 = bytes / 16;
  const unsigned blocks = static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>((n16 + 255) / 256, 512)));
  k_ipc_pull<<<dim3(blocks), dim3(256), 0, s>>>(flags, me, reinterpret_cast<uint4*>(dst_up),
                                                reinterpret_cast<const uint4*>(src_up),
                                                reinterpret_cast<uint4*>(dst_down),
                                                reinterpret_cast<const uint4*>(src_down), n16);
  PCONV_HIP_CHECK(hipGetLastError());
}

void launch_ipc_signal_wait(IpcFlags* flags, int me, int up, int down, uint64_t timeout_ticks, hipStream_t s) {
  k_ipc_signal_wait<<<dim3(1), dim3(64), 0, s>>>(flags, me, up, down, timeout_ticks);
  PCONV_HIP_CHECK(hipGetLastError());
}

void launch_ipc_ack_wait(IpcFlags* flags, int me, int up, int down, uint64_t timeout_ticks, hipStream_t s) {
  k_ipc_ack_wait<<<dim3(1), dim3(64), 0, s>>>(flags, me, up, down, timeout_ticks);
  PCONV_HIP_CHECK(hipGetLastError());
}

}  // namespace pconv
