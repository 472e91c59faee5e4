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

// Copy of `n16` 16-byte granules per side by `nthreads` threads starting
// at thread `t0`: four loads in flight per side before their stores (a
// remote source costs a round trip per load; restrict lets the loads run
// ahead of the stores).
__device__ __forceinline__ void pull_rows(uint4* __restrict__ dst_up, const uint4* __restrict__ src_up,
                                          uint4* __restrict__ dst_down, const uint4* __restrict__ src_down,
                                          int64_t n16, int64_t t0, int64_t nthreads) {
  constexpr int U = 4;
  int64_t i = t0;
  for (; i + (U - 1) * nthreads < n16; i += U * nthreads) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (src_up) a[u] = src_up[i + u * nthreads];
      if (src_down) b[u] = src_down[i + u * nthreads];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (src_up) dst_up[i + u * nthreads] = a[u];
      if (src_down) dst_down[i + u * nthreads] = b[u];
    }
  }
  for (; i < n16; i += nthreads) {
    if (src_up) dst_up[i] = src_up[i];
    if (src_down) dst_down[i] = src_down[i];
  }
}

// Grid form: G workgroups, ONE dispatch.  `count` changes only at the very
// end of an exchange (by its last workgroup), so every workgroup of this
// dispatch reads the same exchange number n = count + 1 at its start (the
// previous exchange's dispatch completed before this one started: stream
// order).  Workgroup 0 publishes level = n (this rank's rows came from
// earlier kernels, released at their end).  Every workgroup's thread 0 waits
// for the neighbours' level >= n with its OWN system-scope acquire, which
// invalidates the caches of its CU and XCD before the workgroup loads the
// neighbours' rows (one acquire per workgroup: a workgroup on another XCD
// is not covered by anyone else's).  After its slice the workgroup arrives
// on a device-memory counter; the last one resets it, publishes count = n
// and ack = n (system-scope release) and waits for the neighbours' acks, so
// the dispatch ends only once they have copied this rank's rows.
__global__ __launch_bounds__(256) void k_ipc_exchange_grid(IpcFlags* f, uint32_t* arrive, int me, int up, int down,
                                                           uint64_t timeout, uint4* __restrict__ dst_up,
                                                           const uint4* __restrict__ src_up,
                                                           uint4* __restrict__ dst_down,
                                                           const uint4* __restrict__ src_down, int64_t n16) {
  __shared__ int ok_s;
  if (threadIdx.x == 0) {
    const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
    const uint32_t n = load_sys(&f[me].count) + 1;
    if (blockIdx.x == 0) store_sys(&f[me].level, n);
    bool ok = true;
    if (up >= 0) ok = wait_ge(&f[up].level, n, t0, timeout);
    if (ok && down >= 0) ok = wait_ge(&f[down].level, n, t0, timeout);
    if (!ok) store_sys(&f[me].err, 1u);
    ok_s = ok;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the acquire's invalidate, before the barrier
  }
  __syncthreads();
  if (ok_s)
    pull_rows(dst_up, src_up, dst_down, src_down, n16,
              static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
              static_cast<int64_t>(gridDim.x) * blockDim.x);
  __syncthreads();  // every load of this workgroup has returned
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 == gridDim.x) {
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
      const uint32_t n = load_sys(&f[me].count) + 1;
      store_sys(&f[me].count, n);
      // a timed-out level wait: no ack (the neighbours' ack waits time out too)
      if (__hip_atomic_load(&f[me].err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0) {
        store_sys(&f[me].ack, n);
        bool ok = true;
        if (up >= 0) ok = wait_ge(&f[up].ack, n, t0, timeout);
        if (ok && down >= 0) ok = wait_ge(&f[down].ack, n, t0, timeout);
        if (!ok) store_sys(&f[me].err, 2u);
      }
    }
  }
}

// Single form: the whole exchange as ONE dispatch (one workgroup): thread 0 publishes and
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

int ipc_grid_workgroups(int64_t bytes) {
  // ~8 KB per workgroup and side (two passes of 256 lanes x 16 B), 8..64
  return static_cast<int>(std::min<int64_t>(64, std::max<int64_t>(8, (bytes / 16 + 511) / 512)));
}

void launch_ipc_exchange(IpcPull form, IpcFlags* f, uint32_t* arrive, int me, int up, int down, uint64_t timeout,
                         uint8_t* dst_up, const uint8_t* src_up, uint8_t* dst_down, const uint8_t* src_down,
                         int64_t bytes, hipStream_t s, int workgroups) {
  PCONV_CHECK(bytes % 16 == 0, "ipc exchange: rows must span whole 16-byte granules");
  for (const void* p : {static_cast<const void*>(dst_up), static_cast<const void*>(src_up),
                        static_cast<const void*>(dst_down), static_cast<const void*>(src_down)})
    PCONV_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "ipc exchange: unaligned row pointer");
  PCONV_CHECK((!src_up || dst_up) && (!src_down || dst_down), "ipc exchange: source without destination");
  auto* du = reinterpret_cast<uint4*>(dst_up);
  auto* dd = reinterpret_cast<uint4*>(dst_down);
  const auto* su = reinterpret_cast<const uint4*>(src_up);
  const auto* sd = reinterpret_cast<const uint4*>(src_down);
  switch (form) {
    case IpcPull::Grid: {
      PCONV_CHECK(arrive != nullptr, "ipc exchange: the grid form needs its arrival counter");
      const int g = workgroups > 0 ? std::min(workgroups, 256) : ipc_grid_workgroups(bytes);
      k_ipc_exchange_grid<<<dim3(g), dim3(256), 0, s>>>(f, arrive, me, up, down, timeout, du, su, dd, sd, bytes / 16);
      break;
    }
    case IpcPull::Single:
      k_ipc_exchange<<<dim3(1), dim3(1024), 0, s>>>(f, me, up, down, timeout, du, su, dd, sd, bytes / 16);
      break;
    case IpcPull::Sdma:
      k_ipc_signal_wait<<<dim3(1), dim3(64), 0, s>>>(f, me, up, down, timeout);
      PCONV_HIP_CHECK(hipGetLastError());
      if (src_up) PCONV_HIP_CHECK(hipMemcpyAsync(dst_up, src_up, static_cast<size_t>(bytes), hipMemcpyDefault, s));
      if (src_down)
        PCONV_HIP_CHECK(hipMemcpyAsync(dst_down, src_down, static_cast<size_t>(bytes), hipMemcpyDefault, s));
      k_ipc_ack_wait<<<dim3(1), dim3(64), 0, s>>>(f, me, up, down, timeout);
      break;
  }
  PCONV_HIP_CHECK(hipGetLastError());
}

}  // namespace pconv
