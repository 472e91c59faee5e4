// Kernels of the HIP-IPC halo protocol (include/pconv/ipc_halo.hpp).
//
// Signalling words live in device-memory mailboxes: a rank stores into its
// neighbours' mailboxes (release, system scope: the store may cross xGMI)
// and polls only its own (acquire, system scope, local HBM).  Every wait is
// bounded by a wall-clock timeout (wall_clock64, constant rate): on expiry
// the rank's host-visible error word is set and the kernel returns, so no
// wave ever spins without end.
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
    __builtin_amdgcn_s_sleep(1);
  }
  return true;
}

// Step 1 (thread 0): publish "my rows of exchange n are final" into the
// neighbours' mailboxes (publish = false: another workgroup of this
// dispatch does it) and wait for theirs; false on timeout.
__device__ bool signal_wait(IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb, uint32_t n, bool publish,
                            uint64_t timeout) {
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  if (publish) {
    if (up_mb) store_sys(&up_mb->level_down, n);  // I am my upper neighbour's lower neighbour
    if (down_mb) store_sys(&down_mb->level_up, n);
  }
  bool ok = true;
  if (up_mb) ok = wait_ge(&mine->level_up, n, t0, timeout);
  if (ok && down_mb) ok = wait_ge(&mine->level_down, n, t0, timeout);
  return ok;
}

// Step 3 (thread 0): count = n, publish "copied" into the neighbours'
// mailboxes, wait for theirs.  Skipped after a timed-out level wait (the
// neighbours' ack waits time out too).
__device__ void ack_wait(IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb, uint32_t* err, uint32_t n,
                         uint64_t timeout) {
  store_sys(&mine->count, n);
  if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
  if (up_mb) store_sys(&up_mb->ack_down, n);
  if (down_mb) store_sys(&down_mb->ack_up, n);
  bool ok = true;
  if (up_mb) ok = wait_ge(&mine->ack_up, n, t0, timeout);
  if (ok && down_mb) ok = wait_ge(&mine->ack_down, n, t0, timeout);
  if (!ok) store_sys(err, 2u);
}

// Copy of `n16` 16-byte granules per side by `nthreads` threads starting
// at thread `t0`: four loads per side in flight before their stores.  A
// remote source costs a round trip per dependent load, and with the grid
// form's sizing a thread has ~2 granules per side, so the slice must be ONE
// round trip: the sides are template parameters and neither loads nor
// stores are predicated (past the end an index wraps to an earlier granule,
// which is copied again with the same bytes) — with per-side or
// per-granule branches the compiler sank every load into its store's block
// behind its own s_waitcnt vmcnt(0), one round trip per granule.
__device__ __forceinline__ int64_t wrap(int64_t j, int64_t n) { return j < n ? j : min(j - n, n - 1); }

template <bool UP, bool DOWN>
__device__ __forceinline__ void pull_sides(uint4* __restrict__ dst_up, const uint4* __restrict__ src_up,
                                           uint4* __restrict__ dst_down, const uint4* __restrict__ src_down,
                                           int64_t n16, int64_t t0, int64_t nthreads) {
  constexpr int U = 4;
  for (int64_t i = t0; i < n16; i += U * nthreads) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = wrap(i + u * nthreads, n16);
      if constexpr (UP) a[u] = src_up[j];
      if constexpr (DOWN) b[u] = src_down[j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t j = wrap(i + u * nthreads, n16);
      if constexpr (UP) dst_up[j] = a[u];
      if constexpr (DOWN) dst_down[j] = b[u];
    }
  }
}

__device__ __forceinline__ void pull_rows(uint4* __restrict__ dst_up, const uint4* __restrict__ src_up,
                                          uint4* __restrict__ dst_down, const uint4* __restrict__ src_down,
                                          int64_t n16, int64_t t0, int64_t nthreads) {
  if (src_up && src_down)
    pull_sides<true, true>(dst_up, src_up, dst_down, src_down, n16, t0, nthreads);
  else if (src_up)
    pull_sides<true, false>(dst_up, src_up, dst_down, src_down, n16, t0, nthreads);
  else if (src_down)
    pull_sides<false, true>(dst_up, src_up, dst_down, src_down, n16, t0, nthreads);
}

// Grid form: G workgroups, ONE dispatch.  `count` changes only at the very
// end of an exchange (by its last workgroup), so every workgroup reads the
// same exchange number n = count + 1 (the previous exchange's dispatch
// completed before this one started: stream order).  Workgroup 0 publishes;
// every workgroup's thread 0 waits with its OWN system-scope acquire, which
// invalidates the caches of its CU and XCD before the workgroup loads the
// neighbours' rows (a workgroup on another XCD is covered by no one else's
// acquire); after its slice the workgroup arrives on the mailbox's counter
// and the last one resets it and performs the ack.
__global__ __launch_bounds__(256) void k_ipc_exchange_grid(IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb,
                                                           uint32_t* err, uint64_t timeout,
                                                           uint4* __restrict__ dst_up, const uint4* __restrict__ src_up,
                                                           uint4* __restrict__ dst_down,
                                                           const uint4* __restrict__ src_down, int64_t n16) {
  __shared__ int ok_s;
  __shared__ uint32_t n_s;
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_load(&mine->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const bool ok = signal_wait(mine, up_mb, down_mb, n, blockIdx.x == 0, timeout);
    if (!ok) store_sys(err, 1u);
    ok_s = ok;
    n_s = n;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the acquire's invalidate, before the barrier
  }
  __syncthreads();
  if (ok_s)
    pull_rows(dst_up, src_up, dst_down, src_down, n16, static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
              static_cast<int64_t>(gridDim.x) * blockDim.x);
  __syncthreads();  // every load of this workgroup has returned
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(&mine->arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 == gridDim.x) {
      __hip_atomic_store(&mine->arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ack_wait(mine, up_mb, down_mb, err, n_s, timeout);
    }
  }
}

// Single form: the whole exchange in ONE workgroup.
__global__ __launch_bounds__(1024) void k_ipc_exchange(IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb,
                                                       uint32_t* err, uint64_t timeout, uint4* __restrict__ dst_up,
                                                       const uint4* __restrict__ src_up, uint4* __restrict__ dst_down,
                                                       const uint4* __restrict__ src_down, int64_t n16) {
  __shared__ int ok_s;
  __shared__ uint32_t n_s;
  if (threadIdx.x == 0) {
    const uint32_t n = __hip_atomic_load(&mine->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
    const bool ok = signal_wait(mine, up_mb, down_mb, n, true, timeout);
    if (!ok) store_sys(err, 1u);
    ok_s = ok;
    n_s = n;
    // the acquire's cache invalidate completes asynchronously: wait for it
    // before the barrier releases the other waves' loads of the neighbours'
    // rows (CDNA4 guide, Guideline 16)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (ok_s) pull_rows(dst_up, src_up, dst_down, src_down, n16, threadIdx.x, blockDim.x);
  __syncthreads();
  if (threadIdx.x == 0) ack_wait(mine, up_mb, down_mb, err, n_s, timeout);
}

// Sdma form: one thread before and one after the SDMA copies.
__global__ __launch_bounds__(64) void k_ipc_signal_wait(IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb,
                                                        uint32_t* err, uint64_t timeout) {
  if (threadIdx.x != 0) return;
  const uint32_t n = __hip_atomic_load(&mine->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  if (!signal_wait(mine, up_mb, down_mb, n, true, timeout)) store_sys(err, 1u);
}

__global__ __launch_bounds__(64) void k_ipc_ack_wait(IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb,
                                                     uint32_t* err, uint64_t timeout) {
  if (threadIdx.x != 0) return;
  const uint32_t n = __hip_atomic_load(&mine->count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  ack_wait(mine, up_mb, down_mb, err, n, timeout);
}

}  // namespace

int ipc_grid_workgroups(int64_t bytes) {
  // 16 KB per workgroup and side: every lane's four granules per side in
  // flight at once (pull_sides), 8..64 workgroups
  return static_cast<int>(std::min<int64_t>(64, std::max<int64_t>(8, (bytes / 16 + 1023) / 1024)));
}

void launch_ipc_exchange(IpcPull form, IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb, uint32_t* err,
                         uint64_t timeout, uint8_t* dst_up, const uint8_t* src_up, uint8_t* dst_down,
                         const uint8_t* src_down, int64_t bytes, hipStream_t s, int workgroups) {
  PCONV_CHECK(mine != nullptr && err != nullptr, "ipc exchange: no mailbox / error word");
  PCONV_CHECK(bytes % 16 == 0, "ipc exchange: rows must span whole 16-byte granules");
  for (const void* p : {static_cast<const void*>(dst_up), static_cast<const void*>(src_up),
                        static_cast<const void*>(dst_down), static_cast<const void*>(src_down)})
    PCONV_CHECK(reinterpret_cast<uintptr_t>(p) % 16 == 0, "ipc exchange: unaligned row pointer");
  // rows need their neighbour's mailbox; a mailbox without rows only as this
  // rank's own (a self-neighbour signalling both sides)
  PCONV_CHECK((!src_up || up_mb) && (!src_down || down_mb) && (src_up || !up_mb || up_mb == mine) &&
                  (src_down || !down_mb || down_mb == mine),
              "ipc exchange: rows without a mailbox (or the reverse)");
  PCONV_CHECK((!src_up || dst_up) && (!src_down || dst_down), "ipc exchange: source without destination");
  auto* du = reinterpret_cast<uint4*>(dst_up);
  auto* dd = reinterpret_cast<uint4*>(dst_down);
  const auto* su = reinterpret_cast<const uint4*>(src_up);
  const auto* sd = reinterpret_cast<const uint4*>(src_down);
  switch (form) {
    case IpcPull::Grid: {
      const int g = workgroups > 0 ? std::min(workgroups, 256) : ipc_grid_workgroups(bytes);
      k_ipc_exchange_grid<<<dim3(g), dim3(256), 0, s>>>(mine, up_mb, down_mb, err, timeout, du, su, dd, sd,
                                                         bytes / 16);
      break;
    }
    case IpcPull::Single:
      k_ipc_exchange<<<dim3(1), dim3(1024), 0, s>>>(mine, up_mb, down_mb, err, timeout, du, su, dd, sd, bytes / 16);
      break;
    case IpcPull::Sdma:
      k_ipc_signal_wait<<<dim3(1), dim3(64), 0, s>>>(mine, up_mb, down_mb, err, timeout);
      PCONV_HIP_CHECK(hipGetLastError());
      if (src_up) PCONV_HIP_CHECK(hipMemcpyAsync(dst_up, src_up, static_cast<size_t>(bytes), hipMemcpyDefault, s));
      if (src_down)
        PCONV_HIP_CHECK(hipMemcpyAsync(dst_down, src_down, static_cast<size_t>(bytes), hipMemcpyDefault, s));
      k_ipc_ack_wait<<<dim3(1), dim3(64), 0, s>>>(mine, up_mb, down_mb, err, timeout);
      break;
  }
  PCONV_HIP_CHECK(hipGetLastError());
}

}  // namespace pconv
