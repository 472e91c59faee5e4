// One image as ONE persistent launch: H2D by the CUs, every level of the
// temporal-blocked gaussian, D2H by the CUs (schedule.hpp: plan_wave).
//
// What it replaces: the reference's GPU_convolution() is a serial chain of
// cudaMemcpy -> `reps` launches -> cudaMemcpy (cuda/cuda_convolution.cu:
// 60-97); the row-streamed image (engine.cpp enqueue_streamed) overlaps the
// three across streams but pays 15-22 us per cross-stream hand-off.  Here the
// workgroups of one resident grid take tasks in ticket order:
//   * load: host rows -> frame 0 (16-byte loads straight from pinned host
//     memory over PCIe, 16 in flight per lane);
//   * level tile: one SWAR temporal tile (the k_swar_pf tile of
//     stencil_swar.hip: 4-byte lanes, buffer-op loads with the range check
//     doing the zero padding, `steps` repetitions in registers with LDS
//     boundary rows) of level j, frame (j-1) % 2 -> frame j % 2;
//   * store: final rows -> host.
// A task first waits for the row tiles it depends on (plan_wave: the tiles it
// reads and the tiles that still read what it overwrites), each complete when
// its counter holds the level's task count.  Hand-offs follow the agent-scope
// recipe of the CDNA4 guide (per-XCD L2s are not coherent): producer — every
// wave drains its stores (s_waitcnt vmcnt(0)), workgroup barrier, one lane
// releases (buffer_wbl2 sc1), waits again, then adds to the counter;
// consumer — one lane polls the counters with relaxed agent loads (s_sleep
// between polls), ONE acquire (buffer_inv sc1) + wait, workgroup barrier,
// then plain loads.  Every poll is bounded by a wall-clock timeout: a
// timed-out wait sets the abort word, every workgroup leaves at its next
// ticket, and the host raises (BandEngine::synchronize).
// Tickets come from one device-scope counter; the plan's ticket order is
// topological, so a workgroup only ever waits on tasks already claimed by
// running workgroups and the grid drains at any residency.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "pconv/device.hpp"
#include "pconv/kernels.hpp"
#include "pconv/schedule.hpp"
#include "swar_device.hpp"

namespace pconv {
namespace {

typedef __attribute__((address_space(1))) uint32_t gu32;
// A native 16-byte vector (HIP's uint4 is a struct: an array of them is not
// promoted to registers and went through scratch).
typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// Shared words are accessed as GLOBAL (not flat) agent-scope atomics.
__device__ __forceinline__ gu32* gptr(const uint32_t* p) { return (gu32*)(const_cast<uint32_t*>(p)); }

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(gptr(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Rows [a, b) of `row_bytes` bytes from src (pitch sp) to dst (pitch dp), by
// the whole workgroup over the flattened (row, granule) space: 16-byte
// granules (4-byte when the rows are not 16-byte aligned), U loads in flight
// per lane before the first store — a PCIe read from pinned host memory
// takes microseconds, so the bytes in flight set the rate (the first form,
// one row per wave, ran at 2-3 GB/s per workgroup: profiles/r04/wave2/).
template <int U, typename T>
__device__ __forceinline__ void copy_flat(const uint8_t* src, int64_t sp, uint8_t* dst, int64_t dp, int a, int b,
                                          int g) {
  const int n = (b - a) * g;
  const int nt = static_cast<int>(blockDim.x);
  for (int i0 = static_cast<int>(threadIdx.x); i0 < n; i0 += nt * U) {
    // Indices past the end are clamped to the last granule: those lanes load
    // and store it again (the same bytes to the same place), so neither loop
    // branches and the U values stay in registers.
    T v[U];
    int r[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * nt, n - 1);
      r[u] = i / g;
      c[u] = i - r[u] * g;
      v[u] = reinterpret_cast<const T*>(src + static_cast<int64_t>(a + r[u]) * sp)[c[u]];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) reinterpret_cast<T*>(dst + static_cast<int64_t>(a + r[u]) * dp)[c[u]] = v[u];
  }
}

// Host rows -> frame rows [a, b) with buffer stores (sc1 = write-through
// when `wt`: the published rows then need no release fence).
template <int U>
__device__ __forceinline__ void load_rows_to_frame(const uint8_t* src, int64_t sp, uint8_t* frame, int dp, int a,
                                                   int b, int g, bool wt) {
  const int n = (b - a) * g;
  const int nt = static_cast<int>(blockDim.x);
  const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(frame + static_cast<int64_t>(a) * dp, 0, (b - a) * dp,
                                                      0x00020000);
  for (int i0 = static_cast<int>(threadIdx.x); i0 < n; i0 += nt * U) {
    v4u32 v[U];
    int r[U], c[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * nt, n - 1);
      r[u] = i / g;
      c[u] = i - r[u] * g;
      v[u] = reinterpret_cast<const v4u32*>(src + static_cast<int64_t>(a + r[u]) * sp)[c[u]];
    }
    if (wt) {
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rsrc, r[u] * dp + c[u] * 16, 0, 16);
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) __builtin_amdgcn_raw_buffer_store_b128(v[u], rsrc, r[u] * dp + c[u] * 16, 0, 0);
    }
  }
}

__device__ __forceinline__ void copy_rows(const uint8_t* src, int64_t sp, uint8_t* dst, int64_t dp, int a, int b,
                                          int row_bytes) {
  const bool wide = (row_bytes % 16 == 0) && (sp % 16 == 0) && (dp % 16 == 0) &&
                    (reinterpret_cast<uintptr_t>(src) % 16 == 0) && (reinterpret_cast<uintptr_t>(dst) % 16 == 0);
  if (wide)
    copy_flat<8, v4u32>(src, sp, dst, dp, a, b, row_bytes / 16);
  else
    copy_flat<16, uint32_t>(src, sp, dst, dp, a, b, row_bytes / 4);  // the wave path requires row_bytes % 4 == 0
}

// One tile of k_swar_pf (stencil_swar.hip) as a device function: output rows
// [r0, r1) (r1 - r0 <= NW*M - 2*steps), column strip pair `col`.
template <int CH, int M, int NW, bool ALT>
__device__ __forceinline__ void wave_tile(const uint8_t* src, uint8_t* dst, int pitch, int row_bytes, int r0, int r1,
                                          int steps, int g_row0, int height, int col,
                                          uint4 (&lds)[2][NW][2][1][64], bool wt) {
  constexpr int LW = 4, NP = 4;
  constexpr u32 kOut = 0x80000000u;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int hl = (steps * CH + LW - 1) / LW;
  const int vbytes = (64 - 2 * hl) * LW;
  const int nstrips = (row_bytes + vbytes - 1) / vbytes;
  const int pair_stride = (nstrips + 1) / 2;
  const int lo_ok = max(r0 - steps, -g_row0), hi_ok = min(r1 + steps, height - g_row0);
  const int st_end = min(r1, height - g_row0);
  const auto srsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src) + static_cast<int64_t>(lo_ok) * pitch,
                                                       0, max(hi_ok - lo_ok, 0) * pitch, 0x00020000);
  const auto drsrc = __builtin_amdgcn_make_buffer_rsrc(dst + static_cast<int64_t>(r0) * pitch, 0,
                                                       max(st_end - r0, 0) * pitch, 0x00020000);
  const int sB = col + pair_stride;
  const int baseA = col * vbytes - hl * LW, baseB = sB * vbytes - hl * LW;
  const int pa = baseA + lane * LW, pb = baseB + lane * LW;
  const int xA = (pa >= 0 && pa < row_bytes) ? pa : -1;
  const int xB = (sB < nstrips && pb >= 0 && pb < row_bytes) ? pb : -1;
  const bool needs_mask = baseA < 0 || baseA + 64 * LW > row_bytes || sB >= nstrips || baseB + 64 * LW > row_bytes;
  const int row_base = r0 - steps + w * M;
  u32 D[M][NP];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    const bool rok = fr >= lo_ok && fr < hi_ok;
    const u32 ro = static_cast<u32>(fr - lo_ok) * static_cast<u32>(pitch);
    const u32 a = __builtin_amdgcn_raw_buffer_load_b32(srsrc, (rok && xA >= 0) ? ro + xA : kOut, 0, 0);
    const u32 b = __builtin_amdgcn_raw_buffer_load_b32(srsrc, (rok && xB >= 0) ? ro + xB : kOut, 0, 0);
    unpack<NP>(a, b, D[i]);
  }
  u32 cm[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k)
    cm[k] = (xA >= 0 && xA + k < row_bytes ? 0xffffu : 0u) | (xB >= 0 && xB + k < row_bytes ? 0xffff0000u : 0u);
  const int out_top = min(max(-g_row0 - row_base, 0), M);
  const int out_bot = min(max(height - g_row0 - row_base, 0), M);
  if constexpr (ALT) {
    int s = 0;
    for (; s + 2 <= steps; s += 2) {
      swar_step<CH, NP, M, NW, 1>(D, lds, 0, w, lane, needs_mask, cm, out_top, out_bot);
      swar_step<CH, NP, M, NW, 2>(D, lds, 1, w, lane, needs_mask, cm, out_top, out_bot);
    }
    if (s < steps) swar_step<CH, NP, M, NW, 0>(D, lds, 0, w, lane, needs_mask, cm, out_top, out_bot);
  } else {
    for (int s = 0; s < steps; ++s) swar_step<CH, NP, M, NW, 0>(D, lds, s & 1, w, lane, needs_mask, cm, out_top, out_bot);
  }
  const bool lane_in = lane >= hl && lane < 64 - hl;
  const int st_hi = min(r0 + NW * M - 2 * steps, st_end);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const int fr = row_base + i;
    const bool rst = fr >= r0 && fr < st_hi;
    const u32 ro = static_cast<u32>(fr - r0) * static_cast<u32>(pitch);
    u32 a, bb;
    pack<NP>(D[i], a, bb);
    if (wt) {  // sc1: write-through, no release fence needed before the arrival
      __builtin_amdgcn_raw_buffer_store_b32(a, drsrc, (rst && lane_in && xA >= 0) ? ro + xA : kOut, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b32(bb, drsrc, (rst && lane_in && xB >= 0) ? ro + xB : kOut, 0, 16);
    } else {
      __builtin_amdgcn_raw_buffer_store_b32(a, drsrc, (rst && lane_in && xA >= 0) ? ro + xA : kOut, 0, 0);
      __builtin_amdgcn_raw_buffer_store_b32(bb, drsrc, (rst && lane_in && xB >= 0) ? ro + xB : kOut, 0, 0);
    }
  }
}

struct WaveLevelDev {
  int steps;
  int arrivals;      // tasks per row tile of this level
  int counter_base;  // first tile counter of this level
  int qbase, qcount; // dynamic mode: this level's tasks in the level-tile section
  int pad[3];
};
static_assert(sizeof(WaveLevelDev) == 32, "8 ints per level");

struct WaveArgs {
  const WaveTask* tasks;   // [loads | level tiles | stores], each part in ticket order
  int nload, ncomp, nstore;
  int loaders, storers;    // workgroups dedicated to loads / stores (the first claimers of a role ticket)
  int levels;
  uint32_t* ctl;  // [0] level-tile ticket, [1] abort, [2] role ticket, [3] load ticket, [4] store ticket; counters from ctl + 8
  const WaveLevelDev* lv;
  const uint8_t* host_in;  // row r of the input at host_in + (r - in_r0) * row_bytes
  int in_r0;
  uint8_t* host_out;       // owned row r at host_out + r * row_bytes
  uint8_t* frame0;         // frames at (row 0, column 0)
  uint8_t* frame1;
  int pitch, row_bytes, g_row0, height;
  uint64_t timeout;        // wall-clock ticks
  uint32_t* err;           // pinned host word: 1 = a wait timed out
  int poll_sleep;          // s_sleep(8) (~0.2 us) per unsuccessful poll
  uint64_t* trace;         // nullable: per task {claimed, deps met, done, workgroup | xcc << 32} (wall clock)
  int write_through;       // published rows stored sc1 (no release fence) instead of plain + release
  int dyn;                 // level tiles claimed only when ready (per-level heads) instead of one ticket queue
  int ncounters;           // tile counters; the per-level heads follow them
};

// Dependencies of `k` complete (relaxed agent loads; the caller acquires).
__device__ __forceinline__ bool deps_ready(const WaveTask& k, const WaveLevelDev& d, const uint32_t* counters) {
  for (int x = k.dep_lo; x <= k.dep_hi; ++x)
    if (static_cast<int>(ld_agent(counters + d.counter_base + x)) < d.arrivals) return false;
  return true;
}

// Roles: the first `loaders` workgroups to start stream the input (no
// dependencies: uploads run at the link's rate whatever the levels are
// doing — one CU keeps only a few KB of PCIe reads in flight, ~2 GB/s, so the
// uploads need many CUs at once: profiles/r04/wave3/), the next `storers`
// stream finished rows out, every other workgroup takes level tiles.  Roles
// come from a ticket taken when the workgroup starts, so every loader is
// running: level tiles wait only on loads and earlier level tiles, stores
// only on level tiles — no cycle, whatever the residency.
template <int CH, int M, int NW, bool ALT>
__global__ __launch_bounds__(64 * NW) void k_wave(WaveArgs A) {
  __shared__ uint4 lds[2][NW][2][1][64];
  __shared__ int sh[3];
  const int tid = threadIdx.x;
  uint32_t* counters = A.ctl + 8;
  if (tid == 0) {
    const int r = static_cast<int>(__hip_atomic_fetch_add(gptr(A.ctl + 2), 1u, __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT));
    sh[2] = r < A.loaders ? 0 : r < A.loaders + A.storers ? 2 : 1;
  }
  __syncthreads();
  const int role = sh[2];
  const int base = role == 0 ? 0 : role == 1 ? A.nload : A.nload + A.ncomp;
  const int count = role == 0 ? A.nload : role == 1 ? A.ncomp : A.nstore;
  uint32_t* ticket = A.ctl + (role == 0 ? 3 : role == 1 ? 0 : 4);
  uint32_t* heads = counters + A.ncounters;
  const bool dyn = role == 1 && A.dyn;
  while (true) {
    if (tid == 0) {
      int t = count;
      if (dyn) {
        // Dynamic: claim a level tile only once its dependencies are complete
        // (deepest level first), so no workgroup holds a task while it
        // waits; give up after the timeout without progress.
        const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
        while (true) {
          bool left = false;
          int got = -1;
          for (int j = A.levels; j >= 1 && got < 0; --j) {
            const WaveLevelDev d = A.lv[j];
            uint32_t h = ld_agent(heads + j);
            while (static_cast<int>(h) < d.qcount) {
              left = true;
              const WaveTask c = A.tasks[base + d.qbase + static_cast<int>(h)];
              if (!deps_ready(c, A.lv[j - 1], counters)) break;
              if (__hip_atomic_compare_exchange_strong(gptr(heads + j), &h, h + 1, __ATOMIC_RELAXED,
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                got = d.qbase + static_cast<int>(h);
                break;
              }  // lost the race: h holds the new head, look at that task
            }
          }
          if (got >= 0) {
            t = got;
            break;
          }
          if (!left) break;  // every level tile claimed: done
          if (static_cast<uint64_t>(wall_clock64()) - t0 > A.timeout || ld_agent(A.ctl + 1) != 0) {
            __hip_atomic_store(gptr(A.ctl + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
          }
          for (int z = 0; z < A.poll_sleep; ++z) __builtin_amdgcn_s_sleep(8);
        }
      } else {
        t = static_cast<int>(__hip_atomic_fetch_add(gptr(ticket), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
      if (ld_agent(A.ctl + 1) != 0) t = count;  // another workgroup gave up: drain
      sh[0] = t;
    }
    __syncthreads();
    if (sh[0] >= count) break;  // uniform
    const int ti = base + sh[0];
    const WaveTask k = A.tasks[ti];
    uint64_t tr_claim = 0;
    if (A.trace && tid == 0) tr_claim = static_cast<uint64_t>(wall_clock64());
    if (tid == 0) {
      int ok = 1;
      if (k.kind != 0) {
        const WaveLevelDev d = A.lv[k.level - 1];
        const uint64_t t0 = static_cast<uint64_t>(wall_clock64());
        for (int x = k.dep_lo; x <= k.dep_hi && ok; ++x) {
          const uint32_t* c = counters + d.counter_base + x;
          while (static_cast<int>(ld_agent(c)) < d.arrivals) {
            if (static_cast<uint64_t>(wall_clock64()) - t0 > A.timeout || ld_agent(A.ctl + 1) != 0) {
              ok = 0;
              break;
            }
            for (int z = 0; z < A.poll_sleep; ++z) __builtin_amdgcn_s_sleep(8);
          }
        }
        if (!ok) {
          __hip_atomic_store(gptr(A.ctl + 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(A.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      sh[1] = ok;
    }
    uint64_t tr_ready = 0;
    if (A.trace && tid == 0) tr_ready = static_cast<uint64_t>(wall_clock64());
    __syncthreads();
    if (!sh[1]) break;  // uniform: a dependency never completed
    if (k.kind == 0) {
      const uint8_t* hin = A.host_in - static_cast<int64_t>(A.in_r0) * A.row_bytes;
      if (A.row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(hin) % 16 == 0)
        load_rows_to_frame<8>(hin, A.row_bytes, A.frame0, A.pitch, k.a, k.b, A.row_bytes / 16, A.write_through != 0);
      else
        copy_rows(hin, A.row_bytes, A.frame0, A.pitch, k.a, k.b, A.row_bytes);
    } else if (k.kind == 1) {
      const int s = A.lv[k.level].steps;
      const uint8_t* src = (k.level - 1) & 1 ? A.frame1 : A.frame0;
      uint8_t* dst = k.level & 1 ? A.frame1 : A.frame0;
      wave_tile<CH, M, NW, ALT>(src, dst, A.pitch, A.row_bytes, k.a, k.b, s, A.g_row0, A.height, k.part, lds,
                                A.write_through != 0);
    } else {
      copy_rows(A.levels & 1 ? A.frame1 : A.frame0, A.pitch, A.host_out, A.row_bytes, k.a, k.b, A.row_bytes);
    }
    if (k.kind != 2) {
      // publish: every wave's stores drained, then (plain stores) one release,
      // and the arrival.  Write-through (sc1) payload needs no release; the
      // row copy of an unaligned input keeps plain stores and the release.
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        const bool plain = !A.write_through ||
                           (k.kind == 0 && !(A.row_bytes % 16 == 0 && reinterpret_cast<uintptr_t>(A.host_in) % 16 == 0));
        if (plain) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(gptr(counters + A.lv[k.level].counter_base + k.tile), 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (A.trace && tid == 0) {
      uint32_t xcc = 0;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
      uint64_t* t = A.trace + 4 * static_cast<int64_t>(ti);
      t[0] = tr_claim;
      t[1] = tr_ready;
      t[2] = static_cast<uint64_t>(wall_clock64());
      t[3] = static_cast<uint64_t>(blockIdx.x) | (static_cast<uint64_t>(xcc) << 32);
    }
    __syncthreads();  // LDS and sh[] are reused by the next task
  }
}

constexpr int kWaveM = 8, kWaveNW = 8;

template <int CH>
const void* wave_fn() {
  return reinterpret_cast<const void*>(&k_wave<CH, kWaveM, kWaveNW, true>);
}

int wave_resident(const void* fn) {
  static std::mutex mu;
  static std::map<const void*, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(fn);
  if (it != cache.end()) return it->second;
  int per_cu = 0, dev = 0, cus = 0;
  PCONV_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 64 * kWaveNW, 0));
  PCONV_HIP_CHECK(hipGetDevice(&dev));
  PCONV_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int n = std::max(1, per_cu) * std::max(1, cus);
  cache.emplace(fn, n);
  return n;
}

}  // namespace

int wave_tile_rows(int max_steps) { return kWaveM * kWaveNW - 2 * max_steps; }

int wave_col_groups(int channels, int steps, int64_t row_bytes) {
  const int hl = (steps * channels + 3) / 4;
  const int vbytes = (64 - 2 * hl) * 4;
  if (vbytes <= 0) return 0;
  const int64_t nstrips = (row_bytes + vbytes - 1) / vbytes;
  return static_cast<int>((nstrips + 1) / 2);
}

void launch_wave_image(const WaveLaunch& w, hipStream_t s) {
  PCONV_CHECK(w.ctl_bytes >= 32 && w.tasks && w.levels_dev && w.ctl && w.err && w.frame0 && w.frame1 && w.host_in && w.host_out,
              "wave launch: missing buffers");
  PCONV_CHECK(w.row_bytes % 4 == 0 && w.pitch % 16 == 0, "wave launch: rows must be whole dwords");
  PCONV_CHECK(w.nload > 0 && w.ncomp > 0 && w.nstore > 0 && w.levels >= 1, "wave launch: empty plan");
  PCONV_HIP_CHECK(hipMemsetAsync(w.ctl, 0, static_cast<size_t>(w.ctl_bytes), s));
  const void* fn = w.channels == 1 ? wave_fn<1>() : w.channels == 3 ? wave_fn<3>() : wave_fn<4>();
  int grid = std::min(w.nload + w.ncomp + w.nstore, wave_resident(fn));
  if (w.max_workgroups > 0) grid = std::min(grid, w.max_workgroups);
  grid = std::max(grid, 3);  // a loader, a storer and a level-tile workgroup at least
  WaveArgs A;
  A.tasks = w.tasks;
  A.nload = w.nload;
  A.ncomp = w.ncomp;
  A.nstore = w.nstore;
  A.loaders = std::max(1, std::min(w.loaders > 0 ? w.loaders : grid / 8, (grid - 1) / 2));
  A.storers = std::max(1, std::min(w.storers > 0 ? w.storers : grid / 8, grid - 1 - A.loaders));
  A.levels = w.levels;
  A.ctl = w.ctl;
  A.lv = reinterpret_cast<const WaveLevelDev*>(w.levels_dev);
  A.host_in = w.host_in;
  A.in_r0 = static_cast<int>(w.in_r0);
  A.host_out = w.host_out;
  A.frame0 = w.frame0;
  A.frame1 = w.frame1;
  A.pitch = static_cast<int>(w.pitch);
  A.row_bytes = static_cast<int>(w.row_bytes);
  A.g_row0 = static_cast<int>(w.g_row0);
  A.height = static_cast<int>(std::min<int64_t>(w.height, int64_t(1) << 30));
  A.timeout = w.timeout_ticks;
  A.err = w.err;
  A.poll_sleep = std::max(1, w.poll_sleep);
  A.trace = w.trace;
  A.write_through = w.write_through ? 1 : 0;
  A.dyn = w.dynamic ? 1 : 0;
  A.ncounters = w.ncounters;
  const dim3 g(static_cast<unsigned>(std::max(1, grid))), b(64 * kWaveNW);
  switch (w.channels) {
    case 1: k_wave<1, kWaveM, kWaveNW, true><<<g, b, 0, s>>>(A); break;
    case 3: k_wave<3, kWaveM, kWaveNW, true><<<g, b, 0, s>>>(A); break;
    case 4: k_wave<4, kWaveM, kWaveNW, true><<<g, b, 0, s>>>(A); break;
    default: PCONV_FAIL("wave launch: channels must be 1, 3 or 4");
  }
  PCONV_HIP_CHECK(hipGetLastError());
}

}  // namespace pconv
