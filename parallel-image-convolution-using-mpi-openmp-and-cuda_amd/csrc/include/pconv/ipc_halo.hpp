// Device-side inter-process halo exchange over HIP IPC.
//
// Replaces the reference's MPI_Isend/Irecv of boundary rows and the
// MPI_Wait pairs around them (mpi/mpi_convolution.c:157-234) for ranks that
// are processes on ONE node: every rank exports its two frames with
// hipIpcGetMemHandle once, opens its neighbours' frames with
// hipIpcOpenMemHandle (same GPU, or a peer GPU mapped over xGMI), and an
// exchange PULLS the neighbours' boundary rows straight into its own ghost
// rows with device copies — no communication library kernel, no host
// staging, nothing on the host path after set-up.
//
// Three pull forms (IpcPull, chosen per transport; docs/PERFORMANCE.md has
// the measurements that pick the default):
//   * Grid (default): ONE dispatch of G workgroups.  Every workgroup's
//     thread 0 waits for the neighbours' level flags with its own
//     system-scope acquire (so each CU's and each XCD's caches are
//     invalidated for the rows it reads), the workgroup copies its slice,
//     and the workgroups meet on a device-memory arrival counter; the last
//     one to arrive publishes `count` / `ack` and waits for the neighbours'
//     acks.  G workgroups keep G times the single form's bytes in flight —
//     what a pull over xGMI (microseconds per round trip) needs.
//   * Single: the same in ONE workgroup (round 4's form: one acquire
//     covers it; latency-bound on a remote source).
//   * Sdma: a one-thread signal / wait kernel, the rows moved by SDMA
//     (hipMemcpyAsync peer copies, no CU involved), a one-thread ack / wait
//     kernel.  The copies cannot be skipped after a timed-out wait: a
//     neighbour that stalls (but keeps its frames mapped) yields stale
//     rows and the raised error, as in the other forms.
// The rows a neighbour reads always come from an earlier kernel of its
// stream, whose end-of-kernel release wrote them back on every XCD.
// Ordering across processes is device-side, through flag words in a shared
// host-memory segment (POSIX shm, registered with hipHostRegister so every
// rank's GPU reads and writes it with system-scope atomics).  Per (rank,
// slot): `count` (exchanges done by this transport), `level` (its rows for
// exchange #count are final) and `ack` (it has copied its neighbours' rows of
// exchange #count).  One exchange, all in stream order on the caller's
// stream:
//   1. signal kernel: count += 1; level = count; wait until every
//      neighbour's level >= count (their rows are final);
//   2. pull kernel: the neighbours' rows (same frame parity: bands advance
//      in lockstep) copied into this rank's ghost rows by the CUs, reading
//      the neighbours' memory directly (skipped after a timeout);
//   3. ack kernel: ack = count; wait until every neighbour's ack >= count
//      (they have copied this rank's rows, so later launches may overwrite
//      them — the reference's wait on its sends before the swap).
// The exchange number lives in device-visible memory, so a captured graph
// replays correctly.  Every wait has a timeout: an expired wait sets the
// rank's error word and returns (no wave spins forever); check() raises.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <vector>

#include "pconv/engine.hpp"

namespace pconv {

// Flag words of one (rank, slot), padded to a cache line.
struct IpcFlags {
  uint32_t count;
  uint32_t level;
  uint32_t ack;
  uint32_t err;
  uint32_t pad[12];
};
static_assert(sizeof(IpcFlags) == 64, "one cache line per flag block");

// Create (rank 0) / map (every rank) the shared flag segment of a job:
// world x slots flag blocks, zeroed at creation.
void ipc_create_segment(const std::string& name, int world, int slots);
void ipc_unlink_segment(const std::string& name);

enum class IpcPull { Grid, Single, Sdma };
IpcPull parse_ipc_pull(const std::string& s);  // "grid" | "single" | "sdma"
const char* ipc_pull_name(IpcPull p);

// One exchange in stream order on `s` (kernels/ipc_flags.hip).  `flags` is
// the device pointer of the segment's block array; dst_* are this rank's
// ghost rows, src_* the neighbours' boundary rows (null: no neighbour on that
// side), `bytes` per side, a multiple of 16.  Grid needs `arrive` (one zeroed
// device word per transport, left zeroed by every exchange) and uses
// `workgroups` (0: chosen from the size).
void launch_ipc_exchange(IpcPull form, IpcFlags* flags, uint32_t* arrive, int me, int up, int down,
                         uint64_t timeout_ticks, uint8_t* dst_up, const uint8_t* src_up, uint8_t* dst_down,
                         const uint8_t* src_down, int64_t bytes, hipStream_t s, int workgroups = 0);
// Workgroups the Grid form uses for `bytes` per side.
int ipc_grid_workgroups(int64_t bytes);

// Cost of one exchange of each pull form without a neighbour process: a flag
// block in pinned host memory (self-neighbour protocol, up = down = me),
// `bytes` per side pulled from a pinned HOST buffer (host_source: the
// stand-in for a peer GPU's HBM behind xGMI — PCIe round trips of
// microseconds) or from this GPU's HBM; ms per exchange over `iters`
// back-to-back exchanges on one stream.
double ipc_pull_probe(const std::string& form, int64_t bytes, bool host_source, int iters, int device,
                      int workgroups = 0);

class IpcHaloTransport : public HaloTransport {
 public:
  // The engine's frames are exported; `slot` selects this transport's flag
  // blocks (slot k of every rank exchanges with slot k of its neighbours).
  IpcHaloTransport(BandEngine& e, const std::string& segment, int slot, int slots, double timeout_s = 30.0,
                   IpcPull pull = IpcPull::Grid);
  ~IpcHaloTransport() override;
  IpcHaloTransport(const IpcHaloTransport&) = delete;
  IpcHaloTransport& operator=(const IpcHaloTransport&) = delete;

  // hipIpcMemHandle_t of frame 0 and frame 1, back to back.
  std::vector<uint8_t> local_handles() const { return handles_; }
  // Open the neighbours' frames (empty vector: no neighbour on that side).
  void connect(const std::vector<uint8_t>& up_handles, const std::vector<uint8_t>& down_handles);
  bool connected() const { return connected_; }

  void exchange(BandEngine& e, int64_t depth, hipStream_t stream) override;
  const char* name() const override { return "ipc"; }
  IpcPull pull() const { return pull_; }
  bool capturable() const override { return true; }

  // Exchanges enqueued so far; the device-side count after the stream drained.
  int64_t enqueued() const { return enqueued_; }
  uint32_t device_count() const;
  // Throws if a wait of this rank timed out (call after the stream drained).
  void check() const;

 private:
  BandEngine* eng_;
  int rank_, world_, slot_, slots_;
  std::string segment_;
  size_t seg_bytes_ = 0;
  void* host_ = nullptr;       // mapped segment
  IpcFlags* dflags_ = nullptr;  // its device address
  uint64_t timeout_ticks_ = 0;
  std::vector<uint8_t> handles_;
  uint8_t* peer_up_[2] = {nullptr, nullptr};    // neighbour frames (base of the allocation)
  uint8_t* peer_down_[2] = {nullptr, nullptr};
  FrameLayout lay_up_, lay_down_;
  bool connected_ = false;
  bool own_ = false;  // a neighbour is this engine itself (one-process emulation)
  IpcPull pull_ = IpcPull::Grid;
  DeviceBuffer arrive_;  // Grid form: the workgroups' arrival counter
  uint8_t* own_base_[2] = {nullptr, nullptr};  // this engine's frames (the destructor never touches the engine)
  int64_t enqueued_ = 0;
};

}  // namespace pconv
