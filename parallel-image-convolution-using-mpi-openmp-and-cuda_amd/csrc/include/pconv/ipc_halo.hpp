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
// One dispatch per exchange by default (k_ipc_exchange: the three steps in
// one workgroup; the rows a neighbour reads always come from an earlier
// kernel of its stream, whose end-of-kernel release wrote them back on every
// XCD); PCONV_IPC_KERNELS=3 splits it into three dispatches.
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

// Device kernels of the protocol (kernels/ipc_flags.hip).  `flags` is the
// device pointer of the segment's block array.
void launch_ipc_signal_wait(IpcFlags* flags, int me, int up, int down, uint64_t timeout_ticks, hipStream_t s);
void launch_ipc_ack_wait(IpcFlags* flags, int me, int up, int down, uint64_t timeout_ticks, hipStream_t s);
// Copy `bytes` from each neighbour's rows into this rank's ghost rows (null
// source: no neighbour on that side); a no-op once this rank's wait timed out.
void launch_ipc_pull(const IpcFlags* flags, int me, uint8_t* dst_up, const uint8_t* src_up, uint8_t* dst_down,
                     const uint8_t* src_down, int64_t bytes, hipStream_t s);
// Signal + wait, pull and ack + wait as ONE single-workgroup dispatch (the
// default; PCONV_IPC_KERNELS=3 issues the three kernels above instead).
void launch_ipc_exchange(IpcFlags* flags, int me, int up, int down, uint64_t timeout_ticks, uint8_t* dst_up,
                         const uint8_t* src_up, uint8_t* dst_down, const uint8_t* src_down, int64_t bytes,
                         hipStream_t s);

class IpcHaloTransport : public HaloTransport {
 public:
  // The engine's frames are exported; `slot` selects this transport's flag
  // blocks (slot k of every rank exchanges with slot k of its neighbours).
  IpcHaloTransport(BandEngine& e, const std::string& segment, int slot, int slots, double timeout_s = 30.0);
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
  bool split_kernels_ = false;  // PCONV_IPC_KERNELS=3: signal / pull / ack as three dispatches
  uint8_t* own_base_[2] = {nullptr, nullptr};  // this engine's frames (the destructor never touches the engine)
  int64_t enqueued_ = 0;
};

}  // namespace pconv
