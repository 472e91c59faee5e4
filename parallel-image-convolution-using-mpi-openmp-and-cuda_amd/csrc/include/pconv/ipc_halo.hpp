// Device-side inter-process halo exchange over HIP IPC.
//
// Replaces the reference's MPI_Isend/Irecv of boundary rows and the
// MPI_Wait pairs around them (mpi/mpi_convolution.c:157-234) for ranks that
// are processes on ONE node: every rank exports its two frames and a small
// device-memory MAILBOX with hipIpcGetMemHandle once, opens its neighbours'
// (same GPU, or a peer GPU mapped over xGMI), and an exchange PULLS the
// neighbours' boundary rows straight into its own ghost rows — no
// communication library kernel, no host staging, nothing on the host path
// after set-up.
//
// Signalling is push-to-the-poller: a rank WRITES its exchange number into
// its neighbours' mailboxes (one remote store each) and POLLS only its own
// mailbox (local HBM), so no poll ever crosses PCIe or xGMI.  Per rank and
// slot the mailbox holds `count` (exchanges done, written by the rank
// itself), `level_up` / `level_down` (the upper / lower neighbour's rows of
// exchange #n are final) and `ack_up` / `ack_down` (that neighbour has copied
// this rank's rows), each on its own cache line.  One exchange, n = count+1,
// in stream order on the caller's stream:
//   1. signal: level_down of the upper neighbour's mailbox = n, level_up of
//      the lower one's = n; wait until this mailbox's level_up / level_down
//      >= n (the neighbours' rows are final: they came from earlier kernels
//      of their streams, whose end-of-kernel release wrote them back);
//   2. pull: the neighbours' rows (same frame parity: bands advance in
//      lockstep) into this rank's ghost rows (skipped after a timeout);
//   3. ack: count = n; ack_down / ack_up of the neighbours' mailboxes = n;
//      wait until this mailbox's acks >= n (they have copied this rank's
//      rows, so later launches may overwrite them — the reference's wait on
//      its sends before the swap).
// Three forms (IpcPull; docs/PERFORMANCE.md has the measurements):
//   * Grid (default): ONE dispatch of G workgroups; every workgroup's thread
//     0 waits with its own system-scope acquire (each CU's and XCD's caches
//     invalidated for the rows it reads), copies its slice, and arrives on a
//     counter in the mailbox; the last one performs step 3.  G workgroups
//     keep G times the single form's bytes in flight — what a pull over
//     xGMI (microseconds per round trip) needs.
//   * Single: the same in ONE workgroup (round 4's form).
//   * Sdma: one-thread signal and ack kernels around SDMA peer copies.  The
//     copies cannot be skipped after a timed-out wait: a neighbour that
//     stalls (but keeps its frames mapped) yields stale rows and the raised
//     error, as in the other forms.
// Visibility across devices.  The mailbox is UNCACHED device memory
// (hipDeviceMallocUncached; fine-grained if the runtime cannot export that):
// a neighbour's system-scope release store into it travels over xGMI to this
// GPU's memory, and this rank's system-scope acquire poll reads memory, not a
// cache line — no L2 of either GPU can hold a stale word.  The rows: the
// neighbour's earlier kernels wrote them into its (coarse-grained) frames and
// their end-of-kernel release wrote its L2 back before its signal store was
// issued (stream order, and the store is a release); this rank's acquire
// invalidates its own L2, so the pull reads the rows from the neighbour's
// memory, not a line cached by an earlier exchange.  self_test() checks all of
// it once at connect.
// Sdma form and a neighbour that EXITS: its copies run even after a timed-out
// wait, so a neighbour gone with its frames unmapped can fault a replay.  It
// is never the default or a fallback; check() after every drain raises
// before the next image is issued.
// The exchange number lives in device memory, so a captured graph replays
// correctly.  Every wait has a wall-clock timeout: an expired wait sets the
// rank's error word (a host shared-memory segment the host checks) and
// returns (no wave spins forever); check() raises.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <string>
#include <vector>

#include "pconv/engine.hpp"

namespace pconv {

// Host-visible words of one (rank, slot), padded to a cache line: the
// error word (1: a level wait timed out, 2: an ack wait timed out).
struct IpcFlags {
  uint32_t err;
  uint32_t pad[15];
};
static_assert(sizeof(IpcFlags) == 64, "one cache line per flag block");

// Device-memory mailbox of one (rank, slot); one cache line per word.
struct IpcMailbox {
  uint32_t count, pad0[15];
  uint32_t level_up, pad1[15];    // written by the upper neighbour
  uint32_t level_down, pad2[15];  // written by the lower neighbour
  uint32_t ack_up, pad3[15];
  uint32_t ack_down, pad4[15];
  uint32_t arrive, pad5[15];      // grid form: workgroups done with this exchange
};
static_assert(sizeof(IpcMailbox) == 384, "six cache lines");

// hipIpcMemHandle_t of frame 0, frame 1 and the mailbox, back to back.
constexpr size_t kIpcHandleBytes = 3 * sizeof(hipIpcMemHandle_t);

// Create (rank 0) / map (every rank) the shared flag segment of a job:
// world x slots flag blocks, zeroed at creation.
void ipc_create_segment(const std::string& name, int world, int slots);
void ipc_unlink_segment(const std::string& name);

enum class IpcPull { Grid, Single, Sdma };
IpcPull parse_ipc_pull(const std::string& s);  // "grid" | "single" | "sdma"
const char* ipc_pull_name(IpcPull p);

// One exchange in stream order on `s` (kernels/ipc_flags.hip).  `mine` is
// this rank's mailbox, `up_mb` / `down_mb` the neighbours' (null: no
// neighbour on that side; this rank's own for a self-neighbour), `err` the
// device address of this rank's host-visible error word; dst_* are this
// rank's ghost rows, src_* the neighbours' boundary rows, `bytes` per side, a
// multiple of 16.  Grid uses `workgroups` (0: chosen from the size).
void launch_ipc_exchange(IpcPull form, IpcMailbox* mine, IpcMailbox* up_mb, IpcMailbox* down_mb, uint32_t* err,
                         uint64_t timeout_ticks, uint8_t* dst_up, const uint8_t* src_up, uint8_t* dst_down,
                         const uint8_t* src_down, int64_t bytes, hipStream_t s, int workgroups = 0);
// Workgroups the Grid form uses for `bytes` per side.
int ipc_grid_workgroups(int64_t bytes);

// Cost of one exchange of each pull form without a neighbour process: a
// mailbox in device memory and an error word in pinned host memory
// (self-neighbour protocol: this rank is its own upper and lower neighbour),
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

  // kIpcHandleBytes: frame 0, frame 1 and the mailbox.
  std::vector<uint8_t> local_handles() const { return handles_; }
  // Open the neighbours' frames (empty vector: no neighbour on that side).
  void connect(const std::vector<uint8_t>& up_handles, const std::vector<uint8_t>& down_handles);
  bool connected() const { return connected_; }
  // Collective with the neighbours (every rank calls it once per transport,
  // in the same slot order, after every rank connected): one exchange of
  // sentinel rows through the real protocol — signal words stored into the
  // neighbours' mailboxes, rows pulled from their allocations, acks — with a
  // short timeout, the pulled bytes compared.  Raises a named error at once
  // (instead of the first real exchange timing out after timeout_s) when a
  // neighbour's stores or rows are not visible to this rank.
  void self_test(double timeout_s = 5.0);
  bool self_tested() const { return self_tested_; }
  // "uncached" | "fine-grained" | "coarse-grained" (the runtime exported neither)
  const std::string& mailbox_kind() const { return mailbox_kind_; }
  // The neighbours' devices (-1: none on that side; this device for a self-neighbour).
  int peer_device(int side) const { return peer_dev_[side & 1]; }

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
  IpcFlags* dflags_ = nullptr;  // its device address (error words)
  uint64_t timeout_ticks_ = 0;
  std::vector<uint8_t> handles_;
  uint8_t* peer_up_[2] = {nullptr, nullptr};    // neighbour frames (base of the allocation)
  uint8_t* peer_down_[2] = {nullptr, nullptr};
  FrameLayout lay_up_, lay_down_;
  bool connected_ = false;
  bool own_ = false;  // a neighbour is this engine itself (one-process emulation)
  IpcPull pull_ = IpcPull::Grid;
  static constexpr size_t kMailboxBytes = size_t(2) << 20;
  static constexpr int64_t kProbeOffset = 4096, kProbeBytes = 4096;  // self-test rows in the mailbox allocation
  DeviceBuffer mail_;                       // this rank's mailbox (exported)
  std::string mailbox_kind_;
  int peer_dev_[2] = {-1, -1};
  bool self_tested_ = false;
  IpcMailbox* peer_mail_up_ = nullptr;      // the neighbours' mailboxes (opened)
  IpcMailbox* peer_mail_down_ = nullptr;
  uint8_t* own_base_[2] = {nullptr, nullptr};  // this engine's frames (the destructor never touches the engine)
  int64_t enqueued_ = 0;
};

}  // namespace pconv
