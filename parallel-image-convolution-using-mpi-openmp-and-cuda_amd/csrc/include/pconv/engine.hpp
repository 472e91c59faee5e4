// Device engine: one row band of the image resident on one GPU.
//
// Replaces GPU_convolution() (cuda/cuda_convolution.cu:49-102) and the MPI
// rank's rep loop (mpi/mpi_convolution.c:151-240):
//   * two device frames (ping-pong) with zero pad columns and `halo` ghost
//     rows, allocated once and reused across runs (no malloc in the loop);
//   * a compute stream and a communication stream; the interior launch of an
//     exchange phase overlaps the halo exchange, the boundary launches wait on
//     an event (schedule.hpp);
//   * the newest result is always the `src` frame after a run — the reference
//     copied back the stale buffer for odd reps;
//   * optional hipGraph capture of a whole rep loop (launch-bound small images);
//   * hipEvent loop timing + host wall timing per run.
// A whole single-GPU image is simply the band {y0=0, rows=H, no neighbours}.
#pragma once

#include <hip/hip_runtime_api.h>

#include <map>
#include <memory>
#include <tuple>
#include <vector>

#include "pconv/device.hpp"
#include "pconv/filter.hpp"
#include "pconv/image.hpp"
#include "pconv/kernels.hpp"
#include "pconv/partition.hpp"
#include "pconv/schedule.hpp"

namespace pconv {

class BandEngine;

// Moves ghost rows between bands.  `exchange` is enqueued on `stream` and
// must fill ghost rows [-depth, 0) from band.up and [rows, rows+depth) from
// band.down of engine.src_frame(), sending the matching owned rows.
class HaloTransport {
 public:
  virtual ~HaloTransport() = default;
  virtual void exchange(BandEngine& e, int64_t depth, hipStream_t stream) = 0;
  virtual const char* name() const = 0;
  // True when exchange() only enqueues stream-ordered device work (no host
  // synchronisation), so it can be captured into a hipGraph: then a serving
  // step that exchanges halos is still ONE graph launch (process_graph).
  virtual bool capturable() const { return false; }
};

struct EngineOptions {
  int device = 0;
  int halo_depth = 1;      // D
  int fuse = 1;            // T (reps per launch; > 1 needs the temporal kernel)
  bool overlap = true;     // interior || halo
  bool use_graph = false;  // capture the rep loop into a hipGraph (no transport)
  // With use_graph: exchange phases run on the compute stream (no separate
  // communication stream) and, with a capturable transport (RCCL, IPC), are
  // captured with the launches into the cached rep-loop graph — the
  // reference's MPI loop on resident bands as one graph launch per image
  // (bench.py resident_loop).  With `overlap` the engine keeps a
  // communication stream and each exchange phase is captured as a fork: the
  // interior launch beside the exchange, the edge strips after it (the
  // reference's Isend/Irecv + inner compute + Wait + edges, one graph).
  bool capture_exchanges = false;
  KernelVariant variant = KernelVariant::Auto;
  // Borrowed streams (nullptr: the engine creates its own).  A process has
  // few hardware queues (GPU_MAX_HW_QUEUES, 4 by default); pipeline slots
  // share streams so that unrelated streams never alias one queue.
  hipStream_t compute_stream = nullptr;
  hipStream_t comm_stream = nullptr;
  // hipEvent loop timing around every run() (two event records, ~3 us of
  // host time each on ROCm 7: the serving pipeline turns it off).
  bool timing = true;
  // Host <-> frame copies (upload_rows / download_rows) and the initial frame
  // zeroing by kernels of this library instead of SDMA / the runtime's blit
  // programs: a one-shot process (the `conv` CLI) skips their first-use
  // set-up; the serving pipeline keeps SDMA (faster per byte, frees the CUs).
  bool kernel_copies = false;
  // Row streaming within one image (schedule.hpp, plan_streamed): a serving
  // step's rows are uploaded in this many chunks and each level advances as
  // far as the rows on the device allow, so H2D, launches and D2H of ONE
  // image overlap on three streams.  0 / 1: whole-image chain.  Issued
  // directly (BandPipeline's event-ordered mode): captured as one graph with
  // fork/join branches it measured 1.4-4.3x slower per image
  // (profiles/r04/stream_a/).
  int stream_chunks = 0;
  // Relative rows per streamed chunk (one weight per chunk, stream_chunks of
  // them); empty: 5, ..., 5, 6 (stream_cuts).
  std::vector<int> stream_weights;
  // Head streaming only for images of at least this many input bytes: the
  // cross-stream hand-offs of a streamed image cost more than they hide on
  // smaller ones.  One image of the headline split N ways, streamed vs one
  // step graph (profiles/r05/e/burst.jsonl): N=1 14.5 MB 0.58 vs 0.68 ms,
  // N=2 7.5 MB 0.385 vs 0.387, N=4 4.1 MB 0.32 vs 0.23, N=8 2.3 MB 0.28 vs
  // 0.15 — so 8 MiB.
  int64_t stream_min_bytes = int64_t(8) << 20;
  // ---- serving-pipeline policy (BandPipeline, slot-stream mode) ----
  // Slot streams on dedicated hardware queues (created with an all-CU mask):
  // from the runtime's shared pool, 4 slot streams landed on queues of which
  // two ran every launch ~5x longer (profiles/r04/slots_c/).
  bool cu_mask_queues = true;
  // A streamed head image's upload / download run on the next two slots'
  // streams (idle while the pipeline is) instead of two more pool streams
  // (0.56 vs 0.77 ms per image with 4 slots, profiles/r04/head/).
  bool head_on_slot_streams = true;
  // With the head's copies on the slots' streams and >= 4 slots: its chunk
  // uploads alternate between slots k+1 and k+2's streams, so one chunk's
  // copy + event does not leave the copy engine idle before the next.  One
  // image 0.546-0.549 vs 0.559-0.568 ms over 3 interleaved rounds, the
  // driver's window 0.334-0.348 vs 0.337-0.351 ms; alternating the downloads
  // too was slower (0.564-0.580, both 0.602-0.625: profiles/r05/l/).
  bool head_alt_uploads = true;
  // Slot-stream mode with head streaming: a burst's first image is held back
  // until the pipeline knows whether more follow — the next submit issues it
  // as a step graph (a burst), drain / ready / wait_image / marks issue it
  // row-streamed (a single image, the latency case).  The driver's 20-image
  // window 0.3282 / 0.3290 / 0.3300 vs 0.3292 / 0.3315 / 0.3335 ms/step
  // eager (6 interleaved pairs, faster in each), one image 0.5349 vs 0.5351
  // ms (profiles/r06/z/).
  bool lazy_head = true;
};

struct RunStats {
  double loop_ms = 0;      // hipEvent time of the rep loop (device)
  double wall_ms = 0;      // host wall time of the enqueue+sync
  int launches = 0;
  int exchanges = 0;
};

class BandEngine {
 public:
  BandEngine(const ImageGeom& geom, const Band& band, const Filter& filter, const EngineOptions& opt);
  ~BandEngine();

  const ImageGeom& geom() const { return geom_; }
  const Band& band() const { return band_; }
  const Filter& filter() const { return filter_; }
  const FrameLayout& layout() const { return lay_; }
  const EngineOptions& options() const { return opt_; }
  static constexpr size_t kMaxCachedGraphs = 64;
  size_t cached_graphs() const { return graphs_.size() + step_graphs_.size(); }
  size_t cached_step_graphs() const { return step_graphs_.size(); }
  hipStream_t compute_stream() const { return cs_; }
  hipStream_t comm_stream() const { return ms_; }

  void set_transport(std::shared_ptr<HaloTransport> t) { transport_ = std::move(t); }

  // Frame pointers at (owned row 0, data column 0).
  uint8_t* src_frame() const { return frame_[cur_].data() + lay_.offset(0); }
  uint8_t* dst_frame() const { return frame_[cur_ ^ 1].data() + lay_.offset(0); }
  // Frame `which` (0/1) at (owned row 0, data column 0); cur() = the source frame.
  uint8_t* frame_at(int which) const { return frame_[which & 1].data() + lay_.offset(0); }
  // Base of frame `which`'s allocation (hipIpcGetMemHandle needs it).
  uint8_t* frame_base(int which) const { return frame_[which & 1].data(); }
  int cur() const { return cur_; }
  // Start frame of the next step (a step that uploads its whole input may
  // start in either frame).
  void set_cur(int c) { cur_ = c & 1; }

  // Copy frame-local rows [r_begin, r_end) from host (pointer at row r_begin).
  // Rows in the ghost zone are accepted (pre-loaded halos).  Async on the
  // compute stream; `host` should be pinned for true async DMA.
  // `stream` = nullptr means the compute stream.
  void upload_rows(const uint8_t* host, int64_t host_pitch, int64_t r_begin, int64_t r_end,
                   hipStream_t stream = nullptr);
  // Same from a device pointer (e.g. a torch CUDA tensor).
  void upload_rows_device(const uint8_t* dev, int64_t dev_pitch, int64_t r_begin, int64_t r_end);
  // Declare whether the ghost rows currently hold valid neighbour data.
  void set_halo_valid(bool v) { halo_valid_ = v; }
  // Serving-step input rows [in_r0, in_r1): false for exactly the owned rows,
  // true for the owned rows plus the full ghost zone on both sides (clipped at
  // the image edges); throws for any other range (a partial ghost zone).
  bool input_preloaded(int64_t in_r0, int64_t in_r1) const;
  // Copy owned rows [r_begin, r_end) of the newest result to host / device.
  void download_rows(uint8_t* host, int64_t host_pitch, int64_t r_begin, int64_t r_end,
                     hipStream_t stream = nullptr);
  void download_rows_device(uint8_t* dev, int64_t dev_pitch, int64_t r_begin, int64_t r_end);

  // Make the compute stream wait for work already queued on `s` / make `s`
  // wait for everything queued on the compute stream.
  void wait_stream(hipStream_t s);
  void signal_stream(hipStream_t s);

  // Fill all `halo` ghost rows now (transport on `stream`, default: the comm
  // stream) and mark them valid: lets a pipeline exchange image k+1's halos
  // while image k still computes.
  void exchange_now(hipStream_t stream = nullptr);
  bool has_transport() const { return transport_ != nullptr; }

  // Enqueue `reps` repetitions (async).  stats filled after synchronize().
  void run(int reps);
  // One whole serving step — H2D of host rows [in_r0, in_r1) (ghost rows
  // allowed), `reps` repetitions, D2H of the owned rows — as ONE cached
  // hipGraph launched on the compute stream: one host API call per image
  // instead of ~12 (copies, launches, events; tools/ubench/api_cost.hip).
  // A schedule that exchanges halos is captured too when the transport is
  // capturable (RCCL send/recv, D2D copies): when the ghost zone covers all
  // `reps`, ONE exchange of the whole zone follows the upload; otherwise the
  // plan's exchange phases are captured in place.  Host buffers must be
  // pinned and stay valid; the graph is keyed on them.
  void process_graph(const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out, int reps);
  // True when `reps` repetitions with / without pre-loaded ghost rows need no exchange.
  bool exchange_free(int reps, bool halo_preloaded) const;
  // Row-streamed serving step (options().stream_chunks chunks): the plan of
  // one image with input rows [in_r0, in_r1); empty chunks when the image
  // cannot be streamed (exchanges, reps == 0, streaming off).
  StreamPlan stream_plan(int reps, int64_t in_r0, int64_t in_r1) const;
  // Enqueue a streamed image: chunk uploads on `up`, launches on the compute
  // stream, downloads of the finished rows on `down` (cross-stream events per
  // chunk).  The caller orders `up` after any earlier use of these frames.
  // Returns the stream whose completion means the whole image is done.
  // `up2` (optional): odd chunks' uploads alternate onto it.
  hipStream_t enqueue_streamed(const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out,
                               const StreamPlan& sp, hipStream_t up, hipStream_t down, hipStream_t up2 = nullptr);
  // Phase-by-phase execution for multi-band emulation on one device.
  std::vector<Phase> plan(int reps) const;
  void exec_exchange(const Phase& p);
  void exec_compute(const Phase& p);

  void synchronize();
  const RunStats& last_stats() const { return stats_; }

  // Zero both frames (ghost rows, pads and data).
  void clear();

  // Debug / tests: copy FRAME rows [r_begin, r_end) of the current source
  // frame, ghost rows included (r_begin >= -halo, r_end <= rows + halo).
  void read_frame_rows(uint8_t* host, int64_t r_begin, int64_t r_end);

 private:
  friend class LocalCluster;
  void enqueue_phase(const Phase& p);
  void launch(const LaunchSpec& l, hipStream_t s);
  StencilLaunch make_launch(const LaunchSpec& l, int cur) const;
  // Settle per-launch choices (tile-shape tuning) of a plan before capturing it.
  void prepare(const std::vector<Phase>& ph);

  ImageGeom geom_;
  Band band_;
  Filter filter_;
  EngineOptions opt_;
  FrameLayout lay_;
  DeviceBuffer frame_[2];
  int cur_ = 0;
  bool halo_valid_ = false;
  int pre_exchanges_ = 0;  // exchange_now() calls since the last run()
  Stream own_cs_, own_ms_;
  hipStream_t cs_ = nullptr, ms_ = nullptr;
  Event ev_ready_, ev_halo_, ev_t0_, ev_t1_, ev_sync_;
  std::vector<Event> up_evs_, dn_evs_;  // streamed images: per chunk, uploaded / rows final
  bool stream_trace_ = false;
  std::vector<Event> st_ev_;
  size_t st_chunks_ = 0;
 public:
  // Diagnostics: time the next streamed images chunk by chunk (timing events
  // after each chunk's upload, its launches' wait, launches, its download's
  // wait and download); stream_trace() gives, for the latest one, {chunk,
  // upload end, launch wait passed, launches end, download wait passed,
  // download end} in ms from its first upload's issue point (-1: nothing
  // recorded).
  void set_stream_trace(bool on) { stream_trace_ = on; }
  std::vector<std::vector<double>> stream_trace();
  // Create the streamed-image events for `chunks` chunks now (set-up), not
  // inside the first streamed image this engine runs.
  void reserve_stream_events(size_t chunks) {
    while (up_evs_.size() < chunks) up_evs_.push_back(Event::create());
    while (dn_evs_.size() < chunks + 1) dn_evs_.push_back(Event::create());
  }

 private:
  std::shared_ptr<HaloTransport> transport_;
  RunStats stats_;
  double wall_t0_ = 0;
  bool timing_pending_ = false;
  // hipGraph cache: (reps, start buffer) -> executable graph
  std::map<std::pair<int, int>, hipGraphExec_t> graphs_;
  struct StepGraph {
    hipGraphExec_t exec = nullptr;
    int end_cur = 0;
    int launches = 0;
    int exchanges = 0;
  };
  // (reps, start buffer, in, in_r0, in_r1, out) -> whole-step graph.  Keyed
  // on host pointers, so both caches are bounded: past kMaxCachedGraphs
  // entries the stream is drained and the cache is emptied.
  void trim_graph_caches();
  std::map<std::tuple<int, int, const uint8_t*, int64_t, int64_t, uint8_t*>, StepGraph> step_graphs_;
};

// Serving pipeline: S band engines ("slots") so that the H2D copy of image
// k+1, the repetitions of image k and the D2H copy of image k-1 overlap on
// three streams (the reference did copy -> compute -> copy, synchronous and
// pageable, cuda/cuda_convolution.cu:60,94-96).  Slot reuse is ordered by
// events; all slots of a rank share one communication stream.
class BandPipeline {
 public:
  // concurrent: -1 = when the hardware-queue budget allows, 0 = one shared
  // compute stream, 1 = one compute stream per slot.
  // graphs: every image is one hipGraph (H2D + reps + D2H) on its slot's own
  // stream — slots run concurrently, one host call per image; needs
  // exchange-free images (see BandEngine::process_graph).
  // slot_streams: every image runs on its slot's own stream (H2D, reps, D2H
  // stream-ordered, no cross-stream events) — slots overlap each other; needs
  // exchange-free images.  step_graphs: each such image is one cached hipGraph
  // (one host call), otherwise its copies and launches are issued directly.
  // slot_comm (slot-stream mode): every slot also gets its own
  // communication stream and keeps opt.overlap, so an exchange phase splits
  // into the interior launch on the slot stream ‖ the exchange on its comm
  // stream, the edge strips after the halo event — and, captured, the whole
  // image (the reference's Isend/inner/Wait/edges loop for every phase) is
  // ONE graph with a fork/join per exchange.
  BandPipeline(const ImageGeom& geom, const Band& band, const Filter& filter, const EngineOptions& opt, int slots,
               int concurrent = -1, bool slot_streams = false, bool step_graphs = true, bool slot_comm = false);
  ~BandPipeline();
  int slots() const { return static_cast<int>(slots_.size()); }
  BandEngine& slot(int i) { return *slots_.at(i); }
  void set_transport(std::shared_ptr<HaloTransport> t);
  // Slot-stream mode: slot k exchanges its halos through its own transport
  // (e.g. one RCCL communicator per slot, so each communicator's operations
  // stay in one stream's order on every rank).
  void set_slot_transport(int k, std::shared_ptr<HaloTransport> t);
  // Enqueue one image: host_in holds frame rows [in_r0, in_r1) (ghost rows
  // allowed), host_out receives the owned rows.  Host buffers must be pinned
  // and must stay untouched until drain(): submit() never blocks the host, so
  // later submits say nothing about when this image's copies have run.
  void submit(const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out, int reps);
  void drain();
  int64_t submitted() const { return count_; }
  // Images head-streamed so far (submitted to an idle pipeline, at least
  // EngineOptions::stream_min_bytes of input).
  int64_t streamed_heads() const { return streamed_heads_; }
  // True when slots run their repetitions on separate compute streams.
  bool concurrent() const { return concurrent_; }
  bool graphs() const { return graphs_; }
  bool step_graphs() const { return graphs_ && step_graphs_; }
  // Stage timeline of the next `images` submits (not with captured step
  // graphs): per image {slot, H2D start, H2D end, reps end, D2H end} in ms
  // from the first image's H2D start, read after drain().  Timing events
  // between the stages: a few microseconds per image of extra work.
  void enable_trace(int images);
  std::vector<std::vector<double>> trace();
  // Completion marks (any mode, captured step graphs included): the next
  // `images` submits each record a timing event on the stream their image
  // completes on, right after the image's work (a marker between two graph
  // launches; the graphs themselves are untouched), and the first also one
  // before it.  marks() (after drain()) returns per image {slot, ms from the
  // first image's issue to its completion, 1 if it was head-streamed}: a
  // diagnostic pass only (bench.py's window replays), never the timed one.
  void enable_marks(int images);
  std::vector<std::vector<double>> marks();
  // Slot-stream mode: has slot k's latest image completed (its output buffer
  // final)?  wait_image(k) blocks until it has — one image, not the drain.
  bool ready(int k);
  void wait_image(int k);

 private:
  void trace_mark(int stage, hipStream_t s);
  void completion_mark(int k, bool before, bool streamed);
  void submit_image(int k, const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out, int reps);
  // EngineOptions::lazy_head: the held-back first image of a burst; issue it
  // streamed (nothing follows) or as a step graph (a burst follows).
  struct HeldImage {
    const uint8_t* in = nullptr;
    int64_t r0 = 0, r1 = 0;
    uint8_t* out = nullptr;
    int reps = 0;
    bool valid = false;
  };
  HeldImage held_;
  bool force_graph_ = false;
  void issue_held(bool streamed);
  Stream h2d_, d2h_, comm_;
  std::vector<Stream> computes_;
  std::vector<Stream> slot_comms_;  // slot_comm: one communication stream per slot
  bool concurrent_ = false;
  bool graphs_ = false;  // slot-stream mode
  bool step_graphs_ = true;
  std::vector<std::unique_ptr<BandEngine>> slots_;
  std::vector<Event> ev_up_, ev_done_, ev_free_, ev_halo_;
  // step-graph mode with stream_chunks > 1: images submitted while nothing is
  // in flight (after construction / drain) are row-streamed (head streaming)
  int64_t burst_pos_ = 0;  // images submitted since the last drain (0: the pipeline is idle)
  int64_t streamed_heads_ = 0;
  bool head_streaming_ = false;  // stream_chunks > 1 with step graphs
  bool head_on_slots_ = false;   // the head's copies on the next two slots' streams
  Event ev_head_, h2d_wait_;
  std::vector<bool> used_;
  int64_t count_ = 0;
  std::vector<Event> trace_ev_;  // 4 per traced image
  std::vector<int> trace_slot_;
  int64_t trace_first_ = 0;
  std::vector<Event> done_;     // slot-stream mode: per slot, its latest image done (timing events)
  Event burst_start_;           // slot-stream mode: before the first image of the latest burst
  std::vector<Event> mark_ev_;  // [0] = before the first image, [1 + i] = image i done
  std::vector<std::pair<int, bool>> mark_info_;  // (slot, head-streamed) per marked image
  int64_t mark_first_ = 0;
};

// N row bands of one image on ONE device, halos moved by D2D copies.  Used to
// validate the decomposition + schedule on a 1-GPU box: the
// result must equal the single-band result bit for bit.
class LocalCluster {
 public:
  LocalCluster(const ImageGeom& geom, int bands, const Filter& filter, const EngineOptions& opt);
  int size() const { return static_cast<int>(engines_.size()); }
  BandEngine& engine(int i) { return *engines_.at(i); }
  // Host image (contiguous) in/out.
  void upload(const uint8_t* host, bool preload_halo);
  // device_async = false: phase by phase with host synchronisation (exchange,
  // sync, compute, sync).  true: every band enqueues its phases through the
  // production path (comm stream || interior launch, edge launches after the
  // halo event), bands ordered only by per-phase events — the overlap and
  // event ordering of a real multi-GPU rank, with D2D copies as transport.
  void run(int reps, bool device_async = false);
  void download(uint8_t* host);
  void synchronize();

 private:
  ImageGeom geom_;
  std::vector<std::unique_ptr<BandEngine>> engines_;
  std::vector<Event> ev_phase_;  // per band: end of its previous phase
};

// Timing-only transport: moves nothing.  Measures a band's compute schedule
// (launches, shrinking ghost regions) on one GPU without its peers.  Results
// of bands with neighbours are NOT correct under it.
class NullTransport : public HaloTransport {
 public:
  void exchange(BandEngine&, int64_t, hipStream_t) override {}
  const char* name() const override { return "null (timing only)"; }
  bool capturable() const override { return true; }
};

// Transport used by LocalCluster (neighbour engines live on the same device).
// Not capturable: its D2D copies read a peer engine's frame, and only
// LocalCluster's per-phase events order them after the peer's work — a
// captured graph would carry no dependency on the peer's stream.
class LocalTransport : public HaloTransport {
 public:
  explicit LocalTransport(std::vector<BandEngine*> peers) : peers_(std::move(peers)) {}
  void exchange(BandEngine& e, int64_t depth, hipStream_t stream) override;
  const char* name() const override { return "local-d2d"; }
  bool capturable() const override { return false; }

 private:
  std::vector<BandEngine*> peers_;
};

}  // namespace pconv
