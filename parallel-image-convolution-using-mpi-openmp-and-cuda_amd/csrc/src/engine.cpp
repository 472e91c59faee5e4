// BandEngine / LocalCluster (see engine.hpp).
#include "pconv/engine.hpp"

#include <cstring>

#include "pconv/trace.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <thread>

namespace pconv {

namespace {

PlanConfig engine_plan_config(const ImageGeom& geom, const Band& band, const Filter& f, const EngineOptions& opt) {
  PlanConfig c;
  c.fuse = supports_fusion(f, opt.variant) ? opt.fuse : 1;
  c.halo_depth = opt.halo_depth;
  c.overlap = opt.overlap;
  // Every rank must derive the same D and T: clamp against the smallest band.
  const int64_t min_rows = band.world > 1 ? geom.height / band.world : 0;
  return normalize_plan_config(c, min_rows, kMaxFusedSteps);
}

}  // namespace

BandEngine::BandEngine(const ImageGeom& geom, const Band& band, const Filter& filter, const EngineOptions& opt)
    : geom_(geom), band_(band), filter_(filter), opt_(opt) {
  geom_.validate();
  PCONV_CHECK(band.rows >= 1 && band.y0 >= 0 && band.y0 + band.rows <= geom.height, "band outside image");
  const PlanConfig c = engine_plan_config(geom_, band_, filter_, opt_);
  opt_.fuse = c.fuse;
  opt_.halo_depth = c.halo_depth;
  set_device(opt_.device);
  lay_ = FrameLayout::make(geom_.row_bytes(), band_.rows, std::max(1, opt_.halo_depth));
  if (opt_.compute_stream) {
    cs_ = opt_.compute_stream;
  } else {
    own_cs_ = Stream::create(0);
    cs_ = own_cs_.get();
  }
  // Zero the frames on the compute stream (not the null stream: a one-shot
  // process then creates one hardware queue instead of two, ~10 ms each on
  // first use; profiles/r02/raw/init_*.jsonl).
  for (auto& f : frame_) {
    f = DeviceBuffer(static_cast<size_t>(lay_.bytes()));
    if (opt_.kernel_copies)
      launch_fill_zero(f.data(), static_cast<int64_t>(f.size()), cs_);
    else
      PCONV_HIP_CHECK(hipMemsetAsync(f.data(), 0, f.size(), cs_));
  }
  // Communication stream only when the band has neighbours (or is borrowed).
  if (opt_.comm_stream) {
    ms_ = opt_.comm_stream;
  } else if ((band_.up >= 0 || band_.down >= 0) && (!opt_.capture_exchanges || opt_.overlap)) {
    // (captured exchanges with overlap: the interior launch of an exchange
    // phase is forked onto this stream inside the capture, enqueue_phase)
    own_ms_ = Stream::create(-1);  // communication gets the higher priority
    ms_ = own_ms_.get();
  } else {
    ms_ = cs_;
  }
  ev_ready_ = Event::create();
  ev_halo_ = Event::create();
  ev_sync_ = Event::create();
  ev_t0_ = Event::create(true);
  ev_t1_ = Event::create(true);
  PCONV_HIP_CHECK(hipStreamSynchronize(cs_));
}

BandEngine::~BandEngine() {
  // Drain first: a cached graph may still be executing on the stream.
  if (cs_) (void)hipStreamSynchronize(cs_);
  if (ms_ && ms_ != cs_) (void)hipStreamSynchronize(ms_);
  for (auto& kv : graphs_) (void)hipGraphExecDestroy(kv.second);
  for (auto& kv : step_graphs_) (void)hipGraphExecDestroy(kv.second.exec);
}

void BandEngine::trim_graph_caches() {
  // Only the cache that reached its bound is emptied (the other keeps its
  // still-valid graphs).
  const bool g = graphs_.size() >= kMaxCachedGraphs, sg = step_graphs_.size() >= kMaxCachedGraphs;
  if (!g && !sg) return;
  PCONV_HIP_CHECK(hipStreamSynchronize(cs_));  // no cached graph may still be running
  if (g) {
    for (auto& kv : graphs_) PCONV_HIP_CHECK(hipGraphExecDestroy(kv.second));
    graphs_.clear();
  }
  if (sg) {
    for (auto& kv : step_graphs_) PCONV_HIP_CHECK(hipGraphExecDestroy(kv.second.exec));
    step_graphs_.clear();
  }
}

void BandEngine::clear() {
  synchronize();
  for (auto& f : frame_) PCONV_HIP_CHECK(hipMemsetAsync(f.data(), 0, f.size(), cs_));
  PCONV_HIP_CHECK(hipStreamSynchronize(cs_));
  halo_valid_ = false;
}

void BandEngine::upload_rows(const uint8_t* host, int64_t host_pitch, int64_t r_begin, int64_t r_end,
                             hipStream_t stream) {
  PCONV_CHECK(r_begin >= -lay_.halo && r_end <= lay_.rows + lay_.halo && r_begin <= r_end,
              "upload_rows: rows outside frame");
  PCONV_CHECK(host_pitch >= lay_.row_bytes, "upload_rows: host pitch < row bytes");
  // Rows beyond the global image edge must stay zero.
  PCONV_CHECK(band_.y0 + r_begin >= 0 && band_.y0 + r_end <= geom_.height, "upload_rows: rows outside image");
  if (r_end == r_begin) return;
  if (opt_.kernel_copies) {
    launch_copy_rows(host, host_pitch, src_frame() + r_begin * lay_.pitch, lay_.pitch, lay_.row_bytes,
                     r_end - r_begin, stream ? stream : cs_);
    return;
  }
  PCONV_HIP_CHECK(hipMemcpy2DAsync(src_frame() + r_begin * lay_.pitch, lay_.pitch, host, host_pitch, lay_.row_bytes,
                                   r_end - r_begin, hipMemcpyHostToDevice, stream ? stream : cs_));
}

void BandEngine::upload_rows_device(const uint8_t* dev, int64_t dev_pitch, int64_t r_begin, int64_t r_end) {
  PCONV_CHECK(r_begin >= -lay_.halo && r_end <= lay_.rows + lay_.halo && r_begin <= r_end,
              "upload_rows_device: rows outside frame");
  PCONV_CHECK(band_.y0 + r_begin >= 0 && band_.y0 + r_end <= geom_.height, "upload_rows_device: rows outside image");
  if (r_end == r_begin) return;
  PCONV_HIP_CHECK(hipMemcpy2DAsync(src_frame() + r_begin * lay_.pitch, lay_.pitch, dev, dev_pitch, lay_.row_bytes,
                                   r_end - r_begin, hipMemcpyDeviceToDevice, cs_));
}

void BandEngine::download_rows(uint8_t* host, int64_t host_pitch, int64_t r_begin, int64_t r_end,
                               hipStream_t stream) {
  PCONV_CHECK(r_begin >= 0 && r_end <= lay_.rows && r_begin <= r_end, "download_rows: rows outside band");
  if (r_end == r_begin) return;
  if (opt_.kernel_copies) {
    launch_copy_rows(src_frame() + r_begin * lay_.pitch, lay_.pitch, host, host_pitch, lay_.row_bytes, r_end - r_begin,
                     stream ? stream : cs_);
    return;
  }
  PCONV_HIP_CHECK(hipMemcpy2DAsync(host, host_pitch, src_frame() + r_begin * lay_.pitch, lay_.pitch, lay_.row_bytes,
                                   r_end - r_begin, hipMemcpyDeviceToHost, stream ? stream : cs_));
}

void BandEngine::download_rows_device(uint8_t* dev, int64_t dev_pitch, int64_t r_begin, int64_t r_end) {
  PCONV_CHECK(r_begin >= 0 && r_end <= lay_.rows && r_begin <= r_end, "download_rows_device: rows outside band");
  if (r_end == r_begin) return;
  PCONV_HIP_CHECK(hipMemcpy2DAsync(dev, dev_pitch, src_frame() + r_begin * lay_.pitch, lay_.pitch, lay_.row_bytes,
                                   r_end - r_begin, hipMemcpyDeviceToDevice, cs_));
}

void BandEngine::read_frame_rows(uint8_t* host, int64_t r_begin, int64_t r_end) {
  PCONV_CHECK(r_begin >= -lay_.halo && r_end <= lay_.rows + lay_.halo && r_begin <= r_end,
              "read_frame_rows: rows outside frame");
  synchronize();
  if (r_end == r_begin) return;
  PCONV_HIP_CHECK(hipMemcpy2D(host, lay_.row_bytes, src_frame() + r_begin * lay_.pitch, lay_.pitch, lay_.row_bytes,
                              r_end - r_begin, hipMemcpyDeviceToHost));
}

void BandEngine::wait_stream(hipStream_t s) {
  ev_sync_.record(s);
  ev_sync_.wait_on(cs_);
}

void BandEngine::signal_stream(hipStream_t s) {
  ev_sync_.record(cs_);
  ev_sync_.wait_on(s);
}

std::vector<Phase> BandEngine::plan(int reps) const {
  PlanConfig c = engine_plan_config(geom_, band_, filter_, opt_);
  c.halo_preloaded = halo_valid_;
  return plan_band(band_, reps, c);
}

StencilLaunch BandEngine::make_launch(const LaunchSpec& l, int cur) const {
  StencilLaunch a;
  a.src = frame_[cur].data() + lay_.offset(0);
  a.dst = frame_[cur ^ 1].data() + lay_.offset(0);
  a.pitch = lay_.pitch;
  a.row_bytes = lay_.row_bytes;
  a.r0 = l.lo;
  a.r1 = l.hi;
  a.frame_lo = -lay_.halo;
  a.frame_hi = lay_.rows + lay_.halo;
  a.steps = l.steps;
  a.g_row0 = band_.y0;
  a.height = geom_.height;
  return a;
}

void BandEngine::prepare(const std::vector<Phase>& ph) {
  // Tuning times real launches.  Every candidate runs frame_[cur_] ->
  // frame_[cur_ ^ 1] whatever the phase parity: the live input (and its
  // pre-loaded ghost rows) in frame_[cur_] is only ever READ here, and the
  // scratch frame is overwritten by the first phase anyway.  The tune key
  // depends only on (channels, steps, rows, row bytes), not on the frames.
  for (const auto& p : ph)
    for (const auto& l : p.launches)
      prepare_stencil(filter_, geom_.channels, make_launch(l, cur_), cs_, opt_.variant);
}

bool BandEngine::input_preloaded(int64_t in_r0, int64_t in_r1) const {
  if (in_r0 == 0 && in_r1 == band_.rows) return false;
  // Ghost rows are either absent or the full valid depth on BOTH sides
  // (clipped at the global image edge): anything else would leave stale or
  // zero ghost rows that the planner believes valid.
  const int64_t want_lo = -std::min<int64_t>(lay_.halo, band_.y0);
  const int64_t want_hi = band_.rows + std::min<int64_t>(lay_.halo, geom_.height - (band_.y0 + band_.rows));
  PCONV_CHECK(in_r0 == want_lo && in_r1 == want_hi,
              "input rows [" + std::to_string(in_r0) + ", " + std::to_string(in_r1) +
                  ") are neither the owned rows [0, " + std::to_string(band_.rows) +
                  ") nor the owned rows plus the full ghost zone [" + std::to_string(want_lo) + ", " +
                  std::to_string(want_hi) + ")");
  return true;
}

void BandEngine::launch(const LaunchSpec& l, hipStream_t s) {
  const StencilLaunch a = make_launch(l, cur_);
  launch_stencil(filter_, geom_.channels, a, s, opt_.variant);
  ++stats_.launches;
}

void BandEngine::enqueue_phase(const Phase& p) {
  TraceRange tr(p.exchange_depth > 0 ? "pconv.phase.exchange" : "pconv.phase.compute");
  if (p.exchange_depth > 0) {
    PCONV_CHECK(transport_ != nullptr, "band has neighbours but no halo transport is attached");
    hipStream_t ms = comm_stream();
    const bool split = ms != cs_;  // one stream: stream order is the dependency
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (split && hipStreamIsCapturing(cs_, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone) {
      // Inside a graph capture the roles swap: the exchange stays on the
      // capturing stream and the INTERIOR launch goes to the forked one.
      // torch's bundled HIP 7.0 runtime recurses without end (stack overflow
      // in hipStreamEndCapture) on a capture whose RCCL kernel sits on a
      // stream that joined it through an event; ROCm 7.2's runtime does not
      // (profiles/r03/capture/fork/, `rccl_capture_probe(op="*_fork")`).
      ev_ready_.record(cs_);
      ev_ready_.wait_on(ms);
      for (const auto& l : p.launches)
        if (!l.after_halo) launch(l, ms);
      transport_->exchange(*this, p.exchange_depth, cs_);
      for (const auto& l : p.launches)
        if (l.after_halo) launch(l, cs_);
      ev_halo_.record(ms);  // join: the interior rows are final before the next phase
      ev_halo_.wait_on(cs_);
      ++stats_.exchanges;
      cur_ ^= 1;
      return;
    }
    if (split) {
      ev_ready_.record(cs_);
      ev_ready_.wait_on(ms);
    }
    // Interior launch FIRST in host order: it needs no ghost row, so the GPU
    // starts it at once while the host is still inside the transport's
    // enqueue (ncclGroupEnd costs ~10 us of host time); the halo transfer
    // then runs under it instead of ahead of it.
    for (const auto& l : p.launches)
      if (!l.after_halo) launch(l, cs_);
    transport_->exchange(*this, p.exchange_depth, ms);
    if (split) {
      ev_halo_.record(ms);
      ev_halo_.wait_on(cs_);
    }
    for (const auto& l : p.launches)
      if (l.after_halo) launch(l, cs_);
    ++stats_.exchanges;
  } else {
    for (const auto& l : p.launches) launch(l, cs_);
  }
  cur_ ^= 1;
}

void BandEngine::exchange_now(hipStream_t stream) {
  if (band_.up < 0 && band_.down < 0) {
    halo_valid_ = true;
    return;
  }
  PCONV_CHECK(transport_ != nullptr, "band has neighbours but no halo transport is attached");
  transport_->exchange(*this, lay_.halo, stream ? stream : ms_);
  halo_valid_ = true;
  ++pre_exchanges_;
}

void BandEngine::run(int reps) {
  TraceRange tr("pconv.run");
  PCONV_CHECK(reps >= 0, "repetitions must be >= 0");
  const std::vector<Phase> ph = plan(reps);
  stats_ = RunStats{};
  stats_.exchanges = pre_exchanges_;
  pre_exchanges_ = 0;
  wall_t0_ = wall_seconds();
  if (opt_.timing) ev_t0_.record(cs_);
  bool graph = opt_.use_graph && !ph.empty();
  // exchanges join the graph only through a capturable transport
  // (opt_.capture_exchanges): on the compute stream, or — with a
  // communication stream (overlap) — forked: the exchange on the capturing
  // stream beside the interior launch, the edges after it (enqueue_phase)
  const bool cap_x = opt_.capture_exchanges && transport_ && transport_->capturable();
  for (const auto& p : ph) graph = graph && (p.exchange_depth == 0 || cap_x);
  if (graph) {
    const auto key = std::make_pair(reps, cur_);
    auto it = graphs_.find(key);
    if (it == graphs_.end()) {
      trim_graph_caches();
      hipGraph_t g = nullptr;
      prepare(ph);
      PCONV_HIP_CHECK(hipStreamBeginCapture(cs_, hipStreamCaptureModeThreadLocal));
      for (const auto& p : ph) enqueue_phase(p);
      PCONV_HIP_CHECK(hipStreamEndCapture(cs_, &g));
      hipGraphExec_t ex = nullptr;
      PCONV_HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
      PCONV_HIP_CHECK(hipGraphDestroy(g));
      it = graphs_.emplace(key, ex).first;
    } else {
      for (const auto& p : ph) {
        stats_.launches += static_cast<int>(p.launches.size());
        if (p.exchange_depth > 0) ++stats_.exchanges;
        cur_ ^= 1;
      }
    }
    PCONV_HIP_CHECK(hipGraphLaunch(it->second, cs_));
  } else {
    for (const auto& p : ph) enqueue_phase(p);
  }
  if (opt_.timing) {
    ev_t1_.record(cs_);
    timing_pending_ = true;
  }
  halo_valid_ = false;
}

bool BandEngine::exchange_free(int reps, bool halo_preloaded) const {
  PlanConfig c = engine_plan_config(geom_, band_, filter_, opt_);
  c.halo_preloaded = halo_preloaded;
  for (const auto& p : plan_band(band_, reps, c))
    if (p.exchange_depth > 0) return false;
  return true;
}

StreamPlan BandEngine::stream_plan(int reps, int64_t in_r0, int64_t in_r1) const {
  StreamPlan sp;
  if (opt_.stream_chunks < 2 || reps < 1) return sp;
  PlanConfig c = engine_plan_config(geom_, band_, filter_, opt_);
  c.halo_preloaded = input_preloaded(in_r0, in_r1);
  const std::vector<Phase> ph = plan_band(band_, reps, c);
  if (!streamable(ph)) return sp;
  const std::vector<int64_t> cuts = opt_.stream_weights.empty()
                                        ? stream_cuts(in_r0, in_r1, opt_.stream_chunks)
                                        : stream_cuts_weighted(in_r0, in_r1, opt_.stream_weights);
  return plan_streamed(ph, in_r0, in_r1, band_.rows, cuts);
}

hipStream_t BandEngine::enqueue_streamed(const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out,
                                         const StreamPlan& sp, hipStream_t up, hipStream_t down,
                                         hipStream_t up2) {
  TraceRange tr("pconv.streamed_image");
  PCONV_CHECK(!sp.chunks.empty(), "enqueue_streamed: empty stream plan");
  PCONV_CHECK(sp.chunks.front().up_lo == in_r0 && sp.chunks.back().up_hi == in_r1,
              "enqueue_streamed: plan does not match the input rows");
  PCONV_CHECK(band_.y0 + in_r0 >= 0 && band_.y0 + in_r1 <= geom_.height && in_r0 >= -lay_.halo &&
                  in_r1 <= lay_.rows + lay_.halo,
              "enqueue_streamed: input rows outside frame / image");
  const int64_t rb = lay_.row_bytes, p = lay_.pitch;
  stats_ = RunStats{};
  const int c0 = cur_;
  uint8_t* in_frame = frame_at(c0);
  const uint8_t* out_frame = frame_at(c0 + sp.levels);
  const size_t nc = sp.chunks.size();
  reserve_stream_events(nc);
  // Hand-offs by events: stream memory operations instead (the producer
  // writes a sequence number, the consumer's queue waits for the word;
  // hipStreamWriteValue32 / hipStreamWaitValue32) passed the device-side
  // waits sooner but cost more on the host: one image 0.557-0.571 vs
  // 0.534-0.551 ms (profiles/r06/p/).
  // Host issue order: every upload first (the H2D stream then runs them back
  // to back instead of waiting for the host to issue the next one behind the
  // previous chunk's launches), then each chunk's launches behind its
  // upload's event, then each download behind its chunk's event (issuing
  // each download right after its own chunk's launches measured no better:
  // 0.5375-0.5378 vs 0.5197-0.5377 ms per image, profiles/r06/r/).  One event
  // per chunk and direction (no re-recorded event is waited on).
  // Chunk copies are SDMA copies: CU copy kernels beside the launches
  // measured slower (0.76-1.02 vs 0.55 ms per image, profiles/r04/verify/).
  auto copy = [&](uint8_t* dst, int64_t dpitch, const uint8_t* src, int64_t spitch, int64_t rows, hipMemcpyKind kind,
                  hipStream_t s) {
    if (rows > 0) PCONV_HIP_CHECK(hipMemcpy2DAsync(dst, dpitch, src, spitch, rb, rows, kind, s));
  };
  auto launches = [&](const StreamChunk& ch) {
    for (size_t i = 0; i < ch.launches.size(); ++i) {
      launch_stencil(filter_, geom_.channels, make_launch(ch.launches[i], (c0 + ch.levels[i] - 1) & 1),
                     cs_, opt_.variant);
      ++stats_.launches;
    }
  };
  auto download = [&](const StreamChunk& ch, hipStream_t s) {
    if (ch.down_hi > ch.down_lo && host_out)
      copy(host_out + ch.down_lo * rb, rb, out_frame + ch.down_lo * p, p, ch.down_hi - ch.down_lo,
           hipMemcpyDeviceToHost, s);
  };
  auto up_of = [&](size_t c) { return (c & 1) && up2 ? up2 : up; };
  // diagnostics (stream_trace): timing events at the start, after each
  // chunk's upload, launches and download — [0] start, then 3 per chunk
  const bool tr_on = stream_trace_;
  if (tr_on) {
    while (st_ev_.size() < 1 + 5 * nc) st_ev_.push_back(Event::create(true));
    st_chunks_ = nc;
    st_ev_[0].record(up);
  }
  for (size_t c = 0; c < nc; ++c) {
    const StreamChunk& ch = sp.chunks[c];
    copy(in_frame + ch.up_lo * p, p, host_in + (ch.up_lo - in_r0) * rb, rb, ch.up_hi - ch.up_lo,
         hipMemcpyHostToDevice, up_of(c));
    if (up_of(c) != cs_) up_evs_[c].record(up_of(c));
    if (tr_on) st_ev_[1 + 5 * c].record(up_of(c));
  }
  bool pending = false;  // launches not yet covered by a download-side event
  for (size_t c = 0; c < nc; ++c) {
    const StreamChunk& ch = sp.chunks[c];
    if (up_of(c) != cs_) up_evs_[c].wait_on(cs_);
    if (tr_on) st_ev_[2 + 5 * c].record(cs_);
    launches(ch);
    if (tr_on) st_ev_[3 + 5 * c].record(cs_);
    if (!ch.launches.empty()) pending = true;
    if (ch.down_hi > ch.down_lo && host_out) {
      dn_evs_[c].record(cs_);
      pending = false;
    }
  }
  // `down` finishing must mean the whole image is done (the next image of
  // these frames waits on it), also when launches follow the last download.
  if (pending) dn_evs_[nc].record(cs_);
  for (size_t c = 0; c < nc; ++c) {
    const StreamChunk& ch = sp.chunks[c];
    if (!(ch.down_hi > ch.down_lo && host_out)) continue;
    dn_evs_[c].wait_on(down);
    if (tr_on) st_ev_[4 + 5 * c].record(down);
    download(ch, down);
    if (tr_on) st_ev_[5 + 5 * c].record(down);
  }
  if (pending) dn_evs_[nc].wait_on(down);
  cur_ = (c0 + sp.levels) & 1;
  halo_valid_ = false;
  return down;
}

std::vector<std::vector<double>> BandEngine::stream_trace() {
  std::vector<std::vector<double>> out;
  if (!stream_trace_ || st_chunks_ == 0) return out;
  synchronize();
  for (size_t c = 0; c < st_chunks_; ++c) {
    std::vector<double> row{static_cast<double>(c)};
    for (int k = 1; k <= 5; ++k) {
      float ms = -1.f;
      // a chunk without a download never records its events: -1
      if (hipEventElapsedTime(&ms, st_ev_[0].get(), st_ev_[5 * c + static_cast<size_t>(k)].get()) != hipSuccess) {
        (void)hipGetLastError();
        ms = -1.f;
      }
      row.push_back(ms);
    }
    out.push_back(row);
  }
  return out;
}

void BandEngine::process_graph(const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out, int reps) {
  TraceRange tr("pconv.step_graph");
  PCONV_CHECK(reps >= 0, "repetitions must be >= 0");
  // The whole input is uploaded by every step, so the step always starts in
  // frame 0: one cached graph per (reps, buffers) instead of one per start
  // frame (an odd number of launches per image flips the frames, and a step
  // whose start frame was not seen before paid a capture + instantiate
  // inside the first timed images).  All ranks follow the same rule, so
  // neighbours still hold the same time level in the frame of equal parity.
  cur_ = 0;
  halo_valid_ = input_preloaded(in_r0, in_r1);
  std::vector<Phase> ph = plan(reps);
  bool exchanges = false;
  for (const auto& p : ph) exchanges = exchanges || p.exchange_depth > 0;
  // Exchange-mode image: one exchange of the whole ghost zone right after the
  // upload when it covers every repetition, else the plan's exchange phases.
  const bool zone_first = exchanges && reps > 0 && exchange_free(reps, true);
  if (exchanges) {
    PCONV_CHECK(transport_ != nullptr, "band has neighbours but no halo transport is attached");
    PCONV_CHECK(transport_->capturable(),
                std::string("process_graph: this schedule needs halo exchanges and the '") + transport_->name() +
                    "' transport cannot be captured into a graph (pre-load deeper ghost rows or issue directly)");
  }
  if (zone_first) {
    halo_valid_ = true;
    ph = plan(reps);
  }
  const auto key = std::make_tuple(reps, cur_, host_in, in_r0, in_r1, host_out);
  auto it = step_graphs_.find(key);
  stats_ = RunStats{};
  if (it == step_graphs_.end()) {
    trim_graph_caches();
    const int64_t rb = lay_.row_bytes;
    hipGraph_t g = nullptr;
    prepare(ph);  // tile-shape tuning cannot run inside the capture
    PCONV_HIP_CHECK(hipStreamBeginCapture(cs_, hipStreamCaptureModeRelaxed));
    upload_rows(host_in, rb, in_r0, in_r1, cs_);
    if (zone_first) {
      transport_->exchange(*this, lay_.halo, cs_);  // stream order: after the upload, before the launches
      ++stats_.exchanges;
    }
    for (const auto& p : ph) enqueue_phase(p);
    if (host_out) download_rows(host_out, rb, 0, band_.rows, cs_);  // nullptr: the caller downloads itself
    PCONV_HIP_CHECK(hipStreamEndCapture(cs_, &g));
    StepGraph sg;
    PCONV_HIP_CHECK(hipGraphInstantiate(&sg.exec, g, nullptr, nullptr, 0));
    PCONV_HIP_CHECK(hipGraphDestroy(g));
    // its device-side set-up now, not inside the first launch (a slot's graph
    // runs its first image in the warm-up, its second in a timed window)
    PCONV_HIP_CHECK(hipGraphUpload(sg.exec, cs_));
    sg.end_cur = cur_;
    sg.launches = stats_.launches;
    sg.exchanges = stats_.exchanges;
    it = step_graphs_.emplace(key, sg).first;
  } else {
    cur_ = it->second.end_cur;
    stats_.launches = it->second.launches;
    stats_.exchanges = it->second.exchanges;
  }
  PCONV_HIP_CHECK(hipGraphLaunch(it->second.exec, cs_));
  halo_valid_ = false;
}

void BandEngine::exec_exchange(const Phase& p) {
  if (p.exchange_depth <= 0) return;
  PCONV_CHECK(transport_ != nullptr, "band has neighbours but no halo transport is attached");
  transport_->exchange(*this, p.exchange_depth, cs_);
  ++stats_.exchanges;
}

void BandEngine::exec_compute(const Phase& p) {
  for (const auto& l : p.launches) launch(l, cs_);
  cur_ ^= 1;
}

void BandEngine::synchronize() {
  PCONV_HIP_CHECK(hipStreamSynchronize(cs_));
  if (ms_ != cs_) PCONV_HIP_CHECK(hipStreamSynchronize(ms_));
  if (timing_pending_) {
    stats_.loop_ms = Event::elapsed_ms(ev_t0_, ev_t1_);
    stats_.wall_ms = (wall_seconds() - wall_t0_) * 1e3;
    timing_pending_ = false;
  }
}

// --------------------------------------------------------------- BandPipeline

namespace {
// A stream on a hardware queue of its own: created with a CU mask (all CUs),
// it gets a dedicated HSA queue instead of one from the runtime's pool.
Stream own_queue_stream(int device) {
  int n = 0;
  PCONV_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device));
  std::vector<uint32_t> mask(static_cast<size_t>((n + 31) / 32), 0u);
  for (int cu = 0; cu < n; ++cu) mask[static_cast<size_t>(cu / 32)] |= 1u << (cu % 32);
  return Stream::create_cu_masked(mask);
}
}  // namespace

BandPipeline::BandPipeline(const ImageGeom& geom, const Band& band, const Filter& filter, const EngineOptions& opt,
                           int slots, int concurrent, bool graphs, bool step_graphs, bool slot_comm) {
  PCONV_CHECK(slots >= 1 && slots <= 8, "pipeline slots must be in [1, 8]");
  set_device(opt.device);
  if (graphs) {
    // One stream per slot carries that slot's whole image (H2D, reps, D2H) as
    // one graph: slots overlap each other without cross-stream events.
    graphs_ = true;
    step_graphs_ = step_graphs;
    concurrent_ = slots > 1;
    EngineOptions o = opt;
    // Directly issued images (exchange mode) replay their repetitions as the
    // engine's cached rep-loop graph whenever no exchange phase remains.
    o.use_graph = !step_graphs;
    o.timing = false;
    // Without slot_comm an image's exchange and launches share its stream:
    // no split launches.  With it, each slot's exchanges run on the slot's
    // own communication stream beside the interior launch.
    o.overlap = slot_comm && opt.overlap;
    // Slot streams on dedicated hardware queues (opt.cu_mask_queues): a
    // stream created with a CU mask (all CUs) gets its own HSA queue instead
    // of one from the runtime's round-robin pool.  From the pool, 4 slot
    // streams landed on queues of which two ran every stencil launch ~5x
    // longer (p50 47 vs 9.6 us; the 8-way proxy step 0.106 vs 0.055 ms at 3
    // slots); with CU-masked queues 4 slots run at 0.053 ms
    // (docs/PERFORMANCE.md §2, profiles/r04/slots_b/).
    for (int i = 0; i < slots; ++i) {
      computes_.push_back(opt.cu_mask_queues ? own_queue_stream(opt.device) : Stream::create(0));
      o.compute_stream = computes_.back().get();
      if (slot_comm) {
        slot_comms_.push_back(Stream::create(-1));
        o.comm_stream = slot_comms_.back().get();
      } else {
        o.comm_stream = computes_.back().get();
      }
      slots_.push_back(std::make_unique<BandEngine>(geom, band, filter, o));
    }
    if (step_graphs && opt.stream_chunks > 1) {
      // head streaming: copy streams for images submitted to an idle pipeline.
      // With >= 3 slots and opt.head_on_slot_streams the head's upload and
      // download run on the next two slots' streams (idle when the pipeline
      // is; the download on the slot a burst reaches last): no hardware queue
      // beyond the slots'.  Two more queues from the
      // runtime's pool made one image 0.77 ms with 4 slots, dedicated
      // (CU-masked) ones 0.85 ms, the slots' streams 0.56 ms
      // (profiles/r04/head/).  Otherwise: two pool streams.
      head_on_slots_ = opt.head_on_slot_streams && slots >= 3;
      if (!head_on_slots_) {
        h2d_ = Stream::create(0);
        d2h_ = Stream::create(0);
      }
      ev_head_ = Event::create();
      h2d_wait_ = Event::create();
      head_streaming_ = true;
      // Every slot may stream a head image (the window's first slot is
      // count % slots): its events now, and one direct H2D and one direct D2H
      // of a row on every slot stream — the streams a head image borrows for
      // its chunk copies — so no first-use set-up of a stream's copies lands
      // in the first window that borrows it.
      const size_t nchunks = std::max(static_cast<size_t>(std::max(opt.stream_chunks, 0)), opt.stream_weights.size());
      for (auto& e : slots_) e->reserve_stream_events(nchunks + 1);
      const int64_t rb = slots_[0]->layout().row_bytes;
      PinnedBuffer row(static_cast<size_t>(rb));
      std::memset(row.data(), 0, row.size());
      for (auto& e : slots_) {
        e->upload_rows(row.data(), rb, 0, 1, e->compute_stream());
        e->download_rows(row.data(), rb, 0, 1, e->compute_stream());
      }
      for (auto& e : slots_) e->synchronize();
    }
    used_.assign(slots, false);
    for (int i = 0; i < slots; ++i) done_.push_back(Event::create(true));
    burst_start_ = Event::create(true);
    return;
  }
  // Streams: H2D, D2H, communication (only with neighbours) and compute.
  // HIP maps streams round-robin onto GPU_MAX_HW_QUEUES hardware queues (4 by
  // default); two busy streams on one queue serialise falsely.  When the
  // queue budget allows, every slot gets its own compute stream so that
  // consecutive images run their repetitions CONCURRENTLY — a small band (the
  // 8-GPU split of a small image) fills only part of the chip per launch, two
  // images in flight fill it.  Otherwise all slots share one compute stream.
  const bool nb = band.up >= 0 || band.down >= 0;
  int hw_queues = 4;
  if (const char* q = std::getenv("GPU_MAX_HW_QUEUES")) hw_queues = std::max(1, std::atoi(q));
  const int fixed = 2 + (nb ? 1 : 0);
  concurrent_ = concurrent < 0 ? (slots > 1 && hw_queues >= fixed + slots) : (concurrent > 0 && slots > 1);
  h2d_ = Stream::create(0);
  d2h_ = Stream::create(0);
  EngineOptions o = opt;
  o.use_graph = false;  // copies/events interleave with the loop
  o.timing = false;     // host time per image matters here (see tools/ubench/api_cost.hip)
  if (nb) {
    comm_ = Stream::create(-1);
    o.comm_stream = comm_.get();
  }
  for (int i = 0; i < (concurrent_ ? slots : 1); ++i) computes_.push_back(Stream::create(0));
  for (int i = 0; i < slots; ++i) {
    o.compute_stream = computes_[concurrent_ ? i : 0].get();
    slots_.push_back(std::make_unique<BandEngine>(geom, band, filter, o));
    ev_up_.push_back(Event::create());
    ev_done_.push_back(Event::create());
    ev_free_.push_back(Event::create());
    ev_halo_.push_back(Event::create());
  }
  used_.assign(slots, false);
}

BandPipeline::~BandPipeline() {
  if (h2d_.get()) (void)hipStreamSynchronize(h2d_.get());
  for (auto& c : computes_) (void)hipStreamSynchronize(c.get());
  for (auto& c : slot_comms_) (void)hipStreamSynchronize(c.get());
  if (d2h_.get()) (void)hipStreamSynchronize(d2h_.get());
  if (comm_.get()) (void)hipStreamSynchronize(comm_.get());
}

void BandPipeline::set_slot_transport(int k, std::shared_ptr<HaloTransport> t) {
  PCONV_CHECK(graphs_, "per-slot transports need the slot-stream pipeline");
  slots_.at(k)->set_transport(std::move(t));
}

void BandPipeline::set_transport(std::shared_ptr<HaloTransport> t) {
  for (auto& s : slots_) s->set_transport(t);
}

void BandPipeline::submit(const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out, int reps) {
  TraceRange tr("pconv.pipeline.submit");
  if (held_.valid) issue_held(false);  // a burst: its first image as a step graph
  const int k = static_cast<int>(count_ % static_cast<int64_t>(slots_.size()));
  if (graphs_ && step_graphs_ && head_streaming_ && burst_pos_ == 0 && slots_[0]->options().lazy_head) {
    burst_start_.record(slots_[static_cast<size_t>(k)]->compute_stream());
    completion_mark(k, true, false);
    held_ = HeldImage{host_in, in_r0, in_r1, host_out, reps, true};
    return;
  }
  // A burst's first image (nothing in flight) starts behind a timing event on
  // its slot's stream (burst_start_): windows whose first image did so ran
  // 0.3281-0.3309 ms/step against 0.3323-0.3365 without (4 interleaved
  // pairs each, profiles/r06/h/marked_*, plain_*; profiles/r06/i/ shows the
  // per-image completion events below alone do not do it).
  if (graphs_ && burst_pos_ == 0) burst_start_.record(slots_[static_cast<size_t>(k)]->compute_stream());
  completion_mark(k, true, false);
  const int64_t heads = streamed_heads_;
  submit_image(k, host_in, in_r0, in_r1, host_out, reps);
  completion_mark(k, false, streamed_heads_ != heads);
  // The image's completion event, right behind its work on the stream it
  // completes on (ready() / wait_image()).
  if (graphs_) done_[static_cast<size_t>(k)].record(slots_[static_cast<size_t>(k)]->compute_stream());
}

void BandPipeline::issue_held(bool streamed) {
  const HeldImage h = held_;
  held_.valid = false;
  const int k = static_cast<int>(count_ % static_cast<int64_t>(slots_.size()));
  const int64_t heads = streamed_heads_;
  force_graph_ = !streamed;
  submit_image(k, h.in, h.r0, h.r1, h.out, h.reps);
  force_graph_ = false;
  completion_mark(k, false, streamed_heads_ != heads);
  done_[static_cast<size_t>(k)].record(slots_[static_cast<size_t>(k)]->compute_stream());
}

bool BandPipeline::ready(int k) {
  if (held_.valid) issue_held(true);
  const hipError_t e = hipEventQuery(done_.at(static_cast<size_t>(k)).get());
  if (e == hipErrorNotReady) return false;
  PCONV_HIP_CHECK(e);
  return true;
}

void BandPipeline::wait_image(int k) {
  if (held_.valid) issue_held(true);
  done_.at(static_cast<size_t>(k)).sync();
}

void BandPipeline::completion_mark(int k, bool before, bool streamed) {
  if (mark_ev_.empty()) return;
  const int64_t i = count_ - mark_first_ - (before ? 0 : 1);  // this image's index among the marked ones
  if (i < 0 || i + 1 >= static_cast<int64_t>(mark_ev_.size())) return;
  if (before && i != 0) return;
  hipStream_t s = graphs_ ? slots_[static_cast<size_t>(k)]->compute_stream() : (before ? h2d_.get() : d2h_.get());
  if (before) {
    mark_ev_[0].record(s);
    return;
  }
  mark_ev_[static_cast<size_t>(i + 1)].record(s);
  mark_info_.emplace_back(k, streamed);
}

void BandPipeline::enable_marks(int images) {
  PCONV_CHECK(images >= 0, "mark capacity must be >= 0");
  mark_ev_.clear();
  mark_info_.clear();
  if (images == 0) return;
  for (int i = 0; i <= images; ++i) mark_ev_.push_back(Event::create(true));
  mark_first_ = count_;
}

std::vector<std::vector<double>> BandPipeline::marks() {
  drain();
  std::vector<std::vector<double>> out;
  for (size_t i = 0; i < mark_info_.size(); ++i)
    out.push_back({static_cast<double>(mark_info_[i].first), Event::elapsed_ms(mark_ev_[0], mark_ev_[i + 1]),
                   mark_info_[i].second ? 1.0 : 0.0});
  mark_ev_.clear();
  mark_info_.clear();
  return out;
}

void BandPipeline::submit_image(int k, const uint8_t* host_in, int64_t in_r0, int64_t in_r1, uint8_t* host_out,
                                int reps) {
  BandEngine& e = *slots_[static_cast<size_t>(k)];
  if (graphs_ && !step_graphs_) {
    // Everything of this image on the slot's stream; halo exchanges (if the
    // ghost rows are not pre-loaded) through this slot's own transport, in
    // stream order between the upload and the launches.
    const bool preloaded = e.input_preloaded(in_r0, in_r1);
    hipStream_t cs = e.compute_stream();
    trace_mark(0, cs);
    e.upload_rows(host_in, e.layout().row_bytes, in_r0, in_r1);
    trace_mark(1, cs);
    if (!preloaded && e.exchange_free(reps, true)) {
      // The ghost zone covers all `reps`: ONE exchange of the whole zone in
      // stream order, then the repetitions need none and run() launches them
      // as one cached graph — an image costs the upload, the transport's
      // calls, one graph launch and the download on the host.
      e.exchange_now(cs);
    } else {
      e.set_halo_valid(preloaded);
    }
    e.run(reps);
    trace_mark(2, cs);
    e.download_rows(host_out, e.layout().row_bytes, 0, e.band().rows);
    trace_mark(3, cs);
    used_[k] = true;
    ++count_;
    return;
  }
  if (graphs_) {
    PCONV_CHECK(trace_ev_.empty(), "pipeline trace needs directly issued images (graph capture off)");
    const int64_t in_bytes = (in_r1 - in_r0) * e.layout().row_bytes;
    // Only the first image of a burst is streamed: streaming the first two
    // (the second on the first head's streams) measured no better — 0.3315-
    // 0.3353 vs 0.3288-0.3328 ms/step, the second head's slot 0.04 ms late
    // in every window (profiles/r06/h/h2_*) — and was removed.
    if (burst_pos_ == 0 && head_streaming_ && !force_graph_ && in_bytes >= e.options().stream_min_bytes) {
      // Head streaming: nothing is in flight, so this image's rows stream
      // (chunked H2D ‖ launches ‖ D2H of finished rows, schedule.hpp
      // plan_streamed) instead of waiting for its whole upload and its
      // whole loop before the first byte comes back — the head of a burst
      // and every single image (latency).  Images behind it run as step
      // graphs; the slot's stream waits for the streamed image's last
      // download before its next graph touches these frames.
      const StreamPlan sp = e.stream_plan(reps, in_r0, in_r1);
      if (!sp.chunks.empty()) {
        e.set_cur(0);  // like process_graph: the whole input is uploaded, start in frame 0
        // The downloads wait on every chunk's launches, so they go on the
        // stream of the slot a burst reaches LAST (k - 1): the burst's next
        // images do not queue behind the head's whole loop.  The uploads are
        // done early and go on slot k + 1's.
        const int n = slots();
        hipStream_t up = head_on_slots_ ? computes_[static_cast<size_t>((k + 1) % n)].get() : h2d_.get();
        hipStream_t down = head_on_slots_ ? computes_[static_cast<size_t>((k + n - 1) % n)].get() : d2h_.get();
        // odd chunks' uploads on slot k+2's stream (EngineOptions::head_alt_uploads)
        hipStream_t up2 = head_on_slots_ && n >= 4 && e.options().head_alt_uploads
                              ? computes_[static_cast<size_t>((k + 2) % n)].get()
                              : nullptr;
        h2d_wait_.record(e.compute_stream());  // earlier work of this slot (its previous graph) first
        h2d_wait_.wait_on(up);
        if (up2) h2d_wait_.wait_on(up2);
        hipStream_t done = e.enqueue_streamed(host_in, in_r0, in_r1, host_out, sp, up, down, up2);
        if (done != e.compute_stream()) {
          ev_head_.record(done);
          ev_head_.wait_on(e.compute_stream());
        }
        ++burst_pos_;
        used_[k] = true;
        ++count_;
        ++streamed_heads_;
        return;
      }
    }
    e.process_graph(host_in, in_r0, in_r1, host_out, reps);
    ++burst_pos_;
    used_[k] = true;
    ++count_;
    return;
  }
  const bool preloaded = e.input_preloaded(in_r0, in_r1);
  // H2D into slot k once its previous image has been downloaded.
  if (used_[k]) ev_free_[k].wait_on(h2d_.get());
  if (e.options().stream_chunks > 1 && trace_ev_.empty()) {
    // Rows streamed within the image: chunk uploads on the H2D stream,
    // launches on the compute stream, finished rows downloaded on the D2H
    // stream, one event pair per chunk (exchange-free images only).
    const StreamPlan sp = e.stream_plan(reps, in_r0, in_r1);
    if (!sp.chunks.empty()) {
      hipStream_t done = e.enqueue_streamed(host_in, in_r0, in_r1, host_out, sp, h2d_.get(), d2h_.get());
      ev_free_[k].record(done);
      used_[k] = true;
      ++count_;
      return;
    }
  }
  trace_mark(0, h2d_.get());
  e.upload_rows(host_in, e.layout().row_bytes, in_r0, in_r1, h2d_.get());
  trace_mark(1, h2d_.get());
  ev_up_[k].record(h2d_.get());
  e.set_halo_valid(preloaded);
  if (!preloaded && comm_.get() && e.has_transport() && reps > 0) {
    // Exchange this image's ghost rows as soon as it is uploaded — on the
    // comm stream, concurrently with the previous image's repetitions.
    ev_up_[k].wait_on(comm_.get());
    e.exchange_now(comm_.get());
    ev_halo_[k].record(comm_.get());
    ev_halo_[k].wait_on(e.compute_stream());
  } else {
    ev_up_[k].wait_on(e.compute_stream());
  }
  // reps on the shared compute stream (later exchanges on the comm stream)
  e.run(reps);
  trace_mark(2, e.compute_stream());
  ev_done_[k].record(e.compute_stream());
  // D2H of the owned rows
  ev_done_[k].wait_on(d2h_.get());
  e.download_rows(host_out, e.layout().row_bytes, 0, e.band().rows, d2h_.get());
  trace_mark(3, d2h_.get());
  ev_free_[k].record(d2h_.get());
  used_[k] = true;
  ++count_;
}

void BandPipeline::enable_trace(int images) {
  PCONV_CHECK(images >= 0, "trace capacity must be >= 0");
  PCONV_CHECK(!step_graphs(), "pipeline trace needs directly issued images (graph capture off)");
  trace_ev_.clear();
  trace_slot_.clear();
  for (int i = 0; i < 4 * images; ++i) trace_ev_.push_back(Event::create(true));
  trace_first_ = count_;
}

void BandPipeline::trace_mark(int stage, hipStream_t s) {
  const int64_t i = count_ - trace_first_;
  if (i < 0 || 4 * i + 3 >= static_cast<int64_t>(trace_ev_.size())) return;
  if (stage == 0) trace_slot_.push_back(static_cast<int>(count_ % static_cast<int64_t>(slots_.size())));
  trace_ev_[4 * i + stage].record(s);
}

std::vector<std::vector<double>> BandPipeline::trace() {
  drain();
  std::vector<std::vector<double>> out;
  for (size_t i = 0; i < trace_slot_.size(); ++i) {
    std::vector<double> row{static_cast<double>(trace_slot_[i])};
    for (int st = 0; st < 4; ++st) row.push_back(Event::elapsed_ms(trace_ev_[0], trace_ev_[4 * i + st]));
    out.push_back(row);
  }
  return out;
}

// Blocking syncs: polling the streams instead (hipStreamQuery in a loop)
// measured within noise for one image (0.5169-0.5411 vs 0.5197-0.5377 ms,
// profiles/r06/r/) and costs a core.
void BandPipeline::drain() {
  if (held_.valid) issue_held(true);  // a single image: row-streamed
  if (h2d_.get()) PCONV_HIP_CHECK(hipStreamSynchronize(h2d_.get()));
  for (auto& s : slots_) s->synchronize();
  if (d2h_.get()) PCONV_HIP_CHECK(hipStreamSynchronize(d2h_.get()));
  burst_pos_ = 0;
}

// --------------------------------------------------------------- LocalCluster

void LocalTransport::exchange(BandEngine& e, int64_t depth, hipStream_t stream) {
  const FrameLayout& L = e.layout();
  const Band& b = e.band();
  const int64_t pitch = L.pitch;
  uint8_t* mine = e.src_frame() - kPadLeft;  // row 0, pitch-aligned start
  // Bands of one cluster advance in lockstep (same phase count per run), so
  // the peer's frame of the same parity holds the same time level — read by
  // parity, not through the peer's current frame, which a device-async run
  // may already have flipped to the next phase.
  const int par = e.cur();
  if (b.up >= 0) {
    BandEngine& p = *peers_.at(b.up);
    PCONV_CHECK(p.layout().pitch == pitch && p.band().rows >= depth, "local halo: incompatible peer");
    const uint8_t* from = p.frame_at(par) - kPadLeft + (p.band().rows - depth) * pitch;
    PCONV_HIP_CHECK(hipMemcpyAsync(mine - depth * pitch, from, depth * pitch, hipMemcpyDeviceToDevice, stream));
  }
  if (b.down >= 0) {
    BandEngine& p = *peers_.at(b.down);
    PCONV_CHECK(p.layout().pitch == pitch && p.band().rows >= depth, "local halo: incompatible peer");
    const uint8_t* from = p.frame_at(par) - kPadLeft;
    PCONV_HIP_CHECK(hipMemcpyAsync(mine + b.rows * pitch, from, depth * pitch, hipMemcpyDeviceToDevice, stream));
  }
}

LocalCluster::LocalCluster(const ImageGeom& geom, int bands, const Filter& filter, const EngineOptions& opt)
    : geom_(geom) {
  const auto bs = row_bands(geom.height, bands);
  std::vector<BandEngine*> peers;
  for (const auto& b : bs) {
    engines_.push_back(std::make_unique<BandEngine>(geom, b, filter, opt));
    peers.push_back(engines_.back().get());
    ev_phase_.push_back(Event::create());
  }
  auto t = std::make_shared<LocalTransport>(peers);
  for (auto& e : engines_) e->set_transport(t);
}

void LocalCluster::upload(const uint8_t* host, bool preload_halo) {
  const int64_t rb = geom_.row_bytes();
  for (auto& e : engines_) {
    const Band& b = e->band();
    const int64_t d = e->layout().halo;
    int64_t rb0 = 0, re = b.rows;
    if (preload_halo) {
      rb0 = -std::min<int64_t>(d, b.y0);
      re = b.rows + std::min<int64_t>(d, geom_.height - (b.y0 + b.rows));
    }
    e->upload_rows(host + (b.y0 + rb0) * rb, rb, rb0, re);
    e->set_halo_valid(preload_halo);
  }
  synchronize();
}

void LocalCluster::run(int reps, bool device_async) {
  std::vector<std::vector<Phase>> plans;
  for (auto& e : engines_) plans.push_back(e->plan(reps));
  const size_t n = plans.front().size();
  for (const auto& p : plans) PCONV_CHECK(p.size() == n, "local cluster: band plans diverge");
  if (device_async) {
    // Every band runs the production phase path (BandEngine::enqueue_phase):
    // the D2D halo copy on its comm stream, the interior launch concurrently
    // on its compute stream, the edge launches after ev_halo — nothing waits
    // on the host.  The only cross-band ordering is one event per band per
    // phase (the MPI_Wait pairs of mpi/mpi_convolution.c:199-234): before
    // phase i a band waits for its neighbours to finish phase i-1, which
    // (a) makes their owned rows final before its exchange reads them and
    // (b) makes their phase i-1 exchange, which read ITS owned rows, done
    // before its phase i launches overwrite that frame.
    const size_t nb = engines_.size();
    for (size_t i = 0; i < n; ++i) {
      for (size_t k = 0; k < nb; ++k) ev_phase_[k].record(engines_[k]->compute_stream());
      for (size_t k = 0; k < nb; ++k) {
        const Band& b = engines_[k]->band();
        for (int peer : {b.up, b.down})
          if (peer >= 0) ev_phase_.at(peer).wait_on(engines_[k]->compute_stream());
      }
      // LocalTransport reads a peer's frame by the exchanging band's parity
      // (frame_at(e.cur())), so enqueueing band k after band k-1 has flipped
      // its frames is safe.
      for (size_t k = 0; k < nb; ++k) engines_[k]->enqueue_phase(plans[k][i]);
    }
    synchronize();
    for (auto& e : engines_) e->set_halo_valid(false);
    return;
  }
  for (size_t i = 0; i < n; ++i) {
    for (size_t k = 0; k < engines_.size(); ++k) engines_[k]->exec_exchange(plans[k][i]);
    synchronize();
    for (size_t k = 0; k < engines_.size(); ++k) engines_[k]->exec_compute(plans[k][i]);
    synchronize();
  }
  for (auto& e : engines_) e->set_halo_valid(false);
}

void LocalCluster::download(uint8_t* host) {
  const int64_t rb = geom_.row_bytes();
  for (auto& e : engines_) e->download_rows(host + e->band().y0 * rb, rb, 0, e->band().rows);
  synchronize();
}

void LocalCluster::synchronize() {
  for (auto& e : engines_) e->synchronize();
}

}  // namespace pconv
