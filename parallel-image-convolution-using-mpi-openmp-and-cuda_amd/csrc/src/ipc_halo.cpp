// HIP-IPC halo transport (see ipc_halo.hpp).
#include "pconv/ipc_halo.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstddef>
#include <cstring>

#include "pconv/trace.hpp"

namespace pconv {

namespace {

size_t segment_bytes(int world, int slots) {
  return static_cast<size_t>(world) * static_cast<size_t>(slots) * sizeof(IpcFlags);
}

std::string shm_path(const std::string& name) { return name.empty() || name[0] != '/' ? "/" + name : name; }

}  // namespace

void ipc_create_segment(const std::string& name, int world, int slots) {
  PCONV_CHECK(world >= 1 && slots >= 1, "ipc segment: bad world / slots");
  const std::string p = shm_path(name);
  const int fd = ::shm_open(p.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  PCONV_CHECK(fd >= 0, "ipc segment: shm_open(" + p + ") failed: " + std::strerror(errno));
  const size_t n = segment_bytes(world, slots);
  const bool ok = ::ftruncate(fd, static_cast<off_t>(n)) == 0;  // zero-filled
  ::close(fd);
  if (!ok) {
    ::shm_unlink(p.c_str());
    PCONV_FAIL("ipc segment: ftruncate failed: " + std::string(std::strerror(errno)));
  }
}

void ipc_unlink_segment(const std::string& name) { (void)::shm_unlink(shm_path(name).c_str()); }

IpcPull parse_ipc_pull(const std::string& s) {
  if (s == "grid") return IpcPull::Grid;
  if (s == "single") return IpcPull::Single;
  if (s == "sdma") return IpcPull::Sdma;
  PCONV_FAIL("unknown IPC pull form '" + s + "' (grid|single|sdma)");
}

const char* ipc_pull_name(IpcPull p) {
  switch (p) {
    case IpcPull::Grid: return "grid";
    case IpcPull::Single: return "single";
    case IpcPull::Sdma: return "sdma";
  }
  return "?";
}

IpcHaloTransport::IpcHaloTransport(BandEngine& e, const std::string& segment, int slot, int slots, double timeout_s,
                                   IpcPull pull)
    : eng_(&e), rank_(e.band().rank), world_(e.band().world), slot_(slot), slots_(slots), segment_(segment),
      pull_(pull) {
  PCONV_CHECK(slot >= 0 && slot < slots, "ipc transport: slot out of range");
  seg_bytes_ = segment_bytes(world_, slots_);
  const std::string p = shm_path(segment);
  const int fd = ::shm_open(p.c_str(), O_RDWR, 0600);
  PCONV_CHECK(fd >= 0, "ipc transport: shm_open(" + p + ") failed: " + std::strerror(errno));
  struct stat st {};
  PCONV_CHECK(::fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= seg_bytes_,
              "ipc transport: flag segment smaller than world x slots blocks");
  host_ = ::mmap(nullptr, seg_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  PCONV_CHECK(host_ != MAP_FAILED, "ipc transport: mmap failed");
  set_device(e.options().device);
  PCONV_HIP_CHECK(hipHostRegister(host_, seg_bytes_, hipHostRegisterMapped));
  void* d = nullptr;
  PCONV_HIP_CHECK(hipHostGetDevicePointer(&d, host_, 0));
  dflags_ = static_cast<IpcFlags*>(d);
  int khz = 0;
  PCONV_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, e.options().device));
  timeout_ticks_ = static_cast<uint64_t>(timeout_s * static_cast<double>(khz > 0 ? khz : 100000) * 1000.0);
  // The mailbox: a whole 2 MiB allocation (never sub-allocated by the
  // runtime, so its IPC handle names exactly this buffer) of UNCACHED device
  // memory — neighbours on other GPUs store into it over xGMI, and no cache
  // of either side may keep a stale copy (ipc_halo.hpp, "Visibility").
  // Fine-grained memory is the second choice; plain (coarse-grained) memory
  // only if the runtime exports neither, and then the connect self-test is
  // what stands between a visibility gap and a 30 s timeout.
  hipIpcMemHandle_t mh{};
  const std::pair<unsigned, const char*> kinds[] = {{hipDeviceMallocUncached, "uncached"},
                                                    {hipDeviceMallocFinegrained, "fine-grained"}};
  for (const auto& k : kinds) {
    void* p = nullptr;
    if (hipExtMallocWithFlags(&p, kMailboxBytes, k.first) != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    if (hipIpcGetMemHandle(&mh, p) != hipSuccess) {
      (void)hipGetLastError();
      (void)hipFree(p);
      continue;
    }
    (void)hipFree(p);  // exportable: allocate it for real (RAII) below
    mail_ = DeviceBuffer(kMailboxBytes, k.first);
    mailbox_kind_ = k.second;
    break;
  }
  if (mailbox_kind_.empty()) {
    mail_ = DeviceBuffer(kMailboxBytes);
    mailbox_kind_ = "coarse-grained";
  }
  PCONV_HIP_CHECK(hipMemset(mail_.data(), 0, kMailboxBytes));
  PCONV_HIP_CHECK(hipDeviceSynchronize());  // zeroed before any neighbour can store into it
  handles_.resize(kIpcHandleBytes);
  for (int i = 0; i < 3; ++i) {
    hipIpcMemHandle_t h;
    void* base = i < 2 ? static_cast<void*>(e.frame_base(i)) : static_cast<void*>(mail_.data());
    if (i < 2) own_base_[i] = e.frame_base(i);
    PCONV_HIP_CHECK(hipIpcGetMemHandle(&h, base));
    std::memcpy(handles_.data() + i * sizeof(h), &h, sizeof(h));
  }
}

IpcHaloTransport::~IpcHaloTransport() {
  for (uint8_t** side : {peer_up_, peer_down_})
    for (int i = 0; i < 2; ++i)
      if (side[i] && side[i] != own_base_[i]) (void)hipIpcCloseMemHandle(side[i]);
  for (IpcMailbox* m : {peer_mail_up_, peer_mail_down_})
    if (m && m != static_cast<void*>(mail_.data())) (void)hipIpcCloseMemHandle(m);
  if (host_ && host_ != MAP_FAILED) {
    (void)hipHostUnregister(host_);
    ::munmap(host_, seg_bytes_);
  }
}

void IpcHaloTransport::connect(const std::vector<uint8_t>& up_handles, const std::vector<uint8_t>& down_handles) {
  PCONV_CHECK(!connected_, "ipc transport: already connected");
  const Band& b = eng_->band();
  const FrameLayout& L = eng_->layout();
  const int dev = eng_->options().device;
  // A self-neighbour is self on EVERY side that has a neighbour (one-process
  // emulation): exchange() then signals this rank's own mailbox on both
  // sides.  A band with one self side and one real peer would signal itself
  // instead of that peer and read the peer's rows without its level word.
  const bool self_up = b.up >= 0 && up_handles == handles_, self_down = b.down >= 0 && down_handles == handles_;
  PCONV_CHECK(!(self_up || self_down) || ((b.up < 0 || self_up) && (b.down < 0 || self_down)),
              "ipc transport: a self-neighbour on one side and a peer rank on the other");
  // Returns true for a self-neighbour.
  auto open = [&](const std::vector<uint8_t>& hs, uint8_t** out, IpcMailbox** mail, int* peer_dev) {
    PCONV_CHECK(hs.size() == kIpcHandleBytes, "ipc transport: bad handle blob");
    if (hs == handles_) {
      // This engine is its own neighbour (one-process emulation of a rank
      // whose halos move: the band's own rows come back as its ghost rows,
      // like RCCL send/recv to self).  A process cannot open its own handle.
      for (int i = 0; i < 2; ++i) out[i] = own_base_[i];
      *mail = reinterpret_cast<IpcMailbox*>(mail_.data());
      *peer_dev = dev;
      own_ = true;
      return true;
    }
    for (int i = 0; i < 3; ++i) {
      hipIpcMemHandle_t h;
      std::memcpy(&h, hs.data() + i * sizeof(h), sizeof(h));
      void* p = nullptr;
      PCONV_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
      if (i < 2)
        out[i] = static_cast<uint8_t*>(p);
      else
        *mail = static_cast<IpcMailbox*>(p);
    }
    // The neighbour's device: on another GPU its frames and mailbox are
    // reached over xGMI, which needs peer access between the two devices.
    hipPointerAttribute_t at{};
    PCONV_HIP_CHECK(hipPointerGetAttributes(&at, out[0]));
    *peer_dev = at.device;
    if (at.device != dev && at.device >= 0) {
      int can = 0;
      PCONV_HIP_CHECK(hipDeviceCanAccessPeer(&can, dev, at.device));
      PCONV_CHECK(can != 0, "ipc transport: device " + std::to_string(dev) + " cannot access the neighbour's device " +
                                std::to_string(at.device) + " (no peer path for its frames and mailbox)");
    }
    return false;
  };
  // The neighbour's frame layout: a peer rank's band of the row split, or —
  // for a self-neighbour — this engine's own frames.  (The emulated band of
  // a W-way split carries world 1, so row_band(height, 1, 0) would describe
  // the whole image: the first version read the "neighbour's" boundary rows
  // that far past the band's own frame.)
  auto peer_layout = [&](bool self, int peer) {
    return self ? L : FrameLayout::make(L.row_bytes, row_band(eng_->geom().height, world_, peer).rows, L.halo);
  };
  if (b.up >= 0) {
    PCONV_CHECK(!up_handles.empty(), "ipc transport: band has an upper neighbour but no handles");
    lay_up_ = peer_layout(open(up_handles, peer_up_, &peer_mail_up_, &peer_dev_[0]), b.up);
    PCONV_CHECK(lay_up_.pitch == L.pitch && lay_up_.halo == L.halo, "ipc transport: neighbour frame layout differs");
  }
  if (b.down >= 0) {
    PCONV_CHECK(!down_handles.empty(), "ipc transport: band has a lower neighbour but no handles");
    lay_down_ = peer_layout(open(down_handles, peer_down_, &peer_mail_down_, &peer_dev_[1]), b.down);
    PCONV_CHECK(lay_down_.pitch == L.pitch && lay_down_.halo == L.halo,
                "ipc transport: neighbour frame layout differs");
  }
  connected_ = true;
}

void IpcHaloTransport::exchange(BandEngine& e, int64_t depth, hipStream_t stream) {
  TraceRange tr("pconv.halo.ipc");
  PCONV_CHECK(connected_ && &e == eng_, "ipc transport: not connected to this engine");
  const FrameLayout& L = e.layout();
  const Band& b = e.band();
  PCONV_CHECK(depth >= 1 && depth <= L.halo && depth <= b.rows, "ipc halo: bad depth");
  PCONV_CHECK((b.up < 0 || depth <= lay_up_.rows) && (b.down < 0 || depth <= lay_down_.rows),
              "ipc halo: depth exceeds a neighbour's band");
  const int me = rank_ * slots_ + slot_;
  const int up = b.up >= 0 ? b.up * slots_ + slot_ : -1;
  const int down = b.down >= 0 ? b.down * slots_ + slot_ : -1;
  const int par = e.cur();  // neighbours hold the same time level in the frame of the same parity
  const size_t n = static_cast<size_t>(depth * L.pitch);
  uint8_t* mine = e.frame_base(par);
  // up: its last `depth` owned rows -> my ghost rows [-depth, 0); down: its
  // first `depth` owned rows -> my ghost rows [rows, rows + depth).  Whole
  // pitch-aligned rows (pads included: zero in every frame).
  const uint8_t* src_up = up >= 0 ? peer_up_[par] + lay_up_.offset(lay_up_.rows - depth) - kPadLeft : nullptr;
  const uint8_t* src_down = down >= 0 ? peer_down_[par] + lay_down_.offset(0) - kPadLeft : nullptr;
  uint8_t* dst_up = up >= 0 ? mine + L.offset(-depth) - kPadLeft : nullptr;
  uint8_t* dst_down = down >= 0 ? mine + L.offset(b.rows) - kPadLeft : nullptr;
  (void)up;
  (void)down;
  // A self-neighbour (one-process emulation) copies within its own frame
  // allocations, which the runtime refuses as a captured SDMA copy: the grid
  // form pulls instead.
  const IpcPull form = pull_ == IpcPull::Sdma && own_ ? IpcPull::Grid : pull_;
  // Mailboxes: the neighbours'.  A self-neighbour signals its own mailbox on
  // BOTH sides, rows or not: an emulated edge band has one neighbour (itself),
  // and there is no upper rank to store the "lower neighbour's rows final"
  // word its one-sided wait reads (the first version timed out).
  auto* mine_mb = reinterpret_cast<IpcMailbox*>(mail_.data());
  IpcMailbox* mb_up = own_ ? mine_mb : (up >= 0 ? peer_mail_up_ : nullptr);
  IpcMailbox* mb_down = own_ ? mine_mb : (down >= 0 ? peer_mail_down_ : nullptr);
  launch_ipc_exchange(form, mine_mb, mb_up, mb_down, &dflags_[me].err, timeout_ticks_, dst_up, src_up, dst_down,
                      src_down, static_cast<int64_t>(n), stream);
  ++enqueued_;
}

namespace {

// Connect self-test sentinel: byte i of (rank, slot)'s probe rows.
uint8_t probe_byte(int rank, int slot, int64_t i) {
  return static_cast<uint8_t>((rank * 131 + slot * 17 + i * 7 + 1) & 0xff);
}

}  // namespace

void IpcHaloTransport::self_test(double timeout_s) {
  TraceRange tr("pconv.halo.ipc_self_test");
  PCONV_CHECK(connected_, "ipc transport: self-test before connect");
  const Band& b = eng_->band();
  if (b.up < 0 && b.down < 0) return;
  set_device(eng_->options().device);
  // Probe rows in the mailbox allocation past the signalling words: [out]
  // this rank's sentinel, [in_up] / [in_down] what it pulls from its
  // neighbours' [out].  The frames are never touched (they may hold data).
  constexpr int64_t P = kProbeBytes;
  uint8_t* base = mail_.data();
  std::vector<uint8_t> out(static_cast<size_t>(P));
  for (int64_t i = 0; i < P; ++i) out[static_cast<size_t>(i)] = probe_byte(rank_, slot_, i);
  PCONV_HIP_CHECK(hipMemcpy(base + kProbeOffset, out.data(), out.size(), hipMemcpyHostToDevice));
  PCONV_HIP_CHECK(hipMemset(base + kProbeOffset + P, 0, static_cast<size_t>(2 * P)));
  PCONV_HIP_CHECK(hipDeviceSynchronize());
  auto peer_probe = [&](IpcMailbox* m) { return reinterpret_cast<const uint8_t*>(m) + kProbeOffset; };
  const uint8_t* src_up = b.up >= 0 ? peer_probe(peer_mail_up_) : nullptr;
  const uint8_t* src_down = b.down >= 0 ? peer_probe(peer_mail_down_) : nullptr;
  uint8_t* dst_up = b.up >= 0 ? base + kProbeOffset + P : nullptr;
  uint8_t* dst_down = b.down >= 0 ? base + kProbeOffset + 2 * P : nullptr;
  auto* mine_mb = reinterpret_cast<IpcMailbox*>(mail_.data());
  IpcMailbox* mb_up = own_ ? mine_mb : (b.up >= 0 ? peer_mail_up_ : nullptr);
  IpcMailbox* mb_down = own_ ? mine_mb : (b.down >= 0 ? peer_mail_down_ : nullptr);
  int khz = 0;
  PCONV_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, eng_->options().device));
  const uint64_t ticks = static_cast<uint64_t>(timeout_s * static_cast<double>(khz > 0 ? khz : 100000) * 1000.0);
  const IpcPull form = pull_ == IpcPull::Sdma && own_ ? IpcPull::Grid : pull_;
  Stream st = Stream::create(0);
  launch_ipc_exchange(form, mine_mb, mb_up, mb_down, &dflags_[rank_ * slots_ + slot_].err, ticks, dst_up, src_up,
                      dst_down, src_down, P, st.get());
  ++enqueued_;
  PCONV_HIP_CHECK(hipStreamSynchronize(st.get()));
  const auto* f = static_cast<const volatile IpcFlags*>(host_);
  const uint32_t err = f[rank_ * slots_ + slot_].err;
  const std::string who = "ipc transport connect self-test (rank " + std::to_string(rank_) + ", slot " +
                          std::to_string(slot_) + ", device " + std::to_string(eng_->options().device) +
                          ", neighbours' devices " + std::to_string(peer_dev_[0]) + " / " +
                          std::to_string(peer_dev_[1]) + ", " + mailbox_kind_ + " mailbox): ";
  PCONV_CHECK(err == 0, who + (err == 1 ? "no neighbour's level word became visible within " : "no neighbour's ack "
                                                                                                "became visible within ") +
                            std::to_string(timeout_s) + " s (a neighbour that is not running its self-test, or a "
                                                        "store across devices this GPU's poll never observes)");
  std::vector<uint8_t> in(static_cast<size_t>(2 * P));
  PCONV_HIP_CHECK(hipMemcpy(in.data(), base + kProbeOffset + P, in.size(), hipMemcpyDeviceToHost));
  for (int side = 0; side < 2; ++side) {
    const int peer = side == 0 ? b.up : b.down;
    if (peer < 0) continue;
    const int pr = own_ ? rank_ : peer;
    for (int64_t i = 0; i < P; ++i)
      PCONV_CHECK(in[static_cast<size_t>(side * P + i)] == probe_byte(pr, slot_, i),
                  who + "the sentinel rows pulled from the " + (side == 0 ? "upper" : "lower") +
                      " neighbour differ at byte " + std::to_string(i) + " (a read across devices returned stale data)");
  }
  self_tested_ = true;
}

uint32_t IpcHaloTransport::device_count() const {
  uint32_t v = 0;
  PCONV_HIP_CHECK(hipMemcpy(&v, mail_.data() + offsetof(IpcMailbox, count), sizeof(v), hipMemcpyDeviceToHost));
  return v;
}

void IpcHaloTransport::check() const {
  const auto* f = static_cast<const volatile IpcFlags*>(host_);
  const uint32_t err = f[rank_ * slots_ + slot_].err;
  PCONV_CHECK(err == 0, std::string("ipc halo: rank ") + std::to_string(rank_) + " slot " + std::to_string(slot_) +
                            (err == 1 ? ": timed out waiting for a neighbour's rows"
                                      : ": timed out waiting for a neighbour to copy this rank's rows"));
}

}  // namespace pconv

namespace pconv {

double ipc_pull_probe(const std::string& form, int64_t bytes, bool host_source, int iters, int device,
                      int workgroups) {
  PCONV_CHECK(bytes > 0 && bytes % 16 == 0 && iters >= 1, "ipc_pull_probe: bytes must be a positive multiple of 16");
  const IpcPull p = parse_ipc_pull(form);
  set_device(device);
  // the error word in coherent (fine-grained) mapped host memory, like the
  // shared segment the transport registers; the mailbox in device memory
  void* fh = nullptr;
  PCONV_HIP_CHECK(hipHostMalloc(&fh, sizeof(IpcFlags), hipHostMallocCoherent | hipHostMallocMapped));
  struct FreeHost {
    void* p;
    ~FreeHost() { (void)hipHostFree(p); }
  } free_flags{fh};
  std::memset(fh, 0, sizeof(IpcFlags));
  void* fd = nullptr;
  PCONV_HIP_CHECK(hipHostGetDevicePointer(&fd, fh, 0));
  DeviceBuffer mail(sizeof(IpcMailbox)), dst(static_cast<size_t>(2 * bytes));
  PCONV_HIP_CHECK(hipMemset(mail.data(), 0, mail.size()));
  PinnedBuffer hsrc;
  DeviceBuffer dsrc;
  uint8_t* src = nullptr;
  if (host_source) {
    hsrc = PinnedBuffer(static_cast<size_t>(2 * bytes));
    std::memset(hsrc.data(), 0x5a, hsrc.size());
    void* d = nullptr;
    PCONV_HIP_CHECK(hipHostGetDevicePointer(&d, hsrc.data(), 0));
    src = static_cast<uint8_t*>(d);
  } else {
    dsrc = DeviceBuffer(static_cast<size_t>(2 * bytes));
    PCONV_HIP_CHECK(hipMemset(dsrc.data(), 0x5a, dsrc.size()));
    src = dsrc.data();
  }
  int khz = 0;
  PCONV_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
  const uint64_t timeout = static_cast<uint64_t>(5.0 * static_cast<double>(khz > 0 ? khz : 100000) * 1000.0);
  Stream st = Stream::create(0);
  auto* err = &static_cast<IpcFlags*>(fd)->err;
  auto* mb = reinterpret_cast<IpcMailbox*>(mail.data());
  auto one = [&] {
    launch_ipc_exchange(p, mb, mb, mb, err, timeout, dst.data(), src + bytes, dst.data() + bytes, src, bytes,
                        st.get(), workgroups);
  };
  for (int i = 0; i < 3; ++i) one();
  PCONV_HIP_CHECK(hipStreamSynchronize(st.get()));
  Event e0 = Event::create(true), e1 = Event::create(true);
  e0.record(st.get());
  for (int i = 0; i < iters; ++i) one();
  e1.record(st.get());
  PCONV_HIP_CHECK(hipStreamSynchronize(st.get()));
  const auto* fl = reinterpret_cast<const volatile IpcFlags*>(fh);
  PCONV_CHECK(fl->err == 0, "ipc_pull_probe: a self-neighbour wait timed out");
  uint32_t count = 0;
  PCONV_HIP_CHECK(hipMemcpy(&count, mail.data() + offsetof(IpcMailbox, count), sizeof(count), hipMemcpyDeviceToHost));
  PCONV_CHECK(count == static_cast<uint32_t>(iters + 3), "ipc_pull_probe: exchange count mismatch");
  std::vector<uint8_t> back(static_cast<size_t>(2 * bytes));
  PCONV_HIP_CHECK(hipMemcpy(back.data(), dst.data(), back.size(), hipMemcpyDeviceToHost));
  for (uint8_t v : back) PCONV_CHECK(v == 0x5a, "ipc_pull_probe: pulled bytes differ from the source");
  return Event::elapsed_ms(e0, e1) / iters;
}

}  // namespace pconv
