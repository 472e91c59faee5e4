// RCCL communicator and halo transport (see rccl_comm.hpp).
#include "pconv/rccl_comm.hpp"
#include "pconv/trace.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <sstream>
#include <thread>

#include "pconv/selftest.hpp"

namespace pconv {

namespace {

// librccl is loaded on first use (dlopen), not at process start: the library
// is ~570 MB with a large symbol table, and a 1-GPU `conv` run or a Python
// process that never builds a communicator should not pay its load and
// relocation in its start-up (the reference's CUDA program, timed end to end
// by cuda/main.c:20-49, links no communication library at all).
struct RcclApi {
  decltype(&::ncclGetVersion) GetVersion = nullptr;
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRank) CommInitRank = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclCommAbort) CommAbort = nullptr;
  decltype(&::ncclGetErrorString) GetErrorString = nullptr;
  decltype(&::ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&::ncclAllReduce) AllReduce = nullptr;
  decltype(&::ncclSend) Send = nullptr;
  decltype(&::ncclRecv) Recv = nullptr;
  decltype(&::ncclGroupStart) GroupStart = nullptr;
  decltype(&::ncclGroupEnd) GroupEnd = nullptr;
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  static std::string err;
  std::call_once(once, [] {
    std::vector<std::string> names;
    if (const char* p = std::getenv("PCONV_RCCL_LIB")) names.emplace_back(p);
    names.emplace_back("librccl.so.1");
    names.emplace_back("librccl.so");
    const char* rocm = std::getenv("ROCM_PATH");
    names.emplace_back(std::string(rocm ? rocm : "/opt/rocm") + "/lib/librccl.so.1");
    void* h = nullptr;
    for (const auto& n : names)
      if ((h = dlopen(n.c_str(), RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) {
      const char* e = dlerror();
      err = std::string("cannot load librccl (") + (e ? e : "not found") + ")";
      return;
    }
    auto sym = [&](const char* name) {
      void* f = dlsym(h, name);
      if (!f) err = std::string("librccl lacks ") + name;
      return f;
    };
    api.GetVersion = reinterpret_cast<decltype(api.GetVersion)>(sym("ncclGetVersion"));
    api.GetUniqueId = reinterpret_cast<decltype(api.GetUniqueId)>(sym("ncclGetUniqueId"));
    api.CommInitRank = reinterpret_cast<decltype(api.CommInitRank)>(sym("ncclCommInitRank"));
    api.CommDestroy = reinterpret_cast<decltype(api.CommDestroy)>(sym("ncclCommDestroy"));
    api.CommAbort = reinterpret_cast<decltype(api.CommAbort)>(sym("ncclCommAbort"));
    api.GetErrorString = reinterpret_cast<decltype(api.GetErrorString)>(sym("ncclGetErrorString"));
    api.CommGetAsyncError = reinterpret_cast<decltype(api.CommGetAsyncError)>(sym("ncclCommGetAsyncError"));
    api.AllReduce = reinterpret_cast<decltype(api.AllReduce)>(sym("ncclAllReduce"));
    api.Send = reinterpret_cast<decltype(api.Send)>(sym("ncclSend"));
    api.Recv = reinterpret_cast<decltype(api.Recv)>(sym("ncclRecv"));
    api.GroupStart = reinterpret_cast<decltype(api.GroupStart)>(sym("ncclGroupStart"));
    api.GroupEnd = reinterpret_cast<decltype(api.GroupEnd)>(sym("ncclGroupEnd"));
  });
  PCONV_CHECK(err.empty(), err);
  return api;
}

}  // namespace

bool rccl_loaded() {
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
  if (h) dlclose(h);
  return h != nullptr;
}

std::string rccl_library_path() {
  if (!rccl_loaded()) return "";
  Dl_info info{};
  if (dladdr(reinterpret_cast<void*>(rccl().GetVersion), &info) == 0 || info.dli_fname == nullptr) return "";
  return info.dli_fname;
}

#define PCONV_RCCL_CHECK(expr)                                                                            \
  do {                                                                                                    \
    ncclResult_t _r = (expr);                                                                             \
    if (_r != ncclSuccess && _r != ncclInProgress)                                                        \
      ::pconv::raise_error(__FILE__, __LINE__, std::string(#expr) + ": " + rccl().GetErrorString(_r));    \
  } while (0)

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  PCONV_RCCL_CHECK(rccl().GetUniqueId(&id));
  std::vector<uint8_t> v(kUniqueIdBytes);
  std::memcpy(v.data(), id.internal, kUniqueIdBytes);
  return v;
}

std::string rccl_version() {
  int v = 0;
  PCONV_RCCL_CHECK(rccl().GetVersion(&v));
  return std::to_string(v / 10000) + "." + std::to_string((v / 100) % 100) + "." + std::to_string(v % 100);
}

RcclComm::RcclComm(const std::vector<uint8_t>& unique_id, int rank, int world, int device)
    : rank_(rank), world_(world), device_(device) {
  PCONV_CHECK(unique_id.size() == kUniqueIdBytes, "RCCL unique id must be 128 bytes");
  PCONV_CHECK(world >= 1 && rank >= 0 && rank < world, "bad RCCL rank/world");
  set_error_rank(rank);
  set_device(device);
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id.data(), kUniqueIdBytes);
  ncclComm_t c = nullptr;
  PCONV_RCCL_CHECK(rccl().CommInitRank(&c, world, id, rank));
  comm_ = c;
  stream_ = Stream::create(0);
  scratch_ = DeviceBuffer(64);
}

RcclComm::~RcclComm() {
  if (comm_) (void)rccl().CommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::check_async_error() {
  ncclResult_t r = ncclSuccess;
  PCONV_RCCL_CHECK(rccl().CommGetAsyncError(static_cast<ncclComm_t>(comm_), &r));
  if (r != ncclSuccess && r != ncclInProgress) {
    (void)rccl().CommAbort(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
    PCONV_FAIL(std::string("RCCL asynchronous error: ") + rccl().GetErrorString(r));
  }
}

void RcclComm::wait(hipStream_t stream, double timeout_s) {
  const double t0 = wall_seconds();
  for (;;) {
    const hipError_t q = hipStreamQuery(stream);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) PCONV_HIP_CHECK(q);
    check_async_error();
    if (timeout_s > 0 && wall_seconds() - t0 > timeout_s) {
      (void)rccl().CommAbort(static_cast<ncclComm_t>(comm_));
      comm_ = nullptr;
      PCONV_FAIL("RCCL wait timed out after " + std::to_string(timeout_s) + " s (peer hung or died?)");
    }
    std::this_thread::yield();
  }
}

double RcclComm::allreduce(double v, int op) {
  PCONV_HIP_CHECK(hipMemcpyAsync(scratch_.data(), &v, sizeof(double), hipMemcpyHostToDevice, stream_.get()));
  PCONV_RCCL_CHECK(rccl().AllReduce(scratch_.data(), scratch_.data(), 1, ncclFloat64, static_cast<ncclRedOp_t>(op),
                                 static_cast<ncclComm_t>(comm_), stream_.get()));
  double out = 0;
  PCONV_HIP_CHECK(hipMemcpyAsync(&out, scratch_.data(), sizeof(double), hipMemcpyDeviceToHost, stream_.get()));
  wait(stream_.get(), 600.0);
  return out;
}

double RcclComm::allreduce_max(double v) { return allreduce(v, ncclMax); }
double RcclComm::allreduce_sum(double v) { return allreduce(v, ncclSum); }
void RcclComm::barrier() { (void)allreduce(0.0, ncclSum); }

void RcclTransport::exchange(BandEngine& e, int64_t depth, hipStream_t stream) {
  TraceRange tr("pconv.halo.rccl");
  const FrameLayout& L = e.layout();
  const Band& b = e.band();
  const int64_t pitch = L.pitch;
  PCONV_CHECK(depth >= 1 && depth <= L.halo && depth <= b.rows, "rccl halo: bad depth");
  uint8_t* row0 = e.src_frame() - kPadLeft;  // pitch-aligned start of owned row 0
  const size_t n = static_cast<size_t>(depth * pitch);
  auto comm = static_cast<ncclComm_t>(comm_->handle());
  PCONV_CHECK(comm != nullptr, "rccl halo: communicator was aborted");
  PCONV_RCCL_CHECK(rccl().GroupStart());
  if (b.up >= 0) {
    PCONV_RCCL_CHECK(rccl().Send(row0, n, ncclUint8, b.up, comm, stream));                     // my top rows
    PCONV_RCCL_CHECK(rccl().Recv(row0 - depth * pitch, n, ncclUint8, b.up, comm, stream));     // ghost above
  }
  if (b.down >= 0) {
    PCONV_RCCL_CHECK(rccl().Send(row0 + (b.rows - depth) * pitch, n, ncclUint8, b.down, comm, stream));
    PCONV_RCCL_CHECK(rccl().Recv(row0 + b.rows * pitch, n, ncclUint8, b.down, comm, stream));  // ghost below
  }
  PCONV_RCCL_CHECK(rccl().GroupEnd());
}

std::string rccl_capture_probe(const std::string& op, const std::string& mode, int64_t bytes, int device,
                               int launches) {
  PCONV_CHECK(op == "sendrecv" || op == "allreduce" || op == "sendrecv_fork" || op == "allreduce_fork",
              "rccl_capture_probe: op must be sendrecv, allreduce, sendrecv_fork or allreduce_fork");
  // *_fork: the RCCL call goes to a SECOND stream that joined the capture
  // through an event (record on the origin, wait on the second stream; joined
  // back the same way) — how a split exchange phase is captured.
  const bool fork = op.size() > 5 && op.compare(op.size() - 5, 5, "_fork") == 0;
  const std::string base = fork ? op.substr(0, op.size() - 5) : op;
  PCONV_CHECK(bytes >= 8 && bytes % 8 == 0, "rccl_capture_probe: bytes must be a positive multiple of 8");
  hipStreamCaptureMode cm = hipStreamCaptureModeGlobal;
  const bool capture = mode != "none";
  if (mode == "thread_local")
    cm = hipStreamCaptureModeThreadLocal;
  else if (mode == "relaxed")
    cm = hipStreamCaptureModeRelaxed;
  else
    PCONV_CHECK(mode == "global" || mode == "none", "rccl_capture_probe: mode must be global|thread_local|relaxed|none");
  auto step = [&](const char* what) {
    std::fprintf(stderr, "[rccl_capture_probe %s/%s] %s\n", op.c_str(), mode.c_str(), what);
    std::fflush(stderr);
  };
  set_device(device);
  step("communicator");
  RcclComm comm(rccl_unique_id(), 0, 1, device);
  auto c = static_cast<ncclComm_t>(comm.handle());
  const size_t n = static_cast<size_t>(bytes);
  DeviceBuffer a(n), b(n);
  std::vector<uint8_t> pat(n), got(n);
  for (size_t i = 0; i < n; ++i) pat[i] = static_cast<uint8_t>((i * 131 + 7) & 0x7f);  // no sum overflow
  PCONV_HIP_CHECK(hipMemcpy(a.data(), pat.data(), n, hipMemcpyHostToDevice));
  PCONV_HIP_CHECK(hipMemset(b.data(), 0, n));
  Stream s = Stream::create(0);
  Stream s2 = Stream::create(-1);
  Event ev_fork = Event::create(), ev_join = Event::create();
  auto enqueue = [&] {
    hipStream_t t = s.get();
    if (fork) {
      ev_fork.record(s.get());
      ev_fork.wait_on(s2.get());
      t = s2.get();
    }
    if (base == "sendrecv") {
      PCONV_RCCL_CHECK(rccl().GroupStart());
      PCONV_RCCL_CHECK(rccl().Send(a.data(), n, ncclUint8, 0, c, t));
      PCONV_RCCL_CHECK(rccl().Recv(b.data(), n, ncclUint8, 0, c, t));
      PCONV_RCCL_CHECK(rccl().GroupEnd());
    } else {
      PCONV_RCCL_CHECK(rccl().AllReduce(a.data(), b.data(), n, ncclUint8, ncclSum, c, t));
    }
    if (fork) {
      ev_join.record(s2.get());
      ev_join.wait_on(s.get());
    }
  };
  hipGraphExec_t ex = nullptr;
  size_t nodes = 0;
  if (capture) {
    step("begin capture");
    PCONV_HIP_CHECK(hipStreamBeginCapture(s.get(), cm));
    step("enqueue under capture");
    enqueue();
    hipGraph_t g = nullptr;
    step("end capture");
    PCONV_HIP_CHECK(hipStreamEndCapture(s.get(), &g));
    PCONV_HIP_CHECK(hipGraphGetNodes(g, nullptr, &nodes));
    step("instantiate");
    PCONV_HIP_CHECK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    PCONV_HIP_CHECK(hipGraphDestroy(g));
  }
  for (int i = 0; i < launches; ++i) {
    PCONV_HIP_CHECK(hipMemsetAsync(b.data(), 0, n, s.get()));
    step(capture ? "graph launch" : "direct enqueue");
    if (capture)
      PCONV_HIP_CHECK(hipGraphLaunch(ex, s.get()));
    else
      enqueue();
    comm.wait(s.get(), 60.0);
    PCONV_HIP_CHECK(hipMemcpy(got.data(), b.data(), n, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (size_t k = 0; k < n; ++k) bad += got[k] != pat[k];
    PCONV_CHECK(bad == 0, "rccl_capture_probe " + op + "/" + mode + ": " + std::to_string(bad) +
                              " bytes differ after launch " + std::to_string(i));
  }
  if (ex) PCONV_HIP_CHECK(hipGraphExecDestroy(ex));
  step("ok");
  std::ostringstream os;
  os << "{\"probe\": \"rccl_capture\", \"op\": \"" << op << "\", \"mode\": \"" << mode << "\", \"bytes\": " << bytes
     << ", \"graph_nodes\": " << nodes << ", \"launches\": " << launches << ", \"status\": \"ok\", \"rccl_version\": \""
     << rccl_version() << "\", \"rccl_path\": \"" << json_escape(rccl_library_path()) << "\"}";
  return os.str();
}

}  // namespace pconv
