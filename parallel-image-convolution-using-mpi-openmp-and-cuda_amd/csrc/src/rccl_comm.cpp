// RCCL communicator and halo transport (see rccl_comm.hpp).
#include "pconv/rccl_comm.hpp"
#include "pconv/trace.hpp"

#include <rccl/rccl.h>

#include <cstring>
#include <thread>

namespace pconv {

#define PCONV_RCCL_CHECK(expr)                                                                      \
  do {                                                                                              \
    ncclResult_t _r = (expr);                                                                       \
    if (_r != ncclSuccess && _r != ncclInProgress)                                                  \
      ::pconv::raise_error(__FILE__, __LINE__, std::string(#expr) + ": " + ncclGetErrorString(_r)); \
  } while (0)

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  PCONV_RCCL_CHECK(ncclGetUniqueId(&id));
  std::vector<uint8_t> v(kUniqueIdBytes);
  std::memcpy(v.data(), id.internal, kUniqueIdBytes);
  return v;
}

std::string rccl_version() {
  int v = 0;
  PCONV_RCCL_CHECK(ncclGetVersion(&v));
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
  PCONV_RCCL_CHECK(ncclCommInitRank(&c, world, id, rank));
  comm_ = c;
  stream_ = Stream::create(0);
  scratch_ = DeviceBuffer(64);
}

RcclComm::~RcclComm() {
  if (comm_) (void)ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::check_async_error() {
  ncclResult_t r = ncclSuccess;
  PCONV_RCCL_CHECK(ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &r));
  if (r != ncclSuccess && r != ncclInProgress) {
    (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
    comm_ = nullptr;
    PCONV_FAIL(std::string("RCCL asynchronous error: ") + ncclGetErrorString(r));
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
      (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
      comm_ = nullptr;
      PCONV_FAIL("RCCL wait timed out after " + std::to_string(timeout_s) + " s (peer hung or died?)");
    }
    std::this_thread::yield();
  }
}

double RcclComm::allreduce(double v, int op) {
  PCONV_HIP_CHECK(hipMemcpyAsync(scratch_.data(), &v, sizeof(double), hipMemcpyHostToDevice, stream_.get()));
  PCONV_RCCL_CHECK(ncclAllReduce(scratch_.data(), scratch_.data(), 1, ncclFloat64, static_cast<ncclRedOp_t>(op),
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
  PCONV_RCCL_CHECK(ncclGroupStart());
  if (b.up >= 0) {
    PCONV_RCCL_CHECK(ncclSend(row0, n, ncclUint8, b.up, comm, stream));                     // my top rows
    PCONV_RCCL_CHECK(ncclRecv(row0 - depth * pitch, n, ncclUint8, b.up, comm, stream));     // ghost above
  }
  if (b.down >= 0) {
    PCONV_RCCL_CHECK(ncclSend(row0 + (b.rows - depth) * pitch, n, ncclUint8, b.down, comm, stream));
    PCONV_RCCL_CHECK(ncclRecv(row0 + b.rows * pitch, n, ncclUint8, b.down, comm, stream));  // ghost below
  }
  PCONV_RCCL_CHECK(ncclGroupEnd());
}

}  // namespace pconv
