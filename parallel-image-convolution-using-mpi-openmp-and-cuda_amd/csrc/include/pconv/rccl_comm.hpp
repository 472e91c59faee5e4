// RCCL (ROCm NCCL) communicator + halo transport over xGMI.
//
// Reference communication (mpi/mpi_convolution.c): 6 MPI_Bcast of the config
// (:65-70), derived row/column datatypes (:75-83), per-rep MPI_Isend/Irecv to
// <=4 neighbours with tag 0 (:157-192), MPI_Wait (:199-234), and a hand-rolled
// Send/Recv max-gather of the loop time (:264-275).
//
// pconv: one process per GPU; a communicator is bootstrapped from a 128-byte
// unique id that the launcher distributes (torch.distributed/gloo, or the
// native fork launcher's shared memory).  A halo exchange is ONE grouped
// ncclSend/ncclRecv pair per neighbour of `depth * pitch` contiguous bytes on
// the engine's communication stream (row bands need no datatypes and no
// corners).  The loop-time max is an ncclAllReduce(ncclMax) of one double.
// Asynchronous RCCL errors are polled with a timeout (failure detection).
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <vector>

#include "pconv/engine.hpp"

namespace pconv {

constexpr int kUniqueIdBytes = 128;

// Generate a fresh unique id (call on ONE rank, distribute the bytes).
std::vector<uint8_t> rccl_unique_id();
std::string rccl_version();
// True once librccl is mapped into this process (it is dlopen'ed on the first
// RCCL call, never at start-up).
bool rccl_loaded();
// Path of the librccl this process mapped ("" while none is mapped): in a
// torch process `librccl.so.1` resolves to torch's bundled copy, in the `conv`
// CLI to ROCm's.
std::string rccl_library_path();

class RcclComm {
 public:
  // Collective over all ranks; `device` must already be the rank's GPU.
  RcclComm(const std::vector<uint8_t>& unique_id, int rank, int world, int device);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  int rank() const { return rank_; }
  int world() const { return world_; }
  void* handle() const { return comm_; }

  // Blocking helpers (own stream): max / sum of one double across ranks.
  double allreduce_max(double v);
  double allreduce_sum(double v);
  void barrier();

  // Throws if RCCL reported an asynchronous error (and aborts the comm).
  void check_async_error();
  // Wait for `stream` while polling for RCCL errors; throws after timeout_s.
  void wait(hipStream_t stream, double timeout_s);

 private:
  double allreduce(double v, int op);
  void* comm_ = nullptr;  // ncclComm_t
  int rank_ = 0, world_ = 1, device_ = 0;
  Stream stream_;
  DeviceBuffer scratch_;
};

class RcclTransport : public HaloTransport {
 public:
  explicit RcclTransport(std::shared_ptr<RcclComm> comm) : comm_(std::move(comm)) {}
  void exchange(BandEngine& e, int64_t depth, hipStream_t stream) override;
  const char* name() const override { return "rccl"; }
  // ncclSend/ncclRecv in a group only enqueue kernels on `stream`: capturable
  // (tests/test_gpu_halo.py and `conv --selftest rccl-capture`, both stacks).
  bool capturable() const override { return true; }
  RcclComm& comm() { return *comm_; }

 private:
  std::shared_ptr<RcclComm> comm_;
};

}  // namespace pconv
