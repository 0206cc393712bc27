// Tensor-parallel communicator on RCCL (NCCL API on ROCm, xGMI transport between MI355X GPUs).
//
// The engine owns its own communicator instead of going through ProcessGroupNCCL so that every
// collective is a plain ncclAllReduce / ncclAllGather enqueued on the caller's HIP stream:
// graph-capturable (RCCL supports stream capture), no watchdog/event bookkeeping inside a
// captured region, no allocation per call.  Bootstrapping (the 128-byte unique id) goes through
// torch.distributed once at start-up.
#include "runtime/rccl_comm.h"

#include <rccl/rccl.h>

#include <cstring>
#include <stdexcept>
#include <string>

namespace k8sllm {

namespace {
void ck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
}
ncclDataType_t dt(int code) {
  switch (code) {
    case 0: return ncclBfloat16;
    case 1: return ncclFloat32;
    case 2: return ncclFloat16;
    case 3: return ncclInt32;
    default: throw std::invalid_argument("unsupported dtype code " + std::to_string(code));
  }
}
ncclRedOp_t op(int code) {
  switch (code) {
    case 0: return ncclSum;
    case 1: return ncclMax;
    case 2: return ncclMin;
    default: throw std::invalid_argument("unsupported reduction " + std::to_string(code));
  }
}
}  // namespace

std::vector<uint8_t> RcclComm::unique_id() {
  ncclUniqueId id;
  ck(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id));
}

RcclComm::RcclComm(int world, int rank, const std::vector<uint8_t>& id) : world_(world), rank_(rank) {
  if (id.size() != sizeof(ncclUniqueId)) throw std::invalid_argument("bad unique id size");
  ncclUniqueId uid;
  std::memcpy(&uid, id.data(), sizeof(uid));
  ncclComm_t c;
  ck(ncclCommInitRank(&c, world, uid, rank), "ncclCommInitRank");
  comm_ = c;
}

void RcclComm::abort() {
  if (comm_) (void)ncclCommAbort(static_cast<ncclComm_t>(comm_));
  comm_ = nullptr;
}

RcclComm::~RcclComm() {
  if (comm_) ncclCommDestroy(static_cast<ncclComm_t>(comm_));
}

void RcclComm::all_reduce(const void* send, void* recv, size_t count, int dtype, int red, hipStream_t s) {
  if (!comm_) throw std::runtime_error("RCCL communicator aborted");
  ck(ncclAllReduce(send, recv, count, dt(dtype), op(red), static_cast<ncclComm_t>(comm_), s), "ncclAllReduce");
}

void RcclComm::all_gather(const void* send, void* recv, size_t count, int dtype, hipStream_t s) {
  if (!comm_) throw std::runtime_error("RCCL communicator aborted");
  ck(ncclAllGather(send, recv, count, dt(dtype), static_cast<ncclComm_t>(comm_), s), "ncclAllGather");
}

void RcclComm::reduce_scatter(const void* send, void* recv, size_t count, int dtype, int red, hipStream_t s) {
  if (!comm_) throw std::runtime_error("RCCL communicator aborted");
  ck(ncclReduceScatter(send, recv, count, dt(dtype), op(red), static_cast<ncclComm_t>(comm_), s), "ncclReduceScatter");
}

std::string RcclComm::async_error() const {
  if (!comm_) return "communicator aborted";
  ncclResult_t r = ncclSuccess;
  if (ncclCommGetAsyncError(static_cast<ncclComm_t>(comm_), &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
  return r == ncclSuccess ? std::string() : std::string(ncclGetErrorString(r));
}

void RcclComm::broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s) {
  if (!comm_) throw std::runtime_error("RCCL communicator aborted");
  ck(ncclBroadcast(buf, buf, count, dt(dtype), root, static_cast<ncclComm_t>(comm_), s), "ncclBroadcast");
}

}  // namespace k8sllm
