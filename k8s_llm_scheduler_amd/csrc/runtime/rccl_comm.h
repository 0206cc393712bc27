#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace k8sllm {

class RcclComm {
 public:
  static std::vector<uint8_t> unique_id();
  RcclComm(int world, int rank, const std::vector<uint8_t>& id);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // dtype codes: 0 bf16, 1 f32, 2 f16, 3 i32; reductions: 0 sum, 1 max, 2 min
  void all_reduce(const void* send, void* recv, size_t count, int dtype, int red, hipStream_t s);
  void all_gather(const void* send, void* recv, size_t count_per_rank, int dtype, hipStream_t s);
  // recv[count_per_rank] = this rank's shard of the sum of every rank's send[world * count_per_rank]
  void reduce_scatter(const void* send, void* recv, size_t count_per_rank, int dtype, int red, hipStream_t s);
  void broadcast(void* buf, size_t count, int dtype, int root, hipStream_t s);
  // ncclCommGetAsyncError: "" when healthy, else the error text (a peer died, a transport failed)
  std::string async_error() const;
  // ncclCommAbort: pending operations of this communicator error out (so a stream blocked on a dead
  // peer drains) and the communicator is unusable afterwards; the engine then builds a new one.
  void abort();
  bool aborted() const { return comm_ == nullptr; }
  int world() const { return world_; }
  int rank() const { return rank_; }

 private:
  void* comm_ = nullptr;
  int world_, rank_;
};

}  // namespace k8sllm
