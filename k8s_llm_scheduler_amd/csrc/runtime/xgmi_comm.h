#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace k8sllm {

// Peer-memory communicator for the decode-time collectives (see kernels/xgmi.hip for the protocol).
// Lifecycle: construct on every rank -> exchange handle() bytes (torch.distributed) -> open(all
// handles) -> all_reduce_bf16 / all_gather on any stream, graph-capturable.
class XgmiComm {
 public:
  XgmiComm(int world, int rank, long long slot_bytes, int blocks, double timeout_s);
  ~XgmiComm();
  XgmiComm(const XgmiComm&) = delete;
  XgmiComm& operator=(const XgmiComm&) = delete;

  std::string handle() const;                        // hipIpcMemHandle_t bytes of this rank's region
  void open(const std::vector<std::string>& handles);  // map every peer's region (index = rank)
  // out = sum over ranks of in (+ residual, a bf16 tensor of the same size, when given)
  void all_reduce_bf16(const void* in, void* out, long long bytes, hipStream_t s, const void* residual = nullptr);
  void all_gather(const void* in, void* out, long long bytes_per_rank, hipStream_t s);
  // out[M, N] = residual + sum over ranks of x[M, K] . W[N, K]^T: the row-parallel decode projection with the
  // all-reduce in its epilogue (kernels/gemv.hip GemvAr); W bf16, or fp8 e4m3 with per-row scales wscale.
  // Returns -5 (nothing launched) where the shape does not fit the fused plan.
  int gemv_allreduce(void* out, const void* x, const void* w, const float* wscale, int M, int N, int K,
                     const void* residual, hipStream_t s);
  uint32_t error();                                   // poll-timeout bitmask (synchronizes the device)
  // Health check without an extra sync: enqueue a copy of the error word to pinned host memory on
  // `s`; after the caller's own synchronization of `s`, last_error() is that word.
  void snapshot_error(hipStream_t s);
  uint32_t last_error() const;
  void reset_error();
  // Back to the freshly-constructed protocol state: zero this rank's region (flags, LL rows, slots),
  // the per-workgroup epochs and the error word.  Recovery after a stall: every rank calls it with its
  // device drained, then the ranks pass a barrier before the next collective.
  void reset();

  int world() const { return world_; }
  int rank() const { return rank_; }
  long long slot_bytes() const { return slot_bytes_; }
  int blocks() const { return blocks_; }
  bool is_open() const { return opened_; }
  // Messages up to this size use the LL protocol (flag in every 8-byte word); 0 disables it.
  long long ll_max_bytes() const { return ll_max_bytes_; }
  void set_ll_max_bytes(long long b) { ll_max_bytes_ = b; }
  // Messages of at least this size (and every message above slot_bytes, up to world x slot_bytes) use the
  // two-shot reduce-scatter + all-gather kernel; 0 = only the ones above slot_bytes.
  long long twoshot_min_bytes() const { return twoshot_min_bytes_; }
  void set_twoshot_min_bytes(long long b) { twoshot_min_bytes_ = b; }
  long long max_allreduce_bytes() const { return (long long)world_ * slot_bytes_; }

 private:
  int world_, rank_, blocks_;
  long long slot_bytes_, region_bytes_, timeout_ticks_;
  int device_ = 0;
  void* region_ = nullptr;      // own IPC region (uncached)
  uint32_t* counters_ = nullptr;  // [max_blocks] epochs + 1 error word
  uint32_t* fused_state_ = nullptr;  // gemv_allreduce: [max groups] epochs + [max groups] tickets (uncached)
  long long fused_off_ = 0;          // byte offset of the gemv_allreduce LL rows in every region
  uint32_t* host_err_ = nullptr;  // pinned copy of the error word (snapshot_error)
  std::vector<void*> bases_;    // every rank's region in this address space
  std::vector<bool> mapped_;    // true where bases_[i] came from hipIpcOpenMemHandle
  bool opened_ = false;
  long long ll_max_bytes_ = 64 * 1024;
  long long twoshot_min_bytes_ = 256 * 1024;
};

}  // namespace k8sllm
