// Host side of the xGMI peer-memory communicator: IPC region allocation, handle exchange, launch.
#include "runtime/xgmi_comm.h"

#include <cstring>
#include <stdexcept>

extern "C" {
long long k8s_xgmi_flag_bytes();
int k8s_xgmi_max_blocks();
int k8s_xgmi_allreduce_bf16(void* const* bases, uint32_t* counters, uint32_t* err, const void* in, void* out,
                            long long bytes, long long slot_bytes, int rank, int world, int blocks,
                            long long timeout_ticks, const void* residual, hipStream_t s);
int k8s_xgmi_allreduce_ll_bf16(void* const* bases, uint32_t* counters, uint32_t* err, const void* in, void* out,
                               long long bytes, long long slot_bytes, int rank, int world, int blocks,
                               long long timeout_ticks, const void* residual, hipStream_t s);
int k8s_xgmi_allreduce_2shot_bf16(void* const* bases, uint32_t* counters, uint32_t* err, const void* in, void* out,
                                  long long bytes, long long slot_bytes, int rank, int world, int blocks,
                                  long long timeout_ticks, const void* residual, hipStream_t s);
int k8s_xgmi_allgather(void* const* bases, uint32_t* counters, uint32_t* err, const void* in, void* out,
                       long long bytes, long long slot_bytes, int rank, int world, int blocks,
                       long long timeout_ticks, hipStream_t s);
int k8s_gemv_allreduce(void* out, const void* x, const void* W, const float* wscale, int M, int N_out, int K,
                       const void* residual, void* const* bases, long long row_bytes, uint32_t* epochs,
                       uint32_t* tickets, uint32_t* err, int rank, int world, long long timeout_ticks,
                       hipStream_t stream);
int k8s_gemv_allreduce_max_groups();
}

namespace k8sllm {

namespace {
void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}
void ckrc(int rc, const char* what) {
  if (rc == 0) return;
  if (rc < 0) throw std::invalid_argument(std::string(what) + ": invalid arguments (code " + std::to_string(rc) + ")");
  throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(static_cast<hipError_t>(rc)));
}
}  // namespace

XgmiComm::XgmiComm(int world, int rank, long long slot_bytes, int blocks, double timeout_s)
    : world_(world), rank_(rank), blocks_(blocks), slot_bytes_(slot_bytes) {
  if (world < 2 || world > 8 || rank < 0 || rank >= world) throw std::invalid_argument("XgmiComm: bad world/rank");
  if (slot_bytes <= 0 || (slot_bytes & 4095)) throw std::invalid_argument("XgmiComm: slot_bytes must be a multiple of 4096");
  if (blocks < 1 || blocks > k8s_xgmi_max_blocks()) throw std::invalid_argument("XgmiComm: bad block count");
  // flagged + LL + two-shot (2 phases) + the fused GEMV all-reduce's LL rows (gemv.hip GemvAr)
  fused_off_ = k8s_xgmi_flag_bytes() + 8LL * world * slot_bytes;
  region_bytes_ = fused_off_ + 2LL * world * slot_bytes;
  if (region_bytes_ > 0x7fffffffLL) throw std::invalid_argument("XgmiComm: region larger than 2 GiB");
  timeout_ticks_ = static_cast<long long>(timeout_s * 100e6);  // s_memrealtime runs at 100 MHz
  ck(hipGetDevice(&device_), "hipGetDevice");
  ck(hipExtMallocWithFlags(&region_, region_bytes_, hipDeviceMallocUncached), "hipExtMallocWithFlags(uncached)");
  ck(hipMemset(region_, 0, region_bytes_), "hipMemset");
  ck(hipMalloc(&counters_, (k8s_xgmi_max_blocks() + 1) * sizeof(uint32_t)), "hipMalloc");
  ck(hipMemset(counters_, 0, (k8s_xgmi_max_blocks() + 1) * sizeof(uint32_t)), "hipMemset");
  ck(hipExtMallocWithFlags(reinterpret_cast<void**>(&fused_state_), 2 * k8s_gemv_allreduce_max_groups() * sizeof(uint32_t),
                           hipDeviceMallocUncached), "hipExtMallocWithFlags(fused state)");
  ck(hipMemset(fused_state_, 0, 2 * k8s_gemv_allreduce_max_groups() * sizeof(uint32_t)), "hipMemset");
  ck(hipHostMalloc(reinterpret_cast<void**>(&host_err_), sizeof(uint32_t), hipHostMallocDefault), "hipHostMalloc");
  *host_err_ = 0;
  ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  bases_.assign(world, nullptr);
  mapped_.assign(world, false);
  bases_[rank] = region_;
}

XgmiComm::~XgmiComm() {
  for (int i = 0; i < world_; ++i)
    if (mapped_[i] && bases_[i]) (void)hipIpcCloseMemHandle(bases_[i]);
  if (region_) (void)hipFree(region_);
  if (counters_) (void)hipFree(counters_);
  if (fused_state_) (void)hipFree(fused_state_);
  if (host_err_) (void)hipHostFree(host_err_);
}

std::string XgmiComm::handle() const {
  hipIpcMemHandle_t h;
  ck(hipIpcGetMemHandle(&h, region_), "hipIpcGetMemHandle");
  return std::string(reinterpret_cast<const char*>(&h), sizeof(h));
}

void XgmiComm::open(const std::vector<std::string>& handles) {
  if (opened_) throw std::runtime_error("XgmiComm: already open");
  if ((int)handles.size() != world_) throw std::invalid_argument("XgmiComm::open: need one handle per rank");
  for (int i = 0; i < world_; ++i) {
    if (i == rank_) continue;
    if (handles[i].size() != sizeof(hipIpcMemHandle_t)) throw std::invalid_argument("XgmiComm::open: bad handle size");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handles[i].data(), sizeof(h));
    void* p = nullptr;
    ck(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
    bases_[i] = p;
    mapped_[i] = true;
  }
  opened_ = true;
}

void XgmiComm::all_reduce_bf16(const void* in, void* out, long long bytes, hipStream_t s, const void* residual) {
  if (!opened_) throw std::runtime_error("XgmiComm: not open");
  if (bytes > slot_bytes_ || (twoshot_min_bytes_ > 0 && bytes >= twoshot_min_bytes_)) {
    ckrc(k8s_xgmi_allreduce_2shot_bf16(bases_.data(), counters_, counters_ + k8s_xgmi_max_blocks(), in, out, bytes,
                                       slot_bytes_, rank_, world_, blocks_, timeout_ticks_, residual, s),
         "xgmi all_reduce (two-shot)");
    return;
  }
  if (bytes <= ll_max_bytes_ && 2 * bytes <= slot_bytes_) {
    ckrc(k8s_xgmi_allreduce_ll_bf16(bases_.data(), counters_, counters_ + k8s_xgmi_max_blocks(), in, out, bytes,
                                    slot_bytes_, rank_, world_, blocks_, timeout_ticks_, residual, s),
         "xgmi all_reduce (LL)");
    return;
  }
  ckrc(k8s_xgmi_allreduce_bf16(bases_.data(), counters_, counters_ + k8s_xgmi_max_blocks(), in, out, bytes,
                               slot_bytes_, rank_, world_, blocks_, timeout_ticks_, residual, s),
       "xgmi all_reduce");
}

int XgmiComm::gemv_allreduce(void* out, const void* x, const void* w, const float* wscale, int M, int N, int K,
                             const void* residual, hipStream_t s) {
  if (!opened_) throw std::runtime_error("XgmiComm: not open");
  void* fb[8];
  for (int i = 0; i < world_; ++i) fb[i] = static_cast<char*>(bases_[i]) + fused_off_;
  const int rc = k8s_gemv_allreduce(out, x, w, wscale, M, N, K, residual, fb, slot_bytes_, fused_state_,
                                    fused_state_ + k8s_gemv_allreduce_max_groups(), counters_ + k8s_xgmi_max_blocks(),
                                    rank_, world_, timeout_ticks_, s);
  if (rc == -5) return rc;  // shape outside the fused plan: the caller runs GEMV + all-reduce
  ckrc(rc, "xgmi gemv_allreduce");
  return 0;
}

void XgmiComm::all_gather(const void* in, void* out, long long bytes, hipStream_t s) {
  if (!opened_) throw std::runtime_error("XgmiComm: not open");
  ckrc(k8s_xgmi_allgather(bases_.data(), counters_, counters_ + k8s_xgmi_max_blocks(), in, out, bytes, slot_bytes_,
                          rank_, world_, blocks_, timeout_ticks_, s),
       "xgmi all_gather");
}

uint32_t XgmiComm::error() {
  uint32_t v = 0;
  ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  ck(hipMemcpy(&v, counters_ + k8s_xgmi_max_blocks(), sizeof(v), hipMemcpyDeviceToHost), "hipMemcpy");
  return v;
}

void XgmiComm::snapshot_error(hipStream_t s) {
  ck(hipMemcpyAsync(host_err_, counters_ + k8s_xgmi_max_blocks(), sizeof(uint32_t), hipMemcpyDeviceToHost, s),
     "hipMemcpyAsync(error word)");
}

uint32_t XgmiComm::last_error() const { return *reinterpret_cast<volatile uint32_t*>(host_err_); }

void XgmiComm::reset() {
  ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
  ck(hipMemset(region_, 0, region_bytes_), "hipMemset(region)");
  ck(hipMemset(counters_, 0, (k8s_xgmi_max_blocks() + 1) * sizeof(uint32_t)), "hipMemset(counters)");
  ck(hipMemset(fused_state_, 0, 2 * k8s_gemv_allreduce_max_groups() * sizeof(uint32_t)), "hipMemset(fused state)");
  *host_err_ = 0;
  ck(hipDeviceSynchronize(), "hipDeviceSynchronize");
}

void XgmiComm::reset_error() {
  ck(hipMemset(counters_ + k8s_xgmi_max_blocks(), 0, sizeof(uint32_t)), "hipMemset");
}

}  // namespace k8sllm
