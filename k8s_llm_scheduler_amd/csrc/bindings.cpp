// pybind11 module `_C`: launchers for the gfx950 kernels + native runtime classes.
//
// Tensors cross the boundary as raw device pointers (Python passes tensor.data_ptr()); shape and
// dtype checks live in the Python wrappers (k8s_llm_scheduler_amd/ops/__init__.py).  Kernels are
// launched on the CURRENT PyTorch HIP stream (queried through c10), so they are captured by
// torch.cuda.CUDAGraph (= hipGraph) like any PyTorch op.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <chrono>
#include <cstdint>
#include <cstring>
#include <thread>
#include <stdexcept>
#include <string>

#include "runtime/block_allocator.h"
#include "runtime/rccl_comm.h"
#include "runtime/xgmi_comm.h"

namespace py = pybind11;

extern "C" {
void* k8s_current_stream();
int k8s_rmsnorm(void* out, const void* x, void* residual, const void* w, int rows, int H, float eps, hipStream_t s);
int k8s_rope_kv_write(void* q_out, void* k_cache, void* v_cache, const void* qkv, const float* cos_sin,
                      const int* positions, const int* slot_mapping, const int* context_lens, const int* block_tables,
                      int max_blocks, int block_size, int T, int nq, int nkv, int D, hipStream_t s);
int k8s_paged_decode_attention(void* out, void* part_acc, void* part_ml, const void* q, const void* k_cache,
                               const void* v_cache, const int* block_tables, const int* context_lens, float scale,
                               int B, int nq, int nkv, int D, int block_size, int max_blocks, int part, int pmax,
                               hipStream_t s);
int k8s_paged_prefill_attention(void* out, const void* q, const void* k_cache, const void* v_cache, const int* cu_q,
                                const int* context_lens, const int* block_tables, float scale, int num_seqs,
                                int max_qlen, int nq, int nkv, int D, int block_size, int max_blocks, hipStream_t s);
void k8s_gemv_plan(int M, int N_out, int K, int epi, int mode, int* ks_out, int* splits_out);
int k8s_sgemv(void* out, void* partial, const void* x, const void* W, const float* wscale, const void* res, int M,
              int N, int K, int epi, int norm, float eps, hipStream_t s);
long long k8s_sgemv_workspace(int M, int N, int K, int epi, int fp8);
// checked builds (common.h K8S_CHECKED): every instrumented unit's device record pointer; -1 in release builds
int k8s_check_bind_misc(void* rec);
int k8s_check_bind_rope_kv(void* rec);
int k8s_check_bind_attn_decode_fused(void* rec);
int k8s_check_bind_attn_decode_split(void* rec);
int k8s_check_bind_attn_prefill(void* rec);
int k8s_check_bind_attn_decode(void* rec);
int k8s_gemv_set_loop(int wg_per_cu);
int k8s_gemv_set_wide(int on);
int k8s_pgemm_set_prio(int mode);
int k8s_pgemm_set_row_slabs(int on);
int k8s_gemv_fp8(void* out, void* partial, const void* x, const void* W, const float* wscale, int M, int N_out,
                 int K, int epi, const void* res_in, void* res_out, const void* nw, float eps, hipStream_t s);
int k8s_quantize_fp8_rows(void* q, float* scale, const void* w, int N, int K, hipStream_t s);
int k8s_quantize_act_fp8(void* q, float* scale, const void* x, int T, int K, hipStream_t s);
int k8s_quantize_act_fp8_rms(void* q, float* scale, const void* x, int T, int K, int rms, float eps, hipStream_t s);
int k8s_quantize_act_mx(void* q, void* e8, const void* x, int T, int K, hipStream_t s);
int k8s_dequant_fp8_rows(void* w, const void* q, const float* scale, int N, int K, hipStream_t s);
int k8s_gemv(void* out, void* partial, const void* x, const void* W, int M, int N_out, int K, int epi, hipStream_t s);
int k8s_gemv_rms(void* out, void* partial, const void* x, const void* W, const float* wscale, int M, int N_out, int K,
                 int epi, const void* res_in, void* res_out, float eps, hipStream_t s);
int k8s_gemv_norm(void* out, void* partial, const void* x, const void* W, int M, int N_out, int K, int epi,
                  const void* res_in, void* res_out, const void* nw, float eps, hipStream_t s);
int k8s_decode_attention_fused(void* out, void* part_acc, void* part_ml, const void* qkv, const float* cos_sin,
                               void* k_cache, void* v_cache, const int* block_tables, const int* context_lens,
                               float scale, int B, int nq, int nkv, int D, int block_size, int max_blocks, int pmax, int part,
                               void* oq, void* oe, const int* cas, const float* pre, int ngm, int rec_stride,
                               hipStream_t s);
int k8s_decode_prefix_col_blocks(int B, int nq, int nkv);
int k8s_decode_prefix(void* pre, int rec_stride, const void* qkv, const float* cos_sin, const void* k_cache,
                      const void* v_cache, const int* block_tables, const int* context_lens, const int* cas, float scale,
                      int B, int nq, int nkv, int D, int block_size, int max_blocks, int ngm, hipStream_t s);
long long k8s_decode_split_workspace(int B, int nq, int nkv, int pmax);
int k8s_decode_attention_split(void* out, void* part, uint32_t* counters, const void* qkv, const float* cos_sin,
                               void* k_cache, void* v_cache, const int* block_tables, const int* context_lens,
                               float scale, int B, int nq, int nkv, int D, int block_size, int max_blocks, int pmax,
                               hipStream_t s);
int k8s_sample(int* tokens, const float* logits, int B, int Vs, int shards, const float* temperature,
               const float* top_p, const uint32_t* seeds, const int* counter, int* ctx_inc, int* hist, int hist_stride,
               int* steps, void* scratch, void* nuc_scratch, const int* slots, const int* stop_cls, int* stop_json,
               const int* stop_cfg, const int* stop_forced, const int* stop_forced_len, int stop_fstride,
               int stop_eos_tok, int* stop_done, int id_base, void* keys_out, int nuc_passes, hipStream_t s);
int k8s_sample_nuc_local(int level, const float* logits, int B, int Vs, const float* temperature, const float* top_p,
                         const int* ctx_inc, const int* slots, void* nuc_scratch, void* out, hipStream_t s);
int k8s_sample_nuc_combine(int level, const void* g, int ld, int ranks, int B, const float* temperature,
                           const float* top_p, const int* ctx_inc, const int* slots, void* nuc_scratch, void* mine,
                           hipStream_t s);
int k8s_sample_merge(int* tokens, const void* g, int ld, int ranks, int B, int* ctx_inc, int* hist, int hist_stride,
                     int* steps, const int* slots, const int* stop_cls, int* stop_json, const int* stop_cfg,
                     const int* stop_forced, const int* stop_forced_len, int stop_fstride, int stop_eos_tok,
                     int* stop_done, hipStream_t s);
long long k8s_sample_scratch_bytes(int B);
long long k8s_sample_nucleus_bytes(int B, int shards);
int k8s_embedding(void* out, const int* ids, const void* table, int T, int H, int vocab, void* oq, void* oe,
                  hipStream_t s);
int k8s_silu_mul(void* out, const void* gu, int T, int I, hipStream_t s);
int k8s_prefetch(const void* p, long long bytes, int blocks, void* sink, hipStream_t s);
int k8s_hash_init(void* out, int rows, int cols, long long gcols, long long row0, long long col0, uint32_t seed,
                  uint32_t tensor_id, float scale, float shift, hipStream_t s);
int k8s_mgemm_num_configs();
int k8s_mgemm_lds_bytes(int cfg, int mode);
int k8s_mgemm_config(int cfg, int* bm, int* bn, int* threads, int* lds_bytes, int* swiglu, int* rb);
int k8s_mgemm_plan_info(int M, int N_out, int K, int epi, int fp8, int cfg, int nwg, long long* tiles, int* cmax,
                        long long* ws_elems);
int k8s_mgemm(void* out, float* ws, unsigned* tickets, const void* x, const void* W, const float* xs, const float* wsc,
              int M, int N_out, int K, int epi, int fp8, int cfg, int nwg, int cmax, const void* res, int rms,
              float eps, void* oq, void* oe, int fenced, hipStream_t s);
int k8s_pgemm4_num_configs();
int k8s_pgemm4_config(int cfg, int* bp, int* bq, int* lds_bytes);
int k8s_pgemm4_plan(int M, int N_out, int K, int epi, int cfg, int splits, int* nwg, long long* slab_elems);
int k8s_pgemm4(void* out, float* slab, const void* x, const void* W, int M, int N_out, int K, int epi, int cfg,
               int splits, int group_m, const void* res, int rms, float eps, hipStream_t s);
int k8s_pgemm_num_configs();
int k8s_pgemm_config(int cfg, int* bp, int* bq, int* lds_bytes);
int k8s_pgemm_plan(int M, int N_out, int K, int epi, int fp8, int cfg, int splits, int* nwg, long long* ws_elems,
                   int* tickets);
int k8s_pgemm(void* out, float* ws, unsigned* tickets, const void* x, const void* W, const float* xs, const float* wsc,
              int M, int N_out, int K, int epi, int fp8, int cfg, int splits, int group_m, const void* res, int rms,
              float eps, void* oq, void* oe, hipStream_t s);
}

namespace {

template <typename T = void>
inline T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }

inline hipStream_t S(int64_t s) {
  return s < 0 ? reinterpret_cast<hipStream_t>(k8s_current_stream()) : reinterpret_cast<hipStream_t>(s);
}

inline void check(int rc, const char* what) {
  if (rc == 0) return;
  std::string msg = std::string(what) + " failed: ";
  if (rc < 0) msg += "invalid arguments (code " + std::to_string(rc) + ")";
  else msg += hipGetErrorString(static_cast<hipError_t>(rc));
  throw std::runtime_error(msg);
}

}  // namespace

#ifndef K8S_MODULE_NAME
#define K8S_MODULE_NAME _C
#endif
PYBIND11_MODULE(K8S_MODULE_NAME, m) {
#ifdef K8S_CHECKED
  m.attr("checked") = true;
#else
  m.attr("checked") = false;
#endif
  // point every instrumented unit at one device record (ops.check_*); returns 0, or nonzero in release builds
  m.def("check_bind", [](uintptr_t rec) {
    int rc = 0;
    for (auto f : {k8s_check_bind_misc, k8s_check_bind_rope_kv, k8s_check_bind_attn_decode_fused,
                   k8s_check_bind_attn_decode_split, k8s_check_bind_attn_prefill, k8s_check_bind_attn_decode})
      rc |= f(reinterpret_cast<void*>(rec));
    return rc;
  });
  m.doc() = "gfx950 HIP kernels and native runtime of k8s_llm_scheduler_amd";
  m.attr("ARCH") = "gfx950";

  m.def("rmsnorm", [](uintptr_t out, uintptr_t x, uintptr_t residual, uintptr_t w, int rows, int H, float eps,
                      int64_t s) { check(k8s_rmsnorm(P(out), P(x), P(residual), P(w), rows, H, eps, S(s)), "rmsnorm"); });
  m.def("rope_kv_write", [](uintptr_t q_out, uintptr_t kc, uintptr_t vc, uintptr_t qkv, uintptr_t cos_sin,
                            uintptr_t pos, uintptr_t slots, uintptr_t ctx, uintptr_t bt, int max_blocks, int bs, int T,
                            int nq, int nkv, int D, int64_t s) {
    check(k8s_rope_kv_write(P(q_out), P(kc), P(vc), P(qkv), P<float>(cos_sin), P<int>(pos), P<int>(slots),
                            P<int>(ctx), P<int>(bt), max_blocks, bs, T, nq, nkv, D, S(s)),
          "rope_kv_write");
  });
  m.def("paged_decode_attention", [](uintptr_t out, uintptr_t pacc, uintptr_t pml, uintptr_t q, uintptr_t kc,
                                     uintptr_t vc, uintptr_t bt, uintptr_t ctx, float scale, int B, int nq, int nkv,
                                     int D, int bs, int max_blocks, int part, int pmax, int64_t s) {
    check(k8s_paged_decode_attention(P(out), P(pacc), P(pml), P(q), P(kc), P(vc), P<int>(bt), P<int>(ctx), scale, B,
                                     nq, nkv, D, bs, max_blocks, part, pmax, S(s)),
          "paged_decode_attention");
  });
  m.def("paged_prefill_attention", [](uintptr_t out, uintptr_t q, uintptr_t kc, uintptr_t vc, uintptr_t cu_q,
                                      uintptr_t ctx, uintptr_t bt, float scale, int nseq, int max_qlen, int nq,
                                      int nkv, int D, int bs, int max_blocks, int64_t s) {
    check(k8s_paged_prefill_attention(P(out), P(q), P(kc), P(vc), P<int>(cu_q), P<int>(ctx), P<int>(bt), scale, nseq,
                                      max_qlen, nq, nkv, D, bs, max_blocks, S(s)),
          "paged_prefill_attention");
  });
  // Bounded wait for a recorded hipEvent (torch.cuda.Event.cuda_event) with the GIL released: the engine's per-step
  // device waits must neither block forever (a stalled collective) nor hold the GIL while they poll (the control
  // plane's watch / worker threads run beside the engine loop).  True once the event completed, False at the timeout.
  m.def("event_wait", [](uintptr_t ev, double timeout_s) {
    py::gil_scoped_release nogil;
    const auto e = reinterpret_cast<hipEvent_t>(ev);
    const auto t0 = std::chrono::steady_clock::now();
    for (long spins = 0;; ++spins) {
      const hipError_t r = hipEventQuery(e);
      if (r == hipSuccess) return true;
      if (r != hipErrorNotReady) throw std::runtime_error(std::string("hipEventQuery: ") + hipGetErrorString(r));
      const double waited = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (waited >= timeout_s) return false;
      if (waited < 0.005) std::this_thread::yield();   // decode steps end within milliseconds: stay responsive
      else std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }, py::arg("event"), py::arg("timeout_s"));
  m.def("pgemm_set_prio", [](int mode) { return k8s_pgemm_set_prio(mode); });
  m.def("pgemm_set_row_slabs", [](int on) { return k8s_pgemm_set_row_slabs(on); });
  m.def("gemv_set_wide", [](int on) { return k8s_gemv_set_wide(on); });
  m.def("gemv_set_loop", [](int wg) { return k8s_gemv_set_loop(wg); });
  m.def("gemv_plan", [](int M, int N, int K, int epi, int mode) {
    int ks, sp;
    k8s_gemv_plan(M, N, K, epi, mode, &ks, &sp);
    return py::make_tuple(ks, sp);
  });
  m.def("gemv_fp8", [](uintptr_t out, uintptr_t partial, uintptr_t x, uintptr_t W, uintptr_t wscale, int M, int N,
                       int K, int epi, uintptr_t res_in, uintptr_t res_out, uintptr_t nw, float eps, int64_t s) {
    check(k8s_gemv_fp8(P(out), P(partial), P(x), P(W), P<float>(wscale), M, N, K, epi, P(res_in), P(res_out), P(nw),
                       eps, S(s)),
          "gemv_fp8");
  });
  m.def("quantize_fp8_rows", [](uintptr_t q, uintptr_t scale, uintptr_t w, int N, int K, int64_t s) {
    check(k8s_quantize_fp8_rows(P(q), P<float>(scale), P(w), N, K, S(s)), "quantize_fp8_rows");
  });
  m.def("quantize_act_fp8", [](uintptr_t q, uintptr_t scale, uintptr_t x, int T, int K, int64_t s) {
    check(k8s_quantize_act_fp8(P(q), P<float>(scale), P(x), T, K, S(s)), "quantize_act_fp8");
  });
  m.def("quantize_act_mx", [](uintptr_t q, uintptr_t e8, uintptr_t x, int T, int K, int64_t s) {
    check(k8s_quantize_act_mx(P(q), P(e8), P(x), T, K, S(s)), "quantize_act_mx");
  });
  m.def("quantize_act_fp8_rms", [](uintptr_t q, uintptr_t scale, uintptr_t x, int T, int K, int rms, float eps,
                                   int64_t s) {
    check(k8s_quantize_act_fp8_rms(P(q), P<float>(scale), P(x), T, K, rms, eps, S(s)), "quantize_act_fp8_rms");
  });
  m.def("dequant_fp8_rows", [](uintptr_t w, uintptr_t q, uintptr_t scale, int N, int K, int64_t s) {
    check(k8s_dequant_fp8_rows(P(w), P(q), P<float>(scale), N, K, S(s)), "dequant_fp8_rows");
  });
  m.def("gemv", [](uintptr_t out, uintptr_t partial, uintptr_t x, uintptr_t W, int M, int N, int K, int epi,
                   int64_t s) { check(k8s_gemv(P(out), P(partial), P(x), P(W), M, N, K, epi, S(s)), "gemv"); });
  m.def("gemv_norm", [](uintptr_t out, uintptr_t partial, uintptr_t x, uintptr_t W, int M, int N, int K, int epi,
                        uintptr_t res_in, uintptr_t res_out, uintptr_t nw, float eps, int64_t s) {
    check(k8s_gemv_norm(P(out), P(partial), P(x), P(W), M, N, K, epi, P(res_in), P(res_out), P(nw), eps, S(s)),
          "gemv_norm");
  });
  // small-batch decode GEMV (3..8 rows, x in registers): returns -5 (nothing launched) for a combination it does not
  // instantiate, so the caller can take another kernel
  m.def("sgemv", [](uintptr_t out, uintptr_t partial, uintptr_t x, uintptr_t W, uintptr_t wscale, uintptr_t res, int M,
                    int N, int K, int epi, int norm, float eps, int64_t s) {
    const int rc = k8s_sgemv(P(out), P(partial), P(x), P(W), P<float>(wscale), P(res), M, N, K, epi, norm, eps, S(s));
    if (rc != -5) check(rc, "sgemv");
    return rc;
  });
  m.def("sgemv_workspace", [](int M, int N, int K, int epi, int fp8) { return k8s_sgemv_workspace(M, N, K, epi, fp8); });
  m.def("gemv_rms", [](uintptr_t out, uintptr_t partial, uintptr_t x, uintptr_t W, uintptr_t wscale, int M, int N,
                       int K, int epi, uintptr_t res_in, uintptr_t res_out, float eps, int64_t s) {
    check(k8s_gemv_rms(P(out), P(partial), P(x), P(W), P<float>(wscale), M, N, K, epi, P(res_in), P(res_out), eps, S(s)),
          "gemv_rms");
  });
  m.def("decode_attention_fused", [](uintptr_t out, uintptr_t pacc, uintptr_t pml, uintptr_t qkv, uintptr_t cos_sin,
                                     uintptr_t kc, uintptr_t vc, uintptr_t bt, uintptr_t ctx, float scale, int B, int nq,
                                     int nkv, int D, int bs, int max_blocks, int pmax, int part, int64_t s,
                                     uintptr_t oq, uintptr_t oe, uintptr_t cas, uintptr_t pre, int ngm, int rec_stride) {
    check(k8s_decode_attention_fused(P(out), P(pacc), P(pml), P(qkv), P<float>(cos_sin), P(kc), P(vc), P<int>(bt),
                                     P<int>(ctx), scale, B, nq, nkv, D, bs, max_blocks, pmax, part, P(oq), P(oe),
                                     P<int>(cas), P<float>(pre), ngm, rec_stride, S(s)),
          "decode_attention_fused");
  }, py::arg("out"), py::arg("pacc"), py::arg("pml"), py::arg("qkv"), py::arg("cos_sin"), py::arg("kc"),
     py::arg("vc"), py::arg("bt"), py::arg("ctx"), py::arg("scale"), py::arg("B"), py::arg("nq"), py::arg("nkv"),
     py::arg("D"), py::arg("bs"), py::arg("max_blocks"), py::arg("pmax"), py::arg("part"), py::arg("s"),
     py::arg("oq") = 0, py::arg("oe") = 0, py::arg("cas") = 0, py::arg("pre") = 0, py::arg("ngm") = 0,
     py::arg("rec_stride") = 0);
  m.def("decode_prefix_col_blocks", [](int B, int nq, int nkv) { return k8s_decode_prefix_col_blocks(B, nq, nkv); });
  m.def("decode_prefix", [](uintptr_t pre, int rec_stride, uintptr_t qkv, uintptr_t cos_sin, uintptr_t kc,
                            uintptr_t vc, uintptr_t bt, uintptr_t ctx, uintptr_t cas, float scale, int B, int nq, int nkv,
                            int D, int bs, int max_blocks, int ngm, int64_t s) {
    check(k8s_decode_prefix(P(pre), rec_stride, P(qkv), P<float>(cos_sin), P(kc), P(vc), P<int>(bt), P<int>(ctx),
                            P<int>(cas), scale, B, nq, nkv, D, bs, max_blocks, ngm, S(s)),
          "decode_prefix");
  });
  m.def("decode_split_workspace", [](int B, int nq, int nkv, int pmax) {
    return k8s_decode_split_workspace(B, nq, nkv, pmax);
  });
  m.def("decode_attention_split", [](uintptr_t out, uintptr_t part, uintptr_t counters, uintptr_t qkv,
                                     uintptr_t cos_sin, uintptr_t kc, uintptr_t vc, uintptr_t bt, uintptr_t ctx,
                                     float scale, int B, int nq, int nkv, int D, int bs, int max_blocks, int pmax,
                                     int64_t s) {
    check(k8s_decode_attention_split(P(out), P(part), P<uint32_t>(counters), P(qkv), P<float>(cos_sin), P(kc), P(vc),
                                     P<int>(bt), P<int>(ctx), scale, B, nq, nkv, D, bs, max_blocks, pmax, S(s)),
          "decode_attention_split");
  });
  m.def("sample", [](uintptr_t tokens, uintptr_t logits, int B, int Vs, int shards, uintptr_t temp, uintptr_t top_p,
                     uintptr_t seeds, uintptr_t counter, uintptr_t ctx_inc, uintptr_t hist, int hist_stride,
                     uintptr_t steps, uintptr_t scratch, uintptr_t nuc_scratch, uintptr_t slots, uintptr_t cls,
                     uintptr_t json, uintptr_t cfg, uintptr_t forced, uintptr_t forced_len, int fstride, int eos_tok,
                     uintptr_t done, int64_t s, int id_base, uintptr_t keys_out, int nuc_passes) {
    check(k8s_sample(P<int>(tokens), P<float>(logits), B, Vs, shards, P<float>(temp), P<float>(top_p),
                     P<uint32_t>(seeds), P<int>(counter), P<int>(ctx_inc), P<int>(hist), hist_stride, P<int>(steps),
                     P(scratch), P(nuc_scratch), P<int>(slots), P<int>(cls), P<int>(json), P<int>(cfg), P<int>(forced),
                     P<int>(forced_len), fstride, eos_tok, P<int>(done), id_base, P(keys_out), nuc_passes, S(s)),
          "sample");
  }, py::arg("tokens"), py::arg("logits"), py::arg("B"), py::arg("Vs"), py::arg("shards"), py::arg("temp"),
     py::arg("top_p"), py::arg("seeds"), py::arg("counter"), py::arg("ctx_inc"), py::arg("hist"),
     py::arg("hist_stride"), py::arg("steps"), py::arg("scratch"), py::arg("nuc_scratch"), py::arg("slots"),
     py::arg("cls"), py::arg("json"), py::arg("cfg"), py::arg("forced"), py::arg("forced_len"), py::arg("fstride"),
     py::arg("eos_tok"), py::arg("done"), py::arg("stream"), py::arg("id_base") = 0, py::arg("keys_out") = 0,
     py::arg("nuc_passes") = 1);
  // vocab-parallel sampling stages (sampler.hip): the TP ranks exchange row maxima / bin totals / best keys
  m.def("sample_nuc_local", [](int level, uintptr_t logits, int B, int Vs, uintptr_t temp, uintptr_t top_p,
                               uintptr_t ctx_inc, uintptr_t slots, uintptr_t nuc_scratch, uintptr_t out, int64_t s) {
    check(k8s_sample_nuc_local(level, P<float>(logits), B, Vs, P<float>(temp), P<float>(top_p), P<int>(ctx_inc),
                               P<int>(slots), P(nuc_scratch), P(out), S(s)),
          "sample_nuc_local");
  });
  m.def("sample_nuc_combine", [](int level, uintptr_t g, int ld, int ranks, int B, uintptr_t temp, uintptr_t top_p,
                                 uintptr_t ctx_inc, uintptr_t slots, uintptr_t nuc_scratch, uintptr_t mine, int64_t s) {
    check(k8s_sample_nuc_combine(level, P(g), ld, ranks, B, P<float>(temp), P<float>(top_p), P<int>(ctx_inc),
                                 P<int>(slots), P(nuc_scratch), P(mine), S(s)),
          "sample_nuc_combine");
  });
  m.def("sample_merge", [](uintptr_t tokens, uintptr_t g, int ld, int ranks, int B, uintptr_t ctx_inc, uintptr_t hist,
                           int hist_stride, uintptr_t steps, uintptr_t slots, uintptr_t cls, uintptr_t json,
                           uintptr_t cfg, uintptr_t forced, uintptr_t forced_len, int fstride, int eos_tok,
                           uintptr_t done, int64_t s) {
    check(k8s_sample_merge(P<int>(tokens), P(g), ld, ranks, B, P<int>(ctx_inc), P<int>(hist), hist_stride,
                           P<int>(steps), P<int>(slots), P<int>(cls), P<int>(json), P<int>(cfg), P<int>(forced),
                           P<int>(forced_len), fstride, eos_tok, P<int>(done), S(s)),
          "sample_merge");
  });
  // Host memory the GPU can write (fine-grained, coherent): the decode graphs' done flags, polled by the host
  // between replays without a device synchronisation.
  m.def("host_mapped_alloc", [](size_t bytes) {
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      throw std::runtime_error("hipHostMalloc failed");
    std::memset(p, 0, bytes);
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) throw std::runtime_error("hipHostGetDevicePointer failed");
    return py::make_tuple(reinterpret_cast<uintptr_t>(p), reinterpret_cast<uintptr_t>(d));
  });
  m.def("host_mapped_free", [](uintptr_t p) { (void)hipHostFree(reinterpret_cast<void*>(p)); });
  m.def("sample_scratch_bytes", [](int B) { return k8s_sample_scratch_bytes(B); });
  m.def("sample_nucleus_bytes", [](int B, int shards) { return k8s_sample_nucleus_bytes(B, shards); });
  m.def("embedding", [](uintptr_t out, uintptr_t ids, uintptr_t table, int T, int H, int vocab, int64_t s,
                        uintptr_t oq, uintptr_t oe) {
    check(k8s_embedding(P(out), P<int>(ids), P(table), T, H, vocab, P(oq), P(oe), S(s)), "embedding");
  }, py::arg("out"), py::arg("ids"), py::arg("table"), py::arg("T"), py::arg("H"), py::arg("vocab"), py::arg("s"),
     py::arg("oq") = 0, py::arg("oe") = 0);
  m.def("prefetch", [](uintptr_t p, long long bytes, int blocks, uintptr_t sink, int64_t s) {
    check(k8s_prefetch(P(p), bytes, blocks, P(sink), S(s)), "prefetch");
  });
  m.def("silu_mul", [](uintptr_t out, uintptr_t gu, int T, int I, int64_t s) {
    check(k8s_silu_mul(P(out), P(gu), T, I, S(s)), "silu_mul");
  });
  m.def("hash_init", [](uintptr_t out, int rows, int cols, long long gcols, long long row0, long long col0,
                        uint32_t seed, uint32_t tid, float scale, float shift, int64_t s) {
    check(k8s_hash_init(P(out), rows, cols, gcols, row0, col0, seed, tid, scale, shift, S(s)), "hash_init");
  });

  m.def("mgemm_configs", []() {
    py::list out;
    for (int c = 0; c < k8s_mgemm_num_configs(); ++c) {
      int bm = 0, bn = 0, th = 0, lds = 0, sw = 0, rb = 0;
      k8s_mgemm_config(c, &bm, &bn, &th, &lds, &sw, &rb);
      out.append(py::make_tuple(bm, bn, th, lds, sw != 0, rb));
    }
    return out;
  });
  m.def("mgemm_lds_bytes", [](int cfg, int mode) { return k8s_mgemm_lds_bytes(cfg, mode); });
  m.def("mgemm_plan_info", [](int M, int N, int K, int epi, int fp8, int cfg, int nwg) {
    long long tiles = 0, ws = 0;
    int cmax = 0;
    if (k8s_mgemm_plan_info(M, N, K, epi, fp8, cfg, nwg, &tiles, &cmax, &ws) != 0)
      throw std::invalid_argument("mgemm_plan_info: invalid plan");
    return py::make_tuple(tiles, cmax, ws);
  });
  m.def("mgemm", [](uintptr_t out, uintptr_t ws, uintptr_t tickets, uintptr_t x, uintptr_t W, uintptr_t xs,
                    uintptr_t wsc, int M, int N, int K, int epi, int fp8, int cfg, int nwg, int cmax, uintptr_t res,
                    int rms, float eps, int64_t s, uintptr_t oq, uintptr_t oe, int fenced) {
    check(k8s_mgemm(P(out), P<float>(ws), P<unsigned>(tickets), P(x), P(W), P<float>(xs), P<float>(wsc), M, N, K,
                    epi, fp8, cfg, nwg, cmax, P(res), rms, eps, P(oq), P(oe), fenced, S(s)),
          "mgemm");
  }, py::arg("out"), py::arg("ws"), py::arg("tickets"), py::arg("x"), py::arg("W"), py::arg("xs"), py::arg("wsc"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("fp8"), py::arg("cfg"), py::arg("nwg"),
     py::arg("cmax"), py::arg("res"), py::arg("rms"), py::arg("eps"), py::arg("s"), py::arg("oq") = 0,
     py::arg("oe") = 0, py::arg("fenced") = 0);

  m.def("pgemm4_configs", []() {
    py::list out;
    for (int c = 0; c < k8s_pgemm4_num_configs(); ++c) {
      int bp = 0, bq = 0, lds = 0;
      k8s_pgemm4_config(c, &bp, &bq, &lds);
      out.append(py::make_tuple(bp, bq, lds));
    }
    return out;
  });
  m.def("pgemm4_plan", [](int M, int N, int K, int epi, int cfg, int splits) {
    int nwg = 0;
    long long slab = 0;
    if (k8s_pgemm4_plan(M, N, K, epi, cfg, splits, &nwg, &slab) != 0)
      throw std::invalid_argument("pgemm4_plan: invalid plan");
    return py::make_tuple(nwg, slab);
  });
  m.def("pgemm4", [](uintptr_t out, uintptr_t slab, uintptr_t x, uintptr_t W, int M, int N, int K, int epi, int cfg,
                     int splits, int group_m, uintptr_t res, int rms, float eps, int64_t s) {
    check(k8s_pgemm4(P(out), P<float>(slab), P(x), P(W), M, N, K, epi, cfg, splits, group_m, P(res), rms, eps, S(s)),
          "pgemm4");
  });
  m.def("pgemm_configs", []() {
    py::list out;
    for (int c = 0; c < k8s_pgemm_num_configs(); ++c) {
      int bp = 0, bq = 0, lds = 0;
      k8s_pgemm_config(c, &bp, &bq, &lds);
      out.append(py::make_tuple(bp, bq, lds));
    }
    return out;
  });
  m.def("pgemm_plan", [](int M, int N, int K, int epi, int fp8, int cfg, int splits) {
    int nwg = 0, tickets = 0;
    long long ws = 0;
    if (k8s_pgemm_plan(M, N, K, epi, fp8, cfg, splits, &nwg, &ws, &tickets) != 0)
      throw std::invalid_argument("pgemm_plan: invalid plan");
    return py::make_tuple(nwg, ws, tickets);
  });
  m.def("pgemm", [](uintptr_t out, uintptr_t ws, uintptr_t tickets, uintptr_t x, uintptr_t W, uintptr_t xs,
                    uintptr_t wsc, int M, int N, int K, int epi, int fp8, int cfg, int splits, int group_m,
                    uintptr_t res, int rms, float eps, int64_t s, uintptr_t oq, uintptr_t oe) {
    check(k8s_pgemm(P(out), P<float>(ws), P<unsigned>(tickets), P(x), P(W), P<float>(xs), P<float>(wsc), M, N, K,
                    epi, fp8, cfg, splits, group_m, P(res), rms, eps, P(oq), P(oe), S(s)),
          "pgemm");
  }, py::arg("out"), py::arg("ws"), py::arg("tickets"), py::arg("x"), py::arg("W"), py::arg("xs"), py::arg("wsc"),
     py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("fp8"), py::arg("cfg"), py::arg("splits"),
     py::arg("group_m"), py::arg("res"), py::arg("rms"), py::arg("eps"), py::arg("s"), py::arg("oq") = 0,
     py::arg("oe") = 0);

  using k8sllm::RcclComm;
  py::class_<RcclComm>(m, "RcclComm")
      .def_static("unique_id", []() {
        auto v = RcclComm::unique_id();
        return py::bytes(reinterpret_cast<const char*>(v.data()), v.size());
      })
      .def(py::init([](int world, int rank, py::bytes id) {
             std::string s = id;
             return new RcclComm(world, rank, std::vector<uint8_t>(s.begin(), s.end()));
           }))
      .def("all_reduce", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int red,
                            int64_t s) { c.all_reduce(P(send), P(recv), count, dtype, red, S(s)); })
      .def("all_gather", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int64_t s) {
        c.all_gather(P(send), P(recv), count, dtype, S(s));
      })
      .def("reduce_scatter", [](RcclComm& c, uintptr_t send, uintptr_t recv, size_t count, int dtype, int red,
                                int64_t s) { c.reduce_scatter(P(send), P(recv), count, dtype, red, S(s)); })
      .def("broadcast", [](RcclComm& c, uintptr_t buf, size_t count, int dtype, int root, int64_t s) {
        c.broadcast(P(buf), count, dtype, root, S(s));
      })
      .def("async_error", &RcclComm::async_error)
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def_property_readonly("world", &RcclComm::world)
      .def_property_readonly("rank", &RcclComm::rank);

  using k8sllm::XgmiComm;
  py::class_<XgmiComm>(m, "XgmiComm")
      .def(py::init<int, int, long long, int, double>(), py::arg("world"), py::arg("rank"), py::arg("slot_bytes"),
           py::arg("blocks") = 16, py::arg("timeout_s") = 30.0)
      .def("handle", [](const XgmiComm& c) { return py::bytes(c.handle()); })
      .def("open", [](XgmiComm& c, const std::vector<py::bytes>& hs) {
        std::vector<std::string> v;
        for (const auto& h : hs) v.emplace_back(h);
        c.open(v);
      })
      .def(
          "all_reduce_bf16",
          [](XgmiComm& c, uintptr_t in, uintptr_t out, long long bytes, int64_t s, uintptr_t residual) {
            c.all_reduce_bf16(P(in), P(out), bytes, S(s), P(residual));
          },
          py::arg("inp"), py::arg("out"), py::arg("bytes"), py::arg("stream") = -1, py::arg("residual") = 0)
      .def("all_gather", [](XgmiComm& c, uintptr_t in, uintptr_t out, long long bytes, int64_t s) {
        c.all_gather(P(in), P(out), bytes, S(s));
      })
      .def(
          "gemv_allreduce",
          [](XgmiComm& c, uintptr_t out, uintptr_t x, uintptr_t w, uintptr_t wscale, int M, int N, int K,
             uintptr_t residual, int64_t s) {
            return c.gemv_allreduce(P(out), P(x), P(w), reinterpret_cast<const float*>(wscale), M, N, K, P(residual),
                                    S(s));
          },
          py::arg("out"), py::arg("x"), py::arg("w"), py::arg("wscale"), py::arg("M"), py::arg("N"), py::arg("K"),
          py::arg("residual") = 0, py::arg("stream") = -1)
      .def("error", &XgmiComm::error)
      .def("snapshot_error", [](XgmiComm& c, int64_t s) { c.snapshot_error(S(s)); }, py::arg("stream") = -1)
      .def("last_error", &XgmiComm::last_error)
      .def("reset_error", &XgmiComm::reset_error)
      .def("reset", &XgmiComm::reset, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("world", &XgmiComm::world)
      .def_property_readonly("rank", &XgmiComm::rank)
      .def_property_readonly("slot_bytes", &XgmiComm::slot_bytes)
      .def_property_readonly("blocks", &XgmiComm::blocks)
      .def_property_readonly("is_open", &XgmiComm::is_open)
      .def_property("ll_max_bytes", &XgmiComm::ll_max_bytes, &XgmiComm::set_ll_max_bytes)
      .def_property("twoshot_min_bytes", &XgmiComm::twoshot_min_bytes, &XgmiComm::set_twoshot_min_bytes)
      .def_property_readonly("max_allreduce_bytes", &XgmiComm::max_allreduce_bytes);

  using k8sllm::BlockAllocator;
  py::class_<BlockAllocator::Allocation>(m, "Allocation")
      .def_readonly("blocks", &BlockAllocator::Allocation::blocks)
      .def_readonly("cached_tokens", &BlockAllocator::Allocation::cached_tokens)
      .def_readonly("copy_src", &BlockAllocator::Allocation::copy_src)
      .def_readonly("copy_tokens", &BlockAllocator::Allocation::copy_tokens);
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int, int, bool>(), py::arg("num_blocks"), py::arg("block_size"), py::arg("prefix_caching") = true)
      .def("allocate", &BlockAllocator::allocate)
      .def("can_allocate", &BlockAllocator::can_allocate)
      .def("commit_prefix", &BlockAllocator::commit_prefix)
      .def("release", &BlockAllocator::release)
      .def("reset_prefix_cache", &BlockAllocator::reset_prefix_cache)
      .def_property_readonly("num_blocks", &BlockAllocator::num_blocks)
      .def_property_readonly("block_size", &BlockAllocator::block_size)
      .def_property_readonly("num_free", &BlockAllocator::num_free)
      .def_property_readonly("num_cached", &BlockAllocator::num_cached)
      .def_property_readonly("hits", &BlockAllocator::hits)
      .def_property_readonly("queries", &BlockAllocator::queries)
      .def("refcount", &BlockAllocator::refcount);
}
