// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels.
// Wave = 64 lanes everywhere; bf16 tensors are moved as 16-byte vectors (8 x bf16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace k8sllm {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef uint16_t bf16_t;  // raw storage type on the host/ABI side

constexpr int WAVE = 64;

__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32 (RNE, NaN-preserving) on gfx950
  return __builtin_bit_cast(bf16_t, b);
}
// Unpack 2 bf16 held in one dword.
__device__ __forceinline__ float lo_bf(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float hi_bf(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, WAVE);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, WAVE));
  return v;
}

// OCP MX e4m3 (K16 block-scaled activations; fp8.hip has the format): one E8M0 byte per 32 values, the smallest
// power of two >= max|block| / 448 (127 for an all-zero block, clamped to [1, 253]), and the exact reciprocal.
__device__ __forceinline__ uint32_t mx_e8m0(float amax) {
  const uint32_t b = __float_as_uint(amax * (1.f / 448.f));
  uint32_t e = (b >> 23) + ((b & 0x7fffffu) != 0u);
  if (amax == 0.f) e = 127u;
  return min(max(e, 1u), 253u);
}
__device__ __forceinline__ float mx_inv_scale(uint32_t e) { return __uint_as_float((254u - e) << 23); }
// 4 fp32 values x inv -> 4 e4m3 bytes (one dword), saturated, round-to-nearest-even
__device__ __forceinline__ uint32_t mx_pack4(float a, float b, float c, float d, float inv) {
  auto cl = [&](float t) { return fminf(fmaxf(t * inv, -448.f), 448.f); };
  int p = __builtin_amdgcn_cvt_pk_fp8_f32(cl(a), cl(b), 0, false);
  p = __builtin_amdgcn_cvt_pk_fp8_f32(cl(c), cl(d), p, true);
  return (uint32_t)p;
}
// bf16 rounding of an fp32 value (MX producers quantize the bf16 value the bf16 path would have stored)
__device__ __forceinline__ float bf_round(float f) { return bf2f(f2bf(f)); }
// Byte offset of the E8M0 scale of 32-value block kb of row m in an [M][K] MX tensor.  Layout [K / 128][M][4]: the
// four scales of a 128-value k-tile of a row form one dword, and the dwords of consecutive rows are adjacent -- so a
// GEMM stages one k-tile's scales for a run of rows as one contiguous LDS-DMA (one cache line per 32 rows, not one
// per row).
__device__ __forceinline__ size_t mx_scale_off(size_t m, int kb, int M) {
  return ((size_t)(kb >> 2) * (size_t)M + m) * 4 + (size_t)(kb & 3);
}
// MX store of one value per lane, the 32 lanes of an aligned half-wave holding one block (row m, columns col..,
// col of the half-wave's first lane a multiple of 32): shuffle max, then one e4m3 byte per lane and the block's E8M0.
__device__ __forceinline__ void mx_store_lane(uint8_t* oq, uint8_t* oe, size_t m, int col, int K, int M, float v) {
  float amax = fabsf(v);
#pragma unroll
  for (int o = 1; o < 32; o <<= 1) amax = fmaxf(amax, __shfl_xor(amax, o, 64));
  const uint32_t e = mx_e8m0(amax);
  oq[m * (size_t)K + col] = (uint8_t)(mx_pack4(v, 0.f, 0.f, 0.f, mx_inv_scale(e)) & 0xffu);
  if ((col & 31) == 0) oe[mx_scale_off(m, col >> 5, M)] = (uint8_t)e;
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats of LDS.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = (lane < nw) ? red[lane] : 0.f;
  t = wave_sum(t);
  __syncthreads();
  return t;
}

// 32-bit mixing hash (murmur3 finalizer) used for counter-based RNG and deterministic init.
__device__ __forceinline__ uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
__device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  return fmix32(a ^ fmix32(b + 0x9e3779b9u ^ fmix32(c + 0x7f4a7c15u)));
}
// Uniform in (0, 1): 24 random bits, never 0.
__device__ __forceinline__ float u01(uint32_t h) { return ((h >> 8) + 0.5f) * (1.0f / 16777216.0f); }

// ---- checked builds (python -m k8s_llm_scheduler_amd._build --checked -> ops/_C_checked*.so, loaded with
// K8S_CHECKED=1): every index a kernel derives from DATA (block tables, slot mappings, token ids, context lengths) is
// range-checked before it addresses memory.  A violation is recorded in a device record the host reads after each
// engine step (ops.check_read) and the index is clamped to a valid one, so the kernel finishes without touching
// memory it does not own -- the bounds-assert debug build of SURVEY.md section 5 (race detection / sanitizers), with
// no trap: a trapping kernel would take the device down for every process on it.  Release builds compile none of it.
struct K8sCheck {
  unsigned count;         // violations since the last reset
  unsigned code, line;    // the first one: check code (K8S_CHK_*), source line
  unsigned unit;          // translation unit (K8S_CHK_UNIT_*)
  long long value;        // the offending value
  long long kv_slots;     // bounds, set by the host: KV-cache slots (blocks x block size)
  long long num_blocks;   // KV-cache blocks
  long long vocab;        // embedding rows
};
enum { K8S_CHK_SLOT = 1, K8S_CHK_BLOCK = 2, K8S_CHK_CTX = 3, K8S_CHK_TOKEN = 4 };

}  // namespace k8sllm

#ifdef K8S_CHECKED
// One record pointer per translation unit (kernels are built without relocatable device code); K8S_CHECK_UNIT
// defines the unit's bind function, k8s_check_bind (bindings) points every unit at the same record.
static __device__ k8sllm::K8sCheck* g_k8s_check;
__device__ __forceinline__ static void k8s_check_fail(unsigned unit, unsigned code, unsigned line, long long v) {
  k8sllm::K8sCheck* c = g_k8s_check;
  if (c == nullptr) return;
  // the record is written with vector memory instructions only: the address is forced into VGPRs
  unsigned long long a = reinterpret_cast<unsigned long long>(c);
  asm volatile("" : "+v"(a));
  k8sllm::K8sCheck* cv = reinterpret_cast<k8sllm::K8sCheck*>(a);
  const unsigned old = __hip_atomic_fetch_add(&cv->count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old == 0) {
    __hip_atomic_store(&cv->code, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cv->line, line, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cv->unit, unit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cv->value, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
__device__ __forceinline__ static long long k8s_bound(int code) {
  const k8sllm::K8sCheck* c = g_k8s_check;
  if (c == nullptr) return 0x7fffffffffffffffLL;
  return code == k8sllm::K8S_CHK_SLOT ? c->kv_slots : code == k8sllm::K8S_CHK_BLOCK ? c->num_blocks : c->vocab;
}
// var must lie in [lo, bound(code)); otherwise record it and set var = fallback
#define K8S_CHECK_RANGE(var, lo, code, fallback)                                          \
  do {                                                                                    \
    if ((long long)(var) < (long long)(lo) || (long long)(var) >= k8s_bound(code)) {      \
      k8s_check_fail(K8S_CHK_THIS_UNIT, (code), __LINE__, (long long)(var));              \
      (var) = (fallback);                                                                 \
    }                                                                                     \
  } while (0)
// var must be <= maxv (a bound the kernel knows itself); otherwise record it and set var = maxv
#define K8S_CHECK_MAX(var, maxv, code)                                                    \
  do {                                                                                    \
    if ((long long)(var) > (long long)(maxv)) {                                           \
      k8s_check_fail(K8S_CHK_THIS_UNIT, (code), __LINE__, (long long)(var));              \
      (var) = (maxv);                                                                     \
    }                                                                                     \
  } while (0)
// a condition that must hold (no clamp: the caller handles the failure)
#define K8S_CHECK_TRUE(cond, code, value)                                                 \
  do {                                                                                    \
    if (!(cond)) k8s_check_fail(K8S_CHK_THIS_UNIT, (code), __LINE__, (long long)(value)); \
  } while (0)
#define K8S_CHECK_UNIT(name)                                                              \
  extern "C" int k8s_check_bind_##name(void* rec) {                                       \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_k8s_check), &rec, sizeof(rec));            \
  }
#else
#define K8S_CHECK_RANGE(var, lo, code, fallback) \
  do {                                           \
  } while (0)
#define K8S_CHECK_TRUE(cond, code, value) \
  do {                                    \
  } while (0)
#define K8S_CHECK_MAX(var, maxv, code) \
  do {                                 \
  } while (0)
#define K8S_CHECK_UNIT(name) \
  extern "C" int k8s_check_bind_##name(void*) { return -1; }
#endif

#define K8S_CHECK_LAUNCH() (void)hipGetLastError()
