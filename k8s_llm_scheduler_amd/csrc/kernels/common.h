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

}  // namespace k8sllm

#define K8S_CHECK_LAUNCH() (void)hipGetLastError()
