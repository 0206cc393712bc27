// FP8 weight storage (BASELINE config 5: Llama-3.3-70B with fp8 weights, TP = 4).
//
// Format: OCP e4m3 (gfx950's native fp8, max 448) with one fp32 scale per output row,
// w[n, k] ~= e4m3(q[n, k]) * scale[n].  Row scales keep every output feature's dynamic range and
// cost one multiply per output in the GEMV epilogue.  Conversions use the gfx950 packed
// converters (v_cvt_pk_fp8_f32 / v_cvt_pk_f32_fp8, round-to-nearest-even).
#include "common.h"

namespace k8sllm {

constexpr float FP8_MAX = 448.f;
typedef __attribute__((ext_vector_type(2))) float f2v;

// One workgroup per row: absmax -> scale -> quantize (16 elements per thread-iteration).
__global__ void __launch_bounds__(256) quantize_fp8_rows_kernel(uint8_t* __restrict__ q, float* __restrict__ scale,
                                                                const bf16_t* __restrict__ w, int K) {
  __shared__ float red[16];
  const int n = blockIdx.x;
  const bf16_t* row = w + (size_t)n * K;
  float amax = 0.f;
  for (int c = threadIdx.x; c < K / 8; c += blockDim.x) {
    const u32x4 v = reinterpret_cast<const u32x4*>(row)[c];
#pragma unroll
    for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fmaxf(fabsf(lo_bf(v[j])), fabsf(hi_bf(v[j]))));
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  __syncthreads();
  float m = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, red[i]);
  const float s = m > 0.f ? m / FP8_MAX : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[n] = s;
  for (int c = threadIdx.x; c < K / 16; c += blockDim.x) {
    const u32x4 a = reinterpret_cast<const u32x4*>(row)[2 * c];
    const u32x4 b = reinterpret_cast<const u32x4*>(row)[2 * c + 1];
    u32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const u32x4& src = j < 2 ? a : b;
      const uint32_t d0 = src[(2 * j) & 3], d1 = src[(2 * j + 1) & 3];
      auto cl = [&](float v) { return fminf(fmaxf(v * inv, -FP8_MAX), FP8_MAX); };
      int packed = __builtin_amdgcn_cvt_pk_fp8_f32(cl(lo_bf(d0)), cl(hi_bf(d0)), 0, false);
      packed = __builtin_amdgcn_cvt_pk_fp8_f32(cl(lo_bf(d1)), cl(hi_bf(d1)), packed, true);
      o[j] = (uint32_t)packed;
    }
    reinterpret_cast<u32x4*>(q + (size_t)n * K)[c] = o;
  }
}

__global__ void dequant_fp8_rows_kernel(bf16_t* __restrict__ w, const uint8_t* __restrict__ q,
                                        const float* __restrict__ scale, int N, int K) {
  const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;  // 16-element chunk
  const long long per_row = K / 16;
  if (i >= (long long)N * per_row) return;
  const int n = (int)(i / per_row);
  const float s = scale[n];
  const u32x4 v = reinterpret_cast<const u32x4*>(q)[i];
  u32x4 o0, o1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f2v lo = __builtin_amdgcn_cvt_pk_f32_fp8(v[j], false);
    const f2v hi = __builtin_amdgcn_cvt_pk_f32_fp8(v[j], true);
    const uint32_t p0 = pack_bf2(lo.x * s, lo.y * s), p1 = pack_bf2(hi.x * s, hi.y * s);
    if (j < 2) { o0[2 * j] = p0; o0[2 * j + 1] = p1; }
    else { o1[2 * j - 4] = p0; o1[2 * j - 3] = p1; }
  }
  reinterpret_cast<u32x4*>(w)[2 * i] = o0;
  reinterpret_cast<u32x4*>(w)[2 * i + 1] = o1;
}

// K16: per-token activation quantization for the fp8 prefill / batched-decode GEMMs (pgemm / mgemm on the fp8
// MFMAs, row-wise scales in their epilogues): one workgroup per row, the row kept in registers between the absmax
// and the conversion (one read of x).  sx[t] = max|x[t]| / 448, xq[t, k] = e4m3(x[t, k] / sx[t]).
// RMS (K2 fused in, the norm gamma folded into W): the RMSNorm of the row only rescales it, so e4m3(norm(x)[t] / s')
// with s' = max|norm(x)[t]| / 448 is exactly e4m3(x[t] / sx[t]) -- the same bytes -- and only the scale changes:
// sx[t] = max|x[t]| / 448 * rsqrt(mean(x[t]^2) + eps), the sum of squares taken in the same pass.  No rmsnorm
// kernel and no normalised bf16 copy of the residual stream run before an fp8 pre-norm projection.
template <int VPT, bool RMS>
__global__ void __launch_bounds__(256) quantize_act_fp8_kernel(uint8_t* __restrict__ q, float* __restrict__ scale,
                                                               const bf16_t* __restrict__ x, int K, float eps) {
  __shared__ float red[16];
  __shared__ float red2[16];
  const int t = blockIdx.x;
  const u32x4* row = reinterpret_cast<const u32x4*>(x + (size_t)t * K);
  const int nvec = K / 16;  // 16 elements per thread-item
  u32x4 va[VPT], vb[VPT];
  float amax = 0.f, ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nvec) {
      va[i] = row[2 * c];
      vb[i] = row[2 * c + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        amax = fmaxf(amax, fmaxf(fabsf(lo_bf(va[i][j])), fabsf(hi_bf(va[i][j]))));
        amax = fmaxf(amax, fmaxf(fabsf(lo_bf(vb[i][j])), fabsf(hi_bf(vb[i][j]))));
        if constexpr (RMS) {
          ss += lo_bf(va[i][j]) * lo_bf(va[i][j]) + hi_bf(va[i][j]) * hi_bf(va[i][j]);
          ss += lo_bf(vb[i][j]) * lo_bf(vb[i][j]) + hi_bf(vb[i][j]) * hi_bf(vb[i][j]);
        }
      }
    }
  }
  amax = wave_max(amax);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = amax;
  if constexpr (RMS) {
    ss = wave_sum(ss);
    if ((threadIdx.x & 63) == 0) red2[threadIdx.x >> 6] = ss;
  }
  __syncthreads();
  const float m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = m > 0.f ? m / FP8_MAX : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) {
    if constexpr (RMS) scale[t] = s * rsqrtf((red2[0] + red2[1] + red2[2] + red2[3]) / (float)K + eps);
    else scale[t] = s;
  }
  auto cl = [&](float v) { return fminf(fmaxf(v * inv, -FP8_MAX), FP8_MAX); };
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * 256;
    if (c < nvec) {
      u32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const u32x4& src = j < 2 ? va[i] : vb[i];
        const uint32_t d0 = src[(2 * j) & 3], d1 = src[(2 * j + 1) & 3];
        int packed = __builtin_amdgcn_cvt_pk_fp8_f32(cl(lo_bf(d0)), cl(hi_bf(d0)), 0, false);
        packed = __builtin_amdgcn_cvt_pk_fp8_f32(cl(lo_bf(d1)), cl(hi_bf(d1)), packed, true);
        o[j] = (uint32_t)packed;
      }
      reinterpret_cast<u32x4*>(q + (size_t)t * K)[c] = o;
    }
  }
}

// K16, block-scaled (OCP MX e4m3, "MXFP8"): every 32 consecutive values of a row share one E8M0 scale (a biased
// power-of-two exponent byte), the smallest power of two >= max|block| / 448, so x / 2^(e - 127) is exact in fp32 and
// fits e4m3 without saturating.  The scales feed the scale operand of v_mfma_scale_f32_16x16x128_f8f6f4 directly
// (one byte per lane = one 32-value block of one row; mgemm / pgemm MX mode), and a block is local to any producer
// tile that covers 32 features of a row -- the SwiGLU epilogues and the attention kernels emit this format
// themselves (no per-row absmax pass).  This kernel is the stand-alone form (tests, and producers without a fused
// form): one thread per block.
__global__ void __launch_bounds__(256) quantize_act_mx_kernel(uint8_t* __restrict__ q, uint8_t* __restrict__ e8,
                                                              const bf16_t* __restrict__ x, long long blocks, int M,
                                                              int KB) {
  const long long b = (long long)blockIdx.x * 256 + threadIdx.x;
  if (b >= blocks) return;
  const int m = (int)(b / KB), kb = (int)(b - (long long)m * KB);
  const u32x4* src = reinterpret_cast<const u32x4*>(x + b * 32);
  float v[32];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const u32x4 d = src[c];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      v[c * 8 + 2 * j] = lo_bf(d[j]);
      v[c * 8 + 2 * j + 1] = hi_bf(d[j]);
    }
  }
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(v[i]));
  const uint32_t e = mx_e8m0(amax);
  const float inv = mx_inv_scale(e);
  u32x4 o0, o1;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o0[j] = mx_pack4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3], inv);
    o1[j] = mx_pack4(v[16 + 4 * j], v[17 + 4 * j], v[18 + 4 * j], v[19 + 4 * j], inv);
  }
  reinterpret_cast<u32x4*>(q + b * 32)[0] = o0;
  reinterpret_cast<u32x4*>(q + b * 32)[1] = o1;
  e8[mx_scale_off(m, kb, M)] = (uint8_t)e;
}

}  // namespace k8sllm

using namespace k8sllm;

// x bf16 [T][K] -> q e4m3 [T][K] + e8 E8M0 scales (layout [K / 128][T][4], common.h mx_scale_off; K % 128 == 0).
extern "C" int k8s_quantize_act_mx(void* q, void* e8, const void* x, int T, int K, hipStream_t s) {
  if (T <= 0) return 0;
  if (K <= 0 || K % 128 != 0) return -1;
  const long long blocks = (long long)T * (K / 32);
  quantize_act_mx_kernel<<<(unsigned)((blocks + 255) / 256), 256, 0, s>>>(
      static_cast<uint8_t*>(q), static_cast<uint8_t*>(e8), static_cast<const bf16_t*>(x), blocks, T, K / 32);
  return (int)hipGetLastError();
}

// rms != 0: the row's 1/rms (eps) is folded into its scale (see quantize_act_fp8_kernel).
extern "C" int k8s_quantize_act_fp8_rms(void* q, float* scale, const void* x, int T, int K, int rms, float eps,
                                        hipStream_t s) {
  if (T <= 0) return 0;
  if (K <= 0 || K % 16 != 0 || K > 16 * 256 * 8) return -1;
  const int vpt = (K / 16 + 255) / 256;
  auto* qq = static_cast<uint8_t*>(q);
  auto* xx = static_cast<const bf16_t*>(x);
#define QA(V)                                                                               \
  if (rms) quantize_act_fp8_kernel<V, true><<<T, 256, 0, s>>>(qq, scale, xx, K, eps);       \
  else quantize_act_fp8_kernel<V, false><<<T, 256, 0, s>>>(qq, scale, xx, K, eps);
  if (vpt <= 2) { QA(2) } else if (vpt <= 4) { QA(4) } else { QA(8) }
#undef QA
  return (int)hipGetLastError();
}

extern "C" int k8s_quantize_act_fp8(void* q, float* scale, const void* x, int T, int K, hipStream_t s) {
  return k8s_quantize_act_fp8_rms(q, scale, x, T, K, 0, 0.f, s);
}

extern "C" int k8s_quantize_fp8_rows(void* q, float* scale, const void* w, int N, int K, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % 16 != 0) return -1;
  quantize_fp8_rows_kernel<<<N, 256, 0, s>>>(static_cast<uint8_t*>(q), scale, static_cast<const bf16_t*>(w), K);
  return (int)hipGetLastError();
}

extern "C" int k8s_dequant_fp8_rows(void* w, const void* q, const float* scale, int N, int K, hipStream_t s) {
  if (N <= 0 || K <= 0 || K % 16 != 0) return -1;
  const long long chunks = (long long)N * (K / 16);
  dequant_fp8_rows_kernel<<<(unsigned)((chunks + 255) / 256), 256, 0, s>>>(
      static_cast<bf16_t*>(w), static_cast<const uint8_t*>(q), scale, N, K);
  return (int)hipGetLastError();
}
