// K2: RMSNorm and fused residual-add + RMSNorm.
//   plain : out = x * rsqrt(mean(x^2) + eps) * w
//   fused : r = x + residual; residual <- r; out = r * rsqrt(mean(r^2) + eps) * w
// One workgroup per row; 16-byte vector loads (8 x bf16 per lane), fp32 accumulation, the
// row kept in registers between the reduction and the scale pass (one HBM read per tensor).
#include "common.h"

namespace k8sllm {

template <int VPT, bool FUSED>
__global__ void __launch_bounds__(256) rmsnorm_kernel(bf16_t* __restrict__ out, const bf16_t* __restrict__ x,
                                                      bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
                                                      int H, float eps) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const u32x4* xv = reinterpret_cast<const u32x4*>(x + (size_t)row * H);
  u32x4* rv = reinterpret_cast<u32x4*>(residual + (size_t)row * H);
  const u32x4* wv = reinterpret_cast<const u32x4*>(w);
  u32x4* ov = reinterpret_cast<u32x4*>(out + (size_t)row * H);
  const int nvec = H >> 3;
  float vals[VPT][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      u32x4 a = xv[c];
      if (FUSED) {
        u32x4 b = rv[c];
        u32x4 s;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float l = lo_bf(a[j]) + lo_bf(b[j]);
          float h = hi_bf(a[j]) + hi_bf(b[j]);
          s[j] = pack_bf2(l, h);
        }
        rv[c] = s;
        a = s;  // normalise the bf16-rounded residual, as an unfused graph would
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        vals[i][2 * j] = lo_bf(a[j]);
        vals[i][2 * j + 1] = hi_bf(a[j]);
        ss += vals[i][2 * j] * vals[i][2 * j] + vals[i][2 * j + 1] * vals[i][2 * j + 1];
      }
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)H + eps);
#pragma unroll
  for (int i = 0; i < VPT; ++i) {
    const int c = threadIdx.x + i * blockDim.x;
    if (c < nvec) {
      u32x4 g = wv[c], o;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        o[j] = pack_bf2(vals[i][2 * j] * inv * lo_bf(g[j]), vals[i][2 * j + 1] * inv * hi_bf(g[j]));
      ov[c] = o;
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// residual == nullptr -> plain RMSNorm.  H must be a multiple of 8 and <= 16384.
extern "C" int k8s_rmsnorm(void* out, const void* x, void* residual, const void* w, int rows, int H, float eps,
                           hipStream_t stream) {
  if (H % 8 != 0 || H > 16384 || rows <= 0) return -1;
  const int nvec = H / 8;
  const int threads = nvec >= 256 ? 256 : ((nvec + 63) / 64) * 64;
  const int vpt = (nvec + threads - 1) / threads;
  auto o = (bf16_t*)out;
  auto xi = (const bf16_t*)x;
  auto r = (bf16_t*)residual;
  auto g = (const bf16_t*)w;
#define LAUNCH(V)                                                                                      \
  if (r) rmsnorm_kernel<V, true><<<rows, threads, 0, stream>>>(o, xi, r, g, H, eps);                  \
  else rmsnorm_kernel<V, false><<<rows, threads, 0, stream>>>(o, xi, r, g, H, eps);
  if (vpt <= 1) { LAUNCH(1) } else if (vpt <= 2) { LAUNCH(2) } else if (vpt <= 4) { LAUNCH(4) } else { LAUNCH(8) }
#undef LAUNCH
  return (int)hipGetLastError();
}
