// Skinny GEMM for batched decode: out[M, N] = x[M, K] . W[N, K]^T with 8 < M <= 64 (pending pods
// decided together), bf16 in, fp32 accumulate on MFMA.
//
// At these M the op is still HBM-bound (weights: 2 bytes each, read once; M = 64 is 64 FLOP/byte,
// far below the 2.5 PFLOP/s : 8 TB/s ridge of ~300), so the kernel is a weight stream with
// v_mfma_f32_16x16x32_bf16 doing the arithmetic:
//  * swapped orientation C^T[n, m] = W[n, :] . x[m, :]: the A operand (16 rows x 32 k) is read
//    straight from the weight rows -- lane l holds row (l & 15), 8 consecutive k at 8 * (l >> 4) --
//    so weights go HBM -> VGPR with 16-byte non-temporal loads, never through LDS;
//  * a wave owns 16 weight rows (SWIGLU: 8 gate rows + the matching 8 up rows, so one tile holds
//    both halves of its features) and streams them in chunks of 256 k (8 x 16 B per lane), TWO
//    chunks ahead of the MFMAs;
//  * x is shared by the 4 waves of a workgroup through a double-buffered LDS chunk [M_pad x 256]
//    (rows padded by 16 B); its global loads are issued BEFORE the weight loads of the same
//    iteration so waiting for x never drains the weight stream (vmcnt retires in order);
//  * stream-K: the (64-row tile, 256-k chunk) iterations are split evenly over exactly
//    2 workgroups per CU, so every CU streams the same number of bytes (no tail round); each tile
//    segment adds its fp32 partial tile into a zeroed accumulator with atomics, and a finalize pass
//    applies the epilogue (bf16 / SwiGLU).  The fp32 epilogue accumulates straight into `out`.
#include <cstdlib>

#include "common.h"

namespace k8sllm {

namespace {
constexpr int SK_KC = 256;                  // k per chunk
constexpr int SK_PITCH = SK_KC * 2 + 16;    // LDS row pitch in bytes
constexpr int SK_ROWS = 64;                 // weight rows per tile (4 waves x 16)
enum { SK_BF16 = 0, SK_F32 = 1, SK_SWIGLU = 2 };

__device__ __forceinline__ float sk_silu(float g) { return g / (1.f + __expf(-g)); }

__device__ __forceinline__ bf16x8 as_bf8(u32x4 v) {
  bf16x8 r;
  __builtin_memcpy(&r, &v, 16);
  return r;
}
}  // namespace

struct SkArgs {
  float* acc;             // [M, wrows] fp32 accumulator (zeroed by the launcher)
  const bf16_t* x;        // [M, K]
  const bf16_t* W;        // [wrows, K]
  int M, N_out, K, half_rows, kchunks, total_iters;
  int diag;               // timing-only experiments (K8S_SKINNY_DIAG): bit0 x chunk 0 only, bit1 lane-contiguous W
};

template <int MT, int EPI>
__global__ void __launch_bounds__(256, 2) skinny_mfma_kernel(SkArgs a) {
  constexpr int MP = MT * 16;
  __shared__ __attribute__((aligned(16))) char xs[2][MP * SK_PITCH];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int row = lane & 15, kq = lane >> 4;
  const int it0 = (int)(((long long)blockIdx.x * a.total_iters) / gridDim.x);
  const int it1 = (int)(((long long)(blockIdx.x + 1) * a.total_iters) / gridDim.x);
  if (it0 >= it1) return;
  const int K = a.K;
  const int wrows = (EPI == SK_SWIGLU) ? 2 * a.half_rows : a.N_out;

  // weight row of this lane in tile t
  auto wrow = [&](int t) -> const bf16_t* {
    int n;
    if (EPI == SK_SWIGLU) {
      const int f = min(t * (SK_ROWS / 2) + wid * 8 + (row & 7), a.N_out - 1);
      n = row < 8 ? f : f + a.half_rows;
    } else {
      n = min(t * SK_ROWS + wid * 16 + row, a.N_out - 1);
    }
    return a.W + (size_t)n * K + kq * 8;
  };
  auto load_a = [&](int it, u32x4 (&dst)[8]) {
    const int t = it / a.kchunks, c = it - t * a.kchunks;
    if (a.diag & 2) {  // same bytes per wave, but every instruction reads 1 KB contiguous of one row
      const bf16_t* p = a.W + (size_t)min(t * SK_ROWS + wid * 16, a.N_out - 1) * K + c * SK_KC + lane * 8;
#pragma unroll
      for (int s = 0; s < 8; ++s)
        dst[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + (size_t)(2 * s) * K));
      return;
    }
    const bf16_t* p = wrow(t) + c * SK_KC;
#pragma unroll
    for (int s = 0; s < 8; ++s) dst[s] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 32 * s));
  };
  constexpr int XV = MP * 32 / 256;  // x vectors (16 B) per thread per chunk
  auto load_x = [&](int it, u32x4 (&xr)[XV]) {
    const int c = (a.diag & 1) ? 0 : it % a.kchunks;
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int v = threadIdx.x + 256 * i, m = v >> 5, cv = v & 31;
      // rows >= M re-read row M-1 (unconditional load); they only feed output columns m >= M,
      // which the epilogue never writes
      xr[i] = *reinterpret_cast<const u32x4*>(a.x + (size_t)min(m, a.M - 1) * K + c * SK_KC + cv * 8);
    }
  };
  auto store_x = [&](int buf, const u32x4 (&xr)[XV]) {
#pragma unroll
    for (int i = 0; i < XV; ++i) {
      const int v = threadIdx.x + 256 * i, m = v >> 5, cv = v & 31;
      *reinterpret_cast<u32x4*>(xs[buf] + m * SK_PITCH + cv * 16) = xr[i];
    }
  };

  // Every load below is unconditional (indices clamped to it1 - 1): a load issued on only one
  // path, or a register move out of an in-flight load, makes the waitcnt pass drain the whole
  // weight stream.  Three weight buffers in a statically unrolled ring: while chunk i is
  // multiplied, chunks i+1 and i+2 are in flight; the load of chunk i+3 reuses chunk i's registers.
  const int last = it1 - 1;
  u32x4 A0[8], A1[8], A2[8];
  {
    u32x4 xr[XV];
    load_x(it0, xr);
    load_a(it0, A0);
    load_a(min(it0 + 1, last), A1);
    load_a(min(it0 + 2, last), A2);
    store_x(0, xr);
  }
  __syncthreads();

  f32x4 acc[MT];
#pragma unroll
  for (int j = 0; j < MT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One k-chunk.  Steps past it1 (the ring's tail padding) multiply stale data into `acc`
  // after its final flush; nothing reads it afterwards.
  auto step = [&](int it, u32x4 (&A)[8]) {
    const int buf = (it - it0) & 1;
    u32x4 xr[XV];
    load_x(min(it + 1, last), xr);  // x first: its wait below leaves the weights in flight
    const char* xb = xs[buf] + row * SK_PITCH + kq * 16;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const bf16x8 b = as_bf8(*reinterpret_cast<const u32x4*>(xb + j * 16 * SK_PITCH + s * 64));
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf8(A[s]), b, acc[j], 0, 0, 0);
      }
    }
    load_a(min(it + 3, last), A);
    const int t = it / a.kchunks;
    if (it < it1 && (it + 1 == it1 || (it + 1) % a.kchunks == 0)) {
      // end of this workgroup's segment of tile t: add the partial tile into the accumulator.
      // C^T tile: lane holds rows 4*kq + i (i < 4) of column m = 16*j + row.
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int m = 16 * j + row;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int n;
          if (EPI == SK_SWIGLU) {
            const int r = 4 * kq + i;  // r < 8: gate feature r; r >= 8: up feature r - 8
            const int f = t * (SK_ROWS / 2) + wid * 8 + (r & 7);
            n = f < a.N_out ? (r < 8 ? f : f + a.half_rows) : -1;
          } else {
            n = t * SK_ROWS + wid * 16 + 4 * kq + i;
            if (n >= a.N_out) n = -1;
          }
          if (m < a.M && n >= 0) atomicAdd(a.acc + (size_t)m * wrows + n, acc[j][i]);
        }
        acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    store_x(buf ^ 1, xr);
    __syncthreads();
  };

  for (int it = it0; it < it1; it += 3) {
    step(it, A0);
    step(it + 1, A1);
    step(it + 2, A2);
  }
}

template <int EPI>
__global__ void skinny_finalize_kernel(void* __restrict__ out, const float* __restrict__ acc, int M, int N_out,
                                       int half_rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N_out) return;
  const int m = i / N_out, n = i - m * N_out;
  if (EPI == SK_SWIGLU) {
    const float* r = acc + (size_t)m * 2 * half_rows;
    reinterpret_cast<bf16_t*>(out)[i] = f2bf(sk_silu(r[n]) * r[n + half_rows]);
  } else {
    reinterpret_cast<bf16_t*>(out)[i] = f2bf(acc[i]);
  }
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" int k8s_skinny_supported(int M, int N_out, int K) {
  return M >= 1 && M <= 64 && N_out > 0 && K % SK_KC == 0 && K > 0;
}

// Workspace (fp32 elements) the launcher needs: the accumulator for the bf16 / SwiGLU epilogues.
extern "C" long long k8s_skinny_workspace(int M, int N_out, int epi) {
  if (epi == SK_F32) return 0;
  return (long long)M * N_out * (epi == SK_SWIGLU ? 2 : 1);
}

extern "C" int k8s_skinny_gemm(void* out, void* workspace, const void* x, const void* W, int M, int N_out, int K,
                               int epi, int num_cus, hipStream_t stream) {
  if (!k8s_skinny_supported(M, N_out, K)) return -1;
  if (epi != SK_F32 && workspace == nullptr) return -3;
  SkArgs a;
  a.acc = epi == SK_F32 ? static_cast<float*>(out) : static_cast<float*>(workspace);
  a.x = static_cast<const bf16_t*>(x);
  a.W = static_cast<const bf16_t*>(W);
  a.M = M;
  a.N_out = N_out;
  a.K = K;
  a.half_rows = (epi == SK_SWIGLU) ? N_out : 0;
  a.kchunks = K / SK_KC;
  static const int diag = [] { const char* e = getenv("K8S_SKINNY_DIAG"); return e ? atoi(e) : 0; }();
  a.diag = diag;
  const int feat_per_tile = (epi == SK_SWIGLU) ? SK_ROWS / 2 : SK_ROWS;
  const int tiles = (N_out + feat_per_tile - 1) / feat_per_tile;
  a.total_iters = tiles * a.kchunks;
  const long long acc_elems = (long long)M * N_out * (epi == SK_SWIGLU ? 2 : 1);
  if (hipError_t e = hipMemsetAsync(a.acc, 0, acc_elems * sizeof(float), stream)) return (int)e;
  // >= 4 chunks (1024 k) per workgroup so the fp32 partial tiles stay small next to the weights
  const int min_iters = a.kchunks < 4 ? a.kchunks : 4;
  int grid = (a.total_iters + min_iters - 1) / min_iters;
  if (grid > 2 * num_cus) grid = 2 * num_cus;
  const int mt = (M + 15) / 16;
#define SK(MTT, EE) skinny_mfma_kernel<MTT, EE><<<grid, 256, 0, stream>>>(a)
#define SK_EPI(MTT)                            \
  switch (epi) {                               \
    case SK_BF16: SK(MTT, SK_BF16); break;     \
    case SK_F32: SK(MTT, SK_F32); break;       \
    case SK_SWIGLU: SK(MTT, SK_SWIGLU); break; \
    default: return -2;                        \
  }
  switch (mt) {
    case 1: SK_EPI(1) break;
    case 2: SK_EPI(2) break;
    case 3: SK_EPI(3) break;
    case 4: SK_EPI(4) break;
    default: return -1;
  }
#undef SK_EPI
#undef SK
  if (epi != SK_F32) {
    const int blocks = (M * N_out + 255) / 256;
    if (epi == SK_SWIGLU)
      skinny_finalize_kernel<SK_SWIGLU><<<blocks, 256, 0, stream>>>(out, a.acc, M, N_out, N_out);
    else
      skinny_finalize_kernel<SK_BF16><<<blocks, 256, 0, stream>>>(out, a.acc, M, N_out, 0);
  }
  return (int)hipGetLastError();
}
