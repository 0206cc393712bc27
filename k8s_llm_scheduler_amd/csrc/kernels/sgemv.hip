// K3/K8/K9/K11/K12 for SMALL decode batches (3..8 rows): out[M, N] = epi(x[M, K] . W[N, K]^T), the weights
// streamed from HBM exactly once (the decode GEMV of gemv.hip stages x in LDS, 64-128 KiB per
// workgroup at 4-8 rows, and re-stages it for every 8 output rows; mgemm's MFMA tiles waste 3/4 of a 16-row tile).
//
// Structure (one 256-thread workgroup = 4 waves; KW of them split K, 4 / KW row groups split the rows):
//  * every wave owns ONE k-slice of KPW elements for the whole launch and holds x[0..M)[slice] in registers
//    (CPL 16-byte chunks per lane per row: <= 128 VGPRs at 8 rows), loaded once -- no LDS staging, no per-row-set
//    re-staging, occupancy bound by registers only (2-3 workgroups per CU);
//  * the workgroup walks a band of output rows, NRT weight rows per step (one row set), the next set's loads
//    (non-temporal, 16 B per lane, 1 KiB contiguous per wave instruction) in flight while the current set is
//    consumed by v_dot2_f32_bf16 (bf16) or v_cvt_scalef32_pk_bf16_fp8 + v_dot2 (fp8 e4m3 with per-row scales);
//  * the NRT x M per-lane partial sums of a row set are reduced across the wave by a HALVING butterfly (each
//    xor step exchanges only the half of the values the lane gives away: NRT*M + 2 shuffles instead of 6 per
//    value), and one lane per value parks the wave's total in LDS;
//  * after the band, the KW k-slices are summed in a fixed order (deterministic), the RMS prologue's 1/rms (norm
//    gamma folded into W, statistics from the same x registers), the fp8 row scale and the epilogue (bf16, fp32
//    logits, SwiGLU of the [gate; up] halves, or the residual add in place) are applied and stored.
//  * K longer than one workgroup covers (KW x KPW) is split over G = gridDim.y workgroups: fp32 partial slabs and
//    sgemv_finalize_kernel (fixed order over the slices + epilogue).
#include "common.h"

namespace k8sllm {

namespace {

constexpr int SG_BAND = 64;   // most output rows per workgroup band (LDS partials: KW x 2*BAND x MT floats)
enum SgEpi { SG_BF16 = 0, SG_F32 = 1, SG_SWIGLU = 2 };

__device__ __forceinline__ float sg_dot2(uint32_t w, uint32_t x, float acc) {
  bf16x2 a, b;
  __builtin_memcpy(&a, &w, 4);
  __builtin_memcpy(&b, &x, 4);
  return __builtin_amdgcn_fdot2_f32_bf16(a, b, acc, false);
}
__device__ __forceinline__ float sg_dot8(const u32x4& w, const u32x4& x, float acc) {
  acc = sg_dot2(w.x, x.x, acc);
  acc = sg_dot2(w.y, x.y, acc);
  acc = sg_dot2(w.z, x.z, acc);
  return sg_dot2(w.w, x.w, acc);
}
// Halving butterfly over the 64 lanes for CNT values per lane: at xor offset O a lane keeps half of its values
// (the lower half if bit O of its lane id is clear) and adds the partner's copy of that half.  Once one value is
// left, the remaining offsets are plain xor sums.  Afterwards value index (lane >> (6 - log2 V)) & (V - 1) of the
// ORIGINAL V values is the wave total in v[0] of every lane (all lanes of a group agree).
template <int CNT, int O>
__device__ __forceinline__ void sg_halve(float* v, int lane) {
  if constexpr (O >= 1) {
    if constexpr (CNT > 1) {
      const bool up = (lane & O) != 0;
#pragma unroll
      for (int i = 0; i < CNT / 2; ++i) {
        const float give = up ? v[i] : v[i + CNT / 2];
        const float keep = up ? v[i + CNT / 2] : v[i];
        v[i] = keep + __shfl_xor(give, O, WAVE);
      }
      sg_halve<CNT / 2, O / 2>(v, lane);
    } else {
      v[0] += __shfl_xor(v[0], O, WAVE);
      sg_halve<1, O / 2>(v, lane);
    }
  }
}
template <int V>
constexpr int sg_log2() { return V <= 1 ? 0 : 1 + sg_log2<V / 2>(); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t sg_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)min(bytes, 0x7fffffffLL), 0x00020000);
}

}  // namespace

// MT: rows of x the kernel is built for (4 or 8; the first M are live).  KPW: k elements per wave slice.  KW: waves
// per workgroup that split K.  NORM: 1/rms of each x row (gamma folded into W) from the x registers (needs the
// workgroup to cover all of K: G == 1).  RES: out = res + acc (res may alias out).  FP8: W is e4m3 with per-row
// fp32 scales wscale.
template <int MT, int KPW, int KW, int EPI, bool NORM, bool RES, bool FP8>
__global__ void __launch_bounds__(256) sgemv_kernel(void* __restrict__ out, float* __restrict__ part,
                                                     const bf16_t* __restrict__ x, const void* __restrict__ W,
                                                     const float* __restrict__ wscale, const bf16_t* res, int M,
                                                     int N, int K, float eps, int half_rows, int band_rows) {
  constexpr int EPC = FP8 ? 16 : 8;            // elements per 16-byte weight chunk
  constexpr int CPL = KPW / (64 * EPC);         // chunks per lane
  constexpr int XV = FP8 ? 2 : 1;               // x vectors (u32x4) per chunk and row
  constexpr int NR = (EPI == SG_SWIGLU) ? 1 : 2;   // output rows per step
  constexpr int NRT = (EPI == SG_SWIGLU) ? 2 : NR; // weight rows per step (gate and up)
  constexpr int V = NRT * MT;                   // partial sums per lane per step
  constexpr int LV = sg_log2<V>();
  constexpr int RGN = 4 / KW;                   // row groups
  constexpr int WB = FP8 ? 1 : 2;               // weight bytes
  static_assert(CPL >= 1 && V <= 64 && (V & (V - 1)) == 0, "bad sgemv configuration");
  __shared__ float red[KW][NRT * SG_BAND][MT];
  __shared__ float ssr[KW][MT];

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int kw = wid % KW, rg = wid / KW;
  const int g = blockIdx.y;
  const int nch = K / EPC;                      // chunks per weight row
  const int cb = (g * KW + kw) * (64 * CPL);    // this wave's first chunk
  const bool active = cb < nch;
  const int b0 = blockIdx.x * band_rows;           // band_rows <= SG_BAND (the LDS partials' capacity)
  const int band = min(band_rows, N - b0);
  const int nsets = (band + NR - 1) / NR;
  const char* Wb = reinterpret_cast<const char*>(W);
  const long long row_bytes = (long long)K * WB;

  // ---- x slice into registers (rows >= M and chunks past K read 0 through the buffer bounds)
  u32x4 xr[CPL][MT][XV];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    // one buffer resource per x row, bounded by the row (0 bytes for rows >= M): chunks past K and dead rows load
    // 0 without a branch (a per-load select made the compiler wait for each load separately)
    const auto xs = sg_rsrc(x + (size_t)min(m, M - 1) * K, m < M ? (long long)K * 2 : 0);
#pragma unroll
    for (int j = 0; j < CPL; ++j) {
      const int c = cb + 64 * j + lane;
#pragma unroll
      for (int v = 0; v < XV; ++v) xr[j][m][v] = __builtin_amdgcn_raw_buffer_load_b128(xs, c * EPC * 2 + 16 * v, 0, 0);
    }
  }

  // one row set: NRT weight rows x CPL chunks per lane (clamped to the row: x is 0 there)
  auto load_set = [&](u32x4 (&w)[CPL][NRT], int q) {
#pragma unroll
    for (int r = 0; r < NRT; ++r) {
      const int rl = (EPI == SG_SWIGLU) ? q : q * NR + r;
      const int n = min(b0 + min(rl, band - 1), N - 1) + ((EPI == SG_SWIGLU && r == 1) ? half_rows : 0);
      const u32x4* row = reinterpret_cast<const u32x4*>(Wb + (long long)n * row_bytes);
#pragma unroll
      for (int j = 0; j < CPL; ++j) w[j][r] = __builtin_nontemporal_load(row + min(cb + 64 * j + lane, nch - 1));
    }
  };
  auto consume = [&](const u32x4 (&w)[CPL][NRT], int q) {
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
    for (int j = 0; j < CPL; ++j)
#pragma unroll
      for (int r = 0; r < NRT; ++r) {
        if constexpr (FP8) {
          // the 16 e4m3 weights become 8 exact bf16 pairs ONCE, then meet every x row (not once per row)
          bf16x2 wp[8];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            wp[2 * d] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[j][r][d], 1.0f, false);
            wp[2 * d + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[j][r][d], 1.0f, true);
          }
#pragma unroll
          for (int m = 0; m < MT; ++m) {
            float a = acc[r * MT + m];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t xw = e < 4 ? xr[j][m][0][e] : xr[j][m][1][e - 4];
              bf16x2 xb;
              __builtin_memcpy(&xb, &xw, 4);
              a = __builtin_amdgcn_fdot2_f32_bf16(wp[e], xb, a, false);
            }
            acc[r * MT + m] = a;
          }
        } else {
#pragma unroll
          for (int m = 0; m < MT; ++m) acc[r * MT + m] = sg_dot8(w[j][r], xr[j][m][0], acc[r * MT + m]);
        }
      }
    sg_halve<V, 32>(acc, lane);
    if ((lane & ((1 << (6 - LV)) - 1)) == 0) {
      const int idx = (lane >> (6 - LV)) & (V - 1);
      const int r = idx / MT, m = idx % MT;
      const int rl = (EPI == SG_SWIGLU) ? q + r * SG_BAND : q * NR + r;
      red[kw][rl][m] = acc[0];
    }
  };

  // the first row set's weights go out right behind the x loads, unconditionally (rows and chunks are clamped, so a
  // wave with no set or no slice reads valid bytes it ignores): a branch here let the compiler sink them below the
  // norm prologue, which then waited for every x load before a single weight byte was requested
  u32x4 wa[CPL][NRT], wb[CPL][NRT];
  int q = rg;
  asm volatile("" ::: "memory");   // every x load is issued before the first weight load (in-order retirement)
  load_set(wa, q);
  asm volatile("" ::: "memory");
  // and the x registers become opaque only here, so nothing that reads them (the norm's sum of squares) can be
  // scheduled above the weight loads: its wait is then for the x loads only (counted: the weights stay in flight)
  if constexpr (NORM) {
#pragma unroll
    for (int j = 0; j < CPL; ++j)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int v = 0; v < XV; ++v) asm volatile("" : "+v"(xr[j][m][v]));
  }

  if constexpr (NORM) {   // sum of squares of each live x row over this wave's slice (the weights are in flight)
    float ss[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float s = 0.f;
#pragma unroll
      for (int j = 0; j < CPL; ++j)
#pragma unroll
        for (int v = 0; v < XV; ++v)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = lo_bf(xr[j][m][v][e]), hi = hi_bf(xr[j][m][v][e]);
            s += lo * lo + hi * hi;
          }
      ss[m] = s;
    }
    constexpr int LM = sg_log2<MT>();
    sg_halve<MT, 32>(ss, lane);
    if (rg == 0 && (lane & ((1 << (6 - LM)) - 1)) == 0) ssr[kw][(lane >> (6 - LM)) & (MT - 1)] = ss[0];
  }

  if (active) {
    for (; q < nsets; q += 2 * RGN) {
      if (q + RGN < nsets) load_set(wb, q + RGN);
      consume(wa, q);
      if (q + RGN >= nsets) break;
      if (q + 2 * RGN < nsets) load_set(wa, q + 2 * RGN);
      consume(wb, q + RGN);
    }
  } else {   // a slice past the end of K (the last k-group of a ragged split): contributes zeros
    for (int i = lane; i < NRT * SG_BAND * MT; i += 64) (&red[kw][0][0])[i] = 0.f;
  }
  __syncthreads();

  // ---- combine the k-slices (fixed order), scale, epilogue
  const int G = gridDim.y;
  for (int t = threadIdx.x; t < band * MT; t += 256) {
    const int m = t / band, rl = t - m * band;
    if (m >= M) break;
    const int n = b0 + rl;
    float a = 0.f, u = 0.f;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      a += red[k][rl][m];
      if (EPI == SG_SWIGLU) u += red[k][SG_BAND + rl][m];
    }
    if constexpr (NORM) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < KW; ++k) s += ssr[k][m];
      const float inv = rsqrtf(s / (float)K + eps);
      a *= inv;
      u *= inv;
    }
    if constexpr (FP8) {
      a *= wscale[n];
      if (EPI == SG_SWIGLU) u *= wscale[n + half_rows];
    }
    if (G > 1) {   // partial slab of this k-group; sgemv_finalize_kernel applies the epilogue
      const int wrows = (EPI == SG_SWIGLU) ? 2 * N : N;
      float* slab = part + ((size_t)g * M + m) * wrows;
      slab[n] = a;
      if (EPI == SG_SWIGLU) slab[N + n] = u;
      continue;
    }
    if constexpr (EPI == SG_F32) {
      reinterpret_cast<float*>(out)[(size_t)m * N + n] = a;
    } else if constexpr (EPI == SG_SWIGLU) {
      reinterpret_cast<bf16_t*>(out)[(size_t)m * N + n] = f2bf(a / (1.f + __expf(-a)) * u);
    } else {
      if constexpr (RES) a += bf2f(res[(size_t)m * N + n]);
      reinterpret_cast<bf16_t*>(out)[(size_t)m * N + n] = f2bf(a);
    }
  }
}

template <int EPI, bool RES>
__global__ void sgemv_finalize_kernel(void* __restrict__ out, const float* __restrict__ part, const bf16_t* res,
                                      int M, int N, int G) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  const int m = i / N, n = i - m * N;
  const int wrows = (EPI == SG_SWIGLU) ? 2 * N : N;
  float a = 0.f, u = 0.f;
  for (int g = 0; g < G; ++g) {
    const float* slab = part + ((size_t)g * M + m) * wrows;
    a += slab[n];
    if (EPI == SG_SWIGLU) u += slab[N + n];
  }
  if constexpr (EPI == SG_F32) {
    reinterpret_cast<float*>(out)[i] = a;
  } else if constexpr (EPI == SG_SWIGLU) {
    reinterpret_cast<bf16_t*>(out)[i] = f2bf(a / (1.f + __expf(-a)) * u);
  } else {
    if constexpr (RES) a += bf2f(res[i]);
    reinterpret_cast<bf16_t*>(out)[i] = f2bf(a);
  }
}

}  // namespace k8sllm

using namespace k8sllm;

namespace {
// Launch plan: (k elements per wave slice, waves per workgroup along K, k-groups).  Slices of 2048 elements
// (bf16: 4 chunks per lane = 128 x registers at 8 rows; fp8: 2) split 4 or 2 ways inside the workgroup, the
// split with less idle slice area wins (ties: more waves on K); K <= 1024 takes one 1024-element slice per wave and
// 4 row groups.
struct SgPlan {
  int kpw, kw, g;
};
SgPlan sg_plan(int K) {
  if (K <= 1024) return {1024, 1, 1};
  const int s = (K + 2047) / 2048;                   // 2048-element slices
  const int g4 = (s + 3) / 4, g2 = (s + 1) / 2;
  const int idle4 = g4 * 4 - s, idle2 = g2 * 2 - s;
  if (idle4 <= idle2) return {2048, 4, g4};
  return {2048, 2, g2};
}
}  // namespace

// Workspace floats for the partial slabs (0 when the plan has one k-group).
extern "C" long long k8s_sgemv_workspace(int M, int N, int K, int epi) {
  const SgPlan p = sg_plan(K);
  if (p.g <= 1) return 0;
  return (long long)p.g * M * (epi == SG_SWIGLU ? 2 : 1) * N;
}

// out [M, N] (bf16, or fp32 for epi 1); x [M, K] bf16; W [N, K] (epi 2: [2N, K], gate rows then up rows) bf16, or
// e4m3 bytes when wscale != null (fp32 per weight row); res [M, N] bf16 for the residual epilogue (may be out);
// norm: 1 = multiply by 1/rms of each x row (the norm gamma folded into W).  Returns -5 (nothing launched) for the
// residual add with another epilogue or with the norm, and for a norm over a K that needs more than one k-group.
extern "C" int k8s_sgemv(void* out, void* partial, const void* x, const void* W, const float* wscale, const void* res,
                         int M, int N, int K, int epi, int norm, float eps, hipStream_t stream) {
  if (M < 1 || M > 8 || N <= 0 || K <= 0) return -1;
  const bool fp8 = wscale != nullptr;
  if (K % (fp8 ? 16 : 8) != 0) return -1;
  const SgPlan p = sg_plan(K);
  if (norm && p.g > 1) return -5;
  if (p.g > 1 && partial == nullptr) return -3;
  const bool has_res = res != nullptr;
  // every (epilogue, norm) pair is instantiated; the residual add only with the plain bf16 epilogue
  if (epi < SG_BF16 || epi > SG_SWIGLU) return -1;
  if (has_res && (epi != SG_BF16 || norm)) return -5;
  // rows per workgroup: enough workgroups to put every CU to work (~512 per k-group, 2 per CU), at most SG_BAND;
  // fewer rows per wave re-read x (L2-resident) more often, so the band never drops below 4 rows
  const int nr = epi == SG_SWIGLU ? 1 : 2;
  int band = (N + 511) / 512;
  band = min(SG_BAND, max(4, (band + nr - 1) / nr * nr));
  const dim3 grid((N + band - 1) / band, p.g);
  const int half_rows = epi == SG_SWIGLU ? N : 0;
  float* part = p.g > 1 ? (float*)partial : nullptr;
  const bf16_t* xx = (const bf16_t*)x;
  const bf16_t* rr = (const bf16_t*)res;
#define SGL(MT, KPW, KW, EE, NN, RR, F8)                                                                     \
  sgemv_kernel<MT, KPW, KW, EE, NN, RR, F8><<<grid, 256, 0, stream>>>(out, part, xx, W, wscale, rr, M, N, K, \
                                                                       eps, half_rows, band)
#define SG_COMBO(MT, KPW, KW, F8)                                                           \
  if (epi == SG_BF16 && norm) { SGL(MT, KPW, KW, SG_BF16, true, false, F8); }               \
  else if (epi == SG_BF16 && has_res) { SGL(MT, KPW, KW, SG_BF16, false, true, F8); }       \
  else if (epi == SG_BF16) { SGL(MT, KPW, KW, SG_BF16, false, false, F8); }                 \
  else if (epi == SG_SWIGLU && norm) { SGL(MT, KPW, KW, SG_SWIGLU, true, false, F8); }      \
  else if (epi == SG_SWIGLU) { SGL(MT, KPW, KW, SG_SWIGLU, false, false, F8); }             \
  else if (norm) { SGL(MT, KPW, KW, SG_F32, true, false, F8); }                             \
  else { SGL(MT, KPW, KW, SG_F32, false, false, F8); }
#define SG_PLAN(MT, F8)                                           \
  if (p.kpw == 1024) { SG_COMBO(MT, 1024, 1, F8) }                \
  else if (p.kw == 4) { SG_COMBO(MT, 2048, 4, F8) }               \
  else { SG_COMBO(MT, 2048, 2, F8) }
  if (M <= 4) {
    if (fp8) { SG_PLAN(4, true) } else { SG_PLAN(4, false) }
  } else {
    if (fp8) { SG_PLAN(8, true) } else { SG_PLAN(8, false) }
  }
#undef SG_PLAN
#undef SG_COMBO
#undef SGL
  if (p.g > 1) {
    const int total = M * N, blocks = (total + 255) / 256;
    if (epi == SG_SWIGLU) sgemv_finalize_kernel<SG_SWIGLU, false><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, p.g);
    else if (epi == SG_F32) sgemv_finalize_kernel<SG_F32, false><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, p.g);
    else if (has_res) sgemv_finalize_kernel<SG_BF16, true><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, p.g);
    else sgemv_finalize_kernel<SG_BF16, false><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, p.g);
  }
  return (int)hipGetLastError();
}
