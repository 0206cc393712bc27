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
#include <atomic>
#include <cstdlib>

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

// 5..16 decode rows on the MATRIX cores.  At 8 rows the v_dot2 form above issues 32 VALU dot2 per 16 weight bytes
// (fp8: 72 with the conversions): VALU-bound at ~5 TB/s (fp8 ~3 TB/s), and it cannot hold 16 rows of x.  Here the
// products run on v_mfma_f32_4x4x4bf16_1k -- 16 independent 4x4x4 blocks, lane 4b + i holding row i of block b
// (A: weights, items = 4 k; B: x, column j = lane & 3; D: item i of lane 4b + j = D[i][j]; checked on the chip by
// tools/experiments/mfma4_layout.hip) -- so the VALU is free and the kernel is a pure weight stream again:
//  * one 16-byte-per-lane load covers 4 weight rows x 256 contiguous bytes (lane l: row l & 3, chunk l >> 2): the
//    16 blocks are 16 consecutive chunks of the same 4 rows, each chunk two (bf16) or four (fp8) k-quads.  That
//    access shape streams at ~6.2 TB/s where the 16x16x32 MFMA's A operand (16 rows x 64 B per load) manages ~5.0
//    (tools/experiments/ldpat.hip, profiles/sgemv_load_patterns_r4.txt);
//  * x lives in registers for the whole launch (B operand: x row 4 xg + (l & 3), the same chunks), MT / 4 groups
//    of 4 rows; fp8 weights become bf16 k-quads with v_cvt_scalef32_pk_bf16_fp8 (x stays bf16, the row scale
//    lands in the epilogue);
//  * 512 threads = 8 waves, ALL splitting the workgroup's k range (jw steps of 16 chunks each); the workgroup
//    walks its band in quads of 4 rows (SwiGLU: gate quads then up quads), register sets of 4 loads (4 KiB per
//    wave) double-buffered -- the shallow queue streams best (the probe: 4-8 KiB per wave beats 16-32 KiB);
//  * at the end of a quad the 16 blocks' partial products are summed by a halving butterfly (4 x MT / 4 values per
//    lane, offsets 32..4) and parked in LDS; after the band the 8 k-slices are summed in a fixed order
//    (deterministic) and the norm / scale / epilogue applied as in the v_dot2 form;
//  * band sized for about one workgroup per CU and k-group; steps past a wave's slice and rows past the band are
//    out of range of the load's buffer (0, no traffic) instead of branches, so every wait is a counted one.
constexpr int SM_KW = 8;   // waves per workgroup

template <int CNT, int O>
__device__ __forceinline__ void sm_halve(float* v, int lane) {   // sg_halve that stops at offset 4 (j = lane & 3)
  if constexpr (O >= 4) {
    if constexpr (CNT > 1) {
      const bool up = (lane & O) != 0;
#pragma unroll
      for (int i = 0; i < CNT / 2; ++i) {
        const float give = up ? v[i] : v[i + CNT / 2];
        const float keep = up ? v[i + CNT / 2] : v[i];
        v[i] = keep + __shfl_xor(give, O, WAVE);
      }
      sm_halve<CNT / 2, O / 2>(v, lane);
    } else {
      v[0] += __shfl_xor(v[0], O, WAVE);
      sm_halve<1, O / 2>(v, lane);
    }
  }
}

template <int EPI, bool RES>
__device__ __forceinline__ void sm_store(void* out, size_t o, float a, float u, float rv) {
  if constexpr (EPI == SG_F32) {
    reinterpret_cast<float*>(out)[o] = a;
  } else if constexpr (EPI == SG_SWIGLU) {
    reinterpret_cast<bf16_t*>(out)[o] = f2bf(a / (1.f + __expf(-a)) * u);
  } else {
    if constexpr (RES) a += rv;
    reinterpret_cast<bf16_t*>(out)[o] = f2bf(a);
  }
}

// Tickets of the in-kernel k-group reduction: zero at load, each range returned to zero by the last workgroup of
// every launch that used it.  Launches draw ranges of SM_TICKET_RANGE in rotation, so kernels that overlap on
// different streams do not share counters.
constexpr int SM_TICKET_RANGE = 256, SM_TICKET_RANGES = 256;
__device__ unsigned sm_tickets[SM_TICKET_RANGE * SM_TICKET_RANGES];

template <int MT, int JT, int EPI, bool NORM, bool RES, bool FP8>
__global__ void __launch_bounds__(512) smfma_kernel(void* __restrict__ out, float* __restrict__ part,
                                                     const bf16_t* __restrict__ x, const void* __restrict__ W,
                                                     const float* __restrict__ wscale, const bf16_t* res, int M,
                                                     int N, int K, float eps, int band_rows, int jw,
                                                     unsigned* tickets) {
  constexpr int EPC = FP8 ? 16 : 8;                // k per 16-byte weight chunk
  constexpr int XG = MT / 4;                       // x groups of 4 rows (the B operand's 4 columns)
  constexpr int KQ = EPC / 4;                      // k-quads per chunk
  constexpr int XV = FP8 ? 2 : 1;                  // x u32x4 per chunk and row
  constexpr int Q = 4;                             // loads per register set
  constexpr int QPU = JT >= Q ? 1 : Q / JT;        // quads per set
  constexpr int NSB = JT >= Q ? JT / Q : 1;        // sets per quad block
  constexpr int QMAX = 512 / MT;                   // quads per workgroup (LDS partials: 64 KiB)
  constexpr int V = 4 * XG;                        // partial products per lane and quad
  constexpr int LV = sg_log2<V>();
  constexpr int WB = FP8 ? 1 : 2;
  static_assert((JT & (JT - 1)) == 0 && JT <= 8 && V <= 16, "bad smfma configuration");
  __shared__ float red[SM_KW][QMAX][4][MT];
  __shared__ float ssw[SM_KW][MT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int kw = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wave-uniform: the step masks below are scalar)
  const int r4 = lane & 3, cb = lane >> 2;         // row in the quad / x row in the group; chunk = block
  const int g = blockIdx.y;
  const int C16 = K / (16 * EPC);                  // steps (16 chunks) per weight row
  const int sb = (g * SM_KW + kw) * jw;            // this wave's first step
  const int jv = max(0, min(jw, C16 - sb));        // its live steps (0: a slice past K)
  const int b0 = blockIdx.x * band_rows;
  const int band = min(band_rows, N - b0);
  const int qg = (band + 3) >> 2;                  // quads of output rows
  const int nq = (EPI == SG_SWIGLU) ? 2 * qg : qg;
  const unsigned row_bytes = (unsigned)K * WB;
  constexpr unsigned OOB = 0x80000000u;            // past every buffer below: the load returns 0, no traffic

  // ---- x -> registers: xr[s][xg] = x[4 xg + r4][chunk 16 (sb + s) + cb]; rows >= M / dead steps read 0
  u32x4 xr[JT][XG][XV];
  {
    const auto xs = sg_rsrc(x, (long long)M * K * 2);
#pragma unroll
    for (int s = 0; s < JT; ++s)
#pragma unroll
      for (int xg = 0; xg < XG; ++xg) {
        const unsigned off =
            s < jv ? (unsigned)(4 * xg + r4) * K * 2 + (unsigned)(16 * (sb + s) + cb) * EPC * 2 : OOB;
#pragma unroll
        for (int v = 0; v < XV; ++v) xr[s][xg][v] = __builtin_amdgcn_raw_buffer_load_b128(xs, off + 16 * v, 0, 0);
      }
  }

  // the band's weight rows through one buffer per half (gate rows; SwiGLU: up rows)
  const char* Wc = reinterpret_cast<const char*>(W);
  const auto wg = sg_rsrc(Wc + (size_t)b0 * row_bytes, (long long)band * row_bytes);
  const auto wu = sg_rsrc(Wc + ((EPI == SG_SWIGLU) ? (size_t)(N + b0) * row_bytes : 0),
                          (EPI == SG_SWIGLU) ? (long long)band * row_bytes : 0);
  const unsigned lane_off = (unsigned)r4 * row_bytes + (unsigned)(16 * sb + cb) * 16;
  // element e of set i of quad block qb: (quad, step), both compile-time but the block
  auto quad_of = [](int qb, int e) { return qb * QPU + (JT >= Q ? 0 : e / JT); };
  auto step_of = [](int i, int e) { return JT >= Q ? i * Q + e : e % JT; };
  auto load_set = [&](u32x4 (&w)[Q], int qb, int i) {
#pragma unroll
    for (int e = 0; e < Q; ++e) {
      const int quad = quad_of(qb, e), s = step_of(i, e);
      const bool up = EPI == SG_SWIGLU && quad >= qg;
      const unsigned off = s < jv ? (unsigned)(4 * (up ? quad - qg : quad)) * row_bytes + lane_off + 256u * s : OOB;
      w[e] = __builtin_amdgcn_raw_buffer_load_b128(up ? wu : wg, off, 0, 2);   // (aux 2: non-temporal)
    }
  };
  auto consume = [&](const u32x4 (&w)[Q], int i, f32x4 (&acc)[QPU][XG]) {
#pragma unroll
    for (int e = 0; e < Q; ++e) {
      const int qq = JT >= Q ? 0 : e / JT, s = step_of(i, e);
#pragma unroll
      for (int kq = 0; kq < KQ; ++kq) {
        uint32_t a0, a1;
        if constexpr (FP8) {
          a0 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[e][kq], 1.0f, false));
          a1 = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[e][kq], 1.0f, true));
        } else {
          a0 = w[e][2 * kq];
          a1 = w[e][2 * kq + 1];
        }
        const bf16x4 a = __builtin_bit_cast(bf16x4, (uint2){a0, a1});
#pragma unroll
        for (int xg = 0; xg < XG; ++xg) {
          const u32x4& xv = xr[s][xg][kq / 2];
          const bf16x4 b = __builtin_bit_cast(bf16x4, (uint2){xv[2 * (kq & 1)], xv[2 * (kq & 1) + 1]});
          acc[qq][xg] = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, b, acc[qq][xg], 0, 0, 0);
        }
      }
    }
  };
  auto park = [&](const f32x4 (&acc)[QPU][XG], int qb) {   // sum the 16 blocks, one lane per (row, x row) to LDS
#pragma unroll
    for (int qq = 0; qq < QPU; ++qq) {
      float v[V];
#pragma unroll
      for (int xg = 0; xg < XG; ++xg)
#pragma unroll
        for (int it = 0; it < 4; ++it) v[xg * 4 + it] = acc[qq][xg][it];
      sm_halve<V, 32>(v, lane);
      const int idx = (lane >> (6 - LV)) & (V - 1);
      if (((lane >> 2) & ((1 << (4 - LV)) - 1)) == 0) red[kw][qb * QPU + qq][idx & 3][4 * (idx >> 2) + r4] = v[0];
    }
  };

  u32x4 wbuf[2][Q];
  asm volatile("" ::: "memory");   // every x load is issued before the first weight load (in-order retirement)
  load_set(wbuf[0], 0, 0);         // (every launched workgroup has >= 1 quad)
  asm volatile("" ::: "memory");
  if constexpr (NORM) {   // sum of squares of each x row over this wave's slice, the first weights in flight
#pragma unroll
    for (int s = 0; s < JT; ++s)
#pragma unroll
      for (int xg = 0; xg < XG; ++xg)
#pragma unroll
        for (int v = 0; v < XV; ++v) asm volatile("" : "+v"(xr[s][xg][v]));
    float ss[XG];
#pragma unroll
    for (int xg = 0; xg < XG; ++xg) {
      float t = 0.f;
#pragma unroll
      for (int s = 0; s < JT; ++s)
#pragma unroll
        for (int v = 0; v < XV; ++v)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float lo = lo_bf(xr[s][xg][v][e]), hi = hi_bf(xr[s][xg][v][e]);
            t += lo * lo + hi * hi;
          }
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) t += __shfl_xor(t, o, WAVE);
      ss[xg] = t;
    }
    if (lane < 4) {
#pragma unroll
      for (int xg = 0; xg < XG; ++xg) ssw[kw][4 * xg + lane] = ss[xg];
    }
  }

  // the first epilogue pass's residual and row scales are requested now, behind the first weight set (clamped, so no
  // load sits under a branch): their latency hides under the weight stream instead of ending the kernel
  float pre_res = 0.f, pre_sa = 1.f, pre_su = 1.f;
  asm volatile("" ::: "memory");
  {
    const int idx = min(tid, band * M - 1);
    const int m = idx / band, n = b0 + idx - m * band;
    if constexpr (RES) pre_res = bf2f(res[(size_t)m * N + n]);
    if constexpr (FP8) {
      pre_sa = wscale[n];
      if constexpr (EPI == SG_SWIGLU) pre_su = wscale[N + n];
    }
  }

  // quad blocks two at a time so the register set of every (block, set) pair is a compile-time choice; an odd
  // count runs a phantom block, and the last block prefetches the (out-of-range) block after it: no load sits
  // under a branch, so every wait stays a counted one
  const int nqb = (nq + QPU - 1) / QPU;
  const int nqbp = (nqb + 1) & ~1;   // (host: nqbp * QPU <= QMAX)
  for (int qb = 0; qb < nqbp; qb += 2) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int qbc = qb + tt;
      f32x4 acc[QPU][XG];
#pragma unroll
      for (int qq = 0; qq < QPU; ++qq)
#pragma unroll
        for (int xg = 0; xg < XG; ++xg) acc[qq][xg] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < NSB; ++i) {
        const int par = (tt * NSB + i) & 1;
        const int nb = i + 1 < NSB ? qbc : qbc + 1, ni = i + 1 < NSB ? i + 1 : 0;
        if (par) load_set(wbuf[0], nb, ni); else load_set(wbuf[1], nb, ni);
        // the next set's loads go out before this set's MFMAs (and their waits): the barrier keeps the loads
        // above it, the opaque accumulators (and, for fp8, the current set feeding the conversions) the math below
        asm volatile("" ::: "memory");
#pragma unroll
        for (int qq = 0; qq < QPU; ++qq)
#pragma unroll
          for (int xg = 0; xg < XG; ++xg) asm volatile("" : "+v"(acc[qq][xg]));
        if constexpr (FP8) {
#pragma unroll
          for (int q = 0; q < Q; ++q) {
            if (par) asm volatile("" : "+v"(wbuf[1][q])); else asm volatile("" : "+v"(wbuf[0][q]));
          }
        }
        if (par) consume(wbuf[1], i, acc); else consume(wbuf[0], i, acc);
      }
      park(acc, qbc);
    }
  }
  __syncthreads();

  // ---- combine the 8 k-slices (fixed order), scale, epilogue
  const int G = gridDim.y;
  for (int idx = tid; idx < band * M; idx += 512) {
    const int m = idx / band, lr = idx - m * band;
    const int n = b0 + lr, qd = lr >> 2, i = lr & 3;
    float a = 0.f, u = 0.f;
#pragma unroll
    for (int k = 0; k < SM_KW; ++k) {
      a += red[k][qd][i][m];
      if (EPI == SG_SWIGLU) u += red[k][qg + qd][i][m];
    }
    if constexpr (NORM) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < SM_KW; ++k) s += ssw[k][m];
      const float inv = rsqrtf(s / (float)K + eps);
      a *= inv;
      u *= inv;
    }
    const bool first = idx == tid;
    if constexpr (FP8) {
      a *= first ? pre_sa : wscale[n];
      if (EPI == SG_SWIGLU) u *= first ? pre_su : wscale[N + n];
    }
    if (G > 1) {   // device-coherent stores (write-through past the XCD's L2): read back by another workgroup
      const int wrows = (EPI == SG_SWIGLU) ? 2 * N : N;
      float* slab = part + ((size_t)g * M + m) * wrows;
      __hip_atomic_store(slab + n, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (EPI == SG_SWIGLU) __hip_atomic_store(slab + N + n, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    const size_t o = (size_t)m * N + n;
    sm_store<EPI, RES>(out, o, a, u, RES ? (first ? pre_res : bf2f(res[o])) : 0.f);
  }
  if (G == 1 || tickets == nullptr) return;   // (no tickets: sgemv_finalize_kernel sums the slabs)

  // ---- k-groups: the LAST workgroup of this band to finish sums the G slabs (fixed order, as the finalize kernel
  // would) and stores the result -- no second launch.  No cache-wide fences: the slab stores above are device-coherent
  // (write-through), every wave waits for its own stores to land before the workgroup counts its arrival with one
  // device-scope add, and the last workgroup reads the slabs with device-coherent loads.
  __shared__ int sm_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's slab stores have landed
  __syncthreads();
  if (tid == 0)
    sm_last = __hip_atomic_fetch_add(&tickets[blockIdx.x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
              (unsigned)(G - 1);
  __syncthreads();
  if (!sm_last) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // (compiler ordering: the loads stay below the add)
  const int wrows = (EPI == SG_SWIGLU) ? 2 * N : N;
  for (int idx = tid; idx < band * M; idx += 512) {
    const int m = idx / band, n = b0 + idx - m * band;
    float a = 0.f, u = 0.f;
    for (int k = 0; k < G; ++k) {
      const float* slab = part + ((size_t)k * M + m) * wrows;
      a += __hip_atomic_load(slab + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (EPI == SG_SWIGLU) u += __hip_atomic_load(slab + N + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const size_t o = (size_t)m * N + n;
    sm_store<EPI, RES>(out, o, a, u, RES ? (idx == tid ? pre_res : bf2f(res[o])) : 0.f);
  }
  if (tid == 0)   // ready for the next launch that draws this ticket range
    __hip_atomic_store(&tickets[blockIdx.x], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// MFMA plan (smfma_kernel): JT register steps per wave (1, 2, 4, 8; a step = 16 chunks of every row of a quad),
// jw live steps, G k-groups.  Needs whole steps (K % 128 bf16, K % 256 fp8); one k-group covers 8 waves x 8 steps
// (8192 k) -- fp8 4 steps (8192 k: an fp8 step holds twice the x of a bf16 one).
struct SmPlan {
  int jt, jw, g;
};
static bool sm_plan(int K, bool fp8, SmPlan& p) {
  const int epc = fp8 ? 16 : 8;
  if (K % (16 * epc) != 0) return false;
  const int c16 = K / (16 * epc), jmax = fp8 ? 4 : 8;
  const int g = (c16 + SM_KW * jmax - 1) / (SM_KW * jmax);
  const int jw = (c16 + SM_KW * g - 1) / (SM_KW * g);
  p = {jw <= 1 ? 1 : (jw <= 2 ? 2 : (jw <= 4 ? 4 : 8)), jw, g};
  return true;
}
// rows from which the matrix-core form takes over from the register dot2 form (K8S_SGEMV_MFMA_MIN_M, default 3:
// every sgemv row count -- at 4 rows it ties or beats the dot2 form, profiles/sgemv_mfma4_kernel_trace_r4.txt; 5
// keeps 3..4 rows on dot2; 17 turns it off: 9..16 rows then go back to mgemm).  The dot2 form remains the path
// for K that is not a whole number of 16-chunk steps.
static int sm_min_m() {
  static const int v = [] { const char* e = getenv("K8S_SGEMV_MFMA_MIN_M"); return e ? atoi(e) : 3; }();
  return v;
}
static int sm_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return v;
}
static bool sm_take(int M, int K, bool fp8, SmPlan& p) { return M >= sm_min_m() && M <= 16 && sm_plan(K, fp8, p); }

// Workspace floats for the partial slabs (0 when the plan has one k-group).
// The same plan k8s_sgemv takes for these operands (fp8: e4m3 weights), so the slabs always fit.
extern "C" long long k8s_sgemv_workspace(int M, int N, int K, int epi, int fp8) {
  SmPlan sp;
  const int g = sm_take(M, K, fp8 != 0, sp) ? sp.g : sg_plan(K).g;
  if (g <= 1) return 0;
  return (long long)g * M * (epi == SG_SWIGLU ? 2 : 1) * N;
}

static void sg_finalize(void* out, float* part, const bf16_t* rr, int M, int N, int G, int epi, bool has_res,
                        hipStream_t stream) {
  const int total = M * N, blocks = (total + 255) / 256;
  if (epi == SG_SWIGLU) sgemv_finalize_kernel<SG_SWIGLU, false><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, G);
  else if (epi == SG_F32) sgemv_finalize_kernel<SG_F32, false><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, G);
  else if (has_res) sgemv_finalize_kernel<SG_BF16, true><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, G);
  else sgemv_finalize_kernel<SG_BF16, false><<<blocks, 256, 0, stream>>>(out, part, rr, M, N, G);
}

// Workgroups of the MFMA form per CU the band is sized for: what the kernel's registers allow (one for every form
// since the epilogue prefetch took the 8-row kernels past 128 VGPRs), capped by K8S_SGEMV_WG_PER_CU (default 1: at 2 the 70B QKV / gate/up / down ran 9 / 3 / 3 %
// slower -- twice the workgroups re-read x -- and O 3 % faster; profiles/sgemv_mfma4_kernel_trace_r4.txt).
static int sm_wg_cap() {
  static const int v = [] { const char* e = getenv("K8S_SGEMV_WG_PER_CU"); return e ? max(1, atoi(e)) : 1; }();
  return v;
}
static std::atomic<unsigned> g_sm_next_range{0};   // one rotation for every instantiation (launches on any stream)

template <int MT, int JT, int EE, bool NN, bool RR, bool F8>
static bool sm_launch(void* out, void* partial, const bf16_t* x, const void* W, const float* wscale, const bf16_t* res,
                      int M, int N, int K, float eps, const SmPlan& sp, hipStream_t stream) {
  static const int occ = [] {
    int n = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&smfma_kernel<MT, JT, EE, NN, RR, F8>),
                                                     512, 0) != hipSuccess)
      n = 1;
    return max(1, min(n, sm_wg_cap()));
  }();
  // ~occ workgroups per CU and k-group, at least 16 rows (x is re-read per workgroup), at most the LDS partials'
  // quads (SwiGLU: gate + up quads, with the phantom rounding)
  constexpr int qmax = 512 / MT;
  const int bandmax = 4 * qmax / (EE == SG_SWIGLU ? 2 : 1);
  const int per = max(1, sm_cus() * occ / sp.g);
  int band = max(min(16, N), (N + per - 1) / per);
  if (band > bandmax) {
    int nb = (N + bandmax - 1) / bandmax;
    nb = (nb + per - 1) / per * per;   // whole rounds of workgroups
    band = (N + nb - 1) / nb;
  }
  const dim3 grid((N + band - 1) / band, sp.g);
  float* part = sp.g > 1 ? (float*)partial : nullptr;
  unsigned* tk = nullptr;   // k-groups: the in-kernel reduction's ticket range (rotating), if the bands fit one
  if (sp.g > 1 && grid.x <= (unsigned)SM_TICKET_RANGE) {
    unsigned* base = nullptr;
    if (hipGetSymbolAddress((void**)&base, HIP_SYMBOL(sm_tickets)) == hipSuccess)
      tk = base + (size_t)(g_sm_next_range.fetch_add(1) % SM_TICKET_RANGES) * SM_TICKET_RANGE;
  }
  smfma_kernel<MT, JT, EE, NN, RR, F8><<<grid, 512, 0, stream>>>(out, part, x, W, wscale, res, M, N, K, eps, band,
                                                                 sp.jw, tk);
  return tk != nullptr;
}

// out [M, N] (bf16, or fp32 for epi 1); x [M, K] bf16; W [N, K] (epi 2: [2N, K], gate rows then up rows) bf16, or
// e4m3 bytes when wscale != null (fp32 per weight row); res [M, N] bf16 for the residual epilogue (may be out);
// partial: k8s_sgemv_workspace floats.  norm: scale row m by 1/rms(x[m]) (the gamma folded into W).
// Returns 0, a negative argument error, or -5 when this kernel does not take the call (the caller routes it to
// mgemm).
extern "C" int k8s_sgemv(void* out, void* partial, const void* x, const void* W, const float* wscale, const void* res,
                         int M, int N, int K, int epi, int norm, float eps, hipStream_t stream) {
  if (M < 1 || M > 16 || N <= 0 || K <= 0) return -1;
  const bool fp8 = wscale != nullptr;
  if (K % (fp8 ? 16 : 8) != 0) return -1;
  if (epi < SG_BF16 || epi > SG_SWIGLU) return -1;
  const bool has_res = res != nullptr;
  if (has_res && (epi != SG_BF16 || norm)) return -5;
  const bf16_t* xx = (const bf16_t*)x;
  const bf16_t* rr = (const bf16_t*)res;
  SmPlan sp;
  if (sm_take(M, K, fp8, sp)) {
    if (norm && sp.g > 1) return -5;
    if (sp.g > 1 && partial == nullptr) return -3;
#define SMK(MT, JT, EE, NN, RR, F8) \
  g_last = sm_launch<MT, JT, EE, NN, RR, F8>(out, partial, xx, W, wscale, rr, M, N, K, eps, sp, stream)
#define SMK_COMBO(MT, JT, F8)                                                           \
  if (epi == SG_BF16 && norm) { SMK(MT, JT, SG_BF16, true, false, F8); }                \
  else if (epi == SG_BF16 && has_res) { SMK(MT, JT, SG_BF16, false, true, F8); }        \
  else if (epi == SG_BF16) { SMK(MT, JT, SG_BF16, false, false, F8); }                  \
  else if (epi == SG_SWIGLU && norm) { SMK(MT, JT, SG_SWIGLU, true, false, F8); }       \
  else if (epi == SG_SWIGLU) { SMK(MT, JT, SG_SWIGLU, false, false, F8); }              \
  else if (norm) { SMK(MT, JT, SG_F32, true, false, F8); }                              \
  else { SMK(MT, JT, SG_F32, false, false, F8); }
#define SMK_JT(MT)                                           \
  if (fp8) {   /* (sm_plan keeps fp8 at <= 4 steps) */      \
    if (sp.jt == 1) { SMK_COMBO(MT, 1, true) }               \
    else if (sp.jt == 2) { SMK_COMBO(MT, 2, true) }          \
    else { SMK_COMBO(MT, 4, true) }                          \
  } else if (sp.jt == 1) { SMK_COMBO(MT, 1, false) }         \
  else if (sp.jt == 2) { SMK_COMBO(MT, 2, false) }           \
  else if (sp.jt == 4) { SMK_COMBO(MT, 4, false) }           \
  else { SMK_COMBO(MT, 8, false) }
    bool g_last = false;   // (true: the launch reduces its k-groups itself)
    if (M <= 8) { SMK_JT(8) } else { SMK_JT(16) }
#undef SMK_JT
#undef SMK_COMBO
#undef SMK
    if (sp.g > 1 && !g_last) sg_finalize(out, (float*)partial, rr, M, N, sp.g, epi, has_res, stream);
    return (int)hipGetLastError();
  }
  if (M > 8) return -5;
  SgPlan p = sg_plan(K);
  if (norm && p.g > 1) return -5;
  if (p.g > 1 && partial == nullptr) return -3;
  // rows per workgroup: enough workgroups to put every CU to work (~512 per k-group, 2 per CU), at most SG_BAND;
  // fewer rows per wave re-read x (L2-resident) more often, so the band never drops below 4 rows
  const int nr = epi == SG_SWIGLU ? 1 : 2;
  int band = (N + 511) / 512;
  band = min(SG_BAND, max(4, (band + nr - 1) / nr * nr));
  const dim3 grid((N + band - 1) / band, p.g);
  const int half_rows = epi == SG_SWIGLU ? N : 0;
  float* part = p.g > 1 ? (float*)partial : nullptr;
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
  if (p.g > 1) sg_finalize(out, part, rr, M, N, p.g, epi, has_res, stream);
  return (int)hipGetLastError();
}
