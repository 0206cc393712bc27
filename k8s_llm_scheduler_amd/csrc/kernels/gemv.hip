// K3/K8/K9/K11/K12 decode path: skinny GEMM out[M, N] = x[M, K] . W[N, K]^T for M <= 8 rows
// (decode batch), bf16 weights streamed from HBM exactly once.
//
// The weight stream is the whole cost (HBM-bound: 2 bytes per weight, ~1 FLOP/byte at M = 1),
// so the kernel is built around keeping many 16-byte weight loads in flight per lane:
//  * one wave owns RPW output rows; a workgroup = 4 waves shares one K-slice of x staged in
//    LDS (x is re-read by every row, the LDS read is 256 B/clk/CU vs the L1's 64),
//  * weights are loaded with non-temporal hints (read once: keep them out of L2/MALL),
//  * bf16 pairs are multiplied with v_dot2_f32_bf16 (fp32 accumulate),
//  * when N alone gives too few workgroups to fill 256 CUs, K is split (grid.y) and partial
//    fp32 slabs are combined by a finalize kernel that also applies the epilogue;
//  * for small N (e.g. the TP = 8 QKV / gate-up slices) KW waves of a workgroup share one row
//    set and split its K range (reduced through LDS), so every wave's share of the weight
//    stream is in flight at once instead of taking several dependent rounds.
// Epilogues: BF16 store, FP32 store (logits), SWIGLU: W = [gate; up] (2I rows) and the output is
// silu(gate_j) * up_j (SURVEY.md K10 fused into K9).
// FP8 weights (BASELINE config 5): W holds OCP e4m3 bytes with one fp32 scale per row; a 16-byte
// load carries 16 weights (half the HBM bytes of bf16); every dword of four e4m3 is converted to two
// bf16 pairs with v_cvt_scalef32_pk_bf16_fp8 (exact) and fed to v_dot2_f32_bf16 against the packed
// activations; the row scale is applied once in the epilogue.
#include <cstdlib>

#include "common.h"

namespace k8sllm {

enum Epi { EPI_BF16 = 0, EPI_F32 = 1, EPI_SWIGLU = 2 };

__device__ __forceinline__ float dot2(uint32_t w, uint32_t x, float acc) {
  // bf16 pairs -> v_dot2c_f32_bf16.  (Passing the 16-byte vectors by reference and bit-casting
  // their elements miscompiled to a single-dword load under ROCm 7.2 -- keep scalars here.)
  bf16x2 a, b;
  __builtin_memcpy(&a, &w, 4);
  __builtin_memcpy(&b, &x, 4);
  return __builtin_amdgcn_fdot2_f32_bf16(a, b, acc, false);
}
__device__ __forceinline__ float dot8(u32x4 w, u32x4 x, float acc) {
  acc = dot2(w.x, x.x, acc);
  acc = dot2(w.y, x.y, acc);
  acc = dot2(w.z, x.z, acc);
  return dot2(w.w, x.w, acc);
}

// 16 fp8 weights (one 16-byte load) against 16 bf16 activations (two 16-byte LDS vectors): each
// dword of 4 e4m3 weights becomes two bf16 pairs with gfx950's v_cvt_scalef32_pk_bf16_fp8 (exact:
// e4m3 fits bf16) and meets its activation pairs in v_dot2_f32_bf16 -- 16 VALU ops per 16 weights
// and no activation unpacking (the f32 path needed ~40).
__device__ __forceinline__ float dot16_fp8(u32x4 w, u32x4 x0, u32x4 x1, float acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x2 lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[j], 1.0f, false);  // bytes 0, 1
    const bf16x2 hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[j], 1.0f, true);   // bytes 2, 3
    const uint32_t xa = j < 2 ? x0[2 * j] : x1[2 * j - 4];
    const uint32_t xb = j < 2 ? x0[2 * j + 1] : x1[2 * j - 3];
    bf16x2 a, b;
    __builtin_memcpy(&a, &xa, 4);
    __builtin_memcpy(&b, &xb, 4);
    acc = __builtin_amdgcn_fdot2_f32_bf16(lo, a, acc, false);
    acc = __builtin_amdgcn_fdot2_f32_bf16(hi, b, acc, false);
  }
  return acc;
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// Tensor-parallel all-reduce fused into a row-parallel projection (o_proj / down at TP > 1 decode; SURVEY
// K8 / K11 + K14 + K2): out = residual + sum over ranks of x_r . W_r^T, without a collective kernel.
// Each wave owns two adjacent output rows, so its bf16-rounded partials for one input row are one 32-bit
// word; lanes t < world push that word as an LL granule {word, epoch} (one 8-byte system-coherent store,
// arrives untorn) into source row `rank` of rank t's fused-LL region (own rank included).  Workgroups are
// grouped; the last workgroup of a group to finish (an arrival ticket) polls the group's granules from
// all world sources in its own region until every tag equals the epoch, sums them in rank order 0..W-1
// (fp32) plus the residual and rounds once: the same bits as the separate LL all-reduce, on every rank.
// Only one workgroup per group ever waits for peers, after its own share of the weight stream is done.
// Epochs are per group (identical on every rank: same grid, same call sequence); two parities per
// (source, word) are enough for the reason the separate LL kernel gives (xgmi.hip).  Polls are bounded:
// a timeout sets a bit of *err and the kernel drains.
constexpr int GAR_MAX_WORLD = 8;
constexpr int GAR_MAX_GROUPS = 64;
constexpr int GAR_SYS = 1 | 16;  // buffer-op aux: sc0 | sc1 (system coherence)
struct GemvAr {
  char* base[GAR_MAX_WORLD];  // fused-LL region of every rank, mapped in this process
  long long row_bytes;        // capacity of one (parity, source) row
  uint32_t* epochs;           // [GAR_MAX_GROUPS] per-group epochs (uncached)
  uint32_t* tickets;          // [GAR_MAX_GROUPS] arrival tickets, zero between calls (uncached)
  uint32_t* err;              // poll-timeout bitmask
  const bf16_t* res;          // [M, N_out] residual (may alias out)
  long long timeout_ticks;    // s_memrealtime ticks (100 MHz)
  int rank, world, group;     // group: workgroups per arrival group
};

// Fused pre-norm prologue (NORM): the GEMV input is rmsnorm(x + res_in) * nw, computed by every
// workgroup from the full rows (L2-resident, M x K x 4 bytes), and workgroup (0, 0) writes the
// updated residual r = x + res_in to res_out.  res_in and res_out must be different buffers
// (the model ping-pongs two residual buffers) because other workgroups are still reading res_in.
template <int M>
__device__ __forceinline__ void norm_row_chunk(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res_in,
                                               int m, int K, int c, u32x4& r) {
  const u32x4 a = *reinterpret_cast<const u32x4*>(x + (size_t)m * K + c * 8);
  if (res_in == nullptr) { r = a; return; }
  const u32x4 b = *reinterpret_cast<const u32x4*>(res_in + (size_t)m * K + c * 8);
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = pack_bf2(lo_bf(a[j]) + lo_bf(b[j]), hi_bf(a[j]) + hi_bf(b[j]));
}

// NORM: 0 = plain input x; 1 = rmsnorm(x + res_in) * nw applied in the prologue; 2 = the norm weight is
// folded into W (W' = W * nw, done once at model load): the prologue only stages r = x + res_in and
// its sum of squares, and the per-row 1/rms scales the accumulator in the epilogue -- no
// normalisation pass and no barrier between the row statistics and the weight stream.
// LOOP: every wave owns row sets s, s + S, s + 2 S, ... (S = waves in the grid) instead of one: x is staged into
// LDS once per workgroup for several row sets, and the first weight block of the next row set is in flight while
// the current one's last block is consumed (one-row-set waves have no such overlap -- an fp8 row of 8192 weights
// is a single round of loads per lane).  Single K slice, one wave per row set, no fused all-reduce.
template <int M, int RPW, int EPI, int NORM, bool FP8, int KW, int NT = 256, bool AR = false, bool LOOP = false>
__global__ void __launch_bounds__(NT) gemv_kernel(void* __restrict__ out, float* __restrict__ partial,
                                                   const bf16_t* __restrict__ x, const void* __restrict__ W,
                                                   int N_out, int K, int KS, int half_rows,
                                                   const bf16_t* __restrict__ res_in, bf16_t* __restrict__ res_out,
                                                   const bf16_t* __restrict__ nw, float eps,
                                                   const float* __restrict__ wscale, GemvAr ar) {
  constexpr int EPC = FP8 ? 16 : 8;  // weights per 16-byte chunk
  constexpr int WB = FP8 ? 1 : 2;    // bytes per weight
  static_assert(!AR || (EPI == EPI_BF16 && RPW == 2 && KW == 1 && NORM == 0), "fused all-reduce: plain 2-row waves");
  static_assert(!LOOP || (KW == 1 && NORM != 1), "row-set loop: one wave per row set, no prologue norm");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  u32x4* xs = reinterpret_cast<u32x4*>(smem);  // [M][KS/8]
  constexpr int NWV = NT / 64;  // waves per workgroup; NWV / KW row sets
  __shared__ float nred[NWV][M];
  __shared__ uint32_t ar_state[2];  // AR: [epoch, last-arriver flag]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (AR && threadIdx.x == 0)
    ar_state[0] = __hip_atomic_load(ar.epochs + blockIdx.x / ar.group, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  const int kb = blockIdx.y * KS;
  const int klen = min(KS, K - kb);
  const int nch = klen / EPC;  // 16-byte weight chunks in this slice
  const int xch = klen >> 3;   // 16-byte x chunks (8 bf16) in this slice

  constexpr int NR = (EPI == EPI_SWIGLU) ? 2 * RPW : RPW;  // weight rows per wave
  constexpr int U = (NR >= 4) ? 2 : ((NR >= 2) ? 4 : 8);  // chunks per lane in flight per row
  // LOOP: lper row sets per wave; workgroup b owns the contiguous row sets [b NWV lper, (b + 1) NWV lper), its wave w
  // the sets b NWV lper + w + NWV j (contiguous bands keep the fused all-reduce's arrival groups contiguous)
  int lper = 1;
  if constexpr (LOOP) lper = ((N_out + RPW - 1) / RPW + (int)gridDim.x * NWV - 1) / ((int)gridDim.x * NWV);
  const int r0 = ((int)blockIdx.x * (NWV / KW) * lper + wid / KW) * RPW;  // first output row of this wave
  const bool active = r0 < N_out;
  const int kpart = wid % KW;                                // this wave's share of the K chunks
  const int per = (nch + KW - 1) / KW;
  const int cb = kpart * per, ce = min(nch, cb + per), clast = max(min(ce, nch) - 1, 0);
  const char* wrow[NR];
  const char* Wb = static_cast<const char*>(W);
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int n = min(r0 + r, N_out - 1);
    wrow[r] = Wb + ((size_t)n * K + kb) * WB;
    if (EPI == EPI_SWIGLU) wrow[RPW + r] = Wb + ((size_t)(n + half_rows) * K + kb) * WB;
  }
  // NORM: the norm weights and the first NL row chunks of x (+ res_in) per thread are loaded BEFORE
  // the weight stream: vmcnt retires in order, so the prologue's waits then do not sit behind the
  // weights' HBM latency and the reduction overlaps the first weight round trip
  constexpr int NL = M <= 2 ? 4 : (M <= 4 ? 2 : 1);
  constexpr int GI = (1024 + NT - 1) / NT;  // norm-weight chunks per thread held in registers (xch <= 1024)
  const int nkc = K >> 3;
  u32x4 g[GI];
  // the first pass's x (and residual) chunks: every load issued before any is consumed -- the add of
  // x + res_in happens after the weight stream has been started (norm_row_chunk's own add would wait
  // for each chunk in turn, a serial chain of L2 round trips ahead of the first weight load)
  u32x4 pre[NL][M], preb[NL][M];
  const bool has_res = res_in != nullptr;
  if (NORM != 0) {
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      if (NORM != 1) break;
      const int c = threadIdx.x + NT * i;
      if (c < xch) g[i] = reinterpret_cast<const u32x4*>(nw + kb)[c];
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int c = min((int)threadIdx.x + u * (int)blockDim.x, nkc - 1);
#pragma unroll
      for (int m = 0; m < M; ++m) pre[u][m] = *reinterpret_cast<const u32x4*>(x + (size_t)m * K + c * 8);
    }
    if (has_res) {
#pragma unroll
      for (int u = 0; u < NL; ++u) {
        const int c = min((int)threadIdx.x + u * (int)blockDim.x, nkc - 1);
#pragma unroll
        for (int m = 0; m < M; ++m) preb[u][m] = *reinterpret_cast<const u32x4*>(res_in + (size_t)m * K + c * 8);
      }
    }
  }
  // plain input: the first XP x chunks per thread (XP = 4 at M <= 2: a whole 8192-wide row at 256 threads) are loaded
  // BEFORE the weight stream too, so staging them into LDS waits for x only, not for the first
  // weight block (loads retire in order: a wait for x issued after the weights is a wait for both)
  constexpr int XP = M <= 2 ? 4 : (M <= 4 ? 2 : 1);   // px holds XP x M x 4 registers: cap it at ~32 for any M
  u32x4 px[XP][M];
  if (NORM == 0) {
    // unconditional buffer loads bounded by the slice: a chunk past it reads 0 without a memory access
    // (a branch per chunk made the compiler copy the whole array per branch and wait on each load)
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x + kb), 0,
                                                     (M - 1) * K * 2 + xch * 16, 0x00020000);
#pragma unroll
    for (int p = 0; p < XP; ++p) {
      const int i = (int)threadIdx.x + p * NT;
#pragma unroll
      for (int m = 0; m < M; ++m)
        px[p][m] = __builtin_amdgcn_raw_buffer_load_b128(xr, m * K * 2 + i * 16, 0, 0);
    }
  }
  // weights do not depend on x: start streaming them before the x staging / norm prologue
  u32x4 wv[U][NR];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int r = 0; r < NR; ++r)
      wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow[r]) + min(cb + lane + 64 * u, clast));
  // keep the x staging below the weight issue: the compiler would otherwise merge each x chunk's
  // `if (i < xch)` load and LDS store into one block ahead of the weights and wait per chunk
  asm volatile("" ::: "memory");

  float inv[M];
  if (NORM != 0) {
    // One global pass: r = x + res_in over the whole row (the sum of squares needs all of it),
    // this slice of r parked in LDS, this thread's norm-weight chunks prefetched into registers;
    // after the reduction the slice is normalised in place in LDS (no second global read).
    const bool writer = blockIdx.x == 0 && blockIdx.y == 0 && res_out != nullptr;
    const int kc0 = kb >> 3;
    float ss[M];
#pragma unroll
    for (int m = 0; m < M; ++m) ss[m] = 0.f;
    // NL row chunks per thread per pass, all loaded before any is consumed.  The first pass was issued
    // before the weight stream and is consumed here in straight-line code, so the compiler's wait
    // counts only its own loads (inside a loop the header wait would be vmcnt(0), i.e. also wait for
    // the first weight block); at K = 8192 and M <= 2 the whole row is this one pass.
    auto consume = [&](int c0, u32x4 (&r)[NL][M]) {
#pragma unroll
      for (int u = 0; u < NL; ++u) {
        const int c = c0 + u * (int)blockDim.x;
        if (c >= nkc) break;
        const int cs = c - kc0;
#pragma unroll
        for (int m = 0; m < M; ++m) {
          if (writer) reinterpret_cast<u32x4*>(res_out + (size_t)m * K)[c] = r[u][m];
          if (cs >= 0 && cs < xch) xs[m * (KS >> 3) + cs] = r[u][m];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float l = lo_bf(r[u][m][j]), h = hi_bf(r[u][m][j]);
            ss[m] += l * l + h * h;
          }
        }
      }
    };
    if (has_res) {
#pragma unroll
      for (int u = 0; u < NL; ++u)
#pragma unroll
        for (int m = 0; m < M; ++m)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            pre[u][m][j] = pack_bf2(lo_bf(pre[u][m][j]) + lo_bf(preb[u][m][j]),
                                    hi_bf(pre[u][m][j]) + hi_bf(preb[u][m][j]));
    }
    consume((int)threadIdx.x, pre);
    if (nkc > (int)blockDim.x * NL) {   // rows longer than one pass (K > 8192 at M <= 2)
      for (int c0 = threadIdx.x + blockDim.x * NL; c0 < nkc; c0 += blockDim.x * NL) {
        u32x4 r[NL][M];
#pragma unroll
        for (int u = 0; u < NL; ++u) {
          const int c = min(c0 + u * (int)blockDim.x, nkc - 1);
#pragma unroll
          for (int m = 0; m < M; ++m) norm_row_chunk<M>(x, res_in, m, K, c, r[u][m]);
        }
        consume(c0, r);
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float t = wave_sum(ss[m]);
      if (lane == 0) nred[wid][m] = t;
    }
  }
  if (NORM == 1) {
    __syncthreads();
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t += nred[w][m];
      inv[m] = rsqrtf(t / (float)K + eps);
    }
#pragma unroll
    for (int i = 0; i < GI; ++i) {
      const int c = threadIdx.x + NT * i;
      if (c >= xch) break;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const u32x4 r = xs[m * (KS >> 3) + c];
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = pack_bf2(lo_bf(r[j]) * inv[m] * lo_bf(g[i][j]), hi_bf(r[j]) * inv[m] * hi_bf(g[i][j]));
        xs[m * (KS >> 3) + c] = o;
      }
    }
    for (int c = threadIdx.x + NT * GI; c < xch; c += blockDim.x) {  // slices longer than 8192
      const u32x4 gw = reinterpret_cast<const u32x4*>(nw + kb)[c];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const u32x4 r = xs[m * (KS >> 3) + c];
        u32x4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          o[j] = pack_bf2(lo_bf(r[j]) * inv[m] * lo_bf(gw[j]), hi_bf(r[j]) * inv[m] * hi_bf(gw[j]));
        xs[m * (KS >> 3) + c] = o;
      }
    }
  } else if (NORM == 0) {
    // stage x[:, kb:kb+klen] into LDS: the chunks loaded ahead of the weights, then any remainder
#pragma unroll
    for (int p = 0; p < XP; ++p) {
      const int i = (int)threadIdx.x + p * NT;
      if (i < xch) {
#pragma unroll
        for (int m = 0; m < M; ++m) xs[m * (KS >> 3) + i] = px[p][m];
      }
    }
    for (int i = threadIdx.x + XP * NT; i < xch; i += NT) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        xs[m * (KS >> 3) + i] = *reinterpret_cast<const u32x4*>(x + (size_t)m * K + kb + i * 8);
    }
  }
  __syncthreads();

  // main loop: software-pipelined weight stream (the loads of block i+1 are in flight while block
  // i is consumed); the first block was issued before the x / norm prologue
  float acc[NR][M];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;

  if constexpr (LOOP) {
    const int nsets = (N_out + RPW - 1) / RPW;
    const int set_end = min(nsets, ((int)blockIdx.x + 1) * NWV * lper);
    const int bpr = (nch + 64 * U - 1) / (64 * U);      // weight blocks per row set
    int set = (int)blockIdx.x * NWV * lper + wid;
    if (NORM == 2) {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < NWV; ++w) t += nred[w][m];
        inv[m] = rsqrtf(t / (float)K + eps);
      }
    }
    const char* nrow[NR];
    for (int j = 0; set < set_end;) {
      u32x4 cur[U][NR];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < NR; ++r) cur[u][r] = wv[u][r];
      // issue the next block: the rest of this row set, or the first block of the wave's next row set
      int nj = j + 1, nset = set;
      if (nj == bpr) {
        nj = 0;
        nset = set + NWV;
      }
      if (nset < set_end) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
          const int n = min(nset * RPW + r, N_out - 1);
          nrow[r] = Wb + (size_t)n * K * WB;
          if (EPI == EPI_SWIGLU) nrow[RPW + r] = Wb + ((size_t)(n + half_rows) * K) * WB;
        }
        const int cn = nj * 64 * U + lane;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < NR; ++r)
            wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(nrow[r]) + min(cn + 64 * u, clast));
      }
      const int c = j * 64 * U + lane;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (c + 64 * u < nch) {
#pragma unroll
          for (int m = 0; m < M; ++m) {
            if (FP8) {
              const u32x4 x0 = xs[m * (KS >> 3) + 2 * (c + 64 * u)];
              const u32x4 x1 = xs[m * (KS >> 3) + 2 * (c + 64 * u) + 1];
#pragma unroll
              for (int r = 0; r < NR; ++r) acc[r][m] = dot16_fp8(cur[u][r], x0, x1, acc[r][m]);
            } else {
              const u32x4 xv = xs[m * (KS >> 3) + c + 64 * u];
#pragma unroll
              for (int r = 0; r < NR; ++r) acc[r][m] = dot8(cur[u][r], xv, acc[r][m]);
            }
          }
        }
      }
      if (nj == 0) {  // row set `set` is complete: reduce, scale, store, start the next one
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int m = 0; m < M; ++m) {
            float v = wave_sum(acc[r][m]);
            if (NORM == 2) v *= inv[m];
            acc[r][m] = v;
          }
        if constexpr (AR) {   // push this row set's partial words to every peer (see the non-loop push below)
          typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
          const uint32_t e = ar_state[0];
          if (lane < ar.world) {
            const int rr = set * RPW, nwd = N_out >> 1;
            const auto rs = __builtin_amdgcn_make_buffer_rsrc(
                ar.base[lane] + ((long long)(e & 1) * ar.world + ar.rank) * ar.row_bytes, 0, (int)ar.row_bytes, 0x00020000);
            const float s0 = FP8 ? wscale[rr] : 1.f, s1 = FP8 ? wscale[rr + 1] : 1.f;
#pragma unroll
            for (int m = 0; m < M; ++m) {
              const u32x2 g = u32x2{pack_bf2(acc[0][m] * s0, acc[1][m] * s1), e};
              __builtin_amdgcn_raw_buffer_store_b64(g, rs, (m * nwd + (rr >> 1)) * 8, 0, GAR_SYS);
            }
          }
        } else if (lane == 0) {
#pragma unroll
          for (int r = 0; r < RPW; ++r) {
            const int n = set * RPW + r;
            if (n >= N_out) break;
            const float sg = FP8 ? wscale[n] : 1.f;
            const float su = (FP8 && EPI == EPI_SWIGLU) ? wscale[n + half_rows] : 1.f;
#pragma unroll
            for (int m = 0; m < M; ++m) {
              const float a = acc[r][m] * sg;
              if (EPI == EPI_F32) {
                reinterpret_cast<float*>(out)[(size_t)m * N_out + n] = a;
              } else if (EPI == EPI_SWIGLU) {
                reinterpret_cast<bf16_t*>(out)[(size_t)m * N_out + n] = f2bf(silu(a) * (acc[RPW + r][m] * su));
              } else {
                reinterpret_cast<bf16_t*>(out)[(size_t)m * N_out + n] = f2bf(a);
              }
            }
          }
        }
#pragma unroll
        for (int r = 0; r < NR; ++r)
#pragma unroll
          for (int m = 0; m < M; ++m) acc[r][m] = 0.f;
        set = nset;
      }
      j = nj;
    }
    if constexpr (!AR) return;
  }
  if constexpr (!LOOP) {
  for (int c = cb + lane; active && c < ce; c += 64 * U) {
    u32x4 cur[U][NR];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int r = 0; r < NR; ++r) cur[u][r] = wv[u][r];
    const int cn = c + 64 * U;
    if (cn < ce) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < NR; ++r)
          wv[u][r] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(wrow[r]) + min(cn + 64 * u, clast));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (c + 64 * u < ce) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          if (FP8) {
            const u32x4 x0 = xs[m * (KS >> 3) + 2 * (c + 64 * u)];
            const u32x4 x1 = xs[m * (KS >> 3) + 2 * (c + 64 * u) + 1];
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r][m] = dot16_fp8(cur[u][r], x0, x1, acc[r][m]);
          } else {
            const u32x4 xv = xs[m * (KS >> 3) + c + 64 * u];
#pragma unroll
            for (int r = 0; r < NR; ++r) acc[r][m] = dot8(cur[u][r], xv, acc[r][m]);
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = wave_sum(acc[r][m]);
  }

  if constexpr (AR) {
    typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
    const uint32_t e = ar_state[0];
    const int W = ar.world, nwd = N_out >> 1;  // LL words per input row
    const long long par = (long long)(e & 1) * W;
    // 1. push: lane t < W sends this wave's M words to rank t (row `rank` of its parity-(e & 1) slot); the loop
    // variant pushed every row set's words as it finished them
    if (!LOOP && active && lane < W) {
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(ar.base[lane] + (par + ar.rank) * ar.row_bytes, 0,
                                                        (int)ar.row_bytes, 0x00020000);
      const float s0 = FP8 ? wscale[r0] : 1.f, s1 = FP8 ? wscale[r0 + 1] : 1.f;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const u32x2 g = u32x2{pack_bf2(acc[0][m] * s0, acc[1][m] * s1), e};
        __builtin_amdgcn_raw_buffer_store_b64(g, rs, (m * nwd + (r0 >> 1)) * 8, 0, GAR_SYS);
      }
    }
    // 2. arrival ticket of this workgroup's group; the last arriver reduces the group's rows
    const int grp = blockIdx.x / ar.group;
    const int g0 = grp * ar.group, gn = min((int)gridDim.x, g0 + ar.group);
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t old = __hip_atomic_fetch_add(ar.tickets + grp, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      ar_state[1] = old == (uint32_t)(gn - g0 - 1);
    }
    __syncthreads();
    if (!ar_state[1]) return;
    if (threadIdx.x == 0) {  // every workgroup of the group has read its epoch and arrived: reset for the next call
      __hip_atomic_store(ar.tickets + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ar.epochs + grp, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // 3. words [w0, w1) of every input row, summed over the W sources in rank order, + residual, one rounding
    const int ROWS_WG = (NT / 64) * RPW * lper;
    const int w0 = g0 * ROWS_WG / 2, w1 = min(nwd, gn * ROWS_WG / 2), nw = w1 - w0;
    const char* mine = ar.base[ar.rank] + par * ar.row_bytes;
    const uint32_t* res = reinterpret_cast<const uint32_t*>(ar.res);
    uint32_t* o = reinterpret_cast<uint32_t*>(out);
    for (int i = threadIdx.x; i < M * nw; i += NT) {
      const int m = i / nw, wi = m * nwd + w0 + (i - m * nw);
      u32x2 g[GAR_MAX_WORLD];
#pragma unroll
      for (int t = 0; t < GAR_MAX_WORLD; ++t)
        if (t < W)
          g[t] = __builtin_amdgcn_raw_buffer_load_b64(
              __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(mine) + t * ar.row_bytes, 0, (int)ar.row_bytes,
                                                0x00020000), wi * 8, 0, GAR_SYS);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      float lo = 0.f, hi = 0.f;
#pragma unroll
      for (int t = 0; t < GAR_MAX_WORLD; ++t) {
        if (t >= W) break;
        while (g[t].y != e) {
          __builtin_amdgcn_s_sleep(1);
          if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > ar.timeout_ticks) {
            __hip_atomic_fetch_or(ar.err, 1u << t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
          g[t] = __builtin_amdgcn_raw_buffer_load_b64(
              __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(mine) + t * ar.row_bytes, 0, (int)ar.row_bytes,
                                                0x00020000), wi * 8, 0, GAR_SYS);
        }
        lo += lo_bf(g[t].x);
        hi += hi_bf(g[t].x);
      }
      if (res != nullptr) {
        const uint32_t rv = res[wi];
        lo += lo_bf(rv);
        hi += hi_bf(rv);
      }
      o[wi] = pack_bf2(lo, hi);
    }
    return;
  }

  if (KW > 1) {  // combine the K parts of the waves sharing these rows
    __shared__ float kred[NWV][NR][M];
    if (lane == 0) {
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) kred[wid][r][m] = acc[r][m];
    }
    __syncthreads();
    if (kpart != 0 || lane != 0 || !active) return;
#pragma unroll
    for (int j = 1; j < KW; ++j)
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int m = 0; m < M; ++m) acc[r][m] += kred[wid + j][r][m];
  } else if (lane != 0 || !active) {
    return;
  }
  const int wrows = (EPI == EPI_SWIGLU) ? 2 * half_rows : N_out;  // weight rows (slab width)
  if (NORM == 2) {  // 1/rms of each input row (the statistics are in LDS since the pre-loop barrier)
#pragma unroll
    for (int m = 0; m < M; ++m) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) t += nred[w][m];
      inv[m] = rsqrtf(t / (float)K + eps);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int m = 0; m < M; ++m) acc[r][m] *= inv[m];
  }
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int n = r0 + r;
    if (n >= N_out) break;
    if (FP8) {
      const float sg = wscale[n];
      const float su = EPI == EPI_SWIGLU ? wscale[n + half_rows] : 0.f;
#pragma unroll
      for (int m = 0; m < M; ++m) {
        acc[r][m] *= sg;
        if (EPI == EPI_SWIGLU) acc[RPW + r][m] *= su;
      }
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
      if (partial != nullptr) {
        float* slab = partial + ((size_t)blockIdx.y * M + m) * wrows;
        slab[n] = acc[r][m];
        if (EPI == EPI_SWIGLU) slab[n + half_rows] = acc[RPW + r][m];
      } else if (EPI == EPI_F32) {
        reinterpret_cast<float*>(out)[(size_t)m * N_out + n] = acc[r][m];
      } else if (EPI == EPI_SWIGLU) {
        reinterpret_cast<bf16_t*>(out)[(size_t)m * N_out + n] = f2bf(silu(acc[r][m]) * acc[RPW + r][m]);
      } else {
        reinterpret_cast<bf16_t*>(out)[(size_t)m * N_out + n] = f2bf(acc[r][m]);
      }
    }
  }
}

template <int EPI>
__global__ void gemv_finalize_kernel(void* __restrict__ out, const float* __restrict__ partial, int M, int N_out,
                                     int splits, int half_rows) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N_out) return;
  const int m = i / N_out, n = i - m * N_out;
  const int wrows = (EPI == EPI_SWIGLU) ? 2 * half_rows : N_out;
  float a = 0.f, b = 0.f;
  for (int s = 0; s < splits; ++s) {
    const float* slab = partial + ((size_t)s * M + m) * wrows;
    a += slab[n];
    if (EPI == EPI_SWIGLU) b += slab[n + half_rows];
  }
  if (EPI == EPI_F32) reinterpret_cast<float*>(out)[i] = a;
  else if (EPI == EPI_SWIGLU) reinterpret_cast<bf16_t*>(out)[i] = f2bf(silu(a) * b);
  else reinterpret_cast<bf16_t*>(out)[i] = f2bf(a);
}

}  // namespace k8sllm

using namespace k8sllm;

// Plan the launch: returns the K-slice length (multiple of 512) and the split count.
// Rows per wave: 2 from M = 4 on.  Below, the plain (no norm prologue, no SwiGLU) projections with
// N >= 8192 outputs (o_proj, down at every TP degree) also take 2: half as many workgroups, twice the
// weight loads in flight per lane (measured TP = 8: o_proj 4.8 -> 3.6 us, down 10.8 -> 9.9 us; it
// loses on the small-N QKV and on gate/up, profiles/kbench_*).  K8S_GEMV_RPW1 = 1 / 2 forces M < 4.
static int gemv_rpw(int M, int N_out = 0, int epi = 0, int mode = 0) {
  static const int env = [] { const char* e = getenv("K8S_GEMV_RPW1"); return e ? atoi(e) : 0; }();
  if (M >= 4) return 2;
  if (env == 1 || env == 2) return env;
  return (mode == 0 && epi != EPI_SWIGLU && N_out >= 8192) ? 2 : 1;
}

extern "C" void k8s_gemv_plan(int M, int N_out, int K, int epi, int mode, int* ks_out, int* splits_out) {
  const int rpw = gemv_rpw(M, N_out, epi, mode);
  const int rows_per_wg = 4 * rpw;
  const int n_wg = (N_out + rows_per_wg - 1) / rows_per_wg;
  const int lds_cap_elems = 65536 / (2 * M);  // <= 64 KiB of x per workgroup (M=1: K up to 32768 unsplit)
  int splits = 1;
  const int target = 256;  // split K only when N alone cannot give every CU a workgroup
  if (n_wg < target) splits = (target + n_wg - 1) / n_wg;
  int ks = (K + splits - 1) / splits;
  ks = ((ks + 511) / 512) * 512;
  if (ks < 512) ks = 512;
  while (ks > lds_cap_elems) ks -= 512;
  if (ks > K) ks = ((K + 7) / 8) * 8;
  splits = (K + ks - 1) / ks;
  (void)epi;
  *ks_out = ks;
  *splits_out = splits;
}

// partial: fp32 workspace of splits * M * wrows floats (wrows = N_out, or 2*N_out for SWIGLU);
// may be null when the plan has a single split.
// wscale != null: W is fp8 (OCP e4m3, one fp32 scale per weight row); K must be a multiple of 16.
// mode: 0 plain, 1 norm weight nw applied in the prologue, 2 norm weight folded into W (nw unused)
// Row-set loop (LOOP): workgroups per CU the grid is cut to (0 = one row set per wave; -1 = default: 2 for fp8
// weights; for bf16 weights 2 on the plain bf16 epilogue (QKV, O, down) and off for SwiGLU / fp32 (gate/up, LM
// head)).  Measured on the 70B decode (profiles/gemv_loop_probe_r3.txt, bench A/B in
// profiles/bench_r3_gemv_loop_ab.txt): fp8 decode -0.6 %; bf16 with the loop everywhere +1.3 % (slower), on the
// plain-epilogue projections only -0.3 %.
// K8S_GEMV_LOOP sets it at load; k8s_gemv_set_loop changes it (tests, A/B probes).
static int g_gemv_loop = [] { const char* e = getenv("K8S_GEMV_LOOP"); return e ? atoi(e) : -1; }();
static int g_gemv_wide = [] { const char* e = getenv("K8S_GEMV_WIDE"); return e ? atoi(e) : 1; }();
extern "C" int k8s_gemv_set_wide(int on) {
  const int old = g_gemv_wide;
  if (on >= 0) g_gemv_wide = on;
  return old;
}
// bf16 SwiGLU (gate/up) GEMVs take the loop (2 workgroups per CU) when their one-row-set grid has at most this many
// workgroups: TP = 4 / 8 shapes (K8S_GEMV_LOOP_SWIGLU_MAX).  At one TP = 8 rank's shapes decode 4.554 -> 4.466
// ms/token (profiles/bench_r3_gemv_loop_ab.txt); at TP = 1 (7168 workgroups) the loop measured slower.
static int g_gemv_loop_swiglu_max = [] {
  const char* e = getenv("K8S_GEMV_LOOP_SWIGLU_MAX");
  return e ? atoi(e) : 2048;
}();
// smallest matrix (Mi weights) the fp8 / plain-epilogue loop takes (K8S_GEMV_LOOP_MIN_MI): 65 keeps the 70B O
// projection (exactly 64 Mi) off it -- +1.3 % end to end (profiles/bench_r3_gemv_loop_ab.txt)
static int g_gemv_loop_min_mi = [] { const char* e = getenv("K8S_GEMV_LOOP_MIN_MI"); return e ? atoi(e) : 65; }();
// default for bf16 weights with the plain bf16 epilogue (QKV, O, down -- not gate/up nor the LM head)
static int g_gemv_loop_bf16 = [] { const char* e = getenv("K8S_GEMV_LOOP_BF16"); return e ? atoi(e) : 2; }();
extern "C" int k8s_gemv_set_loop(int wg_per_cu) {   // returns the previous setting; < -1 only reads it
  const int old = g_gemv_loop;
  if (wg_per_cu >= -1) g_gemv_loop = wg_per_cu;
  return old;
}

static int gemv_launch(int mode, void* out, void* partial, const void* x, const void* W, const float* wscale, int M,
                       int N_out, int K, int epi, const void* res_in, void* res_out, const void* nw, float eps,
                       hipStream_t stream) {
  if (M < 1 || M > 8 || K % 8 != 0 || N_out <= 0) return -1;
  const bool fp8 = wscale != nullptr;
  if (fp8 && K % 16 != 0) return -1;
  int ks, splits;
  k8s_gemv_plan(M, N_out, K, epi, mode, &ks, &splits);
  if (splits > 1 && partial == nullptr) return -3;
  float* part = splits > 1 ? (float*)partial : nullptr;
  const int rpw = gemv_rpw(M, N_out, epi, mode);
  // KW: waves per row set (K8S_GEMV_KW = 2 / 4 splits a row set's K over that many waves).  One wave per row
  // set is the default: the two-wave split the small-N projections (TP = 8 QKV, LM head) used to take measured
  // slower end to end (TP = 8 shapes 4.28 -> 4.26 ms/token with one wave, 8B and TP = 1 unchanged,
  // profiles/gemv_kw_ab.txt).
  static const int kw_env = [] { const char* e = getenv("K8S_GEMV_KW"); return e ? atoi(e) : 0; }();
  const int kw = (kw_env == 2 || kw_env == 4) ? kw_env : 1;
  // The norm variants keep 4 row sets per workgroup when they split K (8 waves, 512 threads):
  // the per-workgroup norm prologue is then shared by twice the waves instead of being repeated.
  const int nt = (mode != 0 && kw == 2 && M <= 4) ? 512 : 256;
  const int rows_per_wg = (nt / 64 / kw) * rpw;
  dim3 grid((N_out + rows_per_wg - 1) / rows_per_wg, splits);
  const size_t lds = (size_t)M * ks * 2;
  const int half_rows = (epi == EPI_SWIGLU) ? N_out : 0;
  const bf16_t* xx = (const bf16_t*)x;
  const void* ww = W;
  const bf16_t* ri = (const bf16_t*)res_in;
  bf16_t* ro = (bf16_t*)res_out;
  const bf16_t* gw = (const bf16_t*)nw;
  const bool swiglu_loop = epi == EPI_SWIGLU && (int)grid.x <= g_gemv_loop_swiglu_max;
  // the loop only on matrices of >= 64 Mi weights (the 70B's at TP = 1, gate/up at TP = 4): on the smaller ones
  // (Llama-3-8B, fp8 at TP = 4) it measured slower
  const bool big = (long long)(epi == EPI_SWIGLU ? 2 * N_out : N_out) * K >= ((long long)g_gemv_loop_min_mi << 20);
  const bool plain_loop = epi == EPI_BF16 && big;
  const int loop_wg = g_gemv_loop >= 0 ? g_gemv_loop
                                       : (fp8 ? (big ? 2 : 0) : (plain_loop ? g_gemv_loop_bf16 : (swiglu_loop ? 2 : 0)));
  if (loop_wg > 0 && splits == 1 && kw == 1 && mode != 1 && M <= 2 && (int)grid.x > 256 * loop_wg) {
    // wide: 8-wave workgroups for the plain bf16-epilogue projections whose x slice takes >= 32 KiB of LDS (the
    // down projection, K = 28672: 56 KiB): LDS, not waves, bounds those at 2 workgroups per CU, so twice the waves
    // per workgroup put twice the weight loads in flight per CU (K8S_GEMV_WIDE = 0 turns it off)
    const bool wide = g_gemv_wide && mode == 0 && epi == EPI_BF16 && (long long)M * K * 2 >= 32768;
    if (wide) {
      const int wgs = (N_out + 8 * rpw - 1) / (8 * rpw);
      {
        const int per = (wgs + 256 * loop_wg - 1) / (256 * loop_wg);   // >= 1
        const dim3 wgrid((wgs + per - 1) / per, 1);
#define GW(MM, RR, F8)                                                                                              \
  gemv_kernel<MM, RR, EPI_BF16, 0, F8, 1, 512, false, true><<<wgrid, 512, lds, stream>>>(                           \
      out, nullptr, xx, ww, N_out, K, ks, half_rows, ri, ro, gw, eps, wscale, GemvAr{})
#define GW2(MM, RR) \
  if (fp8) { GW(MM, RR, true); } else { GW(MM, RR, false); }
        if (M == 1) { if (rpw == 2) { GW2(1, 2) } else { GW2(1, 1) } }
        else { if (rpw == 2) { GW2(2, 2) } else { GW2(2, 1) } }
#undef GW2
#undef GW
        return (int)hipGetLastError();
      }
    }
    const int per = ((int)grid.x + 256 * loop_wg - 1) / (256 * loop_wg);   // row sets per wave
    const dim3 lgrid(((int)grid.x + per - 1) / per, 1);
#define GL(MM, RR, EE, F8, NN)                                                                                     \
  gemv_kernel<MM, RR, EE, NN, F8, 1, 256, false, true><<<lgrid, 256, lds, stream>>>(out, nullptr, xx, ww, N_out, K, \
                                                                                     ks, half_rows, ri, ro, gw, eps, \
                                                                                     wscale, GemvAr{})
#define GL2(MM, RR, EE)                                             \
  if (fp8) { if (mode == 2) { GL(MM, RR, EE, true, 2); } else { GL(MM, RR, EE, true, 0); } }    \
  else { if (mode == 2) { GL(MM, RR, EE, false, 2); } else { GL(MM, RR, EE, false, 0); } }
#define GLE(MM, RR)                                      \
  switch (epi) {                                         \
    case EPI_BF16: GL2(MM, RR, EPI_BF16); break;         \
    case EPI_F32: GL2(MM, RR, EPI_F32); break;           \
    case EPI_SWIGLU: GL2(MM, RR, EPI_SWIGLU); break;     \
    default: return -2;                                  \
  }
    if (M == 1) { if (rpw == 2) { GLE(1, 2) } else { GLE(1, 1) } }
    else { if (rpw == 2) { GLE(2, 2) } else { GLE(2, 1) } }
#undef GLE
#undef GL2
#undef GL
    return (int)hipGetLastError();
  }
#define G4(MM, RR, EE, F8, KK, NTT)                                                                            \
  if (mode == 1) gemv_kernel<MM, RR, EE, 1, F8, KK, NTT><<<grid, NTT, lds, stream>>>(                          \
      out, part, xx, ww, N_out, K, ks, half_rows, ri, ro, gw, eps, wscale, GemvAr{});                            \
  else if (mode == 2) gemv_kernel<MM, RR, EE, 2, F8, KK, NTT><<<grid, NTT, lds, stream>>>(                     \
      out, part, xx, ww, N_out, K, ks, half_rows, ri, ro, gw, eps, wscale, GemvAr{});                            \
  else gemv_kernel<MM, RR, EE, 0, F8, KK><<<grid, 256, lds, stream>>>(out, part, xx, ww, N_out, K, ks,          \
                                                                       half_rows, ri, ro, gw, eps, wscale, GemvAr{})
#define G3(MM, RR, EE, F8, KK)                  \
  if constexpr (KK == 2 && MM <= 4) {           \
    G4(MM, RR, EE, F8, KK, 512);                \
  } else {                                      \
    G4(MM, RR, EE, F8, KK, 256);                \
  }
#define G2(MM, RR, EE, F8)                      \
  if (kw == 4) { G3(MM, RR, EE, F8, 4); }        \
  else if (kw == 2) { G3(MM, RR, EE, F8, 2); }   \
  else { G3(MM, RR, EE, F8, 1); }
#define G(MM, RR, EE)        \
  if (fp8) { G2(MM, RR, EE, true); } \
  else { G2(MM, RR, EE, false); }
#define BY_EPI(MM, RR)                  \
  switch (epi) {                        \
    case EPI_BF16: G(MM, RR, EPI_BF16); break;       \
    case EPI_F32: G(MM, RR, EPI_F32); break;         \
    case EPI_SWIGLU: G(MM, RR, EPI_SWIGLU); break;   \
    default: return -2;                 \
  }
  switch (M) {
    case 1: if (rpw == 2) { BY_EPI(1, 2) } else { BY_EPI(1, 1) } break;
    case 2: if (rpw == 2) { BY_EPI(2, 2) } else { BY_EPI(2, 1) } break;
    case 3: if (rpw == 2) { BY_EPI(3, 2) } else { BY_EPI(3, 1) } break;
    case 4: BY_EPI(4, 2) break;
    case 5: BY_EPI(5, 2) break;
    case 6: BY_EPI(6, 2) break;
    case 7: BY_EPI(7, 2) break;
    case 8: BY_EPI(8, 2) break;
  }
#undef BY_EPI
#undef G
#undef G2
#undef G3
  if (splits > 1) {
    const int total = M * N_out;
    const int blocks = (total + 255) / 256;
    switch (epi) {
      case EPI_BF16: gemv_finalize_kernel<EPI_BF16><<<blocks, 256, 0, stream>>>(out, part, M, N_out, splits, half_rows); break;
      case EPI_F32: gemv_finalize_kernel<EPI_F32><<<blocks, 256, 0, stream>>>(out, part, M, N_out, splits, half_rows); break;
      case EPI_SWIGLU: gemv_finalize_kernel<EPI_SWIGLU><<<blocks, 256, 0, stream>>>(out, part, M, N_out, splits, half_rows); break;
    }
  }
  return (int)hipGetLastError();
}

extern "C" int k8s_gemv_norm_w(void* out, void* partial, const void* x, const void* W, const float* wscale, int M,
                               int N_out, int K, int epi, const void* res_in, void* res_out, const void* nw,
                               float eps, hipStream_t stream) {
  return gemv_launch(nw != nullptr ? 1 : 0, out, partial, x, W, wscale, M, N_out, K, epi, res_in, res_out, nw, eps,
                     stream);
}

// Pre-norm projection with the norm weight folded into W: y = epi((W' . (x + res_in)) / rms(x + res_in)).
extern "C" int k8s_gemv_rms(void* out, void* partial, const void* x, const void* W, const float* wscale, int M,
                            int N_out, int K, int epi, const void* res_in, void* res_out, float eps,
                            hipStream_t stream) {
  return gemv_launch(2, out, partial, x, W, wscale, M, N_out, K, epi, res_in, res_out, nullptr, eps, stream);
}

extern "C" int k8s_gemv_norm(void* out, void* partial, const void* x, const void* W, int M, int N_out, int K,
                             int epi, const void* res_in, void* res_out, const void* nw, float eps,
                             hipStream_t stream) {
  return k8s_gemv_norm_w(out, partial, x, W, nullptr, M, N_out, K, epi, res_in, res_out, nw, eps, stream);
}

extern "C" int k8s_gemv(void* out, void* partial, const void* x, const void* W, int M, int N_out, int K, int epi,
                        hipStream_t stream) {
  return k8s_gemv_norm_w(out, partial, x, W, nullptr, M, N_out, K, epi, nullptr, nullptr, nullptr, 0.f, stream);
}

extern "C" int k8s_gemv_fp8(void* out, void* partial, const void* x, const void* W, const float* wscale, int M,
                            int N_out, int K, int epi, const void* res_in, void* res_out, const void* nw, float eps,
                            hipStream_t stream) {
  if (wscale == nullptr) return -1;
  return k8s_gemv_norm_w(out, partial, x, W, wscale, M, N_out, K, epi, res_in, res_out, nw, eps, stream);
}

// Row-parallel projection with the tensor-parallel all-reduce (and the residual add) in its epilogue:
// out[M, N_out] = residual + sum over ranks of x . W^T (see GemvAr).  Every rank must issue the same sequence of
// these calls with the same shapes (the group epochs advance per call).  Two-row waves, one K slice (the whole
// row of x in LDS), 4-wave workgroups.  Returns -5 where the shape does not fit that plan (the caller then runs
// the GEMV and a separate all-reduce).
extern "C" int k8s_gemv_allreduce(void* out, const void* x, const void* W, const float* wscale, int M, int N_out,
                                  int K, const void* residual, void* const* bases, long long row_bytes,
                                  uint32_t* epochs, uint32_t* tickets, uint32_t* err, int rank, int world,
                                  long long timeout_ticks, hipStream_t stream) {
  constexpr int ROWS_WG = 8;  // 4 waves x 2 rows
  if (M < 1 || M > 8 || K % 16 != 0 || N_out <= 0 || world < 2 || world > GAR_MAX_WORLD || rank < 0 || rank >= world)
    return -1;
  if (N_out % ROWS_WG != 0 || (long long)M * K * 2 > 65536 || (long long)M * N_out * 4 > row_bytes) return -5;
  // row-set loop (K8S_GEMV_LOOP_AR = workgroups per CU, 0 = one row set per wave): each workgroup streams a
  // contiguous band of row sets and pushes each set's words as it finishes it
  static const int loop_ar = [] { const char* e = getenv("K8S_GEMV_LOOP_AR"); return e ? atoi(e) : 0; }();
  const int nwg1 = N_out / ROWS_WG;
  const int per = (loop_ar > 0 && M <= 2 && nwg1 > 256 * loop_ar) ? (nwg1 + 256 * loop_ar - 1) / (256 * loop_ar) : 1;
  const int nwg = (nwg1 + per - 1) / per;
  const int group = (nwg + 31) / 32;  // ~32 arrival groups: one waiting workgroup per group
  if ((nwg + group - 1) / group > GAR_MAX_GROUPS) return -5;
  GemvAr a;
  for (int i = 0; i < GAR_MAX_WORLD; ++i) a.base[i] = i < world ? static_cast<char*>(bases[i]) : nullptr;
  a.row_bytes = row_bytes; a.epochs = epochs; a.tickets = tickets; a.err = err;
  a.res = static_cast<const bf16_t*>(residual); a.timeout_ticks = timeout_ticks;
  a.rank = rank; a.world = world; a.group = group;
  const bool fp8 = wscale != nullptr;
  const size_t lds = (size_t)M * K * 2;
  const bf16_t* xx = static_cast<const bf16_t*>(x);
#define GAR1(MM, LP)                                                                                                \
  if (fp8) gemv_kernel<MM, 2, EPI_BF16, 0, true, 1, 256, true, LP><<<nwg, 256, lds, stream>>>(                      \
      out, nullptr, xx, W, N_out, K, K, 0, nullptr, nullptr, nullptr, 0.f, wscale, a);                               \
  else gemv_kernel<MM, 2, EPI_BF16, 0, false, 1, 256, true, LP><<<nwg, 256, lds, stream>>>(                         \
      out, nullptr, xx, W, N_out, K, K, 0, nullptr, nullptr, nullptr, 0.f, wscale, a)
#define GAR(MM)                                   \
  if constexpr (MM <= 2) {                        \
    if (per > 1) { GAR1(MM, true); }              \
    else { GAR1(MM, false); }                     \
  } else {                                        \
    GAR1(MM, false);                              \
  }
  switch (M) {
    case 1: GAR(1); break;
    case 2: GAR(2); break;
    case 3: GAR(3); break;
    case 4: GAR(4); break;
    case 5: GAR(5); break;
    case 6: GAR(6); break;
    case 7: GAR(7); break;
    case 8: GAR(8); break;
  }
#undef GAR
#undef GAR1
  return (int)hipGetLastError();
}

extern "C" int k8s_gemv_allreduce_max_groups() { return GAR_MAX_GROUPS; }
