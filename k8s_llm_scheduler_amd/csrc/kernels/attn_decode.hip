// K7: paged GQA decode attention with split-KV (flash-decoding), SURVEY.md 2.5.
// One query token per sequence; the G = nq/nkv query heads of a KV head are processed by one
// workgroup so each K/V row is read from HBM once for the whole group.  The context is cut
// into partitions of PART tokens (grid.x); each workgroup writes an un-normalised partial
// output plus its (max, sum) and a second kernel merges the partitions.  When the grid has a
// single partition the first kernel writes the final bf16 output directly.
//
// Layouts: q [B, nq, D] bf16; k/v cache [num_slots, nkv, D] bf16 with
// slot = block_tables[b][i / block_size] * block_size + i % block_size; context_lens[b] counts
// the tokens to attend to (the current token's K/V is already in the cache).
#include "common.h"

#define K8S_CHK_THIS_UNIT 6

namespace k8sllm {

constexpr float LOG2E = 1.4426950408889634f;

template <int D, int G, int PART>
__global__ void __launch_bounds__(256) paged_decode_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_acc, float* __restrict__ part_ml,
    const bf16_t* __restrict__ q, const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ context_lens, float scale, int block_size,
    int max_blocks, int nkv, int pmax) {
  constexpr int LPT = D / 8;          // lanes per key row (16 B each)
  constexpr int TPW = WAVE / LPT;     // tokens per wave per step
  constexpr int NW = 4;               // waves per workgroup
  constexpr int TPH = 256 / G;        // threads per head in the softmax pass
  __shared__ float qs[G][D];
  __shared__ float sc[G][PART];
  __shared__ float red[NW][G][D];
  __shared__ float stat[G][2];
  __shared__ float tmp[16][G];

  const int b = blockIdx.z, kvh = blockIdx.y, p = blockIdx.x;
  int ctx = context_lens[b];
  K8S_CHECK_MAX(ctx, max_blocks * block_size, K8S_CHK_CTX);
  const int start = p * PART;
  if (start >= ctx) return;
  const int n = min(PART, ctx - start);
  const int nq = nkv * G;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const float qscale = scale * LOG2E;

  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i - g * D;
    qs[g][d] = bf2f(q[((size_t)b * nq + kvh * G + g) * D + d]) * qscale;
  }
  __syncthreads();

  const int* bt = block_tables + (size_t)b * max_blocks;
  // ---- scores = q . k (log2 domain).  Wave w owns tokens [w*PART/NW, (w+1)*PART/NW); every
  // K row load of the wave is issued before the first one is consumed (memory-level parallelism
  // instead of a latency chain).
  constexpr int TOK_W = PART / NW;          // tokens per wave
  constexpr int QSTEPS = TOK_W / TPW;       // 16-lane groups per wave, TPW tokens per step
  const int sub = lane % LPT, tok_in_wave = lane / LPT;
  {
    u32x4 kreg[QSTEPS];
#pragma unroll
    for (int st = 0; st < QSTEPS; ++st) {
      const int i = wid * TOK_W + st * TPW + tok_in_wave;
      const int tt = start + min(i, n - 1);
      int blk = bt[tt / block_size];
      K8S_CHECK_RANGE(blk, 0, K8S_CHK_BLOCK, 0);
      const int slot = blk * block_size + tt % block_size;
      kreg[st] = *reinterpret_cast<const u32x4*>(k_cache + ((size_t)slot * nkv + kvh) * D + sub * 8);
    }
#pragma unroll
    for (int st = 0; st < QSTEPS; ++st) {
      const int i = wid * TOK_W + st * TPW + tok_in_wave;
      float kf[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) { kf[2 * j] = lo_bf(kreg[st][j]); kf[2 * j + 1] = hi_bf(kreg[st][j]); }
      float part[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float acc = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += qs[g][sub * 8 + j] * kf[j];
        part[g] = acc;
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
#pragma unroll
        for (int o = LPT / 2; o > 0; o >>= 1) part[g] += __shfl_xor(part[g], o, WAVE);
      }
      if (sub == 0 && i < n) {
#pragma unroll
        for (int g = 0; g < G; ++g) sc[g][i] = part[g];
      }
    }
  }
  __syncthreads();

  // ---- softmax statistics per head (TPH threads per head)
  {
    const int g = tid / TPH, r = tid % TPH;
    float m = -INFINITY;
    for (int i = r; i < n; i += TPH) m = fmaxf(m, sc[g][i]);
    constexpr int SEG = TPH < 64 ? TPH : 64;
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, WAVE));
    if (TPH > 64) {
      if (lane == 0) tmp[wid][0] = m;  // one head spans TPH/64 waves; G <= 2 here
      __syncthreads();
      m = -INFINITY;
      for (int w = g * (TPH / 64); w < (g + 1) * (TPH / 64); ++w) m = fmaxf(m, tmp[w][0]);
      __syncthreads();
    }
    float l = 0.f;
    for (int i = r; i < n; i += TPH) {
      const float e = exp2f(sc[g][i] - m);
      sc[g][i] = e;
      l += e;
    }
#pragma unroll
    for (int o = SEG / 2; o > 0; o >>= 1) l += __shfl_xor(l, o, WAVE);
    if (TPH > 64) {
      if (lane == 0) tmp[wid][1] = l;
      __syncthreads();
      l = 0.f;
      for (int w = g * (TPH / 64); w < (g + 1) * (TPH / 64); ++w) l += tmp[w][1];
    }
    if (r == 0) { stat[g][0] = m; stat[g][1] = l; }
  }
  __syncthreads();

  // ---- acc = p . v : wave w takes its TOK_W tokens, all V row loads issued up front;
  // lane owns dims (2*lane, 2*lane+1)
  float acc[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g][0] = acc[g][1] = 0.f;
  const int d0 = lane * 2;
  if (d0 < D) {
    uint32_t vreg[TOK_W];
#pragma unroll
    for (int k = 0; k < TOK_W; ++k) {
      const int i = wid * TOK_W + k;
      const int tt = start + min(i, n - 1);
      int blk = bt[tt / block_size];
      K8S_CHECK_RANGE(blk, 0, K8S_CHK_BLOCK, 0);
      const int slot = blk * block_size + tt % block_size;
      vreg[k] = *reinterpret_cast<const uint32_t*>(v_cache + ((size_t)slot * nkv + kvh) * D + d0);
    }
#pragma unroll
    for (int k = 0; k < TOK_W; ++k) {
      const int i = wid * TOK_W + k;
      if (i < n) {
        const float v0 = lo_bf(vreg[k]), v1 = hi_bf(vreg[k]);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float pg = sc[g][i];
          acc[g][0] += pg * v0;
          acc[g][1] += pg * v1;
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) { red[wid][g][d0] = acc[g][0]; red[wid][g][d0 + 1] = acc[g][1]; }
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += 256) {
    const int g = i / D, d = i - g * D;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) s += red[w][g][d];
    const int h = kvh * G + g;
    if (pmax == 1) {
      out[((size_t)b * nq + h) * D + d] = f2bf(s / stat[g][1]);
    } else {
      const size_t pi = ((size_t)b * nq + h) * pmax + p;
      part_acc[pi * D + d] = s;
      if (d == 0) { part_ml[pi * 2] = stat[g][0]; part_ml[pi * 2 + 1] = stat[g][1]; }
    }
  }
}

// Merge partitions: one workgroup per (head, batch row), D threads.
template <int D>
__global__ void __launch_bounds__(D) paged_decode_reduce_kernel(bf16_t* __restrict__ out,
                                                               const float* __restrict__ part_acc,
                                                               const float* __restrict__ part_ml,
                                                               const int* __restrict__ context_lens, int part,
                                                               int pmax, int nq) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int ctx = context_lens[b];
  if (ctx <= 0) return;
  const int np = min(pmax, (ctx + part - 1) / part);
  const size_t base = ((size_t)b * nq + h) * pmax;
  float M = -INFINITY;
  for (int p = 0; p < np; ++p) M = fmaxf(M, part_ml[(base + p) * 2]);
  float num = 0.f, den = 0.f;
  for (int p = 0; p < np; ++p) {
    const float w = exp2f(part_ml[(base + p) * 2] - M);
    num += w * part_acc[(base + p) * D + d];
    den += w * part_ml[(base + p) * 2 + 1];
  }
  out[((size_t)b * nq + h) * D + d] = f2bf(num / den);
}

}  // namespace k8sllm

using namespace k8sllm;

K8S_CHECK_UNIT(attn_decode)

// workspace: part_acc [B, nq, pmax, D] fp32 and part_ml [B, nq, pmax, 2] fp32 (unused if pmax == 1)
extern "C" int k8s_paged_decode_attention(void* out, void* part_acc, void* part_ml, const void* q, const void* k_cache,
                                          const void* v_cache, const int* block_tables, const int* context_lens,
                                          float scale, int B, int nq, int nkv, int D, int block_size, int max_blocks,
                                          int part, int pmax, hipStream_t stream) {
  if (B <= 0) return 0;
  if (D != 128 || nq % nkv != 0 || part != 64) return -1;
  const int G = nq / nkv;
  dim3 grid(pmax, nkv, B);
#define L(GG)                                                                                             \
  paged_decode_kernel<128, GG, 64><<<grid, 256, 0, stream>>>(                                            \
      (bf16_t*)out, (float*)part_acc, (float*)part_ml, (const bf16_t*)q, (const bf16_t*)k_cache,           \
      (const bf16_t*)v_cache, block_tables, context_lens, scale, block_size, max_blocks, nkv, pmax)
  switch (G) {
    case 1: L(1); break;
    case 2: L(2); break;
    case 4: L(4); break;
    case 8: L(8); break;
    case 16: L(16); break;
    default: return -2;
  }
#undef L
  if (pmax > 1) {
    paged_decode_reduce_kernel<128><<<dim3(nq, B), 128, 0, stream>>>((bf16_t*)out, (const float*)part_acc,
                                                                     (const float*)part_ml, context_lens, part, pmax,
                                                                     nq);
  }
  return (int)hipGetLastError();
}
