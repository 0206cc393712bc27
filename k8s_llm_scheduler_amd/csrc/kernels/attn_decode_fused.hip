// K4 + K5 + K7 fused for decode: RoPE of the new token's q/k, its paged-KV write, and GQA
// attention over the paged cache, in ONE kernel that reads the QKV projection output directly.
//
// Why: at TP=8 a decode layer is ~70 us of which the small kernels (rope, attention merge) are
// ~4.5 us each of mostly launch gap and dependent-load latency.  Here:
//  * one workgroup (8 waves) covers PART = 1024 context tokens of one (sequence, kv head), so
//    any context up to 1024 tokens (the reference's 3-node prompts are ~0.5k) is a single pass
//    that writes the final output -- no merge kernel work;
//  * longer contexts split into partitions and the merge kernel combines them (it exits at once
//    when the context fits one partition, so a captured graph serves every length);
//  * the workgroup owning the new token's position rotates k, writes k/v into the cache and uses
//    the rotated values from LDS for its own scores (no cross-workgroup ordering needed);
//  * every K row load of a wave is issued before the first is consumed, V loads likewise.
//
// Layouts: qkv [B, (nq + 2*nkv) * D] bf16 (pre-RoPE); cos_sin [max_pos, D] f32 (cos | sin);
// caches [num_slots, nkv, D] bf16; context_lens[b] INCLUDES the new token (pos = ctx - 1).
#include "common.h"

namespace k8sllm {

constexpr float LOG2E_F = 1.4426950408889634f;

template <int D, int G, int PART>
__global__ void __launch_bounds__(512) decode_fused_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_acc, float* __restrict__ part_ml, const bf16_t* __restrict__ qkv,
    const float* __restrict__ cos_sin, bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ context_lens, float scale, int block_size,
    int max_blocks, int nkv, int pmax) {
  constexpr int NW = 8;
  constexpr int NT = NW * WAVE;
  constexpr int LPT = D / 8;        // lanes per K row (16 B each)
  constexpr int TPW = WAVE / LPT;   // K rows per wave per step
  constexpr int TOK_W = PART / NW;  // tokens per wave
  constexpr int KB = 8;             // K loads in flight per lane
  constexpr int VB = 32;            // V loads in flight per lane
  constexpr int HALF = D / 2;
  __shared__ float qs[G][D];
  __shared__ float sc[G][PART];
  __shared__ float red[G][D];
  __shared__ float kcur[D], vcur[D];
  __shared__ float wm[NW][G], wl[NW][G];
  __shared__ float stat[G][2];

  const int b = blockIdx.z, kvh = blockIdx.y, p = blockIdx.x;
  const int ctx = context_lens[b];
  const int start = p * PART;
  if (ctx <= 0 || start >= ctx) return;
  const int n = min(PART, ctx - start);
  const int pos = ctx - 1;
  const bool owner = pos < start + n;  // this partition holds the new token
  const int nq = nkv * G;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const bf16_t* row = qkv + (size_t)b * (nq + 2 * nkv) * D;
  const float* cs = cos_sin + (size_t)pos * D;
  const int* bt = block_tables + (size_t)b * max_blocks;
  const float qscale = scale * LOG2E_F;

  // ---- rotate q (and k / copy v when owner); rotate-half pairs (i, i + D/2)
  for (int i = tid; i < (G + 2) * HALF; i += NT) {
    const int h = i / HALF, d = i - h * HALF;
    if (h < G) {
      const bf16_t* x = row + (size_t)(kvh * G + h) * D;
      const float x1 = bf2f(x[d]), x2 = bf2f(x[d + HALF]);
      const float c = cs[d], s = cs[d + HALF];
      // round to bf16 like the unfused path (q is stored as bf16 there)
      qs[h][d] = bf2f(f2bf(x1 * c - x2 * s)) * qscale;
      qs[h][d + HALF] = bf2f(f2bf(x2 * c + x1 * s)) * qscale;
    } else if (owner) {
      if (h == G) {
        const bf16_t* x = row + (size_t)(nq + kvh) * D;
        const float x1 = bf2f(x[d]), x2 = bf2f(x[d + HALF]);
        const float c = cs[d], s = cs[d + HALF];
        const bf16_t k1 = f2bf(x1 * c - x2 * s), k2 = f2bf(x2 * c + x1 * s);
        kcur[d] = bf2f(k1);
        kcur[d + HALF] = bf2f(k2);
        const int slot = bt[pos / block_size] * block_size + pos % block_size;
        bf16_t* kd = k_cache + ((size_t)slot * nkv + kvh) * D;
        kd[d] = k1;
        kd[d + HALF] = k2;
      } else {
        const bf16_t* x = row + (size_t)(nq + nkv + kvh) * D;
        const bf16_t v1 = x[d], v2 = x[d + HALF];
        vcur[d] = bf2f(v1);
        vcur[d + HALF] = bf2f(v2);
        const int slot = bt[pos / block_size] * block_size + pos % block_size;
        bf16_t* vd = v_cache + ((size_t)slot * nkv + kvh) * D;
        vd[d] = v1;
        vd[d + HALF] = v2;
      }
    }
  }
  for (int i = tid; i < G * D; i += NT) (&red[0][0])[i] = 0.f;
  __syncthreads();

  // ---- scores (log2 domain): wave w owns tokens [w*TOK_W, (w+1)*TOK_W) of the partition
  const int sub = lane % LPT, tiw = lane / LPT;
  const int wbase = wid * TOK_W;
  const int wn = max(0, min(TOK_W, n - wbase));  // valid tokens of this wave
  for (int s0 = 0; s0 < wn; s0 += KB * TPW) {
    u32x4 kreg[KB];
#pragma unroll
    for (int st = 0; st < KB; ++st) {
      const int i = wbase + s0 + st * TPW + tiw;
      const int tt = start + min(i, n - 1);
      const int slot = bt[tt / block_size] * block_size + tt % block_size;
      kreg[st] = *reinterpret_cast<const u32x4*>(k_cache + ((size_t)slot * nkv + kvh) * D + sub * 8);
    }
#pragma unroll
    for (int st = 0; st < KB; ++st) {
      const int i = wbase + s0 + st * TPW + tiw;
      float kf[8];
      if (start + i == pos) {
#pragma unroll
        for (int j = 0; j < 8; ++j) kf[j] = kcur[sub * 8 + j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) { kf[2 * j] = lo_bf(kreg[st][j]); kf[2 * j + 1] = hi_bf(kreg[st][j]); }
      }
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
      if (sub == 0 && i < wbase + wn) {
#pragma unroll
        for (int g = 0; g < G; ++g) sc[g][i] = part[g];
      }
    }
  }
  __syncthreads();

  // ---- per-wave softmax over the wave's own slice (no barrier): local max m_w and sum l_w per
  // head; p = exp2(s - m_w) stays in sc.  The waves are combined once, below.
  float mloc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float m = -INFINITY;
    for (int i = lane; i < wn; i += WAVE) m = fmaxf(m, sc[g][wbase + i]);
    m = wave_max(m);
    const float mu = (m == -INFINITY) ? 0.f : m;
    float l = 0.f;
    for (int i = lane; i < wn; i += WAVE) {
      const float e = exp2f(sc[g][wbase + i] - mu);
      sc[g][wbase + i] = e;
      l += e;
    }
    l = wave_sum(l);
    mloc[g] = m;
    if (lane == 0) { wm[wid][g] = m; wl[wid][g] = l; }
  }

  // ---- p . v : lane owns dims (2*lane, 2*lane+1); V row loads in batches of VB per lane
  float acc[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g][0] = acc[g][1] = 0.f;
  const int d0 = 2 * lane;
  if (d0 < D && wn > 0) {
    for (int k0 = 0; k0 < wn; k0 += VB) {
      uint32_t vreg[VB];
#pragma unroll
      for (int k = 0; k < VB; ++k) {
        const int tt = start + wbase + min(k0 + k, wn - 1);
        const int slot = bt[tt / block_size] * block_size + tt % block_size;
        vreg[k] = *reinterpret_cast<const uint32_t*>(v_cache + ((size_t)slot * nkv + kvh) * D + d0);
      }
#pragma unroll
      for (int k = 0; k < VB; ++k) {
        const int i = wbase + k0 + k;
        if (k0 + k < wn) {
          float v0, v1;
          if (start + i == pos) { v0 = vcur[d0]; v1 = vcur[d0 + 1]; }
          else { v0 = lo_bf(vreg[k]); v1 = hi_bf(vreg[k]); }
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const float pg = sc[g][i];
            acc[g][0] += pg * v0;
            acc[g][1] += pg * v1;
          }
        }
      }
    }
  }
  __syncthreads();  // wm / wl of every wave visible
  if (tid < G) {
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w][tid]);
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w)
      if (wm[w][tid] != -INFINITY) L += wl[w][tid] * exp2f(wm[w][tid] - M);
    stat[tid][0] = M;
    stat[tid][1] = L;
  }
  if (d0 < D && wn > 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float M = -INFINITY;
#pragma unroll
      for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w][g]);
      const float f = exp2f(mloc[g] - M);
      atomicAdd(&red[g][d0], acc[g][0] * f);
      atomicAdd(&red[g][d0 + 1], acc[g][1] * f);
    }
  }
  __syncthreads();
  const bool single = ctx <= PART;
  for (int i = tid; i < G * D; i += NT) {
    const int g = i / D, d = i - g * D;
    const int h = kvh * G + g;
    const float s = red[g][d];
    if (single) {
      out[((size_t)b * nq + h) * D + d] = f2bf(s / stat[g][1]);
    } else {
      const size_t pi = ((size_t)b * nq + h) * pmax + p;
      part_acc[pi * D + d] = s;
      if (d == 0) { part_ml[pi * 2] = stat[g][0]; part_ml[pi * 2 + 1] = stat[g][1]; }
    }
  }
}

template <int D>
__global__ void __launch_bounds__(D) decode_merge_kernel(bf16_t* __restrict__ out, const float* __restrict__ part_acc,
                                                         const float* __restrict__ part_ml,
                                                         const int* __restrict__ context_lens, int part, int pmax,
                                                         int nq) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int ctx = context_lens[b];
  if (ctx <= part) return;  // single-partition rows were finished by the attention kernel
  const int np = min(pmax, (ctx + part - 1) / part);
  const size_t base = ((size_t)b * nq + h) * pmax;
  float M = -INFINITY;
  for (int q = 0; q < np; ++q) M = fmaxf(M, part_ml[(base + q) * 2]);
  float num = 0.f, den = 0.f;
  for (int q = 0; q < np; ++q) {
    const float w = exp2f(part_ml[(base + q) * 2] - M);
    num += w * part_acc[(base + q) * D + d];
    den += w * part_ml[(base + q) * 2 + 1];
  }
  out[((size_t)b * nq + h) * D + d] = f2bf(num / den);
}

}  // namespace k8sllm

using namespace k8sllm;

// part_acc [B, nq, pmax, D] f32 / part_ml [B, nq, pmax, 2] f32 (needed when pmax > 1)
extern "C" int k8s_decode_attention_fused(void* out, void* part_acc, void* part_ml, const void* qkv,
                                          const float* cos_sin, void* k_cache, void* v_cache, const int* block_tables,
                                          const int* context_lens, float scale, int B, int nq, int nkv, int D,
                                          int block_size, int max_blocks, int pmax, hipStream_t stream) {
  if (B <= 0) return 0;
  if (D != 128 || nq % nkv != 0) return -1;
  if (pmax > 1 && (part_acc == nullptr || part_ml == nullptr)) return -3;
  const int G = nq / nkv;
  dim3 grid(pmax, nkv, B);
#define L(GG)                                                                                               \
  decode_fused_kernel<128, GG, 1024><<<grid, 512, 0, stream>>>(                                             \
      (bf16_t*)out, (float*)part_acc, (float*)part_ml, (const bf16_t*)qkv, cos_sin, (bf16_t*)k_cache,       \
      (bf16_t*)v_cache, block_tables, context_lens, scale, block_size, max_blocks, nkv, pmax)
  switch (G) {
    case 1: L(1); break;
    case 2: L(2); break;
    case 4: L(4); break;
    case 8: L(8); break;
    default: return -2;
  }
#undef L
  if (pmax > 1)
    decode_merge_kernel<128><<<dim3(nq, B), 128, 0, stream>>>((bf16_t*)out, (const float*)part_acc,
                                                              (const float*)part_ml, context_lens, 1024, pmax, nq);
  return (int)hipGetLastError();
}
