// K6: causal prefill flash attention over the PAGED KV cache, MFMA bf16 (gfx950).
//
// Reading K/V through the block table (instead of from the chunk's own q/k/v) makes the same
// kernel serve plain prefill, chunked prefill and prefix-cached prompts: query i of sequence s
// sits at absolute position ctx_s - qlen_s + i and attends keys [0, pos].
//
// GQA packing: one workgroup = NW waves = 16 NW (query, head) rows = QT = 16 NW / G consecutive queries x
// the G query heads that share ONE kv head (G = nq / nkv), so every K/V tile is fetched once per
// group instead of once per query head (8x fewer K/V bytes at Llama-3.3-70B's 8:1 GQA), and the
// causal key range of a workgroup ends at its QT-th query instead of its 64th.  Row r of the
// workgroup is query tile * QT + r / G, head kvh * G + r % G.
// NW = 4, 8 or 16 (64 / 128 / 256 rows): every K/V byte a workgroup stages feeds 16 NW rows of MFMA work, so at
// long contexts -- where every workgroup streams the whole causal K/V range through L2 -- wider workgroups cut
// the K/V traffic per FLOP.  The host takes 8 waves when that grid still has >= 256 workgroups (16: opt-in).
//
// Structure:
//  * "swapped" QK^T: S^T = K . Q^T with v_mfma_f32_16x16x32_bf16, so each lane ends up holding
//    16 scores of ONE query row (row = lane & 15): the row max/sum need 2 cross-lane steps and
//    the probabilities feed the P.V MFMA as its A operand straight from registers (the key
//    order inside a 32-key step is permuted identically on the V side, see below).
//  * V tiles (64 keys x 128 d) are staged in LDS with an XOR swizzle and read with the gfx950
//    transposing read ds_read_b64_tr_b16, which delivers 4 keys of one d column per lane --
//    exactly the B-operand layout, so V needs no register transpose.
//  * K and V tiles are fetched one tile AHEAD into registers by all 256 threads (the loads of tile
//    t+1 are in flight during tile t's MFMAs), then stored into swizzled LDS images shared by the
//    4 waves; K fragments are read back with conflict-free ds_read_b128.
//  * online softmax in the log2 domain (scale * log2(e) folded into S).
#include <cstdlib>

#include "common.h"

#define K8S_CHK_THIS_UNIT 5

namespace k8sllm {

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

__device__ __forceinline__ int v_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

template <int D, int G, int NW>
__global__ void __launch_bounds__(64 * NW) paged_prefill_kernel(
    bf16_t* __restrict__ out, const bf16_t* __restrict__ q, const bf16_t* __restrict__ k_cache,
    const bf16_t* __restrict__ v_cache, const int* __restrict__ cu_q, const int* __restrict__ context_lens,
    const int* __restrict__ block_tables, float scale_log2, int nq, int nkv, int block_size, int max_blocks) {
  static_assert(D == 128, "head_dim 128");
  constexpr int KT = 64;             // keys per tile
  constexpr int NT = 64 * NW;        // threads
  constexpr int CPT = KT * D / 8 / NT;  // 16-byte chunks of one tile per thread (K and V each)
  __shared__ __attribute__((aligned(16))) char klds[KT * D * 2];
  __shared__ __attribute__((aligned(16))) char vlds[KT * D * 2];

  constexpr int QT = 16 * NW / G;  // queries per workgroup
  const int s = blockIdx.z, kvh = blockIdx.y, tile = blockIdx.x;
  const int q0 = cu_q[s], qlen = cu_q[s + 1] - q0;
  if (tile * QT >= qlen) return;
  int ctx = context_lens[s];
  K8S_CHECK_MAX(ctx, max_blocks * block_size, K8S_CHK_CTX);
  const int qstart = ctx - qlen;  // absolute position of query 0
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const int* bt = block_tables + (size_t)s * max_blocks;
  const size_t kv_stride = (size_t)nkv * D;

  const int last_row = min(tile * QT + QT - 1, qlen - 1);
  const int kv_end = qstart + last_row + 1;  // keys needed by this workgroup
  const int ntiles = (kv_end + KT - 1) / KT;

  // Tile staging, one tile ahead: thread tid fetches chunks idx = tid + NT c (key row idx/16,
  // 16-byte column chunk idx%16) of K and V into registers while the current tile is computed,
  // then stores them swizzled into LDS.  Keys past the context: K clamped (their scores are
  // masked), V zero (P is 0 there, V must be finite).
  // The block ids of a tile are requested one tile before its K/V (nbt): otherwise every prefetch is two dependent
  // round trips (block id, then K/V) against one tile of math, and long contexts pay that chain once per tile.
  u32x4 kn[CPT], vn[CPT];
  int nbt[CPT];
  auto load_bt = [&](int t) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      nbt[c] = bt[min(t * KT + (tid + NT * c) / (D / 8), ctx - 1) / block_size];
      K8S_CHECK_RANGE(nbt[c], 0, K8S_CHK_BLOCK, 0);
    }
  };
  auto fetch = [&](int t) {   // tile t's K/V with the ids in nbt, then tile t + 1's ids
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int idx = tid + NT * c;
      const int key = t * KT + idx / (D / 8), ch = idx % (D / 8);
      const int kc = min(key, ctx - 1);
      const size_t off = (size_t)(nbt[c] * block_size + kc % block_size) * kv_stride + kvh * D + ch * 8;
      kn[c] = *reinterpret_cast<const u32x4*>(k_cache + off);
      vn[c] = key < ctx ? *reinterpret_cast<const u32x4*>(v_cache + off) : u32x4{0u, 0u, 0u, 0u};
    }
    load_bt(t + 1);   // (keys past the context clamp to the last one: always a valid id)
  };
  load_bt(0);
  fetch(0);

  // my (query, head) row (B operand columns / softmax rows)
  const int wr = wid * 16 + li;
  const int row = tile * QT + wr / G, head = kvh * G + wr % G;
  const int row_c = min(row, qlen - 1);  // clamp padding rows to a valid query
  const int qpos = qstart + row_c;
  bf16x8 qf[D / 32];
  {
    const bf16_t* qp = q + ((size_t)(q0 + row_c) * nq + head) * D;
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(qp + kk * 32 + g * 8);
  }

  f32x4 o[D / 16];
#pragma unroll
  for (int n = 0; n < D / 16; ++n) o[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  for (int t = 0; t < ntiles; ++t) {
    const int kbase = t * KT;
    // ---- tile t: registers -> LDS (both images swizzled: 16-byte chunk ch of row r at ch ^ swz(r))
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const int idx = tid + NT * c;
      const int kr = idx / (D / 8), ch = idx % (D / 8);
      *reinterpret_cast<u32x4*>(klds + kr * (D * 2) + 16 * (ch ^ (kr & 15))) = kn[c];
      *reinterpret_cast<u32x4*>(vlds + kr * (D * 2) + 16 * (ch ^ v_swz(kr))) = vn[c];
    }
    __syncthreads();
    if (t + 1 < ntiles) fetch(t + 1);  // in flight during this tile's math

    // ---- S^T = K . Q^T for 4 key sub-tiles of 16; lane (li, g) reads key row 16m + li, d 32kk + 8g
    f32x4 sacc[KT / 16];
#pragma unroll
    for (int m = 0; m < KT / 16; ++m) {
      const int kr = 16 * m + li;
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) {
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(klds + kr * (D * 2) + 16 * ((4 * kk + g) ^ (kr & 15)));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka, qf[kk], acc, 0, 0, 0);
      }
      sacc[m] = acc;
    }
    // lane holds S[row li][key kbase + 16m + 4g + i]
    float tmax = -INFINITY;
#pragma unroll
    for (int m = 0; m < KT / 16; ++m) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kbase + m * 16 + g * 4 + i;
        float v = sacc[m][i] * scale_log2;
        v = (key <= qpos && key < ctx) ? v : -INFINITY;
        sacc[m][i] = v;
        tmax = fmaxf(tmax, v);
      }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, WAVE));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, WAVE));
    const float m_new = fmaxf(m_run, tmax);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    float rsum = 0.f;
#pragma unroll
    for (int m = 0; m < KT / 16; ++m) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pv = exp2f(sacc[m][i] - m_use);
        sacc[m][i] = pv;
        rsum += pv;
      }
    }
    rsum += __shfl_xor(rsum, 16, WAVE);
    rsum += __shfl_xor(rsum, 32, WAVE);
    l_run = l_run * alpha + rsum;
    m_run = m_new;

    // rescale O rows (row 4g+i of O lives in lanes whose li == 4g+i for the stats)
    float a_i[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) a_i[i] = __shfl(alpha, g * 4 + i, WAVE);
#pragma unroll
    for (int n = 0; n < D / 16; ++n) {
#pragma unroll
      for (int i = 0; i < 4; ++i) o[n][i] *= a_i[i];
    }

    // P as A operand: k-step st covers keys 32st..32st+31 in the permuted order
    // slot j<4 -> key 32st + 4g + j ; slot j>=4 -> key 32st + 16 + 4g + (j-4)
    bf16x8 pa[KT / 32];
#pragma unroll
    for (int st = 0; st < KT / 32; ++st) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[st][j] = (__bf16)sacc[2 * st][j];
        pa[st][4 + j] = (__bf16)sacc[2 * st + 1][j];
      }
    }

    const int qd = li >> 2, pd = li & 3;  // tr-read lane roles: row q, column group p
#pragma unroll
    for (int st = 0; st < KT / 32; ++st) {
      const int r0 = 32 * st + 4 * g + qd;
      const int r1 = r0 + 16;
#pragma unroll
      for (int n = 0; n < D / 16; ++n) {
        const int col = 16 * n + 4 * pd;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const lds_bf16x4* a0 = (const lds_bf16x4*)(vlds + r0 * (D * 2) + 16 * (ch ^ v_swz(r0)) + hb);
        const lds_bf16x4* a1 = (const lds_bf16x4*)(vlds + r1 * (D * 2) + 16 * (ch ^ v_swz(r1)) + hb);
        const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a0);
        const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)a1);
        bf16x8 vb;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vb[j] = v0[j]; vb[4 + j] = v1[j]; }
        o[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[st], vb, o[n], 0, 0, 0);
      }
    }
    __syncthreads();  // before the next tile overwrites the LDS images
  }

  // ---- normalise and store: o[n][i] = O[row 4g+i][d 16n + li]
  float inv_l[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lv = __shfl(l_run, g * 4 + i, WAVE);
    inv_l[i] = lv > 0.f ? 1.f / lv : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int orow = wid * 16 + g * 4 + i;
    const int r = tile * QT + orow / G, oh = kvh * G + orow % G;
    if (r < qlen) {
      bf16_t* op = out + ((size_t)(q0 + r) * nq + oh) * D + li;
#pragma unroll
      for (int n = 0; n < D / 16; ++n) op[16 * n] = f2bf(o[n][i] * inv_l[i]);
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

K8S_CHECK_UNIT(attn_prefill)

extern "C" int k8s_paged_prefill_attention(void* out, const void* q, const void* k_cache, const void* v_cache,
                                           const int* cu_q, const int* context_lens, const int* block_tables,
                                           float scale, int num_seqs, int max_qlen, int nq, int nkv, int D,
                                           int block_size, int max_blocks, hipStream_t stream) {
  if (num_seqs <= 0 || max_qlen <= 0) return 0;
  if (D != 128 || nq % nkv != 0) return -1;
  const int G = nq / nkv;
  const float sl2 = scale * 1.4426950408889634f;
  // 8 waves when that grid still covers every CU, else 4.  The 16-wave form measured no faster than 8 on the 256-node
  // prompts (profiles/bench_r3_nodes256_attn_waves_ab.jsonl) and stays opt-in: K8S_PREFILL_ATTN_WAVES = 4 / 8 / 16.
  static const int waves_env = [] { const char* e = getenv("K8S_PREFILL_ATTN_WAVES"); return e ? atoi(e) : 0; }();
  auto wgs = [&](int nw) { return (long long)((max_qlen + 16 * nw / G - 1) / (16 * nw / G)) * nkv * num_seqs; };
  const int nw = (waves_env == 4 || waves_env == 8 || waves_env == 16) ? waves_env : wgs(8) >= 256 ? 8 : 4;
#define PF(GG, NWW)                                                                                          \
  {                                                                                                          \
    constexpr int QT = 16 * NWW / GG;                                                                        \
    dim3 grid((max_qlen + QT - 1) / QT, nkv, num_seqs);                                                      \
    paged_prefill_kernel<128, GG, NWW><<<grid, 64 * NWW, 0, stream>>>(                                       \
        (bf16_t*)out, (const bf16_t*)q, (const bf16_t*)k_cache, (const bf16_t*)v_cache, cu_q, context_lens,  \
        block_tables, sl2, nq, nkv, block_size, max_blocks);                                                 \
  }
#define PFW(GG) \
  if (nw == 16) PF(GG, 16) else if (nw == 8) PF(GG, 8) else PF(GG, 4)
  switch (G) {  // query heads per kv head (Llama-3.3-70B: 8; Llama-3-8B: 4)
    case 1: PFW(1) break;
    case 2: PFW(2) break;
    case 4: PFW(4) break;
    case 8: PFW(8) break;
    case 16: PFW(16) break;
    default: return -1;
  }
#undef PFW
#undef PF
  return (int)hipGetLastError();
}
