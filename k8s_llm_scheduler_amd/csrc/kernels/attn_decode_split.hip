// K4 + K5 + K7 fused for decode, SMALL-GRID variant: RoPE of the new token's q/k, its paged-KV
// write and GQA attention, for the shapes where only a handful of (sequence, kv head) pairs exist
// (TP = 8 at batch 1: ONE kv head per rank, so the one-workgroup-per-pair kernel of
// attn_decode_fused.hip runs on a single CU and its serial chain is the whole cost).
//
// Here the context is cut into 64-token chunks and every chunk is its own ONE-WAVE workgroup:
//  * the chunk's 4 cache blocks are read from the block table together with the context length,
//    then all K (4 tiles x 16 rows x 256 B) and V (64 rows) loads of the wave are issued at once,
//    straight into registers (one HBM round trip for the whole chunk);
//  * S^T = K . Q^T with v_mfma_f32_16x16x32_bf16 (16 context tokens x 16 query heads of the GQA
//    group, heads >= G zero-padded), softmax statistics by two cross-lane steps, P.V with P in
//    registers as the A operand and V staged through LDS and read with ds_read_b64_tr_b16;
//  * single-chunk contexts (<= 64 tokens) write the final output; otherwise each chunk stores its
//    un-normalised partial (acc, max, sum) with sc1 stores, counts its arrival with one agent-scope
//    atomic, and the chunk whose add comes last merges all partials (sc1 loads) and re-arms the
//    counter -- no second kernel, no grid barrier (MI355X_MICROARCH.md visibility table, row 1);
//  * the chunk holding the new token's position rotates its k, writes k/v to the cache and uses
//    the fresh values itself (the cache write need not be visible to anyone in this launch).
//
// Layouts as in attn_decode_fused.hip: qkv [B, (nq + 2*nkv) * D] bf16 (pre-RoPE); cos_sin
// [max_pos, D] f32 (cos | sin); caches [num_slots, nkv, D] bf16 with 16-token blocks;
// context_lens[b] INCLUDES the new token (pos = ctx - 1).
// At most 64 chunks (contexts up to 4096 tokens; longer ones use attn_decode_fused.hip).
// Workspace: part [B, nkv, pmax, G*D + 2*G] f32; counters [B * nkv] u32, zero before the first
// launch and restored to zero by every launch.
#include "common.h"

#define K8S_CHK_THIS_UNIT 4

namespace k8sllm {

namespace {

constexpr float SPLIT_LOG2E = 1.4426950408889634f;
constexpr int SPLIT_CH = 64;  // context tokens per workgroup (one wave)
constexpr int SC1 = 16;       // buffer-op cache policy: sc1 (L1 bypass, coherent at the L2)
#ifndef SPLIT_QB_LANES
#define SPLIT_QB_LANES 36       // merge: chunk accumulators per round trip x loads per chunk (G = 8: 9 chunks, the
                                // bench's 465-528-token contexts in one round trip; 208 VGPRs, 2 waves / SIMD kept)
#endif
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_split_t;

// Timeline probe (tools/attn_trace.py builds this file with -DK8S_ATTN_TRACE into its own library):
// lane 0 of every workgroup stamps s_memrealtime (100 MHz) at 10 points, after draining its memory
// traffic, into g_attn_trace[workgroup][12].  Compiled out of the production kernel.
#ifdef K8S_ATTN_TRACE
__device__ unsigned long long* g_attn_trace;
#define TR(i)                                                                                  \
  do {                                                                                         \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                \
    if (threadIdx.x == 0)                                                                      \
      g_attn_trace[((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 12 + (i)] = \
          __builtin_amdgcn_s_memrealtime();                                                    \
  } while (0)
#else
#define TR(i) \
  do {        \
  } while (0)
#endif

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t split_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

}  // namespace

// The split-attention work of workgroup (chunk c, kv head kvh, sequence b).
template <int G>
__device__ __forceinline__ void split_body(
    bf16_t* __restrict__ out, float* __restrict__ part, uint32_t* __restrict__ counters,
    const bf16_t* __restrict__ qkv, const float* __restrict__ cos_sin, bf16_t* __restrict__ k_cache,
    bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    float scale, int max_blocks, int nkv, int pmax, int c, int kvh, int b) {
  constexpr int D = 128, HALF = D / 2, CH = SPLIT_CH;
  constexpr int PSTRIDE = G * D + 2 * G;  // floats per (b, kvh, chunk) partial record
  static_assert(G >= 1 && G <= 16, "GQA group of 1..16 heads");
  __shared__ __attribute__((aligned(16))) bf16_t qs[16][D];         // rotated q, zero heads >= G
  __shared__ __attribute__((aligned(16))) char vbuf[2][32 * D * 2];  // V of the two 32-key steps
  __shared__ __attribute__((aligned(16))) bf16_t kcur[D];
  __shared__ __attribute__((aligned(16))) bf16_t vcur[D];

  const int lane = threadIdx.x, li = lane & 15, g4 = lane >> 4;
  const int* bt = block_tables + (size_t)b * max_blocks;
  const size_t kvs = (size_t)nkv * D;
  const int start = c * CH;
  TR(0);

  // context length, the chunk's 4 block ids and the new token's q/k/v (lane p: dims p and p + 64
  // of every q head, of k and of v) are independent loads: one round trip
  // (vector buffer loads, the five values through one opaque statement: otherwise the compiler waits for a scalar
  // load of the length, and branches, before it requests the block ids -- two round trips instead of one)
  int ctx_v = (int)__builtin_amdgcn_raw_buffer_load_b32(split_rsrc(context_lens), b * 4, 0, 0);
  int tblk[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    tblk[t] = (int)__builtin_amdgcn_raw_buffer_load_b32(split_rsrc(bt), min(start / 16 + t, max_blocks - 1) * 4, 0, 0);
  asm volatile("" : "+v"(ctx_v), "+v"(tblk[0]), "+v"(tblk[1]), "+v"(tblk[2]), "+v"(tblk[3]));
  int ctx = __builtin_amdgcn_readfirstlane(ctx_v);
  const int nq = nkv * G;
  const bf16_t* row = qkv + (size_t)b * (nq + 2 * nkv) * D;
  bf16_t xa[G], xb[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    xa[h] = row[(size_t)(kvh * G + h) * D + lane];
    xb[h] = row[(size_t)(kvh * G + h) * D + HALF + lane];
  }
  const bf16_t ka = row[(size_t)(nq + kvh) * D + lane], kb = row[(size_t)(nq + kvh) * D + HALF + lane];
  const bf16_t va = row[(size_t)(nq + nkv + kvh) * D + lane], vb2 = row[(size_t)(nq + nkv + kvh) * D + HALF + lane];
  if (ctx <= 0 || start >= ctx) return;
  K8S_CHECK_MAX(ctx, max_blocks * 16, K8S_CHK_CTX);
#pragma unroll
  for (int t = 0; t < 4; ++t) K8S_CHECK_RANGE(tblk[t], 0, K8S_CHK_BLOCK, 0);
  TR(1);

  // ---- every K and V load of the chunk, issued before anything is consumed
  bf16x8 kf[4][D / 32];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16_t* kp = k_cache + (size_t)(tblk[t] * 16 + li) * kvs + (size_t)kvh * D + g4 * 8;
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) kf[t][kk] = *reinterpret_cast<const bf16x8*>(kp + kk * 32);
  }
  // V goes straight into LDS (LDS-DMA, no VGPRs): instruction q fills vbuf bytes [1 KiB q, 1 KiB (q+1)) =
  // rows 4q..4q+3 of the chunk; lane L lands at row 4q + L/16, 16-byte position L%16, which in the
  // swizzled image holds column chunk (L%16) ^ swz(row % 32) -- so that is the chunk it fetches.  Rows past
  // the context re-read the last valid row: their P is exactly 0, the bytes only have to be finite.
  const int n = min(CH, ctx - start);
  {
    const int lt = (n - 1) >> 4;
    const int last_row = (lt == 0 ? tblk[0] : lt == 1 ? tblk[1] : lt == 2 ? tblk[2] : tblk[3]) * 16 + ((n - 1) & 15);
    char* vflat = &vbuf[0][0];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = 4 * q + g4;
      const int srow = r < n ? tblk[q >> 2] * 16 + (r & 15) : last_row;
      const bf16_t* src = v_cache + (size_t)srow * kvs + (size_t)kvh * D + (li ^ swz(r & 31)) * 8;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(vflat + 1024 * q), 16, 0, 0);
    }
  }
  const int pos = ctx - 1;
  const bool owner = pos < start + n;  // the chunk that holds the new token
  const float* cs = cos_sin + (size_t)pos * D;

  // ---- RoPE: lane p rotates dims (p, p + 64) of every q head (and of the new k in the owner
  // chunk); the cos/sin row is the only load of this phase
  {
    const int p = lane;
    const float cp = cs[p], sp = cs[HALF + p];
    int pblk = owner ? bt[pos / 16] : 0;
    K8S_CHECK_RANGE(pblk, 0, K8S_CHK_BLOCK, 0);
    const int pslot = pblk * 16 + pos % 16;
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      bf16_t lo = 0, hi = 0;
      if (h < G) {
        const float a = bf2f(xa[h]), c2 = bf2f(xb[h]);
        lo = f2bf(a * cp - c2 * sp);
        hi = f2bf(c2 * cp + a * sp);
      }
      qs[h][p] = lo;
      qs[h][HALF + p] = hi;
    }
    if (owner) {
      const float a = bf2f(ka), c2 = bf2f(kb);
      const bf16_t klo = f2bf(a * cp - c2 * sp), khi = f2bf(c2 * cp + a * sp);
      bf16_t* kd = k_cache + (size_t)pslot * kvs + (size_t)kvh * D;
      bf16_t* vd = v_cache + (size_t)pslot * kvs + (size_t)kvh * D;
      kd[p] = klo;
      kd[HALF + p] = khi;
      vd[p] = va;
      vd[HALF + p] = vb2;
      kcur[p] = klo;
      kcur[HALF + p] = khi;
      vcur[p] = va;
      vcur[HALF + p] = vb2;
    }
  }
  __syncthreads();  // one wave: orders the LDS writes above before the reads below
  TR(2);

  // Q^T fragments (B operand): lane holds Q[head li][d = 32kk + 8*g4 + j]
  bf16x8 qf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(&qs[li][kk * 32 + g4 * 8]);

  // ---- S^T = K . Q^T; lane holds S[token 16t + 4*g4 + i][head li]
  const float qscale = scale * SPLIT_LOG2E;
  f32x4 sacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (start + 16 * t + li == pos) {  // the fresh key
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) kf[t][kk] = *reinterpret_cast<const bf16x8*>(&kcur[kk * 32 + g4 * 8]);
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][kk], qf[kk], acc, 0, 0, 0);
    sacc[t] = acc;
  }
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = (16 * t + 4 * g4 + i) < n ? sacc[t][i] * qscale : -INFINITY;
      sacc[t][i] = v;
      m = fmaxf(m, v);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16, WAVE));
  m = fmaxf(m, __shfl_xor(m, 32, WAVE));  // max of head li over the chunk (n >= 1: finite)
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e = exp2f(sacc[t][i] - m);
      sacc[t][i] = e;
      l += e;
    }
  }
  l += __shfl_xor(l, 16, WAVE);
  l += __shfl_xor(l, 32, WAVE);
  TR(3);

  // ---- O = P . V over two 32-key steps.  The V image has landed (the K wait above drained the
  // DMA too); the owner chunk replaces the new token's row, which the cache did not hold yet.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (owner) {   // the new token's row and the padding rows after it, which re-read its stale cache slot
    const int rp = pos - start;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = 4 * q + g4;
      if (r >= rp)
        *reinterpret_cast<u32x4*>(vbuf[r >> 5] + (r & 31) * (D * 2) + 16 * (li ^ swz(r & 31))) =
            *reinterpret_cast<const u32x4*>(&vcur[li * 8]);
    }
  }
  __syncthreads();
  f32x4 o[D / 16];
#pragma unroll
  for (int nn = 0; nn < D / 16; ++nn) o[nn] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qd = li >> 2, pd = li & 3;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    if (32 * st < n) {
      const char* vb = vbuf[st];
      // A operand: P with the key order (4*g4 + j | 16 + 4*g4 + j) of the 32-key step
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = (__bf16)sacc[2 * st][j];
        pa[4 + j] = (__bf16)sacc[2 * st + 1][j];
      }
      const int r0 = 4 * g4 + qd, r1 = r0 + 16;
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) {
        const int col = 16 * nn + 4 * pd;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_split_t*)(vb + r0 * (D * 2) + 16 * (ch ^ swz(r0)) + hb));
        const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_split_t*)(vb + r1 * (D * 2) + 16 * (ch ^ swz(r1)) + hb));
        bf16x8 vbf;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vbf[j] = v0[j]; vbf[4 + j] = v1[j]; }
        o[nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vbf, o[nn], 0, 0, 0);
      }
    }
  }
  // o[nn][i] = O[head 4*g4 + i][d = 16nn + li]; the statistics of head h live in lane h
  float lh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) lh[i] = __shfl(l, 4 * g4 + i, WAVE);
  TR(4);
  // (clamped to the launched chunks: a caller whose max_context is below a row's context gets a wrong row, never a
  // ticket left armed for the next launch)
  const int nlive = min(pmax, (ctx + CH - 1) / CH);
  if (nlive == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 4 * g4 + i;
      if (h < G) {
        bf16_t* op = out + ((size_t)b * nq + kvh * G + h) * D;
        const float inv = 1.f / lh[i];
#pragma unroll
        for (int nn = 0; nn < D / 16; ++nn) {
          op[16 * nn + li] = f2bf(o[nn][i] * inv);
        }
      }
    }
    TR(7);
    return;
  }

  // ---- partial record (sc1 stores), arrival count, last arriver merges
  const size_t pair = (size_t)b * nkv + kvh;
  float* rec = part + (pair * pmax + c) * PSTRIDE;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = 4 * g4 + i;
    if (h < G) {
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn)
        __hip_atomic_store(rec + h * D + 16 * nn + li, o[nn][i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (g4 == 0 && li < G) {
    __hip_atomic_store(rec + G * D + li, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + G * D + G + li, l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores land before its arrival counts
  TR(5);
  uint32_t prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(&counters[pair], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __shfl(prev, 0, WAVE);
  TR(6);
  if (prev != (uint32_t)(nlive - 1)) return;
  if (lane == 0) __hip_atomic_store(&counters[pair], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the add

  // ---- merge.  Lane q parks chunk q's (max, sum) of every head in LDS (the V staging area is
  // free now), then lane (h, d0) combines: QB chunks' accumulators are loaded back to back per
  // round trip instead of one dependent load chain per chunk.
  float* stat = reinterpret_cast<float*>(&vbuf[0][0]);  // [nlive <= 64][2G]
  const auto rs = split_rsrc(part + pair * pmax * PSTRIDE);
  auto ld1 = [&](int idx) -> float {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, idx * 4, 0, SC1));
  };
  constexpr int LPH = 64 / G, DPL = D / LPH;  // lanes per head, d per lane (DPL = 2G)
  constexpr int VW = (DPL % 4 == 0) ? 4 : 2;  // floats per load
  constexpr int NV = DPL / VW;                // loads per chunk
  constexpr int QB = (SPLIT_QB_LANES / NV) > 0 ? SPLIT_QB_LANES / NV : 1;
  const int h = lane / LPH, d0 = (lane % LPH) * DPL;
  float buf[QB][DPL];
  auto load_batch = [&](int q0) {
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
      const int off = (min(q0 + qq, nlive - 1) * PSTRIDE + h * D + d0) * 4;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        if constexpr (VW == 4) {
          const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * v, 0, SC1);
#pragma unroll
          for (int e = 0; e < 4; ++e) buf[qq][4 * v + e] = __uint_as_float(a[e]);
        } else {
          typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
          const u32x2 a = __builtin_amdgcn_raw_buffer_load_b64(rs, off + 8 * v, 0, SC1);
          buf[qq][2 * v] = __uint_as_float(a[0]);
          buf[qq][2 * v + 1] = __uint_as_float(a[1]);
        }
      }
    }
  };
  // the first batch of accumulators and every chunk's statistics in ONE round trip
  load_batch(0);
  float sv[2 * G];
  if (lane < nlive) {
#pragma unroll
    for (int j = 0; j < 2 * G; ++j) sv[j] = ld1(lane * PSTRIDE + G * D + j);
  }
  __syncthreads();  // (one wave) the P.V reads of vbuf are done before it is overwritten
  if (lane < nlive) {
#pragma unroll
    for (int j = 0; j < 2 * G; ++j) stat[lane * 2 * G + j] = sv[j];
  }
  __syncthreads();
  TR(8);
  float M = -INFINITY;
  for (int q = 0; q < nlive; ++q) M = fmaxf(M, stat[q * 2 * G + h]);
  float num[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) num[j] = 0.f;
  float den = 0.f;
  for (int q0 = 0; q0 < nlive; q0 += QB) {
    if (q0 > 0) load_batch(q0);
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
      const int q = q0 + qq;
      if (q < nlive) {
        const float w = exp2f(stat[q * 2 * G + h] - M);
        den += w * stat[q * 2 * G + G + h];
#pragma unroll
        for (int j = 0; j < DPL; ++j) num[j] += w * buf[qq][j];
      }
    }
  }
  TR(9);
  bf16_t* op = out + ((size_t)b * nq + kvh * G + h) * D + d0;
  const float inv = 1.f / den;
#pragma unroll
  for (int j = 0; j < DPL; ++j) op[j] = f2bf(num[j] * inv);
  TR(7);
}

template <int G>
__global__ void __launch_bounds__(64) decode_split_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part, uint32_t* __restrict__ counters,
    const bf16_t* __restrict__ qkv, const float* __restrict__ cos_sin, bf16_t* __restrict__ k_cache,
    bf16_t* __restrict__ v_cache, const int* __restrict__ block_tables, const int* __restrict__ context_lens,
    float scale, int max_blocks, int nkv, int pmax) {
  split_body<G>(out, part, counters, qkv, cos_sin, k_cache, v_cache, block_tables, context_lens, scale, max_blocks,
                nkv, pmax, blockIdx.x, blockIdx.y, blockIdx.z);
}

}  // namespace k8sllm

using namespace k8sllm;

K8S_CHECK_UNIT(attn_decode_split)

#ifdef K8S_ATTN_TRACE
extern "C" int k8s_attn_trace_set(unsigned long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_attn_trace), &p, sizeof(p));
}
#endif

extern "C" long long k8s_decode_split_workspace(int B, int nq, int nkv, int pmax) {
  if (nkv <= 0 || nq % nkv != 0) return -1;
  const long long G = nq / nkv;
  return (long long)B * nkv * pmax * (G * 128 + 2 * G);  // floats
}

// part: k8s_decode_split_workspace floats (may be null when pmax == 1); counters: B * nkv zeroed u32
extern "C" int k8s_decode_attention_split(void* out, void* part, uint32_t* counters, const void* qkv,
                                          const float* cos_sin, void* k_cache, void* v_cache, const int* block_tables,
                                          const int* context_lens, float scale, int B, int nq, int nkv, int D,
                                          int block_size, int max_blocks, int pmax, hipStream_t stream) {
  if (B <= 0) return 0;
  if (D != 128 || nkv <= 0 || nq % nkv != 0) return -1;
  if (block_size != 16) return -4;
  if (pmax < 1 || (pmax > 1 && (part == nullptr || counters == nullptr))) return -3;
  if (pmax > 64) return -6;  // the merge keeps one chunk's statistics per lane
  const long long G = nq / nkv;
  if ((long long)pmax * (G * 128 + 2 * G) * 4 > 0x7fffffffLL) return -5;  // 32-bit merge offsets per pair
  dim3 grid(pmax, nkv, B);
#define L(GG)                                                                                                 \
  decode_split_kernel<GG><<<grid, 64, 0, stream>>>((bf16_t*)out, (float*)part, counters, (const bf16_t*)qkv, \
                                                   cos_sin, (bf16_t*)k_cache, (bf16_t*)v_cache, block_tables, \
                                                   context_lens, scale, max_blocks, nkv, pmax)
  switch (G) {
    case 1: L(1); break;
    case 2: L(2); break;
    case 4: L(4); break;
    case 8: L(8); break;
    case 16: L(16); break;
    default: return -2;
  }
#undef L
  return (int)hipGetLastError();
}
