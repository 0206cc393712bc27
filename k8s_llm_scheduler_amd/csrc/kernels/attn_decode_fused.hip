// K4 + K5 + K7 fused for decode: RoPE of the new token's q/k, its paged-KV write, and GQA
// attention over the paged cache in ONE kernel that reads the QKV projection output directly.
//
// Structure (one workgroup = 16 waves x 64 tokens = PART = 1024 context tokens of one (sequence,
// kv head)): the context length and the wave's 4 block ids are one round trip; then every wave
// holding live tokens issues all its K loads (registers) and the V rows of its first 32 keys
// (LDS-DMA into its staging area) before consuming any; the second 32 keys' V rows are register
// loads issued after the scores, in flight across the softmax exchange and the first P.V step:
//  * MFMA v_mfma_f32_16x16x32_bf16 in the "swapped" orientation S^T = K . Q^T: the 16 rows are
//    16 context tokens, the 16 columns the query heads of the GQA group (G <= 16, padded with
//    zero heads), so each K row is read once for all heads, with 16 rows x 64 B per load
//    instruction (coalesced), and every lane ends up holding 4 scores of ONE head;
//  * softmax statistics: registers -> 2 cross-lane steps -> one LDS exchange between waves;
//  * P.V: P feeds the MFMA A operand straight from registers (keys permuted inside each 32-key
//    step exactly as on the V side); V is staged through LDS (XOR swizzle) and read with the
//    gfx950 transposing read ds_read_b64_tr_b16;
//  * contexts up to 1024 tokens (the reference's prompts are ~0.5k) are a single pass that
//    writes the final output; longer ones split into partitions merged by a second kernel that
//    exits immediately for single-partition rows (one captured graph serves every length);
//  * the workgroup owning the new token's position rotates its k, writes k/v to the cache and
//    substitutes the fresh values for its own use (no cross-workgroup ordering).
//
// Layouts: qkv [B, (nq + 2*nkv) * D] bf16 (pre-RoPE); cos_sin [max_pos, D] f32 (cos | sin);
// caches [num_slots, nkv, D] bf16; context_lens[b] INCLUDES the new token (pos = ctx - 1).
#include "common.h"

#define K8S_CHK_THIS_UNIT 3

namespace k8sllm {

constexpr float LOG2E_F = 1.4426950408889634f;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_t;

__device__ __forceinline__ int vswz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// Cascade decode attention: sh shared 64-token spans are cut into groups of ceil(sh / ngm) spans, one partial
// (max, sum, unnormalised P.V, per query head) per group; every reader derives the same group count from sh.
constexpr int CASCADE_MAX_GROUPS = 32;
__device__ __forceinline__ int cascade_groups(int sh, int ngm) {
  if (sh <= 0 || ngm <= 0) return 0;
  const int spg = (sh + ngm - 1) / ngm;
  return (sh + spg - 1) / spg;
}
// Prefix partial records share attn_decode_split.hip's layout: per (row, kv head) "pair", rec_stride records of
// G * D + 2 G floats (the G heads' unnormalised P.V, then their maxima, then their sums); group k is record k.
// Fold the npre records of one (pair, head g) into (M, num, den) at element d: every load issued up front
// (unconditional, clamped to the last live group -- a loop of dependent waits would cost one round trip per group).
__device__ __forceinline__ void cascade_fold(const float* __restrict__ pre, size_t rec0, int G, int g, int npre, int d,
                                             float& M, float& num, float& den) {
  constexpr int D = 128;
  const size_t ps = (size_t)G * D + 2 * G;
  float pm[CASCADE_MAX_GROUPS], pl[CASCADE_MAX_GROUPS], pa[CASCADE_MAX_GROUPS];
#pragma unroll
  for (int k = 0; k < CASCADE_MAX_GROUPS; ++k) {
    const float* r = pre + (rec0 + (size_t)min(k, npre - 1)) * ps;
    pa[k] = r[g * D + d];
    pm[k] = r[G * D + g];
    pl[k] = r[G * D + G + g];
  }
  float Mt = M;
#pragma unroll
  for (int k = 0; k < CASCADE_MAX_GROUPS; ++k)
    if (k < npre) Mt = fmaxf(Mt, pm[k]);
  const float a = exp2f(M - Mt);   // (M = -inf: no per-row part yet, a = 0)
  num *= a;
  den *= a;
#pragma unroll
  for (int k = 0; k < CASCADE_MAX_GROUPS; ++k) {
    if (k < npre) {
      const float w = exp2f(pm[k] - Mt);
      num += w * pa[k];
      den += w * pl[k];
    }
  }
  M = Mt;
}

template <int D, int G, int PART, int NW>
__global__ void __launch_bounds__(NW * 64) decode_fused_kernel(
    bf16_t* __restrict__ out, float* __restrict__ part_acc, float* __restrict__ part_ml, const bf16_t* __restrict__ qkv,
    const float* __restrict__ cos_sin, bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ context_lens, float scale, int block_size,
    int max_blocks, int nkv, int pmax, uint8_t* __restrict__ oq, uint8_t* __restrict__ oe,
    const int* __restrict__ cas, const float* __restrict__ pre, int ngm, int rec_stride) {
  static_assert(D == 128 && G <= 16, "head_dim 128, group <= 16");
  static_assert(PART / NW == 64, "64 tokens per wave");
  constexpr int NT = NW * WAVE;
  constexpr int TW = PART / NW;   // tokens per wave (64)
  constexpr int NTILE = TW / 16;  // 16-token tiles per wave
  constexpr int HALF = D / 2;
  __shared__ __attribute__((aligned(16))) bf16_t qs[16][D];             // rotated q, zero heads >= G
  __shared__ __attribute__((aligned(16))) char vbuf[NW][32 * D * 2];    // per-wave V stage (32 keys)
  __shared__ __attribute__((aligned(16))) bf16_t kcur[D];
  __shared__ __attribute__((aligned(16))) bf16_t vcur[D];
  __shared__ float red[G][D];
  __shared__ float wm[NW][16], wl[NW][16];

  const int b = blockIdx.z, kvh = blockIdx.y, p = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int li = lane & 15, g4 = lane >> 4;
  const int* bt = block_tables + (size_t)b * max_blocks;
  const size_t kvs = (size_t)nkv * D;
  // cascade (decode_prefix_kernel ran first): the first 64 * sh context tokens are the batch's shared prefix, already
  // attended by that kernel; the partitions start after it (p * PART tokens past it) and the row's prefix partials
  // join the merge.  (sh: one extra round trip before the block ids, cascade launches only)
  const int sh = cas != nullptr ? max(0, __builtin_amdgcn_readfirstlane(*(volatile const int*)cas)) : 0;
  const int pst = 64 * sh;
  const int start = pst + p * PART;
  const int wbase = wid * TW;
  // With 16-token blocks a 16-token tile is exactly one cache block, so the rows of this wave depend only on 4
  // block-table entries.  The context length and those entries are one round trip; then every live wave issues
  // all its K loads (registers) and the V rows of its first 32-key step (LDS-DMA straight into its staging area,
  // no registers) together -- waves past the context load nothing.  The unused tail of a block table holds valid
  // ids, so K tiles past the context within a live wave stay in bounds.
  // (vector buffer loads, all five values through one opaque statement: otherwise the compiler waits for a scalar
  // load of the length, and branches, before it requests the block ids)
  const auto rs_cl = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(context_lens), 0, 0x7fffffff, 0x00020000);
  const auto rs_bt = __builtin_amdgcn_make_buffer_rsrc(const_cast<int*>(bt), 0, 0x7fffffff, 0x00020000);
  int ctx_v = (int)__builtin_amdgcn_raw_buffer_load_b32(rs_cl, b * 4, 0, 0);
  int tblk[NTILE];  // cache block of each 16-token tile of this wave (reused for V)
#pragma unroll
  for (int t = 0; t < NTILE; ++t)
    tblk[t] = (int)__builtin_amdgcn_raw_buffer_load_b32(rs_bt, min((start + wbase) / 16 + t, max_blocks - 1) * 4, 0, 0);
  static_assert(NTILE == 4, "four block ids per wave");
  asm volatile("" : "+v"(ctx_v), "+v"(tblk[0]), "+v"(tblk[1]), "+v"(tblk[2]), "+v"(tblk[3]));
  int ctx = __builtin_amdgcn_readfirstlane(ctx_v);
  if (ctx <= 0 || start >= ctx) return;
  K8S_CHECK_MAX(ctx, max_blocks * 16, K8S_CHK_CTX);
  const int n = min(PART, ctx - start);
  const int wn = max(0, min(TW, n - wbase));  // live tokens of this wave (wave-uniform)
  bf16x8 kf[NTILE][D / 32];
  if (wn > 0) {
#pragma unroll
    for (int t = 0; t < NTILE; ++t) K8S_CHECK_RANGE(tblk[t], 0, K8S_CHK_BLOCK, 0);
#pragma unroll
    for (int t = 0; t < NTILE; ++t) {
      const bf16_t* kp = k_cache + (size_t)(tblk[t] * 16 + li) * kvs + (size_t)kvh * D + g4 * 8;
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) kf[t][kk] = *reinterpret_cast<const bf16x8*>(kp + kk * 32);
    }
    // V of keys 0..31: instruction q fills staging bytes [1 KiB q, 1 KiB (q + 1)) = rows 4q..4q+3; lane L lands
    // at row 4q + L/16, 16-byte slot L%16, which in the swizzled image holds column chunk (L%16) ^ vswz(row) -- so
    // that is the chunk it fetches.  Rows past the wave's live keys re-read its last live row (their P is exactly
    // 0; the bytes only have to be finite).
    const int lr = min(wn, 32) - 1;
    const int last_row = (lr < 16 ? tblk[0] : tblk[1]) * 16 + (lr & 15);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int r = 4 * q + g4;
      const int srow = r < wn ? tblk[q >> 2] * 16 + (r & 15) : last_row;
      const bf16_t* src = v_cache + (size_t)srow * kvs + (size_t)kvh * D + (li ^ vswz(r)) * 8;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(&vbuf[wid][0] + 1024 * q), 16,
                                       0, 0);
    }
  }
  const int pos = ctx - 1;
  const bool owner = pos < start + n;
  const int nq = nkv * G;
  const bf16_t* row = qkv + (size_t)b * (nq + 2 * nkv) * D;
  const float* cs = cos_sin + (size_t)pos * D;
  int pblk = bt[pos / 16];
  K8S_CHECK_RANGE(pblk, 0, K8S_CHK_BLOCK, 0);
  const int pslot = pblk * 16 + pos % 16;

  // ---- prologue: RoPE (two rotation pairs per item), zero padding heads, clear accumulators
  for (int i = tid; i < 16 * (HALF / 2) + 2 * (HALF / 2); i += NT) {
    const int h = i / (HALF / 2), d = 2 * (i - h * (HALF / 2));
    if (h < 16) {
      uint32_t lo_pair = 0, hi_pair = 0;
      if (h < G) {
        const bf16_t* x = row + (size_t)(kvh * G + h) * D;
        const uint32_t a = *reinterpret_cast<const uint32_t*>(x + d);
        const uint32_t c2 = *reinterpret_cast<const uint32_t*>(x + d + HALF);
        const float c0 = cs[d], c1 = cs[d + 1], s0 = cs[d + HALF], s1 = cs[d + HALF + 1];
        lo_pair = pack_bf2(lo_bf(a) * c0 - lo_bf(c2) * s0, hi_bf(a) * c1 - hi_bf(c2) * s1);
        hi_pair = pack_bf2(lo_bf(c2) * c0 + lo_bf(a) * s0, hi_bf(c2) * c1 + hi_bf(a) * s1);
      }
      *reinterpret_cast<uint32_t*>(&qs[h][d]) = lo_pair;
      *reinterpret_cast<uint32_t*>(&qs[h][d + HALF]) = hi_pair;
    } else if (owner) {
      const bool isk = (h == 16);
      const bf16_t* x = row + (size_t)(isk ? nq + kvh : nq + nkv + kvh) * D;
      const uint32_t a = *reinterpret_cast<const uint32_t*>(x + d);
      const uint32_t c2 = *reinterpret_cast<const uint32_t*>(x + d + HALF);
      uint32_t lo_pair = a, hi_pair = c2;
      if (isk) {
        const float c0 = cs[d], c1 = cs[d + 1], s0 = cs[d + HALF], s1 = cs[d + HALF + 1];
        lo_pair = pack_bf2(lo_bf(a) * c0 - lo_bf(c2) * s0, hi_bf(a) * c1 - hi_bf(c2) * s1);
        hi_pair = pack_bf2(lo_bf(c2) * c0 + lo_bf(a) * s0, hi_bf(c2) * c1 + hi_bf(a) * s1);
      }
      bf16_t* dst = (isk ? k_cache : v_cache) + (size_t)pslot * kvs + (size_t)kvh * D;
      *reinterpret_cast<uint32_t*>(dst + d) = lo_pair;
      *reinterpret_cast<uint32_t*>(dst + d + HALF) = hi_pair;
      bf16_t* keep = isk ? kcur : vcur;
      *reinterpret_cast<uint32_t*>(keep + d) = lo_pair;
      *reinterpret_cast<uint32_t*>(keep + d + HALF) = hi_pair;
    }
  }
  for (int i = tid; i < G * D; i += NT) (&red[0][0])[i] = 0.f;
  __syncthreads();

  // Q^T fragments (B operand): lane holds Q[head li][d = 32kk + 8*g4 + j]
  bf16x8 qf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(&qs[li][kk * 32 + g4 * 8]);

  // ---- S^T = K . Q^T over this wave's tokens; lane holds S[token 16t + 4*g4 + i][head li]
  const float qscale = scale * LOG2E_F;
  f32x4 sacc[NTILE];
#pragma unroll
  for (int t = 0; t < NTILE; ++t) {
    if (start + wbase + 16 * t + li == pos) {  // the fresh key (cache write may not be visible yet)
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) kf[t][kk] = *reinterpret_cast<const bf16x8*>(&kcur[kk * 32 + g4 * 8]);
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][kk], qf[kk], acc, 0, 0, 0);
    sacc[t] = acc;
  }
  // V rows of the second 32-key step: register loads issued now (the K registers are free), in flight across
  // the softmax exchange and the first step's P.V; staged into LDS once the first step's reads are done
  u32x4 vv[8];
  const bool two = 32 < wn;  // wave-uniform
  if (two) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int c = lane + 64 * q, r = c >> 4, ch = c & 15;
      const int blk = (r < 16) ? tblk[2] : tblk[3];  // r < 16 <=> q < 4 (lane-independent)
      vv[q] = *reinterpret_cast<const u32x4*>(v_cache + (size_t)(blk * 16 + (r & 15)) * kvs + (size_t)kvh * D + ch * 8);
    }
  }
  // scale, mask, wave-local max per head
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < NTILE; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 16 * t + 4 * g4 + i;
      const float v = k < wn ? sacc[t][i] * qscale : -INFINITY;
      sacc[t][i] = v;
      m = fmaxf(m, v);
    }
  }
  m = fmaxf(m, __shfl_xor(m, 16, WAVE));
  m = fmaxf(m, __shfl_xor(m, 32, WAVE));
  if (g4 == 0) wm[wid][li] = m;
  __syncthreads();
  float M = -INFINITY;
#pragma unroll
  for (int w = 0; w < NW; ++w) M = fmaxf(M, wm[w][li]);
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < NTILE; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e = exp2f(sacc[t][i] - M);
      sacc[t][i] = e;
      l += e;
    }
  }
  l += __shfl_xor(l, 16, WAVE);
  l += __shfl_xor(l, 32, WAVE);
  if (g4 == 0) wl[wid][li] = l;

  // ---- O = P . V over 32-key steps; V staged per wave in LDS (swizzled 16-byte chunks)
  f32x4 o[D / 16];
#pragma unroll
  for (int nn = 0; nn < D / 16; ++nn) o[nn] = f32x4{0.f, 0.f, 0.f, 0.f};
  char* vb = vbuf[wid];
  const int qd = li >> 2, pd = li & 3;
  static_assert(NTILE == 4, "two 32-key steps per wave");
#pragma unroll
  for (int st = 0; st < NTILE / 2; ++st) {
    if (32 * st < wn) {  // wave-uniform
      if (st == 0) {
        // the DMA image of keys 0..31 has landed (only the second step's register loads may still be in flight:
        // loads complete in order); the new token's row -- and the padding rows after it, which re-read its
        // stale cache slot -- take the fresh v
        if (two) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int rp = pos - (start + wbase);
        if (rp >= 0 && rp < 32) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int c = lane + 64 * q, r = c >> 4, ch = c & 15;
            if (r >= rp)
              *reinterpret_cast<u32x4*>(vb + r * (D * 2) + 16 * (ch ^ vswz(r))) =
                  *reinterpret_cast<const u32x4*>(&vcur[ch * 8]);
          }
        }
      } else {
        // stage the 32 keys x 128 d loaded above (fresh token from LDS, keys past the wave zeroed)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int c = lane + 64 * q, r = c >> 4, ch = c & 15;
          const int k = 32 * st + r;
          if (start + wbase + k == pos) vv[q] = *reinterpret_cast<const u32x4*>(&vcur[ch * 8]);
          if (k >= wn) vv[q] = u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int c = lane + 64 * q, r = c >> 4, ch = c & 15;
          *reinterpret_cast<u32x4*>(vb + r * (D * 2) + 16 * (ch ^ vswz(r))) = vv[q];
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
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
            (lds_bf16x4_t*)(vb + r0 * (D * 2) + 16 * (ch ^ vswz(r0)) + hb));
        const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(vb + r1 * (D * 2) + 16 * (ch ^ vswz(r1)) + hb));
        bf16x8 vbf;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vbf[j] = v0[j]; vbf[4 + j] = v1[j]; }
        o[nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vbf, o[nn], 0, 0, 0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();  // tr reads done before the next step overwrites vbuf
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  // o[nn][i] = O[head 4*g4 + i][d = 16nn + li].  Cross-wave sum: every wave parks its partial in
  // the (now idle) V staging area, then each thread adds one (head, d) over the waves -- no LDS
  // atomics (16 waves adding into the same addresses serialise).
  __syncthreads();  // all waves done with vbuf
  float* part = reinterpret_cast<float*>(&vbuf[0][0]);  // [NW][G][D] floats (G*D*4*NW <= sizeof vbuf)
  static_assert(NW * G * D * 4 <= NW * 32 * D * 2, "partials fit in the V staging area");
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int h = 4 * g4 + i;
    if (h < G) {
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) part[(wid * G + h) * D + 16 * nn + li] = wn > 0 ? o[nn][i] : 0.f;
    }
  }
  __syncthreads();
  for (int i = tid; i < G * D; i += NT) {
    float a = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) a += part[w * G * D + i];
    (&red[0][0])[i] = a;
  }
  __syncthreads();
  // (pmax == 1 with a longer context: the caller's max_context is below the row's context -- a precondition
  // violation; the partition's own tokens are written as the output instead of through absent partial buffers)
  const bool single = ctx - pst <= PART || pmax == 1;
  for (int i = tid; i < G * D; i += NT) {
    const int g = i / D, d = i - g * D;
    float L = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) L += wl[w][g];
    const int h = kvh * G + g;
    const float sacc_v = red[g][d];
    if (single) {
      float num = sacc_v, den = L;
      const int npre = cascade_groups(sh, ngm);
      if (npre > 0) {   // the shared prefix's partials (log2 domain, the same scale) join this row's
        float Mw = -INFINITY;
#pragma unroll
        for (int w = 0; w < NW; ++w) Mw = fmaxf(Mw, wm[w][g]);
        cascade_fold(pre, ((size_t)b * nkv + kvh) * rec_stride, G, g, npre, d, Mw, num, den);
      }
      if (oq != nullptr) {   // MX output: the 32 lanes of (head, d / 32) form one half-wave (NT, D: multiples of 32)
        mx_store_lane(oq, oe, b, h * D + d, nq * D, gridDim.z, bf_round(num / den));
      } else {
        out[((size_t)b * nq + h) * D + d] = f2bf(num / den);
      }
    } else {
      float Mx = -INFINITY;
#pragma unroll
      for (int w = 0; w < NW; ++w) Mx = fmaxf(Mx, wm[w][g]);
      const size_t pi = ((size_t)b * nq + h) * pmax + p;
      part_acc[pi * D + d] = sacc_v;
      if (d == 0) { part_ml[pi * 2] = Mx; part_ml[pi * 2 + 1] = L; }
    }
  }
}

// ---- Cascade part 1: the shared prefix of a decode batch, read ONCE for every row that shares it.
// Batched scheduling decides many pods against one cluster snapshot; with the cluster-first prompt layout every
// prompt of a batch starts with the same thousands of tokens, which the prefix cache stores once -- but the
// per-row attention above would still read those K/V bytes once per row (B times per layer and step).  Here one
// workgroup = (group of shared 64-token spans, kv head, 8 x 16 query columns): the 16 columns of a wave are the G
// query heads of 16 / G rows, so one staged K/V span feeds 8 waves x 16 (row, head) columns -- an MFMA-shaped GEMM
// (S^T = K . Q^T, then P . V) instead of B separate GEMVs over the same bytes.
//  * the span's K and V (64 tokens x 256 B each) go HBM -> registers -> LDS (one 16-byte load and one ds_write per
//    thread and operand; the next span's loads in flight under this span's MFMAs), double-buffered, one barrier per
//    span; K rows in an XOR-swizzled image (conflict-free ds_read_b128 A fragments), V in the attention kernel's
//    image for the transposing ds_read_b64_tr_b16 B fragments;
//  * online softmax across the group's spans in the log2 domain (scores x scale x log2 e), the attention kernel's
//    convention, so the partials merge with its own (decode_fused_kernel / decode_merge_kernel above);
//  * q is rotated here (RoPE at each row's own position) from the pre-RoPE QKV rows.
// cas = {sh, r0}: sh spans shared by every active row (the host's longest common block-table prefix, never reaching a
// row's new token), read from row r0's block table.  Partials: record k of pair (row, kv head) in the split
// layout above (cascade_fold), rec_stride records per pair.
template <int G>
__global__ void __launch_bounds__(512) decode_prefix_kernel(
    float* __restrict__ pre, int rec_stride, const bf16_t* __restrict__ qkv,
    const float* __restrict__ cos_sin, const bf16_t* __restrict__ k_cache, const bf16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, const int* __restrict__ context_lens, const int* __restrict__ cas,
    float scale, int B, int nkv, int max_blocks, int ngm) {
  constexpr int D = 128, HALF = D / 2, SPT = 16 / G, ROWB = D * 2;   // rows per 16-column tile, bytes per K/V row
  static_assert(G >= 1 && G <= 16 && 16 % G == 0, "GQA group of 1, 2, 4, 8 or 16 heads");
  __shared__ __attribute__((aligned(16))) char stage[2][2][64 * ROWB];   // [buffer][K | V][64 tokens x 256 B]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, li = lane & 15, g4 = lane >> 4;
  const int sh = cas[0];
  if (sh <= 0) return;
  const int spg = (sh + ngm - 1) / ngm;
  const int s0 = blockIdx.x * spg, s1 = min(s0 + spg, sh);
  if (s0 >= s1) return;
  const int r0 = min(max(cas[1], 0), B - 1);   // (a host value, clamped to the launch's rows)
  const int kvh = blockIdx.y, nq = nkv * G;
  const size_t kvs = (size_t)nkv * D;
  const int* bt0 = block_tables + (size_t)r0 * max_blocks;

  // ---- this lane's query column li: row b = tile * SPT + li / G, head kvh * G + li % G; rotated q as the MFMA B
  // operand (qf[kk][j] = q[d = 32 kk + 8 g4 + j]: d < 64 for kk < 2, so the lane holds both halves of its RoPE pairs)
  const int tile = blockIdx.z * 8 + wid;
  const int bq = tile * SPT + li / G, hq = kvh * G + li % G;
  const int ctxq = bq < B ? context_lens[bq] : 0;
  const bool live = ctxq > 0;
  bf16x8 qf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk)
#pragma unroll
    for (int j = 0; j < 8; ++j) qf[kk][j] = (__bf16)0.f;
  if (live) {
    const bf16_t* x = qkv + (size_t)bq * (nq + 2 * nkv) * D + (size_t)hq * D;
    const float* cs = cos_sin + (size_t)(ctxq - 1) * D;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int d0 = 32 * kk + 8 * g4;
      const u32x4 xl = *reinterpret_cast<const u32x4*>(x + d0);
      const u32x4 xh = *reinterpret_cast<const u32x4*>(x + d0 + HALF);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = (e & 1) ? hi_bf(xl[e >> 1]) : lo_bf(xl[e >> 1]);
        const float c2 = (e & 1) ? hi_bf(xh[e >> 1]) : lo_bf(xh[e >> 1]);
        const float c = cs[d0 + e], sn = cs[d0 + e + HALF];
        qf[kk][e] = (__bf16)(a * c - c2 * sn);
        qf[kk + 2][e] = (__bf16)(c2 * c + a * sn);
      }
    }
  }

  // ---- staging: thread tid moves K and V rows (tid >> 4) and 32 + (tid >> 4), 16-byte chunk tid & 15
  const int srow = tid >> 4, sch = tid & 15;
  auto blk_of = [&](int s, int j) {   // cache block of this thread's row j of span s
    int v = bt0[4 * s + (srow >> 4) + 2 * j];
    K8S_CHECK_RANGE(v, 0, K8S_CHK_BLOCK, 0);
    return v;
  };
  auto load = [&](const int (&bl)[2], u32x4 (&kr)[2], u32x4 (&vr)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const size_t off = (size_t)(bl[j] * 16 + (srow & 15)) * kvs + (size_t)kvh * D + sch * 8;
      kr[j] = *reinterpret_cast<const u32x4*>(k_cache + off);
      vr[j] = *reinterpret_cast<const u32x4*>(v_cache + off);
    }
  };
  auto store = [&](int buf, const u32x4 (&kr)[2], const u32x4 (&vr)[2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = srow + 32 * j;
      *reinterpret_cast<u32x4*>(&stage[buf][0][r * ROWB + 16 * (sch ^ (r & 15))]) = kr[j];
      *reinterpret_cast<u32x4*>(&stage[buf][1][r * ROWB + 16 * (sch ^ vswz(r))]) = vr[j];
    }
  };

  u32x4 kr[2], vr[2];
  int bl[2] = {blk_of(s0, 0), blk_of(s0, 1)};
  load(bl, kr, vr);
  if (s0 + 1 < s1) {
    bl[0] = blk_of(s0 + 1, 0);
    bl[1] = blk_of(s0 + 1, 1);
  }
  store(0, kr, vr);
  __syncthreads();

  const float qscale = scale * LOG2E_F;
  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[D / 16];
#pragma unroll
  for (int nn = 0; nn < D / 16; ++nn) o[nn] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qd = li >> 2, pd = li & 3;
  for (int s = s0; s < s1; ++s) {
    const int buf = (s - s0) & 1;
    const bool more = s + 1 < s1;
    if (more) {   // (block-uniform) the next span's rows in flight under this span's math
      load(bl, kr, vr);
      if (s + 2 < s1) {
        bl[0] = blk_of(s + 2, 0);
        bl[1] = blk_of(s + 2, 1);
      }
    }
    const char* kb = stage[buf][0];
    const char* vb = stage[buf][1];
    // S^T = K . Q^T: lane holds S[token 16 t + 4 g4 + i][column li]
    f32x4 sacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(kb + (16 * t + li) * ROWB + 16 * ((4 * kk + g4) ^ li));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], acc, 0, 0, 0);
      }
      sacc[t] = acc;
    }
    float mloc = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sacc[t][i] *= qscale;
        mloc = fmaxf(mloc, sacc[t][i]);
      }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 16, WAVE));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, WAVE));
    const float m_new = fmaxf(m_run, mloc);
    const float alpha = exp2f(m_run - m_new);   // (0 on the first span: m_run = -inf)
    float lsum = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = exp2f(sacc[t][i] - m_new);
        sacc[t][i] = e;
        lsum += e;
      }
    lsum += __shfl_xor(lsum, 16, WAVE);
    lsum += __shfl_xor(lsum, 32, WAVE);
    l_run = l_run * alpha + lsum;
    m_run = m_new;
    // o[nn][i] holds column 4 g4 + i: its rescale factor lives in lane 4 g4 + i (g4 = 0 there, li = the column)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float ai = __shfl(alpha, 4 * g4 + i, WAVE);
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) o[nn][i] *= ai;
    }
    // O += P . V over the span's two 32-key steps (the attention kernel's key order and V fragments)
#pragma unroll
    for (int st = 0; st < 2; ++st) {
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = (__bf16)sacc[2 * st][j];
        pa[4 + j] = (__bf16)sacc[2 * st + 1][j];
      }
      const int ra = 32 * st + 4 * g4 + qd, rb = ra + 16;
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) {
        const int col = 16 * nn + 4 * pd;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(vb + ra * ROWB + 16 * (ch ^ vswz(ra)) + hb));
        const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(vb + rb * ROWB + 16 * (ch ^ vswz(rb)) + hb));
        bf16x8 vbf;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vbf[j] = v0[j];
          vbf[4 + j] = v1[j];
        }
        o[nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vbf, o[nn], 0, 0, 0);
      }
    }
    if (more) store(buf ^ 1, kr, vr);   // (that buffer's last readers passed the previous span's barrier)
    __syncthreads();                    // next span staged; this one's reads done before it is refilled
  }

  // ---- partials of this group: column c's (max, sum) from lane c, its P.V row from lanes (c / 4 = g4, c % 4 = i)
  const int gi = blockIdx.x;
  constexpr int PS = G * D + 2 * G;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = 4 * g4 + i;
    const bool ok = __shfl((int)live, c, WAVE) != 0;
    if (ok) {
      const int b = tile * SPT + c / G;
      float* dst = pre + (((size_t)b * nkv + kvh) * rec_stride + gi) * PS + (c % G) * D;
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) dst[16 * nn + li] = o[nn][i];
    }
  }
  if (g4 == 0 && live) {
    float* dst = pre + (((size_t)bq * nkv + kvh) * rec_stride + gi) * PS + G * D + li % G;
    dst[0] = m_run;
    dst[G] = l_run;
  }
}

template <int D>
__global__ void __launch_bounds__(D) decode_merge_kernel(bf16_t* __restrict__ out, const float* __restrict__ part_acc,
                                                         const float* __restrict__ part_ml,
                                                         const int* __restrict__ context_lens, int part, int pmax,
                                                         int nq, uint8_t* __restrict__ oq, uint8_t* __restrict__ oe,
                                                         const int* __restrict__ cas, const float* __restrict__ pre,
                                                         int ngm, int rec_stride, int G) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int sh = cas != nullptr ? max(0, cas[0]) : 0;
  const int ctx = context_lens[b] - 64 * sh;   // (cascade: the partitions start after the shared prefix)
  if (context_lens[b] <= 0 || ctx <= part) return;  // single-partition rows were finished by the attention kernel
  const int np = min(pmax, (ctx + part - 1) / part);
  const size_t base = ((size_t)b * nq + h) * pmax;
  const int npre = cascade_groups(sh, ngm);
  float M = -INFINITY;
  for (int q = 0; q < np; ++q) M = fmaxf(M, part_ml[(base + q) * 2]);
  float num = 0.f, den = 0.f;
  for (int q = 0; q < np; ++q) {
    const float w = exp2f(part_ml[(base + q) * 2] - M);
    num += w * part_acc[(base + q) * D + d];
    den += w * part_ml[(base + q) * 2 + 1];
  }
  if (npre > 0) cascade_fold(pre, ((size_t)b * (nq / G) + h / G) * rec_stride, G, h % G, npre, d, M, num, den);
  if (oq != nullptr) mx_store_lane(oq, oe, b, h * D + d, nq * D, gridDim.y, bf_round(num / den));
  else out[((size_t)b * nq + h) * D + d] = f2bf(num / den);
}

}  // namespace k8sllm

using namespace k8sllm;

K8S_CHECK_UNIT(attn_decode_fused)

// part_acc [B, nq, pmax, D] f32 / part_ml [B, nq, pmax, 2] f32 (needed when pmax > 1).
// part: context tokens per workgroup, 1024 (16 waves, ~137 KB of LDS: one workgroup per CU) or 512 (8 waves,
// ~73 KB: two per CU -- for batches whose (sequence, kv head) pairs outnumber the CUs, where the 16-wave
// workgroups would run in two rounds).  pmax = ceil(max context / part).
// oq / oe (optional): the output as MX e4m3 [B][nq * D] + E8M0 scales (common.h mx_scale_off layout) (K16: the fp8 O projection's input
// quantized by its producer) instead of bf16.
// cas / pre / ngm / rec_stride (optional, all or none): the cascade inputs -- k8s_decode_prefix ran on the same
// stream first (records of rec_stride per pair); the rows' first 64 * cas[0] tokens are skipped here and that
// kernel's partials merged instead.
extern "C" int k8s_decode_attention_fused(void* out, void* part_acc, void* part_ml, const void* qkv,
                                          const float* cos_sin, void* k_cache, void* v_cache, const int* block_tables,
                                          const int* context_lens, float scale, int B, int nq, int nkv, int D,
                                          int block_size, int max_blocks, int pmax, int part, void* oq, void* oe,
                                          const int* cas, const float* pre, int ngm, int rec_stride,
                                          hipStream_t stream) {
  if (B <= 0) return 0;
  if (D != 128 || nq % nkv != 0) return -1;
  if (block_size != 16) return -4;  // the speculative K loads assume one 16-token block per tile
  if (pmax > 1 && (part_acc == nullptr || part_ml == nullptr)) return -3;
  if (part != 1024 && part != 512) return -5;
  if (cas != nullptr && (pre == nullptr || ngm < 1 || ngm > CASCADE_MAX_GROUPS || rec_stride < ngm)) return -6;
  const int G = nq / nkv;
  dim3 grid(pmax, nkv, B);
#define L(GG, PP, WW)                                                                                       \
  decode_fused_kernel<128, GG, PP, WW><<<grid, WW * 64, 0, stream>>>(                                        \
      (bf16_t*)out, (float*)part_acc, (float*)part_ml, (const bf16_t*)qkv, cos_sin, (bf16_t*)k_cache,       \
      (bf16_t*)v_cache, block_tables, context_lens, scale, block_size, max_blocks, nkv, pmax, (uint8_t*)oq,   \
      (uint8_t*)oe, cas, pre, ngm, rec_stride)
#define LG(PP, WW)                 \
  switch (G) {                     \
    case 1: L(1, PP, WW); break;   \
    case 2: L(2, PP, WW); break;   \
    case 4: L(4, PP, WW); break;   \
    case 8: L(8, PP, WW); break;   \
    case 16: L(16, PP, WW); break; \
    default: return -2;            \
  }
  if (part == 1024) {
    LG(1024, 16)
  } else {
    LG(512, 8)
  }
#undef LG
#undef L
  if (pmax > 1)
    decode_merge_kernel<128><<<dim3(nq, B), 128, 0, stream>>>((bf16_t*)out, (const float*)part_acc,
                                                              (const float*)part_ml, context_lens, part, pmax, nq,
                                                              (uint8_t*)oq, (uint8_t*)oe, cas, pre, ngm, rec_stride,
                                                              G);
  return (int)hipGetLastError();
}

// Workgroups of k8s_decode_prefix along the query columns: 8 waves x 16 (row, head) columns each.
extern "C" int k8s_decode_prefix_col_blocks(int B, int nq, int nkv) {
  if (nkv <= 0 || nq % nkv != 0 || 16 % (nq / nkv) != 0) return -1;
  const int spt = 16 / (nq / nkv);
  return (B + 8 * spt - 1) / (8 * spt);
}

// Cascade part 1 (decode_prefix_kernel): the batch's shared prefix (cas = {spans, reference row}, device ints the
// host writes before the step) attended once for every row; grid (ngm, nkv, column blocks).  Group k's partial of
// pair (row, kv head) is record k of rec_stride >= ngm records (attn_decode_split.hip's record layout); the per-row
// kernel given the same cas (k8s_decode_attention_fused / _split) merges them.
extern "C" int k8s_decode_prefix(void* pre, int rec_stride, const void* qkv, const float* cos_sin, const void* k_cache,
                                 const void* v_cache, const int* block_tables, const int* context_lens, const int* cas,
                                 float scale, int B, int nq, int nkv, int D, int block_size, int max_blocks, int ngm,
                                 hipStream_t stream) {
  if (B <= 0) return 0;
  if (D != 128 || block_size != 16 || ngm < 1 || ngm > CASCADE_MAX_GROUPS || rec_stride < ngm) return -1;
  if (pre == nullptr || cas == nullptr) return -3;
  const int cb = k8s_decode_prefix_col_blocks(B, nq, nkv);
  if (cb < 1) return -2;
  const dim3 grid(ngm, nkv, cb);
#define LP(GG)                                                                                                   \
  decode_prefix_kernel<GG><<<grid, 512, 0, stream>>>((float*)pre, rec_stride, (const bf16_t*)qkv, cos_sin,        \
                                                     (const bf16_t*)k_cache, (const bf16_t*)v_cache, block_tables,   \
                                                     context_lens, cas, scale, B, nkv, max_blocks, ngm)
  switch (nq / nkv) {
    case 1: LP(1); break;
    case 2: LP(2); break;
    case 4: LP(4); break;
    case 8: LP(8); break;
    case 16: LP(16); break;
    default: return -2;
  }
#undef LP
  return (int)hipGetLastError();
}
