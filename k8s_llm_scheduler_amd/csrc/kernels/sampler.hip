// K13 + K17: sampling over a (possibly vocab-sharded) fp32 logits buffer, fused with the
// decode-state update so a whole decode step can be replayed from a hipGraph.
//
// Logits layout: [shards][B][Vs]; token id v = shard * Vs + j (vocab-parallel LM head output
// after an all-gather, or a single shard).  Per row b:
//   temperature <= 0       -> greedy argmax (lowest index wins ties, like torch.argmax)
//   top_p >= 1             -> Gumbel-max: argmax(l / T + G), G = -log(-log(U)), one pass
//   0 < top_p < 1          -> nucleus, then Gumbel-max inside it.  The nucleus is a threshold on
//                             f(l) = floor((M - l) / T * 65536 / 28): the smallest f* whose tokens
//                             {f <= f*} carry >= top_p of the probability mass (2^-40 fixed point,
//                             integer sums: order-independent, so every TP rank picks the same set).
//                             One fine bin spans 28/65536 of log-probability (0.04 %), so the set is
//                             the exact sorted-cumsum nucleus up to ties inside one such bin.
// U comes from a counter-based hash of (seed[b], counter[b], token) so results do not depend on
// batch composition or on which rank samples (every TP rank draws the same token).
// After sampling: tokens[b] = tok; hist[b][steps[b]] = tok; steps[b]++; ctx[b]++ (optional).
//
// Work split: the per-token work (a hash and two logs for Gumbel) over a 128k vocabulary is
// compute-bound on one CU (~70 us), so every pass spreads the vocabulary over NB workgroups per row
// (each inside one vocab shard).  Greedy / Gumbel: each workgroup reduces its slice to one packed
// 64-bit key (ord(score) << 32 | ~index, so the max key is the best score with the LOWEST index),
// folds it into a per-row atomicMax, and the workgroup whose arrival-counter add comes last
// finalizes the row (agent-scope atomics only) and re-arms the row's key and counter for the next
// graph replay.  Nucleus rows first run three more passes over the same grid (launched only when
// the caller asks for the nucleus path):
//   1. row max (atomicMax of the ordered key);
//   2. mass histogram over the 256 coarse bins f >> 8 per workgroup (LDS, one copy per wave), written
//      with sc1 stores; the last-arriving workgroup sums the NB copies, takes Z and the target mass
//      floor(Z * top_p), and scans for the coarse bin b* where the cumulative mass crosses it;
//   3. the same over the 256 fine bins inside b* -> f*.
// The row state (max key, arrival counters) starts zeroed and the sampling pass's last arriver
// re-arms it, like the argmax key and counter (no memset node in the replayed graph).
#include "common.h"

namespace k8sllm {

constexpr int ST = 256;   // threads per workgroup
constexpr int NB = 32;    // workgroups per row (split over the vocab shards)
constexpr float NUC_FS = 65536.f / 28.f;  // fine-bin scale; exp(-28) * 2^40 < 1: no mass beyond
constexpr int NUC_NONE = 65536;

struct NucRow {             // one per row; maxkey / cnt0 / cnt1 zero between calls
  unsigned long long target, above;
  uint32_t maxkey, bstar, fstar, cnt0, cnt1, pad[7];
};
static_assert(sizeof(NucRow) == 64, "NucRow is 64 bytes");

__device__ __forceinline__ uint32_t ord_key(float f) {  // monotone float -> uint32
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key_float(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k ^ 0x80000000u) : ~k);
}
__device__ __forceinline__ int nuc_fine(float l, float M, float invT) {
  const float x = ((M - l) * invT) * NUC_FS;
  return x < 65536.f ? (int)x : NUC_NONE;  // NaN -> none
}
__device__ __forceinline__ unsigned long long nuc_mass(float l, float M, float invT) {
  return (unsigned long long)(__expf((l - M) * invT) * 1099511627776.0f);
}

struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax better(ArgMax a, ArgMax b) {
  if (b.v > a.v || (b.v == a.v && b.i < a.i)) return b;
  return a;
}
__device__ ArgMax block_argmax(ArgMax a, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax b{__shfl_xor(a.v, o, WAVE), __shfl_xor(a.i, o, WAVE)};
    a = better(a, b);
  }
  if (lane == 0) { sv[wid] = a.v; si[wid] = a.i; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < ST / 64; ++w) a = better(a, ArgMax{sv[w], si[w]});
    sv[0] = a.v;
    si[0] = a.i;
  }
  __syncthreads();
  ArgMax r{sv[0], si[0]};
  __syncthreads();
  return r;
}

__device__ __forceinline__ unsigned long long pack_key(float score, int idx) {
  return ((unsigned long long)ord_key(score) << 32) | (unsigned long long)(0xFFFFFFFFu - (uint32_t)idx);
}

// Device-side stop detection of the decode graphs.  Per token, a class word built once from
// the tokenizer vocabulary: x = eos (bit 0) | net brace delta (int8, bits 8-15) | min running depth relative to
// the entry (int8, 16-23); y = holds a '{' (bit 0) | depth at the end when the first '{' of the answer is in it
// (int8, 8-15) | min depth after that '{' (int8, 16-23).  Per slot: json state (-2: the prefill's first token is
// not classified yet, -1: no '{' yet, d >= 1: depth) and cfg = eos stop (bit 0) | json stop (bit 1) |
// max_tokens << 8.  The naive brace counter is the one of control/jsonextract.py json_object_closed, so the
// device and the host agree on when an answer's first object closes.
struct StopArgs {
  const int2* cls;        // [vocab] token classes, or null (stop detection off)
  int* json;              // [slots]
  const int* cfg;         // [slots]
  const int* forced;      // [slots][fstride] scripted answer tokens, or null
  const int* forced_len;  // [slots]: -1 = sample; >= 0 = write forced[st] (EOS past the end)
  int fstride;
  int eos_tok;
  int* done;              // [slots] host-mapped flags: set when the slot's answer finishes
};

__device__ __forceinline__ int json_step(int state, int2 c, bool& closed) {
  closed = false;
  if (state >= 1) {
    const int amin = (int)(int8_t)((c.x >> 16) & 0xff), adelta = (int)(int8_t)((c.x >> 8) & 0xff);
    if (state + amin <= 0) {
      closed = true;
      return 0;
    }
    return state + adelta;
  }
  if (c.y & 1) {
    const int bmin = (int)(int8_t)((c.y >> 16) & 0xff), bend = (int)(int8_t)((c.y >> 8) & 0xff);
    if (bmin <= 0) {
      closed = true;
      return 0;
    }
    return bend;
  }
  return state;
}

// Decode-state update of state slot s (= the row, or slots[row]): tokens[s] = tok; hist[s][steps[s]] = tok;
// steps[s]++; ctx[s]++ -- or, when the answer finished (EOS, closed JSON object, max_tokens), ctx[s] = 0 (later
// replays skip the slot) and the host-mapped done flag.
__device__ __forceinline__ void write_token(int s, int tok, int* __restrict__ tokens, int* __restrict__ ctx_inc,
                                            int* __restrict__ hist, int hist_stride, int* __restrict__ steps,
                                            const StopArgs& sa) {
  const int st = steps != nullptr ? steps[s] : 0;
  bool fin = false;
  if (sa.cls != nullptr && hist != nullptr && ctx_inc != nullptr) {
    const int cfg = sa.cfg[s], max_new = cfg >> 8;
    int state = sa.json[s];
    bool closed = false;
    if (state == -2) {   // the first token, sampled by the prefill
      const int t0 = hist[(size_t)s * hist_stride];
      state = -1;
      if ((cfg & 1) && (sa.cls[t0].x & 1)) {
        fin = true;
      } else if (cfg & 2) {
        state = json_step(state, sa.cls[t0], closed);
        fin = closed;
      }
      if (!fin && st >= max_new) fin = true;
      if (fin) {   // the answer ended at its first token: emit nothing more
        sa.json[s] = state;
        ctx_inc[s] = 0;
        if (sa.done != nullptr) __hip_atomic_store(&sa.done[s], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
      }
    }
    if (sa.forced != nullptr && sa.forced_len[s] >= 0)
      tok = st < sa.forced_len[s] ? sa.forced[(size_t)s * sa.fstride + st] : sa.eos_tok;
    const int2 c = sa.cls[tok];
    if ((cfg & 1) && (c.x & 1)) {
      fin = true;
    } else {
      if (cfg & 2) {
        state = json_step(state, c, closed);
        fin = closed;
      }
      if (st + 1 >= max_new) fin = true;
    }
    sa.json[s] = state;
  }
  tokens[s] = tok;
  if (hist != nullptr) {
    if (st < hist_stride) hist[(size_t)s * hist_stride + st] = tok;
    steps[s] = st + 1;
  }
  if (ctx_inc != nullptr) ctx_inc[s] = fin ? 0 : ctx_inc[s] + 1;
  if (fin && sa.done != nullptr) __hip_atomic_store(&sa.done[s], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// This workgroup's slice: inside ONE shard (gridDim.x = shards * per_shard), so a token is
// base[j] with id s * Vs + j and no division per token.
struct Slice {
  const float* base;
  int j0, j1, id0;
};
// id_base: global id of this buffer's first token (vocab-parallel sampling: rank * Vs; 0 for a gathered buffer)
__device__ __forceinline__ Slice slice_of(const float* logits, int b, int B, int Vs, int shards, int id_base) {
  const int per_shard = gridDim.x / shards;
  const int s = blockIdx.x / per_shard, q = blockIdx.x - s * per_shard;
  const int per = (Vs + per_shard - 1) / per_shard;
  Slice r;
  r.base = logits + ((size_t)s * B + b) * Vs;
  r.j0 = q * per;
  r.j1 = min(Vs, r.j0 + per);
  r.id0 = id_base + s * Vs;
  return r;
}

__device__ __forceinline__ bool nuc_row(int b, const int* ctx_inc, const int* slots, const float* temperature,
                                        const float* top_p) {
  return (ctx_inc == nullptr || ctx_inc[slots != nullptr ? slots[b] : b] > 0) && temperature[b] > 0.f &&
         top_p[b] < 1.f;
}

// pass 1: row max of the logits (ordered-key atomicMax into maxkey[b * mstride]: the row state's maxkey, or -- vocab
// parallel -- this rank's exported row maxima, combined over the ranks by nuc_import_max_kernel)
__global__ void __launch_bounds__(ST) nuc_max_kernel(const float* __restrict__ logits, int B, int Vs, int shards,
                                                     const float* __restrict__ temperature,
                                                     const float* __restrict__ top_p, const int* __restrict__ ctx_inc,
                                                     const int* __restrict__ slots, uint32_t* __restrict__ maxkey,
                                                     int mstride) {
  __shared__ float red[ST / 64];
  const int b = blockIdx.y;
  if (!nuc_row(b, ctx_inc, slots, temperature, top_p)) return;
  const Slice sl = slice_of(logits, b, B, Vs, shards, 0);
  float m = -INFINITY;
  for (int j = sl.j0 + threadIdx.x; j < sl.j1; j += ST) m = fmaxf(m, sl.base[j]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < ST / 64; ++w) m = fmaxf(m, red[w]);
    __hip_atomic_fetch_max(&maxkey[(size_t)b * mstride], ord_key(m), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Bin totals of one row (thread = bin; every thread of the workgroup calls this): inclusive scan, then the first bin
// where the cumulative mass reaches the target.  LEVEL 0 stores target / mass above b* / b*, LEVEL 1 f* in the row
// state.  sh_sel must be 256 on entry.
template <int LEVEL>
__device__ __forceinline__ void nuc_select(unsigned long long tot, int b, const float* __restrict__ top_p,
                                           NucRow* __restrict__ st, unsigned long long (*scan)[256], int* sh_sel) {
  const int tid = threadIdx.x;
  int cur = 0;
  scan[0][tid] = tot;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const unsigned long long v = scan[cur][tid] + (tid >= o ? scan[cur][tid - o] : 0ull);
    scan[cur ^ 1][tid] = v;
    cur ^= 1;
    __syncthreads();
  }
  const unsigned long long incl = scan[cur][tid];
  unsigned long long target, base;
  if (LEVEL == 0) {
    const unsigned long long Z = scan[cur][255];
    target = (unsigned long long)((double)Z * (double)top_p[b]);
    base = 0ull;
  } else {
    target = __hip_atomic_load(&st[b].target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    base = __hip_atomic_load(&st[b].above, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tot != 0ull && base + incl >= target) atomicMin(sh_sel, tid);
  __syncthreads();
  if (tid == (*sh_sel == 256 ? 255 : *sh_sel)) {
    if (LEVEL == 0) {
      __hip_atomic_store(&st[b].target, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&st[b].above, incl - tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&st[b].bstar, (uint32_t)tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint32_t bstar = __hip_atomic_load(&st[b].bstar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&st[b].fstar, (bstar << 8) | (uint32_t)tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// passes 2 (LEVEL 0: coarse bins f >> 8 over every token) and 3 (LEVEL 1: fine bins f & 255 of the
// tokens in coarse bin b*).  ws: [B][gridDim.x][256] u64 partial histograms.  exp_out (vocab-parallel
// sampling): the last arriver writes this rank's bin totals to exp_out[b][256] instead of selecting --
// nuc_scan_kernel selects from the sum over the ranks (integer masses: the same totals as a gathered row).
template <int LEVEL>
__global__ void __launch_bounds__(ST) nuc_hist_kernel(const float* __restrict__ logits, int B, int Vs, int shards,
                                                      const float* __restrict__ temperature,
                                                      const float* __restrict__ top_p, const int* __restrict__ ctx_inc,
                                                      const int* __restrict__ slots, NucRow* __restrict__ st,
                                                      unsigned long long* __restrict__ ws,
                                                      unsigned long long* __restrict__ exp_out) {
  __shared__ unsigned long long h[ST / 64][256];   // one histogram per wave: 4x fewer colliding atomics
  __shared__ unsigned long long scan[2][256];
  __shared__ uint32_t sh_prev;
  __shared__ int sh_sel;
  const int b = blockIdx.y;
  if (!nuc_row(b, ctx_inc, slots, temperature, top_p)) return;
  const int tid = threadIdx.x, wid = tid >> 6;
  const float invT = 1.f / temperature[b];
  const float M = key_float(__hip_atomic_load(&st[b].maxkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const uint32_t bstar = LEVEL == 1 ? __hip_atomic_load(&st[b].bstar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
#pragma unroll
  for (int w = 0; w < ST / 64; ++w) h[w][tid] = 0ull;
  __syncthreads();
  const Slice sl = slice_of(logits, b, B, Vs, shards, 0);
  for (int j = sl.j0 + tid; j < sl.j1; j += ST) {
    const float l = sl.base[j];
    const int f = nuc_fine(l, M, invT);
    if (f == NUC_NONE) continue;
    if (LEVEL == 1 && (uint32_t)(f >> 8) != bstar) continue;
    const unsigned long long m = nuc_mass(l, M, invT);
    if (m) atomicAdd(&h[wid][LEVEL == 0 ? (f >> 8) : (f & 255)], m);
  }
  __syncthreads();
  unsigned long long mine = 0ull;
#pragma unroll
  for (int w = 0; w < ST / 64; ++w) mine += h[w][tid];
  unsigned long long* row_ws = ws + (size_t)b * gridDim.x * 256;
  __hip_atomic_store(row_ws + (size_t)blockIdx.x * 256 + tid, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores land before the arrival
  __syncthreads();
  if (tid == 0) {
    uint32_t* cnt = LEVEL == 0 ? &st[b].cnt0 : &st[b].cnt1;
    sh_prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    sh_sel = 256;
  }
  __syncthreads();
  if (sh_prev != gridDim.x - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the arrival

  // last arriver: bin totals (thread = bin), inclusive scan, first bin where the target is reached
  // sc1 buffer loads (not atomics): independent, so all NB copies are in flight in one round trip
  unsigned long long tot = 0ull;
  {
    typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(row_ws, 0, 0x7fffffff, 0x00020000);
    constexpr int SC1 = 16;
    for (int w0 = 0; w0 < (int)gridDim.x; w0 += 16) {
      u32x2 v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        v[k] = w0 + k < (int)gridDim.x
                   ? __builtin_amdgcn_raw_buffer_load_b64(rs, ((w0 + k) * 256 + tid) * 8, 0, SC1)
                   : u32x2{0u, 0u};
#pragma unroll
      for (int k = 0; k < 16; ++k) tot += ((unsigned long long)v[k][1] << 32) | v[k][0];
    }
  }
  if (exp_out != nullptr) {
    exp_out[(size_t)b * 256 + tid] = tot;
    return;
  }
  nuc_select<LEVEL>(tot, b, top_p, st, scan, &sh_sel);
}

// ---- vocab-parallel sampling: the combine steps after a (tiny) all-gather over the TP ranks
// Row max: st[b].maxkey = max over the ranks' exported maxima g[r * ld + b]; this rank's export is re-armed to 0
// (the all-gather that read it has run: stream order).  One thread per row.
__global__ void __launch_bounds__(ST) nuc_import_max_kernel(const uint32_t* __restrict__ g, int ld, int ranks, int B,
                                                            const float* __restrict__ temperature,
                                                            const float* __restrict__ top_p,
                                                            const int* __restrict__ ctx_inc,
                                                            const int* __restrict__ slots, NucRow* __restrict__ st,
                                                            uint32_t* __restrict__ mine) {
  const int b = blockIdx.x * ST + threadIdx.x;
  if (b >= B) return;
  mine[b] = 0u;
  if (!nuc_row(b, ctx_inc, slots, temperature, top_p)) return;
  uint32_t m = 0u;
  for (int r = 0; r < ranks; ++r) m = max(m, g[(size_t)r * ld + b]);
  __hip_atomic_store(&st[b].maxkey, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Bin totals summed over the ranks' exports g[r][B][256] (grid B), then the selection of nuc_hist_kernel.
template <int LEVEL>
__global__ void __launch_bounds__(ST) nuc_scan_kernel(const unsigned long long* __restrict__ g, int ranks, int B,
                                                      const float* __restrict__ temperature,
                                                      const float* __restrict__ top_p, const int* __restrict__ ctx_inc,
                                                      const int* __restrict__ slots, NucRow* __restrict__ st) {
  __shared__ unsigned long long scan[2][256];
  __shared__ int sh_sel;
  const int b = blockIdx.x;
  if (!nuc_row(b, ctx_inc, slots, temperature, top_p)) return;
  unsigned long long tot = 0ull;
  for (int r = 0; r < ranks; ++r) tot += g[((size_t)r * B + b) * 256 + threadIdx.x];
  if (threadIdx.x == 0) sh_sel = 256;
  nuc_select<LEVEL>(tot, b, top_p, st, scan, &sh_sel);
}

// grid (nbx, B); row_key [B] u64 and row_cnt [B] u32 must be zero before the first launch (the
// last arriver of each row restores them).  nuc: the nucleus passes' row state, or null (top_p ignored).
__global__ void __launch_bounds__(ST) sample_kernel(int* __restrict__ tokens, const float* __restrict__ logits, int B,
                                                    int Vs, int shards, const float* __restrict__ temperature,
                                                    const float* __restrict__ top_p, const uint32_t* __restrict__ seeds,
                                                    const int* __restrict__ counter, int* __restrict__ ctx_inc,
                                                    int* __restrict__ hist, int hist_stride, int* __restrict__ steps,
                                                    unsigned long long* __restrict__ row_key,
                                                    uint32_t* __restrict__ row_cnt, NucRow* __restrict__ nuc,
                                                    const int* __restrict__ slots, StopArgs sa, int id_base,
                                                    unsigned long long* __restrict__ keys_out) {
  __shared__ float sv[ST / 64];
  __shared__ int si[ST / 64];
  const int b = blockIdx.y;
  const int s = slots != nullptr ? slots[b] : b;       // decode-state slot of this row
  if (ctx_inc != nullptr && ctx_inc[s] <= 0) return;  // padded (or finished) row
  const float T = temperature[b];
  const uint32_t seed = seeds[b];
  const uint32_t ctr = counter ? (uint32_t)counter[b] : 0u;
  const Slice sl = slice_of(logits, b, B, Vs, shards, id_base);
  ArgMax best{-INFINITY, 0x7fffffff};
  if (T <= 0.f) {
    for (int j = sl.j0 + threadIdx.x; j < sl.j1; j += ST) best = better(best, ArgMax{sl.base[j], sl.id0 + j});
  } else {
    const float invT = 1.f / T;
    const bool nucleus = nuc != nullptr && top_p[b] < 1.f;
    float M = 0.f;
    int fstar = NUC_NONE;
    if (nucleus) {
      M = key_float(__hip_atomic_load(&nuc[b].maxkey, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      fstar = (int)__hip_atomic_load(&nuc[b].fstar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    for (int j = sl.j0 + threadIdx.x; j < sl.j1; j += ST) {
      const float l = sl.base[j];
      if (nucleus && nuc_fine(l, M, invT) > fstar) continue;
      const int v = sl.id0 + j;
      const float u = u01(hash3(seed, ctr, (uint32_t)v));
      best = better(best, ArgMax{l * invT - __logf(-__logf(u)), v});
    }
  }
  best = block_argmax(best, sv, si);
  if (threadIdx.x == 0) {
    if (best.i != 0x7fffffff)
      __hip_atomic_fetch_max(&row_key[b], pack_key(best.v, best.i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the max lands before the arrival is counted
    const uint32_t arrived = __hip_atomic_fetch_add(&row_cnt[b], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (arrived == gridDim.x - 1) {  // last arriver: every other workgroup's max is already folded in
      const unsigned long long k = __hip_atomic_load(&row_key[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&row_key[b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&row_cnt[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (nuc != nullptr && T > 0.f && top_p[b] < 1.f) {   // re-arm the nucleus row state (every
        NucRow* w = nuc + b;                                // other workgroup has read it already)
        __hip_atomic_store(&w->maxkey, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&w->cnt0, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&w->cnt1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (keys_out != nullptr) {   // vocab-parallel: this rank's best key; sample_merge_kernel picks over the ranks
        keys_out[b] = k;
      } else {
        write_token(s, (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)), tokens, ctx_inc, hist, hist_stride, steps,
                    sa);
      }
    }
  }
}

// Vocab-parallel sampling, last step: the row's token is the best of the ranks' keys g[r * ld + b] (packed
// score | ~global id: the same maximum as one pass over the gathered logits, ties to the lowest id), then the
// decode-state update of sample_kernel.  Every rank runs it on the same gathered keys: the same token everywhere.
__global__ void __launch_bounds__(64) sample_merge_kernel(int* __restrict__ tokens,
                                                          const unsigned long long* __restrict__ g, int ld, int ranks,
                                                          int B, int* __restrict__ ctx_inc, int* __restrict__ hist,
                                                          int hist_stride, int* __restrict__ steps,
                                                          const int* __restrict__ slots, StopArgs sa) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  const int s = slots != nullptr ? slots[b] : b;
  if (ctx_inc != nullptr && ctx_inc[s] <= 0) return;
  unsigned long long k = 0ull;
  for (int r = 0; r < ranks; ++r) k = max(k, g[(size_t)r * ld + b]);
  write_token(s, (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull)), tokens, ctx_inc, hist, hist_stride, steps, sa);
}

__host__ __device__ inline int grid_x(int shards) { return shards * ((NB + shards - 1) / shards); }

}  // namespace k8sllm

using namespace k8sllm;

// Scratch layouts do not depend on B, so one buffer serves every batch size (decode graph buckets,
// prefill rows, speculative verify rows) in any order:
//   scratch:     row_key [SAMPLE_ROW_CAP] u64 | row_cnt [SAMPLE_ROW_CAP] u32 -- zero-initialised, owned by
//                the caller (one per concurrently captured sampler), restored to zero by every launch.
//   nuc_scratch: (or null: top_p ignored) NucRow [SAMPLE_ROW_CAP] | histograms [B][grid][256] u64 --
//                the row states zero before the first call and left zero; the histograms are fully
//                rewritten by every launch before they are read.
constexpr int SAMPLE_ROW_CAP = 4096;

static bool make_stop_args(StopArgs& sa, const int* cls, int* json, const int* cfg, const int* forced,
                           const int* forced_len, int fstride, int eos_tok, int* done, const int* hist,
                           const int* ctx_inc) {
  sa.cls = reinterpret_cast<const int2*>(cls);
  sa.json = json;
  sa.cfg = cfg;
  sa.forced = forced;
  sa.forced_len = forced_len;
  sa.fstride = fstride;
  sa.eos_tok = eos_tok;
  sa.done = done;
  return !(sa.cls != nullptr && (sa.json == nullptr || sa.cfg == nullptr || hist == nullptr || ctx_inc == nullptr ||
                                 (sa.forced != nullptr && sa.forced_len == nullptr)));
}
// slots (or null): decode-state slot of every row (tokens / ctx_inc / hist / steps / stop state are indexed by
// slot; temperature / top_p / seeds / counter by row).  stop_*: device-side stop detection (null cls = off).
extern "C" int k8s_sample(int* tokens, const float* logits, int B, int Vs, int shards, const float* temperature,
                          const float* top_p, const uint32_t* seeds, const int* counter, int* ctx_inc, int* hist,
                          int hist_stride, int* steps, void* scratch, void* nuc_scratch, const int* slots,
                          const int* stop_cls, int* stop_json, const int* stop_cfg, const int* stop_forced,
                          const int* stop_forced_len, int stop_fstride, int stop_eos_tok, int* stop_done,
                          int id_base, void* keys_out, int nuc_passes, hipStream_t stream) {
  if (B <= 0) return 0;
  if (B > SAMPLE_ROW_CAP) return -2;
  if (hist != nullptr && steps == nullptr) return -1;
  if (scratch == nullptr) return -3;
  if (shards < 1 || Vs < 1) return -2;
  auto* key = static_cast<unsigned long long*>(scratch);
  auto* cnt = reinterpret_cast<uint32_t*>(key + SAMPLE_ROW_CAP);
  const dim3 grid(grid_x(shards), B);
  NucRow* st = nullptr;
  if (nuc_scratch != nullptr) {
    st = static_cast<NucRow*>(nuc_scratch);
    auto* ws = reinterpret_cast<unsigned long long*>(st + SAMPLE_ROW_CAP);
    if (nuc_passes) {   // (vocab-parallel sampling runs them itself, with its combine steps between)
      nuc_max_kernel<<<grid, ST, 0, stream>>>(logits, B, Vs, shards, temperature, top_p, ctx_inc, slots, &st->maxkey,
                                              (int)(sizeof(NucRow) / sizeof(uint32_t)));
      nuc_hist_kernel<0><<<grid, ST, 0, stream>>>(logits, B, Vs, shards, temperature, top_p, ctx_inc, slots, st, ws,
                                                  nullptr);
      nuc_hist_kernel<1><<<grid, ST, 0, stream>>>(logits, B, Vs, shards, temperature, top_p, ctx_inc, slots, st, ws,
                                                  nullptr);
    }
  }
  StopArgs sa;
  if (!make_stop_args(sa, stop_cls, stop_json, stop_cfg, stop_forced, stop_forced_len, stop_fstride, stop_eos_tok,
                      stop_done, hist, ctx_inc))
    return -1;
  sample_kernel<<<grid, ST, 0, stream>>>(tokens, logits, B, Vs, shards, temperature, top_p, seeds, counter, ctx_inc,
                                         hist, hist_stride, steps, key, cnt, st, slots, sa, id_base,
                                         static_cast<unsigned long long*>(keys_out));
  return (int)hipGetLastError();
}

// Vocab-parallel sampling (each TP rank samples its own vocabulary shard; rows exchange a few bytes instead of
// their logits).  Per call, on the local shard [B][Vs] (shards = 1, global ids from id_base):
//   nucleus rows only:  local(-1) -> all-gather u32 [B] -> combine(-1)        (row max)
//                       local(0)  -> all-gather u64 [B][256] -> combine(0)    (coarse bin b*)
//                       local(1)  -> all-gather u64 [B][256] -> combine(1)    (fine bin f*)
//   every row:          k8s_sample(keys_out, nuc_passes = 0) -> all-gather u64 [B] -> k8s_sample_merge
// local: level -1 writes this rank's row maxima to out (u32 [B], zero before the call: combine(-1) re-arms it);
// levels 0 / 1 this rank's bin totals to out (u64 [B][256]).
extern "C" int k8s_sample_nuc_local(int level, const float* logits, int B, int Vs, const float* temperature,
                                    const float* top_p, const int* ctx_inc, const int* slots, void* nuc_scratch,
                                    void* out, hipStream_t stream) {
  if (B <= 0) return 0;
  if (B > SAMPLE_ROW_CAP || Vs < 1 || nuc_scratch == nullptr || out == nullptr) return -2;
  auto* st = static_cast<NucRow*>(nuc_scratch);
  auto* ws = reinterpret_cast<unsigned long long*>(st + SAMPLE_ROW_CAP);
  const dim3 grid(grid_x(1), B);
  auto* o64 = static_cast<unsigned long long*>(out);
  if (level < 0)
    nuc_max_kernel<<<grid, ST, 0, stream>>>(logits, B, Vs, 1, temperature, top_p, ctx_inc, slots,
                                            static_cast<uint32_t*>(out), 1);
  else if (level == 0)
    nuc_hist_kernel<0><<<grid, ST, 0, stream>>>(logits, B, Vs, 1, temperature, top_p, ctx_inc, slots, st, ws, o64);
  else
    nuc_hist_kernel<1><<<grid, ST, 0, stream>>>(logits, B, Vs, 1, temperature, top_p, ctx_inc, slots, st, ws, o64);
  return (int)hipGetLastError();
}

// combine: g = the all-gathered exports ([ranks][ld] u32 for level -1, with mine = this rank's export to re-arm;
// [ranks][B][256] u64 for levels 0 / 1).
extern "C" int k8s_sample_nuc_combine(int level, const void* g, int ld, int ranks, int B, const float* temperature,
                                      const float* top_p, const int* ctx_inc, const int* slots, void* nuc_scratch,
                                      void* mine, hipStream_t stream) {
  if (B <= 0) return 0;
  if (B > SAMPLE_ROW_CAP || ranks < 1 || nuc_scratch == nullptr || g == nullptr) return -2;
  auto* st = static_cast<NucRow*>(nuc_scratch);
  if (level < 0) {
    if (mine == nullptr || ld < B) return -2;
    nuc_import_max_kernel<<<(B + ST - 1) / ST, ST, 0, stream>>>(static_cast<const uint32_t*>(g), ld, ranks, B,
                                                                temperature, top_p, ctx_inc, slots, st,
                                                                static_cast<uint32_t*>(mine));
  } else if (level == 0) {
    nuc_scan_kernel<0><<<B, ST, 0, stream>>>(static_cast<const unsigned long long*>(g), ranks, B, temperature, top_p,
                                             ctx_inc, slots, st);
  } else {
    nuc_scan_kernel<1><<<B, ST, 0, stream>>>(static_cast<const unsigned long long*>(g), ranks, B, temperature, top_p,
                                             ctx_inc, slots, st);
  }
  return (int)hipGetLastError();
}

// merge: g = the all-gathered keys [ranks][ld] u64 (k8s_sample's keys_out of every rank); the decode-state update and
// stop detection of k8s_sample.
extern "C" int k8s_sample_merge(int* tokens, const void* g, int ld, int ranks, int B, int* ctx_inc, int* hist,
                                int hist_stride, int* steps, const int* slots, const int* stop_cls, int* stop_json,
                                const int* stop_cfg, const int* stop_forced, const int* stop_forced_len,
                                int stop_fstride, int stop_eos_tok, int* stop_done, hipStream_t stream) {
  if (B <= 0) return 0;
  if (ld < B || ranks < 1 || g == nullptr) return -2;
  if (hist != nullptr && steps == nullptr) return -1;
  StopArgs sa;
  if (!make_stop_args(sa, stop_cls, stop_json, stop_cfg, stop_forced, stop_forced_len, stop_fstride, stop_eos_tok,
                      stop_done, hist, ctx_inc))
    return -1;
  sample_merge_kernel<<<(B + 63) / 64, 64, 0, stream>>>(tokens, static_cast<const unsigned long long*>(g), ld, ranks,
                                                          B, ctx_inc, hist, hist_stride, steps, slots, sa);
  return (int)hipGetLastError();
}

extern "C" long long k8s_sample_scratch_bytes(int B) {
  (void)B;
  return (long long)SAMPLE_ROW_CAP * 12;
}

extern "C" long long k8s_sample_nucleus_bytes(int B, int shards) {
  if (B <= 0 || shards < 1) return 0;
  return (long long)SAMPLE_ROW_CAP * (long long)sizeof(NucRow) + (long long)B * grid_x(shards) * 256 * 8;
}
