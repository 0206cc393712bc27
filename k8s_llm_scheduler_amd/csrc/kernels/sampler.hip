// K13 + K17: sampling over a (possibly vocab-sharded) fp32 logits buffer, fused with the
// decode-state update so a whole decode step can be replayed from a hipGraph.
//
// Logits layout: [shards][B][Vs]; token id v = shard * Vs + j (vocab-parallel LM head output
// after an all-gather, or a single shard).  Per row b:
//   temperature <= 0       -> greedy argmax (lowest index wins ties, like torch.argmax)
//   top_p >= 1             -> Gumbel-max: argmax(l / T + G), G = -log(-log(U)), one pass
//   0 < top_p < 1          -> nucleus: exact logit threshold by a 4 x 8-bit radix select on
//                             probability MASS (no sort), then Gumbel-max inside the nucleus.
// U comes from a counter-based hash of (seed[b], counter[b], token) so results do not depend on
// batch composition or on which rank samples (every TP rank draws the same token).
// After sampling: tokens[b] = tok; hist[b][steps[b]] = tok; steps[b]++; ctx[b]++ (optional).
//
// Work split: the per-token work (a hash and two logs for Gumbel) over a 128k vocabulary is
// compute-bound on one CU (~70 us), so greedy / Gumbel rows spread the vocabulary over NB
// workgroups: each reduces its slice to one packed 64-bit key (ord(score) << 32 | ~index, so the
// max key is the best score with the LOWEST index), folds it into a per-row atomicMax, and the
// workgroup whose arrival-counter add comes last finalizes the row (agent-scope atomics only:
// the payload is the atomic itself, the last arriver reads it with an agent-scope load) and
// re-arms the row's key and counter for the next graph replay.  Nucleus rows (top_p < 1) need a
// global mass histogram and stay on workgroup 0 of their row with the radix-select path.
#include "common.h"

namespace k8sllm {

constexpr int ST = 256;   // threads per workgroup
constexpr int NB = 32;    // workgroups per row (greedy / Gumbel)

__device__ __forceinline__ uint32_t ord_key(float f) {  // monotone float -> uint32
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
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

__device__ __forceinline__ void write_token(int b, int tok, int* __restrict__ tokens, int* __restrict__ ctx_inc,
                                            int* __restrict__ hist, int hist_stride, int* __restrict__ steps) {
  tokens[b] = tok;
  if (hist != nullptr) {
    const int st = steps[b];
    if (st < hist_stride) hist[(size_t)b * hist_stride + st] = tok;
    steps[b] = st + 1;
  }
  if (ctx_inc != nullptr) ctx_inc[b] += 1;
}

// grid (NB, B); row_key [B] u64 and row_cnt [B] u32 must be zero before the first launch (the
// last arriver of each row restores them).
__global__ void __launch_bounds__(ST) sample_kernel(int* __restrict__ tokens, const float* __restrict__ logits, int B,
                                                    int Vs, int shards, const float* __restrict__ temperature,
                                                    const float* __restrict__ top_p, const uint32_t* __restrict__ seeds,
                                                    const int* __restrict__ counter, int* __restrict__ ctx_inc,
                                                    int* __restrict__ hist, int hist_stride, int* __restrict__ steps,
                                                    unsigned long long* __restrict__ row_key,
                                                    uint32_t* __restrict__ row_cnt) {
  __shared__ float sv[ST / 64];
  __shared__ int si[ST / 64];
  __shared__ unsigned long long hist_mass[256];
  __shared__ unsigned long long sh_z;
  __shared__ uint32_t sh_prefix;
  __shared__ unsigned long long sh_above;
  const int b = blockIdx.y, part = blockIdx.x;
  if (ctx_inc != nullptr && ctx_inc[b] <= 0) return;  // padded row
  const int V = Vs * shards;
  const float T = temperature[b];
  const float P = top_p[b];
  const uint32_t seed = seeds[b];
  const uint32_t ctr = counter ? (uint32_t)counter[b] : 0u;
  auto L = [&](int v) -> float {
    const int s = v / Vs, j = v - s * Vs;
    return logits[((size_t)s * B + b) * Vs + j];
  };

  if (T > 0.f && P < 1.f) {  // ---- nucleus: exact mass threshold (radix select), one workgroup
    if (part != 0) return;
    const float invT = 1.f / T;
    ArgMax mx{-INFINITY, 0};
    for (int v = threadIdx.x; v < V; v += ST) mx = better(mx, ArgMax{L(v), v});
    mx = block_argmax(mx, sv, si);
    const float M = mx.v;
    // Probability mass in 2^-40 fixed point, summed with INTEGER atomics: the histogram, the total
    // and hence the threshold do not depend on the order the adds land in, so every TP rank (same
    // logits) picks the same nucleus and the same token.
    auto mass = [&](float l) -> unsigned long long {
      return (unsigned long long)(__expf((l - M) * invT) * 1099511627776.0f);
    };
    if (threadIdx.x == 0) sh_z = 0ull;
    __syncthreads();
    unsigned long long zl = 0ull;
    for (int v = threadIdx.x; v < V; v += ST) zl += mass(L(v));
    atomicAdd(&sh_z, zl);
    __syncthreads();
    const unsigned long long target = (unsigned long long)((double)sh_z * (double)P);
    uint32_t prefix = 0;
    unsigned long long above = 0ull;  // mass of tokens strictly above the current prefix bucket
    for (int round = 0; round < 4; ++round) {
      const int shift = 24 - 8 * round;
      for (int i = threadIdx.x; i < 256; i += ST) hist_mass[i] = 0ull;
      __syncthreads();
      for (int v = threadIdx.x; v < V; v += ST) {
        const float l = L(v);
        const uint32_t k = ord_key(l);
        const bool match = round == 0 || (k >> (shift + 8)) == (prefix >> (shift + 8));
        if (match) atomicAdd(&hist_mass[(k >> shift) & 255], mass(l));
      }
      __syncthreads();
      if (threadIdx.x == 0) {
        unsigned long long cum = above;
        int bsel = 0;
        for (int bk = 255; bk >= 0; --bk) {
          if (cum + hist_mass[bk] >= target || bk == 0) { bsel = bk; break; }
          cum += hist_mass[bk];
        }
        sh_prefix = prefix | ((uint32_t)bsel << shift);
        sh_above = cum;
      }
      __syncthreads();
      prefix = sh_prefix;
      above = sh_above;
      __syncthreads();
    }
    const uint32_t kthr = prefix;  // include tokens whose ord_key >= kthr
    ArgMax best{-INFINITY, 0x7fffffff};
    for (int v = threadIdx.x; v < V; v += ST) {
      const float l = L(v);
      if (ord_key(l) < kthr) continue;
      const float u = u01(hash3(seed, ctr, (uint32_t)v));
      best = better(best, ArgMax{l * invT - __logf(-__logf(u)), v});
    }
    best = block_argmax(best, sv, si);
    if (threadIdx.x == 0) write_token(b, best.i, tokens, ctx_inc, hist, hist_stride, steps);
    return;
  }

  // ---- greedy / Gumbel-max over this workgroup's vocabulary slice
  const int per = (V + gridDim.x - 1) / gridDim.x;
  const int v0 = part * per, v1 = min(V, v0 + per);
  ArgMax best{-INFINITY, 0x7fffffff};
  if (T <= 0.f) {
    for (int v = v0 + threadIdx.x; v < v1; v += ST) best = better(best, ArgMax{L(v), v});
  } else {
    const float invT = 1.f / T;
    for (int v = v0 + threadIdx.x; v < v1; v += ST) {
      const float u = u01(hash3(seed, ctr, (uint32_t)v));
      best = better(best, ArgMax{L(v) * invT - __logf(-__logf(u)), v});
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
      const int tok = (int)(0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull));
      __hip_atomic_store(&row_key[b], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&row_cnt[b], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      write_token(b, tok, tokens, ctx_inc, hist, hist_stride, steps);
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

// row_key [B] u64 + row_cnt [B] u32: zero-initialised scratch owned by the caller (one per
// concurrently captured sampler), restored to zero by every launch.
extern "C" int k8s_sample(int* tokens, const float* logits, int B, int Vs, int shards, const float* temperature,
                          const float* top_p, const uint32_t* seeds, const int* counter, int* ctx_inc, int* hist,
                          int hist_stride, int* steps, void* scratch, hipStream_t stream) {
  if (B <= 0) return 0;
  if (hist != nullptr && steps == nullptr) return -1;
  if (scratch == nullptr) return -3;
  auto* key = static_cast<unsigned long long*>(scratch);
  auto* cnt = reinterpret_cast<uint32_t*>(key + B);
  dim3 grid(NB, B);
  sample_kernel<<<grid, ST, 0, stream>>>(tokens, logits, B, Vs, shards, temperature, top_p, seeds, counter, ctx_inc,
                                         hist, hist_stride, steps, key, cnt);
  return (int)hipGetLastError();
}

extern "C" long long k8s_sample_scratch_bytes(int B) { return (long long)B * 12; }
