// Layer-persistent decode (VERDICT r4 "next round" item 1; SURVEY K2-K11 of the per-token hot loop): every decoder
// layer of a decode step in ONE launch, for TP = 1 and for one simulated TP rank (collectives skipped).
//
// Why: at one TP = 8 rank's shapes a decode layer streams 214 MB of weights (34 us at 6.3 TB/s) but took 52 us as
// four GEMV launches + split attention: HBM idles while attention runs (8 us on ~270 KB of KV) and every small
// projection pays its own ramp.  Weights do not depend on activations, so here they never wait for them:
//
//  * one 512-thread workgroup per CU (grid = CU count, ~>80 KiB of LDS so no CU takes two);
//  * waves 1..7 ("streamers") stream this CU's slice of every projection of every layer, in order, as 1 KiB
//    pieces (16 B per lane, non-temporal) into a REGISTER ring of RS pieces per wave that is refilled the moment a
//    piece is consumed -- RS x 7 KiB per CU in flight or landed at any time, independent of what the activations do.
//    A streamer that reaches a phase whose input is not ready yet parks on an LDS word while its ring fills up;
//  * wave 0 (the "chain" wave) carries the dependencies: it reduces the streamers' per-row partials (fixed order,
//    deterministic), applies the epilogue (1/rms, SwiGLU, residual add), publishes the CU's output rows as 8-byte
//    data-tagged granules {2 x bf16, epoch} (one sc1 store each: readers poll the data itself, no flags, no fences;
//    MI355X_MICROARCH.md visibility table / R2), gathers the next phase's whole input vector from every CU's
//    granules into LDS (with the RMS statistics where the next projection is pre-norm) and releases the streamers;
//  * attention (RoPE + paged-KV write + GQA, one wave per 64-token chunk, in-launch merge of the chunk partials by
//    the last arriver, as attn_decode_split.hip) runs on the chain waves of a few workgroups while every streamer
//    keeps loading W_o and W_gate_up behind it.
//
// Row ownership: CU c owns row PAIRS [c P / G, (c + 1) P / G) of every projection (P = rows / 2), so each granule
// has one writer.  Gate/up: the gate and up rows of the same pairs (SwiGLU is CU-local).  Pieces of a phase are
// dealt round-robin to the streamers; a wave's pieces of one row are consecutive in its sequence, so each
// (wave, row) partial is written once per phase and the chain wave sums the 7 waves in wave order.
//
// Epochs: every workgroup reads sync[0] at launch; the last workgroup to finish (sync[32] ticket) increments it,
// so each launch's granules carry a fresh tag and a graph replays without any host involvement.  Granule buffers
// are per (layer, hand-off): a tag is written once per launch.  Every wait is bounded (s_memrealtime); a timeout
// sets a bit of sync[64] and an abort word that lets the whole grid drain.
//
// Numerics: fp32 accumulation everywhere; outputs rounded to bf16 once (the residual adds of O / down round the sum
// x + branch once, as the TP > 1 path's all-reduce epilogue does).
#include "common.h"

namespace k8sllm {

namespace {

constexpr int PD_NS = 7;                  // streamer waves per workgroup
constexpr int PD_NT = 64 * (PD_NS + 1);   // + the chain wave (wave 0)
constexpr int PD_RMAX = 128;              // rows of one projection per workgroup (per-wave partials in LDS)
constexpr int PD_SC1 = 16;                // buffer-op aux: sc1 (L1 bypass)
constexpr int PD_NTL = 2;                 // buffer-op aux: nt (weights are read once)
constexpr float PD_LOG2E = 1.4426950408889634f;
// chain-wave trace points per layer: 0 QKV done, 1 attention items done, 2 attention output gathered, 3 O done,
// 4 o gathered, 5 gate/up done, 6 g gathered, 7 down done, 8 next x gathered; 9-12 QKV / O / gate-up / down rows
// published (this workgroup's granule stores issued)
constexpr int PD_TRACE_PTS = 13;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4_pd_t;

struct PdLayer {
  const bf16_t* w[4];   // qkv [Nqkv, H], o [H, nq D], gate_up [2 I, H], down [H, I]
  bf16_t* kc;           // this layer's caches [slots, nkv, D]
  bf16_t* vc;
};

}  // namespace

struct PdArgs {
  const PdLayer* layers;
  const bf16_t* x0;       // [M, H] layer-0 residual stream (embedding output)
  bf16_t* xout;           // [M, H] final residual stream
  const float* cos_sin;
  const int* block_tables;
  const int* context_lens;
  u32x2* gran;            // [L][M][gl] granules
  float* part;            // attention chunk partials [M nkv][pmax][G D + 2 G]
  uint32_t* counters;     // [M nkv] arrival counters (zero between launches)
  uint32_t* sync;         // [0] epoch (>= 1), [32] finish ticket, [64] error bits
  unsigned long long* trace;   // optional: [grid][L][PD_TRACE_PTS] s_memrealtime stamps of the chain waves
  long long timeout_ticks;
  float eps, scale;
  int L, H, nq, nkv, I, max_blocks, pmax, gl;
  int off_resid, off_xin, off_red, off_att, off_ctl;   // LDS layout (bytes)
};

namespace {

__device__ __forceinline__ __amdgpu_buffer_rsrc_t pd_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ float pd_silu(float g) { return g / (1.f + __expf(-g)); }
__device__ __forceinline__ int pd_swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// LDS control words (chain wave <-> streamers of one workgroup)
struct PdCtl {
  uint32_t ready;    // phases whose input is in LDS (phase s is ready when ready > s)
  uint32_t pdone;    // streamer-phase completions (phase s is done when pdone >= NS (s + 1))
  uint32_t abort;    // a wait timed out somewhere in this workgroup: every later wait returns at once
  uint32_t tag;      // this launch's epoch
};

__device__ __forceinline__ uint32_t lds_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Bounded wait for an LDS word to reach `want` (s_sleep between polls keeps issue slots free).  A timeout sets the
// workgroup's abort word (bits: 1 streamer wait, 4 chain wait); the chain wave reports it in sync[64] at the end.
// No vector-memory instruction here: a streamer's only ones are its ring loads (see pd_streamer).
__device__ __forceinline__ void pd_wait_lds(const uint32_t* word, uint32_t want, PdCtl* ctl, const PdArgs& a,
                                           uint32_t errbit) {
  if (lds_ld(word) < want) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (lds_ld(word) < want) {
      if (lds_ld(&ctl->abort)) break;
      __builtin_amdgcn_s_sleep(1);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
        __hip_atomic_fetch_or(&ctl->abort, errbit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
    }
  }
  // the LDS data the word releases is read only after it: the loop's exit depends on the word's value (LDS is one
  // ordered structure per CU), and this keeps the compiler from hoisting those reads above the (relaxed) poll
  asm volatile("" ::: "memory");
}

// This workgroup's share of one projection -- the same in every layer (only the weight base differs).
struct PdGeo {
  int r0;         // first output row (2 x first pair)
  int nrows;      // output rows (gate/up: gate rows = up rows = output rows)
  int ppr;        // 1 KiB pieces per weight row (K / 512)
  int p0;         // pieces of the first region (gate/up: the gate rows)
  int P;          // pieces of the phase
  long long off0;     // byte offset of region 0 from the layer's weight
  long long off1m;    // byte offset of region 1 (the up rows) minus p0 pieces
};

__device__ __forceinline__ PdGeo pd_geo(const PdArgs& a, int ph, int c, int G) {
  const int D = 128, nqD = a.nq * D, nqkv = (a.nq + 2 * a.nkv) * D;
  int K, pairs;
  if (ph == 0) { K = a.H; pairs = nqkv >> 1; }
  else if (ph == 1) { K = nqD; pairs = a.H >> 1; }
  else if (ph == 2) { K = a.H; pairs = a.I >> 1; }
  else { K = a.I; pairs = a.H >> 1; }
  const int q0 = (c * pairs) / G, q1 = ((c + 1) * pairs) / G;
  PdGeo g;
  g.r0 = 2 * q0;
  g.nrows = 2 * (q1 - q0);
  g.ppr = K >> 9;
  g.p0 = g.nrows * g.ppr;
  g.off0 = (long long)g.r0 * K * 2;
  if (ph == 2) {
    g.off1m = (long long)(a.I + g.r0) * K * 2 - (long long)g.p0 * 1024;
    g.P = 2 * g.p0;
  } else {
    g.off1m = g.off0;
    g.P = g.p0;
  }
  return g;
}

__device__ __forceinline__ int pd_count(int P, int s) { return P > s ? (P - s + PD_NS - 1) / PD_NS : 0; }

template <typename T>
__device__ __forceinline__ T pd_sel(int ph, T v0, T v1, T v2, T v3) {
  return ph == 0 ? v0 : (ph == 1 ? v1 : (ph == 2 ? v2 : v3));
}

// ------------------------------------------------------------------------------------------------ streamers
// Streamer s (0..6) of a workgroup: its pieces of phase (l, ph) are p = s, s + 7, s + 14, ... < P; every value here
// is wave-uniform (SGPRs), the weights go straight to a register ring w[RS] (one 16-byte load per lane per piece).
template <int M, int RS>
__device__ __forceinline__ void pd_streamer(const PdArgs& a, char* lds, int s, const PdGeo (&geo)[4]) {
  const int lane = threadIdx.x & 63;
  PdCtl* ctl = reinterpret_cast<PdCtl*>(lds + a.off_ctl);
  const char* resid = lds + a.off_resid;
  const char* xin = lds + a.off_xin;
  float* red = reinterpret_cast<float*>(lds + a.off_red);   // [NS][M][RMAX]
  const int KX = max(a.nq * 128, a.I);
  const int L = a.L;
  const int cnt0 = pd_count(geo[0].P, s), cnt1 = pd_count(geo[1].P, s), cnt2 = pd_count(geo[2].P, s),
            cnt3 = pd_count(geo[3].P, s);

  // ---- issue cursor
  int il = 0, iph = 0, ip = s, ileft = cnt0, ip0 = geo[0].p0;
  const char* ib0 = reinterpret_cast<const char*>(a.layers[0].w[0]) + geo[0].off0;
  const char* ib1 = ib0;
  const char* ilast = ib0;
  auto iseek = [&]() {
    while (ileft == 0 && il < L) {
      if (++iph == 4) { iph = 0; ++il; }
      if (il < L) {
        const char* w = reinterpret_cast<const char*>(a.layers[il].w[iph]);
        ib0 = w + pd_sel(iph, geo[0].off0, geo[1].off0, geo[2].off0, geo[3].off0);
        ib1 = w + pd_sel(iph, geo[0].off1m, geo[1].off1m, geo[2].off1m, geo[3].off1m);
        ip0 = pd_sel(iph, geo[0].p0, geo[1].p0, geo[2].p0, geo[3].p0);
        ileft = pd_sel(iph, cnt0, cnt1, cnt2, cnt3);
        ip = s;
      }
    }
  };
  auto inext = [&]() -> const char* {   // the next piece's address (the last one again once the stream is done)
    if (il < L) {
      ilast = (ip < ip0 ? ib0 : ib1) + (size_t)ip * 1024;
      ip += PD_NS;
      --ileft;
      iseek();
    }
    return ilast;
  };
  iseek();

  u32x4 w[RS];
#pragma unroll
  for (int j = 0; j < RS; ++j) w[j] = __builtin_amdgcn_raw_buffer_load_b128(pd_rsrc(inext()), lane * 16, 0, PD_NTL);

  // ---- consume cursor
  int l = 0, ph = 0, left = 0, row = 0, part = 0, ppr = 1;
  bool started = false;     // the current phase's input is ready and its cursor is set
  const char* xb = resid;
  int xstride = a.H * 2;
  float acc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = 0.f;

  auto enter = [&]() {      // wait for phase (l, ph)'s input; a phase without pieces of this wave is done at once
    while (l < L) {
      pd_wait_lds(&ctl->ready, 4u * l + ph + 1, ctl, a, 1u);
      left = pd_sel(ph, cnt0, cnt1, cnt2, cnt3);
      if (left > 0) break;
      if (lane == 0) __hip_atomic_fetch_add(&ctl->pdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (++ph == 4) { ph = 0; ++l; }
    }
    ppr = pd_sel(ph, geo[0].ppr, geo[1].ppr, geo[2].ppr, geo[3].ppr);
    row = s / ppr;
    part = s - row * ppr;
    const bool in_resid = (ph == 0 || ph == 2);
    xb = in_resid ? resid : xin;
    xstride = in_resid ? a.H * 2 : KX * 2;
    started = true;
  };
  auto flush = [&](int r) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float v = wave_sum(acc[m]);
      if (lane == 0) red[(s * M + m) * PD_RMAX + r] = v;
      acc[m] = 0.f;
    }
  };

  // Every step issues exactly ONE load (the refill is unconditional, and no other vector-memory instruction is ever
  // issued by a streamer), so the compiler's counted waits stay at vmcnt(RS) for every slot of the unrolled ring.
  while (l < L) {
#pragma unroll
    for (int j = 0; j < RS; ++j) {
      if (!started && l < L) enter();
      const bool live = l < L;
      if (live) {
        // piece of row `row`, 512-element part `part` of phase (l, ph)
        const u32x4 wv = w[j];
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const u32x4 xv = *reinterpret_cast<const u32x4*>(xb + m * xstride + ((part << 6) + lane) * 16);
          float t = acc[m];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            t = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, (uint32_t)wv[e]),
                                                 __builtin_bit_cast(bf16x2, (uint32_t)xv[e]), t, false);
          acc[m] = t;
        }
      }
      // refill the slot: the stream runs ahead of the consumer by RS pieces, whatever the phase dependencies
      w[j] = __builtin_amdgcn_raw_buffer_load_b128(pd_rsrc(inext()), lane * 16, 0, PD_NTL);
      if (live) {
        const int prow = row;
        part += PD_NS;
        while (part >= ppr) { part -= ppr; ++row; }
        if (--left == 0) {   // this wave's last piece of the phase
          flush(prow);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // partials stored and x reads done
          if (lane == 0) __hip_atomic_fetch_add(&ctl->pdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          started = false;
          if (++ph == 4) { ph = 0; ++l; }
        } else if (row != prow) {
          flush(prow);
        }
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------ chain wave
// Gather n4 groups of 4 bf16 into dst (LDS, contiguous): group i is the 16-byte pair of granules at byte offset
// srcoff(i) of the hand-off buffer `src` (sc1 loads: the L1 never holds another CU's data).  Every lane keeps up to B
// loads in flight and re-polls ALL its not-yet-published granules together, so a gather ends one round trip after
// its last producer.  Bounded; returns the lane's sum of squares of the gathered values when SS.
template <bool SS, int B, typename F>
__device__ __forceinline__ float pd_gather(const u32x2* src, char* dst, int n4, F srcoff, uint32_t tag, PdCtl* ctl,
                                           const PdArgs& a) {
  const int lane = threadIdx.x & 63;
  const auto rs = pd_rsrc(src);
  float ss = 0.f;
  for (int i0 = 0; i0 < n4; i0 += 64 * B) {
    u32x4 v[B];
    uint32_t pend = 0;
#pragma unroll
    for (int u = 0; u < B; ++u) {
      const int i = i0 + lane + 64 * u;
      if (i < n4) pend |= 1u << u;
      v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, srcoff(min(i, n4 - 1)), 0, PD_SC1);
    }
    uint64_t t0 = 0;
    while (true) {
#pragma unroll
      for (int u = 0; u < B; ++u) {
        if ((pend >> u) & 1u) {
          const u32x4 x = v[u];
          if (x[1] == tag && x[3] == tag) {
            const int i = i0 + lane + 64 * u;
            *reinterpret_cast<u32x2*>(dst + i * 8) = u32x2{x[0], x[2]};
            if (SS) {
              const float p = lo_bf(x[0]), q = hi_bf(x[0]), r = lo_bf(x[2]), t = hi_bf(x[2]);
              ss += p * p + q * q + r * r + t * t;
            }
            pend &= ~(1u << u);
          }
        }
      }
      if (__ballot(pend != 0u) == 0) break;
      if (lds_ld(&ctl->abort)) break;
      const uint64_t now = __builtin_amdgcn_s_memrealtime();
      if (t0 == 0) {
        t0 = now;
      } else if ((long long)(now - t0) > a.timeout_ticks) {
        __hip_atomic_fetch_or(&ctl->abort, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
#pragma unroll
      for (int u = 0; u < B; ++u)
        if ((pend >> u) & 1u)
          v[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, srcoff(i0 + lane + 64 * u), 0, PD_SC1);
    }
  }
  return ss;
}

// Publish rows [r0, r0 + n) of one output vector (values v of lane r = row r0 + r, r < 64 per call) as granules.
__device__ __forceinline__ void pd_publish(u32x2* dst, int r0, int r, int n, float v, uint32_t tag) {
  const float nb = __shfl_down(v, 1, WAVE);
  if (r < n && (r & 1) == 0)
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack_bf2(v, nb), tag}, pd_rsrc(dst), ((r0 + r) >> 1) * 8, 0, PD_SC1);
}

// Sum of the streamers' partials of row r (fixed wave order)
template <int M>
__device__ __forceinline__ float pd_rowsum(const float* red, int m, int r) {
  float t = 0.f;
#pragma unroll
  for (int s = 0; s < PD_NS; ++s) t += red[(s * M + m) * PD_RMAX + r];
  return t;
}

// One attention work item (sequence b, kv head kvh, 64-token chunk ci) of layer l: RoPE of the new token's q/k, its
// paged-KV write (owner chunk) and GQA attention over the chunk; multi-chunk contexts merge their partials in the
// last-arriving chunk (sc1 records + agent-scope counter, as attn_decode_split.hip).  The pair's output (G heads x
// 128) is published as granules into the layer's attention hand-off.  qkvs: the pair's pre-RoPE q (G x 128), k, v.
template <int G>
__device__ __forceinline__ void pd_attention(const PdArgs& a, int l, int b, int kvh, int ci, const bf16_t* qkvs, char* scr,
                             u32x2* gout, uint32_t tag) {
  constexpr int D = 128, HALF = 64, CH = 64;
  constexpr int PSTRIDE = G * D + 2 * G;
  const int lane = threadIdx.x & 63, li = lane & 15, g4 = lane >> 4;
  bf16_t (*qs)[D] = reinterpret_cast<bf16_t (*)[D]>(scr);            // [16][D]
  char* vbuf = scr + 16 * D * 2;                                       // [2][32 rows][256 B]
  bf16_t* kcur = reinterpret_cast<bf16_t*>(vbuf + 2 * 32 * D * 2);     // [D]
  bf16_t* vcur = kcur + D;                                             // [D]
  const PdLayer& ly = a.layers[l];
  bf16_t* k_cache = ly.kc;
  bf16_t* v_cache = ly.vc;
  const int* bt = a.block_tables + (size_t)b * a.max_blocks;
  const size_t kvs = (size_t)a.nkv * D;
  const int start = ci * CH;
  const int ctx = a.context_lens[b];
  const int nq = a.nq;
  const auto gr = pd_rsrc(gout);

  if (ctx <= 0) {   // a padded row: its output is zeros (the O projection still gathers it)
    if (ci == 0) {
      for (int i = lane; i < G * D / 2; i += 64)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{0u, tag}, gr, ((kvh * G * D) / 2 + i) * 8, 0, PD_SC1);
    }
    return;
  }
  if (start >= ctx) return;
  int tblk[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) tblk[t] = bt[min(start / 16 + t, a.max_blocks - 1)];
  bf16_t xa[G], xb[G];
#pragma unroll
  for (int h = 0; h < G; ++h) {
    xa[h] = qkvs[h * D + lane];
    xb[h] = qkvs[h * D + HALF + lane];
  }
  const bf16_t ka = qkvs[G * D + lane], kb = qkvs[G * D + HALF + lane];
  const bf16_t va = qkvs[(G + 1) * D + lane], vb2 = qkvs[(G + 1) * D + HALF + lane];

  bf16x8 kf[4][D / 32];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const bf16_t* kp = k_cache + (size_t)(tblk[t] * 16 + li) * kvs + (size_t)kvh * D + g4 * 8;
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) kf[t][kk] = *reinterpret_cast<const bf16x8*>(kp + kk * 32);
  }
  const int n = min(CH, ctx - start);
  {
    const int lt = (n - 1) >> 4;
    const int last_row = (lt == 0 ? tblk[0] : lt == 1 ? tblk[1] : lt == 2 ? tblk[2] : tblk[3]) * 16 + ((n - 1) & 15);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = 4 * q + g4;
      const int srow = r < n ? tblk[q >> 2] * 16 + (r & 15) : last_row;
      const bf16_t* src = v_cache + (size_t)srow * kvs + (size_t)kvh * D + (li ^ pd_swz(r & 31)) * 8;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(vbuf + 1024 * q), 16, 0, 0);
    }
  }
  const int pos = ctx - 1;
  const bool owner = pos < start + n;
  const float* cs = a.cos_sin + (size_t)pos * D;
  {
    const int p = lane;
    const float cp = cs[p], sp = cs[HALF + p];
    const int pslot = owner ? bt[pos / 16] * 16 + pos % 16 : 0;
#pragma unroll
    for (int h = 0; h < 16; ++h) {
      bf16_t lo = 0, hi = 0;
      if (h < G) {
        const float x0 = bf2f(xa[h]), x1 = bf2f(xb[h]);
        lo = f2bf(x0 * cp - x1 * sp);
        hi = f2bf(x1 * cp + x0 * sp);
      }
      qs[h][p] = lo;
      qs[h][HALF + p] = hi;
    }
    if (owner) {
      const float x0 = bf2f(ka), x1 = bf2f(kb);
      const bf16_t klo = f2bf(x0 * cp - x1 * sp), khi = f2bf(x1 * cp + x0 * sp);
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
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (one wave) LDS writes above before the reads below

  bf16x8 qf[D / 32];
#pragma unroll
  for (int kk = 0; kk < D / 32; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(&qs[li][kk * 32 + g4 * 8]);
  const float qscale = a.scale * PD_LOG2E;
  f32x4 sacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (start + 16 * t + li == pos) {
#pragma unroll
      for (int kk = 0; kk < D / 32; ++kk) kf[t][kk] = *reinterpret_cast<const bf16x8*>(&kcur[kk * 32 + g4 * 8]);
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < D / 32; ++kk) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[t][kk], qf[kk], acc, 0, 0, 0);
    sacc[t] = acc;
  }
  float mx = -INFINITY;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float v = (16 * t + 4 * g4 + i) < n ? sacc[t][i] * qscale : -INFINITY;
      sacc[t][i] = v;
      mx = fmaxf(mx, v);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, WAVE));
  mx = fmaxf(mx, __shfl_xor(mx, 32, WAVE));
  float sum = 0.f;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e = exp2f(sacc[t][i] - mx);
      sacc[t][i] = e;
      sum += e;
    }
  }
  sum += __shfl_xor(sum, 16, WAVE);
  sum += __shfl_xor(sum, 32, WAVE);

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the V image has landed (and the K loads)
  if (owner) {
    const int rp = pos - start;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = 4 * q + g4;
      if (r >= rp)
        *reinterpret_cast<u32x4*>(vbuf + (r >> 5) * (32 * D * 2) + (r & 31) * (D * 2) + 16 * (li ^ pd_swz(r & 31))) =
            *reinterpret_cast<const u32x4*>(&vcur[li * 8]);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  f32x4 o[D / 16];
#pragma unroll
  for (int nn = 0; nn < D / 16; ++nn) o[nn] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int qd = li >> 2, pd = li & 3;
#pragma unroll
  for (int st = 0; st < 2; ++st) {
    if (32 * st < n) {
      const char* vb = vbuf + st * (32 * D * 2);
      bf16x8 pa;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pa[j] = (__bf16)sacc[2 * st][j];
        pa[4 + j] = (__bf16)sacc[2 * st + 1][j];
      }
      const int rr0 = 4 * g4 + qd, rr1 = rr0 + 16;
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) {
        const int col = 16 * nn + 4 * pd;
        const int ch = col >> 3, hb = (col & 7) * 2;
        const bf16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_pd_t*)(vb + rr0 * (D * 2) + 16 * (ch ^ pd_swz(rr0)) + hb));
        const bf16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_pd_t*)(vb + rr1 * (D * 2) + 16 * (ch ^ pd_swz(rr1)) + hb));
        bf16x8 vbf;
#pragma unroll
        for (int j = 0; j < 4; ++j) { vbf[j] = v0[j]; vbf[4 + j] = v1[j]; }
        o[nn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, vbf, o[nn], 0, 0, 0);
      }
    }
  }
  float lh[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) lh[i] = __shfl(sum, 4 * g4 + i, WAVE);
  const int nlive = (ctx + CH - 1) / CH;
  const int obase = (kvh * G * D) / 2;   // granule index of the pair's first output value (row b's hand-off)
  if (nlive == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int h = 4 * g4 + i;
      const float inv = 1.f / lh[i];
#pragma unroll
      for (int nn = 0; nn < D / 16; ++nn) {
        const float v = o[nn][i] * inv, nb = __shfl_down(v, 1, 16);
        if (h < G && (li & 1) == 0)
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack_bf2(v, nb), tag}, gr,
                                                (obase + (h * D + 16 * nn + li) / 2) * 8, 0, PD_SC1);
      }
    }
    return;
  }
  const size_t pair = (size_t)b * a.nkv + kvh;
  float* rec = a.part + (pair * a.pmax + ci) * PSTRIDE;
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
    __hip_atomic_store(rec + G * D + li, mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(rec + G * D + G + li, sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t prev = 0;
  if (lane == 0) prev = __hip_atomic_fetch_add(&a.counters[pair], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  prev = __shfl(prev, 0, WAVE);
  if (prev != (uint32_t)(nlive - 1)) return;
  if (lane == 0) __hip_atomic_store(&a.counters[pair], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // merge (last arriver): chunk statistics parked in LDS, accumulators summed with max-rescaling
  float* stat = reinterpret_cast<float*>(vbuf);   // [nlive][2G]
  const auto rs = pd_rsrc(a.part + pair * a.pmax * PSTRIDE);
  constexpr int LPH = 64 / G, DPL = D / LPH;
  const int h = lane / LPH, d0 = (lane % LPH) * DPL;
  if (lane < nlive) {
#pragma unroll
    for (int j = 0; j < 2 * G; ++j)
      stat[lane * 2 * G + j] =
          __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, (lane * PSTRIDE + G * D + j) * 4, 0, PD_SC1));
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  float M2 = -INFINITY;
  for (int q = 0; q < nlive; ++q) M2 = fmaxf(M2, stat[q * 2 * G + h]);
  float num[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) num[j] = 0.f;
  float den = 0.f;
  constexpr int QB = 4;
  for (int q0 = 0; q0 < nlive; q0 += QB) {
    float buf[QB][DPL];
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
      const int off = (min(q0 + qq, nlive - 1) * PSTRIDE + h * D + d0) * 4;
#pragma unroll
      for (int v = 0; v < DPL; v += 2) {
        const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(rs, off + 4 * v, 0, PD_SC1);
        buf[qq][v] = __uint_as_float(x[0]);
        buf[qq][v + 1] = __uint_as_float(x[1]);
      }
    }
#pragma unroll
    for (int qq = 0; qq < QB; ++qq) {
      const int q = q0 + qq;
      if (q < nlive) {
        const float wgt = exp2f(stat[q * 2 * G + h] - M2);
        den += wgt * stat[q * 2 * G + G + h];
#pragma unroll
        for (int j = 0; j < DPL; ++j) num[j] += wgt * buf[qq][j];
      }
    }
  }
  const float inv = 1.f / den;
#pragma unroll
  for (int j = 0; j < DPL; j += 2)
    __builtin_amdgcn_raw_buffer_store_b64(u32x2{pack_bf2(num[j] * inv, num[j + 1] * inv), tag}, gr,
                                          (obase + (h * D + d0 + j) / 2) * 8, 0, PD_SC1);
}

template <int M, int G>
__device__ __forceinline__ void pd_chain(const PdArgs& a, char* lds, int c, int NG, uint32_t tag,
                                         const PdGeo (&geo)[4]) {
  const int lane = threadIdx.x & 63;
  PdCtl* ctl = reinterpret_cast<PdCtl*>(lds + a.off_ctl);
  char* resid = lds + a.off_resid;
  char* xin = lds + a.off_xin;
  float* red = reinterpret_cast<float*>(lds + a.off_red);
  char* att = lds + a.off_att;
  bf16_t* qkvs = reinterpret_cast<bf16_t*>(att + 16 * 128 * 2 + 2 * 32 * 128 * 2 + 2 * 128 * 2);
  const int D = 128, nqD = a.nq * D, nqkv = (a.nq + 2 * a.nkv) * D, H = a.H, I = a.I;
  const int KX = max(nqD, I);
  const int oq = 0, oa = nqkv / 2, oo = oa + nqD / 2, og = oo + H / 2, ox = og + I / 2;   // granule offsets
  auto gbase = [&](int l, int m) { return a.gran + ((size_t)l * M + m) * a.gl; };
  const auto lin = [](int i) { return i * 16; };   // contiguous hand-off ranges
  auto stamp = [&](int l, int k) {
    if (a.trace != nullptr && lane == 0)
      a.trace[((size_t)c * a.L + l) * PD_TRACE_PTS + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto zero_red = [&](int nrows) {
    for (int i = lane; i < PD_NS * M * PD_RMAX; i += 64) red[i] = 0.f;
    (void)nrows;
  };
  auto release = [&](uint32_t seq) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(&ctl->ready, seq + 1);
  };
  auto wait_done = [&](uint32_t seq) { pd_wait_lds(&ctl->pdone, (uint32_t)PD_NS * (seq + 1), ctl, a, 4u); };

  zero_red(0);
  // layer-0 input: the embedding rows (plain loads: written by an earlier kernel), RMS statistics
  float inv1[M], inv2[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    float ss = 0.f;
    for (int i = lane; i < H / 8; i += 64) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(a.x0 + (size_t)m * H + i * 8);
      *reinterpret_cast<u32x4*>(resid + m * H * 2 + i * 16) = v;
#pragma unroll
      for (int e = 0; e < 4; ++e) ss += lo_bf(v[e]) * lo_bf(v[e]) + hi_bf(v[e]) * hi_bf(v[e]);
    }
    inv1[m] = rsqrtf(wave_sum(ss) / (float)H + a.eps);
  }
  release(0);

  const int n_items = (int)(M * a.nkv * a.pmax);
  for (int l = 0; l < a.L; ++l) {
    const uint32_t s0 = 4u * l;
    // ---- QKV: 1/rms epilogue, publish
    {
      const PdGeo& g = geo[0];
      wait_done(s0);
      stamp(l, 0);
      for (int r0 = 0; r0 < g.nrows; r0 += 64) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int r = r0 + lane;
          const float v = r < g.nrows ? pd_rowsum<M>(red, m, r) * inv1[m] : 0.f;
          pd_publish(gbase(l, m) + oq, g.r0 + r0, lane, g.nrows - r0, v, tag);
        }
      }
      stamp(l, 9);
      zero_red(g.nrows);
    }
    // ---- attention items of this workgroup
    for (int it = NG - 1 - c; it < n_items; it += NG) {
      const int b = it / (a.nkv * a.pmax), kvh = (it / a.pmax) % a.nkv, ci = it % a.pmax;
      // the pair's q (G heads), k and v from the QKV hand-off
      const u32x2* src = gbase(l, b) + oq;
      // q of the G heads, k, v: three ranges of the hand-off, one gather (one round trip)
      // (byte offsets: a hand-off holds 2 values per 8-byte granule, 4 bytes per value)
      const int nqg = G * D / 4, qo = kvh * G * D * 4, ko = (a.nq + kvh) * D * 4, vo = (a.nq + a.nkv + kvh) * D * 4;
      pd_gather<false, (G * D / 4 + D / 2 + 63) / 64>(
          src, reinterpret_cast<char*>(qkvs), nqg + D / 2,
          [=](int i) { return i < nqg ? qo + i * 16 : (i < nqg + D / 4 ? ko + (i - nqg) * 16 : vo + (i - nqg - D / 4) * 16); },
          tag, ctl, a);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (lds_ld(&ctl->abort)) continue;
      pd_attention<G>(a, l, b, kvh, ci, qkvs, att, gbase(l, b) + oa, tag);
    }
    stamp(l, 1);
    // ---- O: input = attention output
#pragma unroll
    for (int m = 0; m < M; ++m) pd_gather<false, 32>(gbase(l, m) + oa, xin + m * KX * 2, nqD / 4, lin, tag, ctl, a);
    release(s0 + 1);
    stamp(l, 2);
    {
      const PdGeo& g = geo[1];
      wait_done(s0 + 1);
      stamp(l, 3);
      for (int r0 = 0; r0 < g.nrows; r0 += 64) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int r = r0 + lane;
          const float v = r < g.nrows
                              ? pd_rowsum<M>(red, m, r) +
                                    bf2f(reinterpret_cast<const bf16_t*>(resid + m * H * 2)[g.r0 + r])
                              : 0.f;
          pd_publish(gbase(l, m) + oo, g.r0 + r0, lane, g.nrows - r0, v, tag);
        }
      }
      stamp(l, 10);
      zero_red(g.nrows);
    }
    // ---- gate/up: input = o (the new residual stream), RMS statistics
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float ss = pd_gather<true, 32>(gbase(l, m) + oo, resid + m * H * 2, H / 4, lin, tag, ctl, a);
      inv2[m] = rsqrtf(wave_sum(ss) / (float)H + a.eps);
    }
    release(s0 + 2);
    stamp(l, 4);
    {
      const PdGeo& g = geo[2];
      wait_done(s0 + 2);
      stamp(l, 5);
      const int n = g.nrows;   // gate rows [0, n), up rows [n, 2n) of the partials
      for (int r0 = 0; r0 < n; r0 += 64) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int r = r0 + lane;
          float v = 0.f;
          if (r < n) {
            const float gt = pd_rowsum<M>(red, m, r) * inv2[m];
            const float up = pd_rowsum<M>(red, m, n + r) * inv2[m];
            v = pd_silu(gt) * up;
          }
          pd_publish(gbase(l, m) + og, g.r0 + r0, lane, n - r0, v, tag);
        }
      }
      stamp(l, 11);
      zero_red(2 * n);
    }
    // ---- down: input = SwiGLU output
#pragma unroll
    for (int m = 0; m < M; ++m) pd_gather<false, 32>(gbase(l, m) + og, xin + m * KX * 2, I / 4, lin, tag, ctl, a);
    release(s0 + 3);
    stamp(l, 6);
    {
      const PdGeo& g = geo[3];
      wait_done(s0 + 3);
      stamp(l, 7);
      const bool last = l == a.L - 1;
      for (int r0 = 0; r0 < g.nrows; r0 += 64) {
#pragma unroll
        for (int m = 0; m < M; ++m) {
          const int r = r0 + lane;
          const float v = r < g.nrows
                              ? pd_rowsum<M>(red, m, r) +
                                    bf2f(reinterpret_cast<const bf16_t*>(resid + m * H * 2)[g.r0 + r])
                              : 0.f;
          if (last) {
            if (r < g.nrows) a.xout[(size_t)m * H + g.r0 + r] = f2bf(v);
          } else {
            pd_publish(gbase(l, m) + ox, g.r0 + r0, lane, g.nrows - r0, v, tag);
          }
        }
      }
      stamp(l, 12);
      zero_red(g.nrows);
    }
    if (l + 1 < a.L) {   // next layer's input: x, RMS statistics
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const float ss = pd_gather<true, 32>(gbase(l, m) + ox, resid + m * H * 2, H / 4, lin, tag, ctl, a);
        inv1[m] = rsqrtf(wave_sum(ss) / (float)H + a.eps);
      }
      release(s0 + 4);
      stamp(l, 8);
    }
  }
}

}  // namespace

template <int M, int RS, int G>
__global__ void __launch_bounds__(PD_NT) decode_persist_kernel(PdArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wid = threadIdx.x >> 6;
  const int c = blockIdx.x, NG = gridDim.x;
  PdCtl* ctl = reinterpret_cast<PdCtl*>(lds + a.off_ctl);
  if (threadIdx.x == 0) {
    ctl->ready = 0;
    ctl->pdone = 0;
    ctl->abort = 0;
    ctl->tag = __hip_atomic_load(a.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  const uint32_t tag = ctl->tag;
  PdGeo geo[4];
#pragma unroll
  for (int ph = 0; ph < 4; ++ph) geo[ph] = pd_geo(a, ph, c, NG);
  if (wid == 0) pd_chain<M, G>(a, lds, c, NG, tag, geo);
  else pd_streamer<M, RS>(a, lds, __builtin_amdgcn_readfirstlane(wid - 1), geo);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's stores (granules, KV, xout) have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t err = lds_ld(&ctl->abort);
    if (err) __hip_atomic_fetch_or(a.sync + 64, err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t prev = __hip_atomic_fetch_add(a.sync + 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (uint32_t)NG - 1) {   // the last workgroup: every other one has read this launch's epoch
      __hip_atomic_store(a.sync + 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.sync, tag + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace k8sllm

using namespace k8sllm;

namespace {
int pd_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return v;
}

struct PdPlan {
  int lds, rs, gl, off_resid, off_xin, off_red, off_att, off_ctl;
};

// Returns 0 and the plan, or a negative code when the shape is outside what the kernel takes.
int pd_plan(int M, int H, int nq, int nkv, int I, int pmax, int grid, PdPlan& p) {
  if (M < 1 || M > 2 || nkv <= 0 || nq % nkv != 0) return -1;
  const int G = nq / nkv;
  if (G != 2 && G != 4 && G != 8) return -2;
  const int nqD = nq * 128, nqkv = (nq + 2 * nkv) * 128;
  if (H % 512 || nqD % 512 || I % 512) return -3;
  if (pmax < 1 || pmax > 64) return -4;
  auto rows = [&](int pairs) { return 2 * ((pairs + grid - 1) / grid); };
  if (rows(nqkv / 2) > PD_RMAX || rows(H / 2) > PD_RMAX || 2 * rows(I / 2) > PD_RMAX) return -5;
  const int KX = nqD > I ? nqD : I;
  p.off_resid = 0;
  p.off_xin = p.off_resid + M * H * 2;
  p.off_red = p.off_xin + M * KX * 2;
  p.off_att = p.off_red + PD_NS * M * PD_RMAX * 4;
  const int att = 16 * 128 * 2 + 2 * 32 * 128 * 2 + 2 * 128 * 2 + (G + 2) * 128 * 2;
  p.off_ctl = p.off_att + ((att + 15) / 16) * 16;
  p.lds = p.off_ctl + 64;
  if (p.lds < 82 * 1024) p.lds = 82 * 1024;   // one workgroup per CU
  if (p.lds > 160 * 1024) return -6;
  p.gl = (nqkv + nqD + 2 * H + I) / 2;
  return 0;
}

static int g_pd_rs = [] { const char* e = getenv("K8S_PERSIST_RS"); return e ? atoi(e) : 12; }();
}  // namespace

extern "C" int k8s_decode_persist_plan(int M, int H, int nq, int nkv, int I, int pmax, int* gl, int* grid) {
  PdPlan p;
  const int g = pd_cus();
  const int rc = pd_plan(M, H, nq, nkv, I, pmax, g, p);
  if (rc == 0) {
    *gl = p.gl;
    *grid = g;
  }
  return rc;
}

// layers: device array of L PdLayer records; gran: L * M * gl granules (8 B, zeroed once); part / counters: as the
// split attention (counters zeroed once); sync: 96 u32, zeroed once with sync[0] = 1.
extern "C" int k8s_decode_persist(const void* layers, int L, const void* x0, void* xout, int M, int H, int nq, int nkv,
                                  int I, float eps, float scale, const float* cos_sin, const int* block_tables,
                                  const int* context_lens, int max_blocks, int pmax, void* gran, void* part,
                                  uint32_t* counters, uint32_t* sync, void* trace, long long timeout_ticks,
                                  hipStream_t stream) {
  PdPlan p;
  const int grid = pd_cus();
  const int rc = pd_plan(M, H, nq, nkv, I, pmax, grid, p);
  if (rc != 0) return rc;
  if (L < 1 || (pmax > 1 && (part == nullptr || counters == nullptr)) || sync == nullptr || gran == nullptr) return -7;
  PdArgs a;
  a.layers = static_cast<const PdLayer*>(layers);
  a.x0 = static_cast<const bf16_t*>(x0);
  a.xout = static_cast<bf16_t*>(xout);
  a.cos_sin = cos_sin;
  a.block_tables = block_tables;
  a.context_lens = context_lens;
  a.gran = static_cast<u32x2*>(gran);
  a.part = static_cast<float*>(part);
  a.counters = counters;
  a.sync = sync;
  a.trace = static_cast<unsigned long long*>(trace);
  a.timeout_ticks = timeout_ticks;
  a.eps = eps;
  a.scale = scale;
  a.L = L; a.H = H; a.nq = nq; a.nkv = nkv; a.I = I; a.max_blocks = max_blocks; a.pmax = pmax; a.gl = p.gl;
  a.off_resid = p.off_resid; a.off_xin = p.off_xin; a.off_red = p.off_red; a.off_att = p.off_att;
  a.off_ctl = p.off_ctl;
  const int G = nq / nkv;
  const int rs = g_pd_rs;
#define PDL(MM, RR, GG)                                                                                          \
  do {                                                                                                           \
    static const bool attr_ok = hipFuncSetAttribute(reinterpret_cast<const void*>(&decode_persist_kernel<MM, RR, GG>), \
                                                    hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess; \
    (void)attr_ok;                                                                                               \
    decode_persist_kernel<MM, RR, GG><<<grid, PD_NT, p.lds, stream>>>(a);                                        \
  } while (0)
#define PDG(MM, RR)                       \
  switch (G) {                            \
    case 2: PDL(MM, RR, 2); break;        \
    case 4: PDL(MM, RR, 4); break;        \
    case 8: PDL(MM, RR, 8); break;        \
    default: return -2;                   \
  }
  if (M == 1 && G == 8 && rs != 12) {   // ring-depth variants (K8S_PERSIST_RS) for the 70B head layout
    if (rs <= 8) PDL(1, 8, 8);
    else PDL(1, 16, 8);
  } else if (M == 1) {
    PDG(1, 12)
  } else {
    PDG(2, 12)
  }
#undef PDG
#undef PDL
  return (int)hipGetLastError();
}

extern "C" int k8s_decode_persist_layer_bytes() { return (int)sizeof(PdLayer); }
extern "C" int k8s_decode_persist_trace_points() { return PD_TRACE_PTS; }
