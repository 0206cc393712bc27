// K3 / K8 / K9(+K10) / K11 / K12 at prefill row counts, bf16: the 4-wave big-tile MFMA GEMM.
//
//     out[M, N_out] = epi( x[M, K] . W[N, K]^T )      epi: bf16 (+ residual) | fp32 | SwiGLU, optional RMS prologue
//
// Why 4 waves (and not pgemm.hip's 8-wave ping-pong): PMC on the 2048 x 8192 x 8192 projection showed the
// 8-wave 128 x 64-per-wave schedule parked 31 % of its wave cycles at barriers (SQ_WAIT_ANY) and issued 1.5x
// the LDS instructions of the library's 256 x 256 kernel, which runs 4 waves of 128 x 128
// (profiles/pmc_pgemm_vs_hipblaslt_M2048_oproj_tp1.txt).  Here every wave owns a 128 x 128 output (64
// fragments of v_mfma_f32_16x16x32_bf16, 256 accumulator registers: the AGPR half of the unified file at one
// wave per SIMD), so per 32-deep k-step a wave issues 16 fragment reads for 64 MFMAs.
//
//  * ring of 4 LDS k-steps (BP + BQ rows x 64 bytes each, 128 KiB at 256 x 256) filled by LDS-DMA
//    (global_load_lds_dwordx4); k-step s+3 is issued right after the barrier of iteration s into the slot
//    k-step s-1 vacated, so three k-steps (two MFMA blocks, ~2k cycles) of DMA are in flight across the raw
//    s_barriers; the one wait per k-step is a counted `s_waitcnt vmcnt` (never 0 in the steady state).
//  * register double buffer: the fragments of k-step s+1 are read (ds_read_b128) before the 64 MFMAs of
//    k-step s, so the LDS latency hides under the matrix pipe of the same wave.
//  * DMA image lane-linear, XOR swizzle on the per-lane global source (16-byte chunk c of row r in slot
//    c ^ ((r >> 2) & 3)): the 16-row fragment reads are conflict-free on 64-byte rows.
//  * swapped orientation C^T = W . x^T: every lane ends with 4 consecutive features of one token (gate/up
//    rows of one feature sit in the same lane for the SwiGLU epilogue).
//  * XCD-aware bijective block remap, group_m m-tiles per n-column group, k-slices of a tile adjacent.
//  * split-K: every slice stores fp32 partial sums into its own slab [M][W rows] (plus the RMS row sums) and
//    pgemm_reduce_kernel sums the slabs in slice order (deterministic) and applies the epilogue -- a
//    parallel reduction over the whole chip instead of one last-arriving workgroup reading every slab.
#include <type_traits>

#include "common.h"

namespace k8sllm {

namespace {
enum { P4_BF16 = 0, P4_F32 = 1, P4_SWIGLU = 2 };
typedef __attribute__((ext_vector_type(2))) uint32_t p4_u32x2;

template <int N>
__device__ __forceinline__ void p4_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void p4_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ float p4_silu(float g) { return g / (1.f + __expf(-g)); }
}  // namespace

struct P4Args {
  void* out;
  const bf16_t* res;     // optional residual (bf16 [M][N_out], may alias out)
  float* slab;           // split-K: [splits][M][W rows] fp32 partial sums, then [splits][M] row sums of squares
  const uint8_t* x;      // [M][K] bf16
  const uint8_t* W;      // [rows][K] bf16
  uint32_t kbytes;       // bytes per row of x and W
  int M, N_out, half_rows, wrows, K;
  int m_tiles, n_tiles, ks, splits, group_m, nwg;
  float eps;
};

template <int FP, int FQ, int EPI, bool RMS, bool K64 = false>
__global__ void __launch_bounds__(256, 1) pgemm4_kernel(P4Args a) {
  constexpr int BP = 32 * FP, BQ = 32 * FQ;          // weight rows, tokens per tile (2 x 2 waves)
  constexpr int ROWS = BP + BQ;
  constexpr int SUB = ROWS * 64;                     // one 32-deep k-step of both operands
  constexpr int G = ROWS / 64;                       // 16-byte DMA instructions per thread per k-step
  constexpr int NSLOT = 4;
  static_assert(ROWS % 64 == 0 && G >= 1, "tile shape");
  // K64: 64-deep LDS stages of 128-byte rows, two of them (the same 4 x 32-deep bytes): every LDS-DMA instruction
  // moves 8 whole 128-byte rows instead of 16 half rows, and one barrier covers 2 x FP x FQ MFMAs
  constexpr int RING = K64 ? 2 * ROWS * 128 : NSLOT * SUB;
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ __attribute__((aligned(16))) char lds[RING + BQ * 8];
  float* rss = reinterpret_cast<float*>(lds + RING);   // [2][BQ] row sums of squares (wave rows)

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int li = lane & 15, g = lane >> 4;

  // ---- block -> (tile, k-slice)
  const int bid = blockIdx.x, q8 = a.nwg >> 3, r8 = a.nwg & 7, xcd = bid & 7, loc = bid >> 3;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const int tile = lid / a.splits, slice = lid - tile * a.splits;
  int mt, nt;
  {
    const int per = a.group_m * a.n_tiles, gi = tile / per, m0 = gi * a.group_m;
    const int gm = min(a.m_tiles - m0, a.group_m), in = tile - gi * per;
    mt = m0 + in % gm;
    nt = in / gm;
  }
  const int ks0 = 2 * (int)((long long)slice * (a.ks / 2) / a.splits);
  const int n = 2 * (int)((long long)(slice + 1) * (a.ks / 2) / a.splits) - ks0;   // even, >= 2

  // ---- per-thread DMA sources: chunk p = j * 256 + tid of the k-step image (rows 0..BP-1 weights, then x);
  // instructions j < GW cover weight rows only, the rest x rows only
  constexpr int GW = BP / 64;
  uint32_t off[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    const int p = j * 256 + tid, r = p >> 2, c = (p & 3) ^ ((r >> 2) & 3);
    const uint32_t col = (uint32_t)(c * 16 + ks0 * 64);
    if (j < GW) {
      const int w = r / (BP / 2), q = r % (BP / 2);
      int row;
      if constexpr (EPI == P4_SWIGLU) {   // wave rows: BP/4 gate rows then the matching BP/4 up rows
        const int f = min(nt * (BP / 2) + w * (BP / 4) + (q % (BP / 4)), a.N_out - 1);
        row = q < BP / 4 ? f : a.half_rows + f;
      } else {
        row = min(nt * BP + r, a.N_out - 1);
      }
      off[j] = (uint32_t)row * a.kbytes + col;
    } else {
      off[j] = (uint32_t)min(mt * BQ + (r - BP), a.M - 1) * a.kbytes + col;
    }
  }
  auto issue = [&](int u) {   // k-step u of this slice into slot u % 4
    char* dst = lds + (u & (NSLOT - 1)) * SUB + wid * 1024;
    const uint32_t kb = (uint32_t)u * 64u;
#pragma unroll
    for (int j = 0; j < G; ++j)
      __builtin_amdgcn_global_load_lds((j < GW ? a.W : a.x) + (off[j] + kb),
                                       (__attribute__((address_space(3))) void*)(dst + j * 4096), 16, 0, 0);
  };

  // ---- fragment reads: row li of a 16-row fragment, chunk g (k 8g .. 8g+7), swizzled
  const int lo = li * 64 + ((g ^ (li >> 2)) << 4);
  const int pb = (wr * (BP / 2)) * 64 + lo, qb = (BP + wc * (BQ / 2)) * 64 + lo;
  bf16x8 A0[FP], B0[FQ], A1[FP], B1[FQ];
  // The fragment reads are inline asm as well: a compiler-visible LDS read ahead of the (opaque) asm MFMAs made the
  // compiler drain lgkmcnt(0) before the first MFMA, exposing the whole read latency every k-step.  Nothing reads
  // An / Bn before the next k-step's p4_sync, whose lgkmcnt(0) retires these reads.
  auto rd = [&](int u, bf16x8* A, bf16x8* B) {
    const char* sb = lds + (u & (NSLOT - 1)) * SUB;
    const uint32_t la = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)(sb + pb));
    const uint32_t lb = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)(sb + qb));
#pragma unroll
    for (int f = 0; f < FP; ++f) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(A[f]) : "v"(la), "i"(f * 1024));
#pragma unroll
    for (int f = 0; f < FQ; ++f) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(B[f]) : "v"(lb), "i"(f * 1024));
  };

  f32x4 acc[FP][FQ];
#pragma unroll
  for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FQ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[FQ];
#pragma unroll
  for (int f = 0; f < FQ; ++f) ss[f] = 0.f;

  // MFMAs of fragment rows [i0, i1) on one k-step's registers (+ the RMS squares of the x fragments)
  auto mma = [&](const bf16x8* A, const bf16x8* B, int i0, int i1) {
#pragma unroll
    for (int i = 0; i < FP; ++i)
      if (i >= i0 && i < i1)
#pragma unroll
        for (int j = 0; j < FQ; ++j)
          // in place, in inline asm: the AGPR tile stays put (with the builtin the register allocator rotated the
          // accumulators through AGPR <-> VGPR copies, 2.2-3.7 per MFMA in every configuration; 11-13 % slower)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(A[i]), "v"(B[j]));
  };
  auto squares = [&](const bf16x8* B, bool sq) {
    if constexpr (RMS) {
      if (sq) {   // the two wave rows hold the same x fragments: each squares every other k-step
#pragma unroll
        for (int f = 0; f < FQ; ++f)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bf16x2 v2 = {B[f][2 * e], B[f][2 * e + 1]};
            ss[f] = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, ss[f], false);
          }
      }
    }
  };
  // One k-step s: make s+1 visible (counted vmcnt + barrier), refill the slot of s-1 with s+3 (LDS-DMA), read
  // s+1 into the other register set, then the 64 MFMAs on s (registers read one k-step earlier).
  // One k-step s: make s+1 visible (counted vmcnt + barrier), then the 64 MFMAs on s (registers read one k-step
  // earlier) with the LDS-DMA refill of s-1's slot by s+3 and the fragment reads of s+1 spread between them: one wave
  // per SIMD, so nothing else would hide a DMA issue or an LDS read (all three are volatile asm or side-effecting
  // builtins, so this program order is the issue order).
  auto step_full = [&](int s, bf16x8* Ac, bf16x8* Bc, bf16x8* An, bf16x8* Bn) {
    p4_vmcnt<G>();
    p4_sync();
    __builtin_amdgcn_sched_barrier(0);
    constexpr int MF = FP * FQ, DR = FP + FQ;
    char* dst = lds + ((s + 3) & (NSLOT - 1)) * SUB + wid * 1024;
    const uint32_t kb = (uint32_t)(s + 3) * 64u;
    const char* sb = lds + ((s + 1) & (NSLOT - 1)) * SUB;
    const uint32_t la = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)(sb + pb));
    const uint32_t lb = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)(sb + qb));
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
    for (int j = 0; j < FQ; ++j) {
      const int k = i * FQ + j;
#pragma unroll
      for (int d = 0; d < G; ++d)
        if (k == d * MF / G)
          __builtin_amdgcn_global_load_lds((d < GW ? a.W : a.x) + (off[d] + kb),
                                           (__attribute__((address_space(3))) void*)(dst + d * 4096), 16, 0, 0);
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(Ac[i]), "v"(Bc[j]));
#pragma unroll
      for (int r = 0; r < DR; ++r)
        if (k == r * MF / DR + MF / (2 * DR)) {
          if (r < FP)
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(An[r]) : "v"(la), "i"(r * 1024));
          else
            asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Bn[r - FP]) : "v"(lb), "i"((r - FP) * 1024));
        }
    }
    squares(Bc, (s & 1) == wr);
  };
  auto step_tail = [&](int s, bf16x8* Ac, bf16x8* Bc, bf16x8* An, bf16x8* Bn) {
    if (s + 1 < n) {
      if (s + 2 < n) p4_vmcnt<G>(); else p4_vmcnt<0>();
      p4_sync();
      if (s + 3 < n) issue(s + 3);
      rd(s + 1, An, Bn);
    }
    mma(Ac, Bc, 0, FP);
    squares(Bc, (s & 1) == wr);
  };

  {   // the inline-asm MFMAs are opaque to the hazard recognizer: every zeroed accumulator passes through an asm
    // tied to it after its write, all before the first MFMA (volatile asm keeps its order)
    asm volatile("s_nop 1" ::: "memory");
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
      for (int j = 0; j < FQ; ++j) asm volatile("s_nop 0" : "+a"(acc[i][j]));
  }
  if constexpr (K64) {
    // ---- 64-deep stages: stage u in slot u & 1, row r at r * 128 bytes, 16-byte chunk c of row r at slot
    // c ^ ((r >> 1) & 7) (the swizzle is applied on the per-lane global source, the DMA image is lane-linear).
    // Sub-step h (k 32 h .. 32 h + 31) of a fragment row li = chunks 4 h + g.  Register sets: R0 = (A0, B0) holds
    // sub-step 0, R1 = (A1, B1) sub-step 1.  Per stage s after the barrier: phase A = the MFMAs of (s - 1, 1) on R1
    // with the reads of (s, 0) into R0 and the LDS-DMA of stage s + 1 (into the slot of s - 1, whose reads every
    // wave retired before the barrier) spread between them; phase P = the MFMAs of (s, 0) on R0 with the reads of
    // (s, 1) into R1.
    constexpr int SUB2 = ROWS * 128, G2 = ROWS / 32, GW2 = BP / 32;
    const int n2 = n / 2;
    uint32_t off2[G2];
#pragma unroll
    for (int j = 0; j < G2; ++j) {
      const int p = j * 256 + tid, r = p >> 3, c = (p & 7) ^ ((r >> 1) & 7);
      const uint32_t col = (uint32_t)(c * 16 + ks0 * 64);
      if (j < GW2) {
        const int w = r / (BP / 2), q = r % (BP / 2);
        int row;
        if constexpr (EPI == P4_SWIGLU) {
          const int f = min(nt * (BP / 2) + w * (BP / 4) + (q % (BP / 4)), a.N_out - 1);
          row = q < BP / 4 ? f : a.half_rows + f;
        } else {
          row = min(nt * BP + r, a.N_out - 1);
        }
        off2[j] = (uint32_t)row * a.kbytes + col;
      } else {
        off2[j] = (uint32_t)min(mt * BQ + (r - BP), a.M - 1) * a.kbytes + col;
      }
    }
    auto dma2 = [&](int u, int d) {   // instruction d of stage u
      __builtin_amdgcn_global_load_lds((d < GW2 ? a.W : a.x) + (off2[d] + (uint32_t)u * 128u),
                                       (__attribute__((address_space(3))) void*)(lds + (u & 1) * SUB2 + wid * 1024 +
                                                                                 d * 4096),
                                       16, 0, 0);
    };
    const int lo0 = li * 128 + ((g ^ (li >> 1)) << 4), lo1 = li * 128 + (((4 + g) ^ (li >> 1)) << 4);
    const int pb2 = wr * (BP / 2) * 128, qb2 = (BP + wc * (BQ / 2)) * 128;
    auto laddr = [&](int u, int off) {
      return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)(lds + (u & 1) * SUB2 + off));
    };
    auto rd2 = [&](int u, int h, bf16x8* A, bf16x8* B) {   // whole sub-step, not interleaved (prologue / tail)
      const uint32_t la = laddr(u, pb2 + (h ? lo1 : lo0)), lb = laddr(u, qb2 + (h ? lo1 : lo0));
#pragma unroll
      for (int f = 0; f < FP; ++f) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(A[f]) : "v"(la), "i"(f * 2048));
#pragma unroll
      for (int f = 0; f < FQ; ++f) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(B[f]) : "v"(lb), "i"(f * 2048));
    };
    // 64 MFMAs on (Ac, Bc) with the reads of sub-step h of stage u into (An, Bn) and (dma) the G2 instructions of
    // stage u + 1 spread between them
    auto phase = [&](const bf16x8* Ac, const bf16x8* Bc, int u, int h, bf16x8* An, bf16x8* Bn, bool rd, bool dma) {
      constexpr int MF = FP * FQ, DR = FP + FQ;
      const uint32_t la = laddr(u, pb2 + (h ? lo1 : lo0)), lb = laddr(u, qb2 + (h ? lo1 : lo0));
#pragma unroll
      for (int i = 0; i < FP; ++i)
#pragma unroll
        for (int j = 0; j < FQ; ++j) {
          const int k = i * FQ + j;
#pragma unroll
          for (int d = 0; d < G2; ++d)
            if (k == d * MF / G2 && dma) dma2(u + 1, d);
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(Ac[i]), "v"(Bc[j]));
#pragma unroll
          for (int r = 0; r < DR; ++r)
            if (k == 4 + r * (MF - 8) / DR && rd) {   // the first read 4 MFMAs in: the previous phase's
                                                       // MFMAs on these registers are long issued
              if (r < FP)
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(An[r]) : "v"(la), "i"(r * 2048));
              else
                asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(Bn[r - FP]) : "v"(lb), "i"((r - FP) * 2048));
            }
        }
    };
    // prologue: stages 0 (and 1) in flight, stage 0 visible, (0, 0) read
#pragma unroll
    for (int d = 0; d < G2; ++d) dma2(0, d);
    p4_vmcnt<0>();
    p4_sync();
    rd2(0, 0, A0, B0);
    if (n2 > 1) {
#pragma unroll
      for (int d = 0; d < G2; ++d) dma2(1, d);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    phase(A0, B0, 0, 1, A1, B1, true, false);           // P_0: (0, 0) on R0, read (0, 1)
    squares(B0, wr == 0);
    for (int s2 = 1; s2 < n2; ++s2) {
      p4_vmcnt<0>();                                     // stage s2 landed (this wave's DMA)
      p4_sync();                                         // ... for every wave; (s2 - 1, 1) reads retired
      __builtin_amdgcn_sched_barrier(0);
      phase(A1, B1, s2, 0, A0, B0, true, s2 + 1 < n2);   // A: (s2 - 1, 1) on R1, read (s2, 0), DMA stage s2 + 1
      squares(B1, wr == 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      phase(A0, B0, s2, 1, A1, B1, true, false);         // P: (s2, 0) on R0, read (s2, 1)
      squares(B0, wr == 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    phase(A1, B1, 0, 0, A0, B0, false, false);           // the last sub-step, (n2 - 1, 1), on R1
    squares(B1, wr == 1);
  } else {
  // n is even (the host splits K in 64-deep units): the loop body is two k-steps with fixed register sets
  issue(0);
  issue(1);
  if (n > 2) issue(2);
  if (n > 2) p4_vmcnt<2 * G>(); else p4_vmcnt<G>();
  p4_sync();
  rd(0, A0, B0);
  int s = 0;
  for (; s + 4 < n; s += 2) {
    step_full(s, A0, B0, A1, B1);
    step_full(s + 1, A1, B1, A0, B0);
  }
  if (s + 2 < n) {
    step_tail(s, A0, B0, A1, B1);
    step_tail(s + 1, A1, B1, A0, B0);
    s += 2;
  }
  step_tail(s, A0, B0, A1, B1);
  step_tail(s + 1, A1, B1, A0, B0);
  }
  p4_vmcnt<0>();
  {   // ... and the last MFMAs' results wait out the MFMA latency before the epilogue reads them:
    // the padding, then one tied empty asm per accumulator (so no read is hoisted above the padding)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
#pragma unroll
    for (int i = 0; i < FP; ++i)
#pragma unroll
      for (int j = 0; j < FQ; ++j) asm volatile("" : "+a"(acc[i][j]));
  }

  if constexpr (RMS) {
#pragma unroll
    for (int f = 0; f < FQ; ++f) {
      ss[f] += __shfl_xor(ss[f], 16, WAVE);
      ss[f] += __shfl_xor(ss[f], 32, WAVE);
    }
    if (g == 0) {
#pragma unroll
      for (int f = 0; f < FQ; ++f) rss[wr * BQ + wc * (BQ / 2) + f * 16 + li] = ss[f];
    }
    __syncthreads();
    if (tid < BQ) rss[tid] += rss[BQ + tid];
    __syncthreads();
  }

  // ---- split-K: raw partial sums into this slice's slab (natural [M][W rows] layout)
  if (a.splits > 1) {
    float* sl = a.slab + (size_t)slice * a.M * a.wrows;
#pragma unroll
    for (int j = 0; j < FQ; ++j) {
      const int m = mt * BQ + wc * (BQ / 2) + j * 16 + li;
      if (m >= a.M) continue;
#pragma unroll
      for (int i = 0; i < FP; ++i) {
        int r0;
        if constexpr (EPI == P4_SWIGLU) {
          const int hf = i / (FP / 2), f = nt * (BP / 2) + wr * (BP / 4) + (i % (FP / 2)) * 16 + 4 * g;
          if (f >= a.N_out) continue;
          r0 = hf ? a.half_rows + f : f;
        } else {
          r0 = nt * BP + wr * (BP / 2) + i * 16 + 4 * g;
          if (r0 >= a.N_out) continue;
        }
        *reinterpret_cast<f32x4*>(sl + (size_t)m * a.wrows + r0) = acc[i][j];
      }
    }
    if (RMS && tid < BQ && mt * BQ + tid < a.M)
      a.slab[(size_t)a.splits * a.M * a.wrows + (size_t)slice * a.M + mt * BQ + tid] = rss[tid];
    return;
  }

  // ---- epilogue: lane holds out[token li of fragment j][features 4 g .. 4 g + 3 of fragment i]
#pragma unroll
  for (int j = 0; j < FQ; ++j) {
    const int mloc = wc * (BQ / 2) + j * 16 + li;
    const int m = mt * BQ + mloc;
    if (m >= a.M) continue;
    float sx = 1.f;
    if constexpr (RMS) sx = rsqrtf(rss[mloc] / (float)a.K + a.eps);
    if constexpr (EPI == P4_SWIGLU) {
#pragma unroll
      for (int i = 0; i < FP / 2; ++i) {
        const int f0 = nt * (BP / 2) + wr * (BP / 4) + i * 16 + 4 * g;
        if (f0 >= a.N_out) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = p4_silu(acc[i][j][e] * sx) * (acc[FP / 2 + i][j][e] * sx);
        const p4_u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
        *reinterpret_cast<p4_u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)m * a.N_out + f0) = o;
      }
    } else {
#pragma unroll
      for (int i = 0; i < FP; ++i) {
        const int n0 = nt * BP + wr * (BP / 2) + i * 16 + 4 * g;
        if (n0 >= a.N_out) continue;
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = acc[i][j][e] * sx;
        if constexpr (EPI == P4_F32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.out) + (size_t)m * a.N_out + n0) =
              f32x4{v[0], v[1], v[2], v[3]};
        } else {
          if (a.res != nullptr) {
            const p4_u32x2 rr = *reinterpret_cast<const p4_u32x2*>(a.res + (size_t)m * a.N_out + n0);
            v[0] += lo_bf(rr[0]);
            v[1] += hi_bf(rr[0]);
            v[2] += lo_bf(rr[1]);
            v[3] += hi_bf(rr[1]);
          }
          const p4_u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
          *reinterpret_cast<p4_u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)m * a.N_out + n0) = o;
        }
      }
    }
  }
#endif
}

// Split-K combine: out[m, 4 q .. 4 q + 3] = epi(sum over slices of the slabs), slices in order.  One thread per
// 4 output features of one token; x scaling (RMS) and the residual as in the main kernel's epilogue.
// MXO (SwiGLU, fp8 weights): the output is MX e4m3 + E8M0 -- the 8 threads of a 32-feature block (adjacent, one
// wave) take the block's max by shuffles.  FP8 with xs == nullptr: MX activations (their scales were the MFMA's).
template <int EPI, bool RMS, bool FP8, bool MXO = false>
__global__ void __launch_bounds__(256) pgemm_reduce_kernel(void* __restrict__ out, const bf16_t* res,
                                                           const float* __restrict__ slab, int splits, int M,
                                                           int N_out, int half_rows, int wrows, int K, float eps,
                                                           const float* __restrict__ xs,
                                                           const float* __restrict__ wsc, uint8_t* __restrict__ oq,
                                                           uint8_t* __restrict__ oe) {
  const long long idx = (long long)blockIdx.x * 256 + threadIdx.x;
  const int qn = N_out / 4;
  if (idx >= (long long)M * qn) return;   // MXO: M * qn is a multiple of 8, so a block's 8 threads exit together
  const int m = (int)(idx / qn), n0 = (int)(idx - (long long)m * qn) * 4;
  const size_t stride = (size_t)M * wrows;
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, u = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < splits; ++k) {
    const float* p = slab + (size_t)k * stride + (size_t)m * wrows;
    s += *reinterpret_cast<const f32x4*>(p + n0);
    if (EPI == P4_SWIGLU) u += *reinterpret_cast<const f32x4*>(p + half_rows + n0);
  }
  float sx = 1.f;
  if (RMS) {
    float t = 0.f;
    for (int k = 0; k < splits; ++k) t += slab[(size_t)splits * stride + (size_t)k * M + m];
    sx = rsqrtf(t / (float)K + eps);
  }
  if (FP8 && xs != nullptr) sx *= xs[m];
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (EPI == P4_SWIGLU) {
      float gt = s[e] * sx, up = u[e] * sx;
      if (FP8) {
        gt *= wsc[n0 + e];
        up *= wsc[half_rows + n0 + e];
      }
      v[e] = p4_silu(gt) * up;
      if (MXO) v[e] = bf_round(v[e]);
    } else {
      v[e] = s[e] * sx * (FP8 ? wsc[n0 + e] : 1.f);
    }
  }
  if constexpr (MXO) {
    float amax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
    amax = fmaxf(amax, __shfl_xor(amax, 1, WAVE));
    amax = fmaxf(amax, __shfl_xor(amax, 2, WAVE));
    amax = fmaxf(amax, __shfl_xor(amax, 4, WAVE));
    const uint32_t e = mx_e8m0(amax);
    *reinterpret_cast<uint32_t*>(oq + (size_t)m * N_out + n0) = mx_pack4(v[0], v[1], v[2], v[3], mx_inv_scale(e));
    if ((n0 & 31) == 0) oe[mx_scale_off(m, n0 >> 5, M)] = (uint8_t)e;
  } else if (EPI == P4_F32) {
    *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(out) + (size_t)m * N_out + n0) = f32x4{v[0], v[1], v[2], v[3]};
  } else {
    if (EPI == P4_BF16 && res != nullptr) {
      const p4_u32x2 rr = *reinterpret_cast<const p4_u32x2*>(res + (size_t)m * N_out + n0);
      v[0] += lo_bf(rr[0]);
      v[1] += hi_bf(rr[0]);
      v[2] += lo_bf(rr[1]);
      v[3] += hi_bf(rr[1]);
    }
    const p4_u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
    *reinterpret_cast<p4_u32x2*>(reinterpret_cast<bf16_t*>(out) + (size_t)m * N_out + n0) = o;
  }
}

}  // namespace k8sllm

using namespace k8sllm;

namespace {
struct P4Cfg {
  int fp, fq;
  bool k64 = false;
};
// tile configurations: BP = 32 FP weight rows x BQ = 32 FQ tokens, 4 waves of (BP / 2) x (BQ / 2)
constexpr P4Cfg kP4Cfgs[] = {
    {8, 8},   // 0: 256 x 256
    {8, 4},   // 1: 256 x 128
    {4, 8},   // 2: 128 x 256
    {4, 4},   // 3: 128 x 128
    {8, 8, true},   // 4: 256 x 256, 64-deep LDS stages (128-byte rows): 1.01-1.10x of config 0 on 29 of 30 70B
                    // TP=1 / TP=8 shapes; the 64-deep forms of configs 1 and 2 were within 2 % of them and were dropped
                    // (profiles/pgemm4_asm_r6.txt)
};
constexpr int kP4NumCfgs = sizeof(kP4Cfgs) / sizeof(kP4Cfgs[0]);

template <int C, int EPI, bool RMS>
int p4_launch(const P4Args& a, hipStream_t s) {
  hipLaunchKernelGGL((pgemm4_kernel<kP4Cfgs[C].fp, kP4Cfgs[C].fq, EPI, RMS, kP4Cfgs[C].k64>), dim3(a.nwg),
                     dim3(256), 0, s, a);
  return (int)hipGetLastError();
}
template <int C>
int p4_epi(const P4Args& a, int epi, int rms, hipStream_t s) {
  if (rms) {
    switch (epi) {
      case P4_BF16: return p4_launch<C, P4_BF16, true>(a, s);
      case P4_F32: return p4_launch<C, P4_F32, true>(a, s);
      case P4_SWIGLU: return p4_launch<C, P4_SWIGLU, true>(a, s);
    }
  } else {
    switch (epi) {
      case P4_BF16: return p4_launch<C, P4_BF16, false>(a, s);
      case P4_F32: return p4_launch<C, P4_F32, false>(a, s);
      case P4_SWIGLU: return p4_launch<C, P4_SWIGLU, false>(a, s);
    }
  }
  return -2;
}
template <int C = 0>
int p4_cfg(const P4Args& a, int cfg, int epi, int rms, hipStream_t s) {
  if constexpr (C < kP4NumCfgs) {
    if (cfg == C) return p4_epi<C>(a, epi, rms, s);
    return p4_cfg<C + 1>(a, cfg, epi, rms, s);
  } else {
    return -4;
  }
}

template <int EPI, bool RMS, bool FP8, bool MXO = false>
int reduce_launch(void* out, const void* res, const float* slab, int splits, int M, int N_out, int half_rows,
                  int wrows, int K, float eps, const float* xs, const float* wsc, void* oq, void* oe, hipStream_t s) {
  const long long items = (long long)M * (N_out / 4);
  hipLaunchKernelGGL((pgemm_reduce_kernel<EPI, RMS, FP8, MXO>), dim3((unsigned)((items + 255) / 256)), dim3(256), 0,
                     s, out, static_cast<const bf16_t*>(res), slab, splits, M, N_out, half_rows, wrows, K, eps, xs,
                     wsc, static_cast<uint8_t*>(oq), static_cast<uint8_t*>(oe));
  return (int)hipGetLastError();
}
}  // namespace

// Split-K combine of pgemm slabs (also used by the fp8 kernel): slab = [splits][M][wrows] fp32, then (rms)
// [splits][M] row sums of squares.
extern "C" int k8s_pgemm_reduce(void* out, const void* res, const float* slab, int splits, int M, int N_out, int K,
                                int epi, int rms, float eps, const float* xs, const float* wsc, void* oq, void* oe,
                                hipStream_t s) {
  if (splits < 1 || M <= 0 || N_out <= 0 || N_out % 4) return -1;
  const int half = epi == P4_SWIGLU ? N_out : 0, wrows = epi == P4_SWIGLU ? 2 * N_out : N_out;
  const bool fp8 = wsc != nullptr;   // (xs == nullptr with fp8: MX activations)
  if (rms && fp8) return -6;
  if (oq != nullptr) {
    if (!fp8 || epi != P4_SWIGLU || oe == nullptr || N_out % 128) return -7;
    return reduce_launch<P4_SWIGLU, false, true, true>(out, res, slab, splits, M, N_out, half, wrows, K, eps, xs, wsc,
                                                      oq, oe, s);
  }
#define K8S_RED(E, R, F) \
  return reduce_launch<E, R, F>(out, res, slab, splits, M, N_out, half, wrows, K, eps, xs, wsc, nullptr, nullptr, s)
  if (fp8) {
    switch (epi) {
      case P4_BF16: K8S_RED(P4_BF16, false, true);
      case P4_F32: K8S_RED(P4_F32, false, true);
      case P4_SWIGLU: K8S_RED(P4_SWIGLU, false, true);
    }
  } else if (rms) {
    switch (epi) {
      case P4_BF16: K8S_RED(P4_BF16, true, false);
      case P4_F32: K8S_RED(P4_F32, true, false);
      case P4_SWIGLU: K8S_RED(P4_SWIGLU, true, false);
    }
  } else {
    switch (epi) {
      case P4_BF16: K8S_RED(P4_BF16, false, false);
      case P4_F32: K8S_RED(P4_F32, false, false);
      case P4_SWIGLU: K8S_RED(P4_SWIGLU, false, false);
    }
  }
#undef K8S_RED
  return -2;
}

extern "C" int k8s_pgemm4_num_configs() { return kP4NumCfgs; }

extern "C" int k8s_pgemm4_config(int cfg, int* bp, int* bq, int* lds_bytes) {
  if (cfg < 0 || cfg >= kP4NumCfgs) return -1;
  *bp = 32 * kP4Cfgs[cfg].fp;
  *bq = 32 * kP4Cfgs[cfg].fq;
  *lds_bytes = 4 * (*bp + *bq) * 64 + *bq * 8;
  return 0;
}

// Launch facts: workgroups and split-K slab elements (0 without split-K).
extern "C" int k8s_pgemm4_plan(int M, int N_out, int K, int epi, int cfg, int splits, int* nwg, long long* slab_elems) {
  if (cfg < 0 || cfg >= kP4NumCfgs || M <= 0 || N_out <= 0 || K <= 0 || splits < 1) return -1;
  if (K % 64 != 0 || N_out % 4 != 0) return -1;
  const int bp = 32 * kP4Cfgs[cfg].fp, bq = 32 * kP4Cfgs[cfg].fq;
  const int feat = epi == P4_SWIGLU ? bp / 2 : bp;
  const int ks = K / 32;
  if (splits > ks / 2) return -1;
  const long long tiles = (long long)((M + bq - 1) / bq) * ((N_out + feat - 1) / feat);
  if (tiles * splits > (1LL << 30)) return -1;
  const long long wrows = epi == P4_SWIGLU ? 2LL * N_out : N_out;
  *nwg = (int)(tiles * splits);
  *slab_elems = splits > 1 ? (long long)splits * M * wrows + (long long)splits * M : 0;
  return 0;
}

extern "C" int k8s_pgemm4(void* out, float* slab, const void* x, const void* W, int M, int N_out, int K, int epi,
                          int cfg, int splits, int group_m, const void* res, int rms, float eps, hipStream_t stream) {
  int nwg;
  long long nsl;
  if (k8s_pgemm4_plan(M, N_out, K, epi, cfg, splits, &nwg, &nsl) != 0) return -1;
  if (splits > 1 && slab == nullptr) return -3;
  const long long kbytes = (long long)K * 2;
  const long long wrows = epi == P4_SWIGLU ? 2LL * N_out : (long long)N_out;
  if (wrows * kbytes >= (1LL << 32) || (long long)M * kbytes >= (1LL << 32)) return -5;   // 32-bit DMA offsets
  if (res != nullptr && epi != P4_BF16) return -6;
  const int bp = 32 * kP4Cfgs[cfg].fp, bq = 32 * kP4Cfgs[cfg].fq;
  const int feat = epi == P4_SWIGLU ? bp / 2 : bp;
  P4Args a;
  a.out = out;
  a.res = static_cast<const bf16_t*>(res);
  a.slab = slab;
  a.x = static_cast<const uint8_t*>(x);
  a.W = static_cast<const uint8_t*>(W);
  a.kbytes = (uint32_t)kbytes;
  a.M = M;
  a.N_out = N_out;
  a.half_rows = epi == P4_SWIGLU ? N_out : 0;
  a.wrows = (int)wrows;
  a.K = K;
  a.m_tiles = (M + bq - 1) / bq;
  a.n_tiles = (N_out + feat - 1) / feat;
  a.ks = K / 32;
  a.splits = splits;
  a.group_m = group_m > 0 ? group_m : 1;
  a.nwg = nwg;
  a.eps = eps;
  int rc = p4_cfg(a, cfg, epi, rms, stream);
  if (rc != 0 || splits == 1) return rc;
  return k8s_pgemm_reduce(out, res, slab, splits, M, N_out, K, epi, rms, eps, nullptr, nullptr, nullptr, nullptr,
                          stream);
}
