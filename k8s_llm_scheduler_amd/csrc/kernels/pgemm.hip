// K3 / K8 / K9(+K10) / K11 / K12 / K15 for prefill-size row counts: the big-tile MFMA GEMM.
//
//     out[M, N_out] = epi( x[M, K] . W[N, K]^T )      epi: bf16 (+ residual) | fp32 | SwiGLU, optional RMS prologue
//
// mgemm.hip owns the weight-streaming regime (batched decode, <= ~128 rows).  This kernel owns prefill chunks
// (hundreds to thousands of rows), where the GEMM is MFMA-bound and the schedule decides everything.  Design:
//
//  * 512-thread workgroups (8 waves, 2 per SIMD), one per CU, output tile BP weight rows x BQ tokens (up to
//    256 x 256).  Waves form a 2 (P) x 4 (Q) grid; wave (wr, wc) owns 2*FP x 2*FQ 16x16 fragments, computed in
//    the swapped orientation C^T = W . x^T on v_mfma_f32_16x16x32_bf16 so every lane ends with 4 consecutive
//    output features of one token (8-byte bf16 stores, gate/up pairs side by side for SwiGLU).
//  * fp8 (OCP e4m3 x and W, per-token / per-row scales in the epilogue): the same tile and LDS image with
//    128-value k-tiles on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales), which runs at
//    twice the bf16 rate -- the non-scaled 16x16x32 fp8 MFMA is only as fast as bf16.
//  * k-tiles of 128 bytes per row (64 bf16 / 128 e4m3), split into four regions: QB0 / QB1 (the first / second FQ
//    fragments of every wave column) and PA0 / PA1 (the first / second FP fragments of every wave row).  The x
//    regions live in a two-stage LDS ring, the weight regions in a WS-stage ring (WS = 2, or 3 where the 160 KiB
//    hold it).  One k-tile is two phases, each two MFMA quadrants:
//        phase 0: read QB0 + QB1 + PA0, MFMA (a0, b0) (a0, b1)      phase 1: read PA1, MFMA (a1, b1) (a1, b0)
//    and each phase refills two regions with LDS-DMA (global_load_lds_dwordx4) at least one phase after their last
//    reader: PA0 + PA1 of k-tile t+WS-1 in phase 0, QB0 + QB1 of t+2 in phase 1.  Each wait is a counted
//    `s_waitcnt vmcnt` one phase before the first reader (never vmcnt(0) in the steady state; pg_window counts
//    the issue sequence).  The four-phase form (one quadrant per phase, one region per phase) ran 1.02-1.19x
//    slower on all 40 TP=1 / TP=8 70B shapes at 256-8192 rows: twice the barriers, and a quarter-k-tile MFMA
//    section too short to hide the partner group's reads (profiles/pgemm_two_phase_r6.txt).
//  * waves 4-7 run one barrier behind waves 0-3 (two barriers per phase): on every SIMD one wave is in its
//    MFMA section while its partner reads LDS and issues the next DMA (8-wave ping-pong).  Every LDS read is
//    retired (lgkmcnt(0)) before the phase's first barrier, which is what makes the one-phase refill legal for
//    both wave groups; the data a phase reads was waited for by every issuing wave one phase earlier.
//  * the DMA image is lane-linear; the XOR swizzle (16-byte chunk c of region row r at slot c ^ ((r >> 1) & 7))
//    is applied on the per-lane global source address, so the 16-row fragment reads (ds_read_b128) are
//    conflict-free.
//  * block -> tile: XCD-aware bijective remap, then group_m m-tiles per n-column group (the x rows and the
//    weight rows of concurrently running tiles share their XCD's L2); k-slices of one tile are adjacent.
//  * split-K (small tile counts, e.g. TP = 8 or 256-row prefill chunks): every slice stores its raw fp32 sums as a
//    row-major slab and k8s_pgemm_reduce (pgemm4.hip) sums the slabs in slice order (deterministic) and runs the
//    epilogue over every CU.  The alternative in-launch form (K8S_PGEMM_ROWSLAB=0) publishes fragment-order slabs
//    (agent release + arrival ticket) and the last arriving slice reduces them; the ticket is reset by the reducer.
//  * MX activations (fp8 = 3; K16 block-scaled, fp8.hip): the x bytes are OCP MX e4m3 and the E8M0 byte of each
//    32-value block is the B scale of the scaled MFMA (the lane holding that block's scale: li + 16 b, see
//    tools/experiments/mx_scale_probe.hip).  The tile's scale dwords (one per token row and k-tile) ride region QB0
//    as one 4-byte LDS-DMA per wave and are read in phase 0 with the QB0 fragments (the region's last reader).
//  * MX output (SwiGLU, mx_out): each wave's features come in 32-feature blocks (fragment pairs), so the epilogue
//    writes e4m3 + E8M0 directly (4-lane shuffle max) -- the down projection's input, quantized by its producer.
//  * RMS prologue (bf16): the un-normalised residual stream is the x operand; the x fragments every wave
//    already holds give the row sums of squares (v_dot2_f32_bf16, waves 0-3 for QB0, 4-7 for QB1), and the
//    epilogue scales by 1 / rms (the norm gamma is folded into W at load time).
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace k8sllm {

namespace {
enum { PG_BF16 = 0, PG_F32 = 1, PG_SWIGLU = 2 };

typedef __attribute__((ext_vector_type(2))) uint32_t pg_u32x2;
typedef __attribute__((ext_vector_type(8))) int pg_i32x8;
typedef __attribute__((ext_vector_type(4))) int pg_i32x4;

template <int N>
__device__ __forceinline__ void pg_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wave-uniform count -> immediate (the tail k-tiles; the steady state uses constants).  A count above the largest
// case waits for more than needed, which is always safe.
template <int N>
__device__ __forceinline__ void pg_vm_wait_chain(int n) {
  if constexpr (N == 0) {
    pg_vmcnt<0>();
  } else {
    if (n >= N) pg_vmcnt<N>();
    else pg_vm_wait_chain<N - 1>(n);
  }
}
__device__ __forceinline__ void pg_vm_wait(int n) { pg_vm_wait_chain<40>(n); }
// retire this wave's LDS reads, then the raw workgroup barrier (LDS-DMA stays in flight across it)
__device__ __forceinline__ void pg_sync_reads() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void pg_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ float pg_silu(float g) { return g / (1.f + __expf(-g)); }

// LDS-DMA issue sequence.  Position s = 4 base + k issues region k: 0 PA0 / 1 PA1 of k-tile base + WS - 1 (both in
// phase 0 of local k-tile base), 2 QB0 / 3 QB1 of k-tile base + 2 (both in phase 1); positions < 0 are the
// prologue.  x regions (QB0 / QB1) live in a two-stage ring (stage u & 1), weight regions (PA0 / PA1) in a
// WS-stage ring (stage u % WS).
__host__ __device__ constexpr int pg_floor4(int s) { return s >= 0 ? s / 4 : -((-s + 3) / 4); }
template <int WS>
__host__ __device__ constexpr int pg_seq_tile(int s) {
  const int base = pg_floor4(s), k = s - 4 * base;
  return base + (k < 2 ? WS - 1 : 2);
}
template <int WS> __host__ __device__ constexpr int pg_pos_pa0(int u) { return 4 * (u - WS + 1); }
template <int WS> __host__ __device__ constexpr int pg_pos_pa1(int u) { return 4 * (u - WS + 1) + 1; }
__host__ __device__ constexpr int pg_pos_qb0(int u) { return 4 * (u - 2) + 2; }
__host__ __device__ constexpr int pg_pos_qb1(int u) { return 4 * (u - 2) + 3; }
// the last position phase j of local k-tile t issues
__host__ __device__ constexpr int pg_issue_end(int j, int t) { return 4 * t + (j == 0 ? 1 : 3); }
// DMA instructions per wave issued at positions (s0, s1] whose k-tile is in [0, n)
template <int GP, int GQ, int GS, int WS>
__host__ __device__ constexpr int pg_window(int s0, int s1, int n) {
  int c = 0;
  for (int s = s0 + 1; s <= s1; ++s) {
    const int u = pg_seq_tile<WS>(s), k = s - 4 * pg_floor4(s);
    if (u >= 0 && u < n) c += k < 2 ? GP : k == 2 ? GQ + GS : GQ;
  }
  return c;
}
__host__ __device__ constexpr int pg_max(int a, int b) { return a > b ? a : b; }
// phase j's wait covers what the next phase reads: phase 0 waits for PA1(t), phase 1 for QB0 / QB1 / PA0 of
// k-tile t + 1 (the latest of their positions)
template <int WS>
__host__ __device__ constexpr int pg_wait_target(int j, int t) {
  return j == 0 ? pg_pos_pa1<WS>(t) : pg_max(pg_pos_qb1(t + 1), pg_pos_pa0<WS>(t + 1));
}
template <int GP, int GQ, int GS, int WS>
__host__ __device__ constexpr int pg_steady(int j) {   // every position of the window exists (t = 16 stands for any)
  return pg_window<GP, GQ, GS, WS>(pg_wait_target<WS>(j, 16), pg_issue_end(j, 16), 1 << 30);
}
__host__ __device__ constexpr int pg_lds_ring(int bp, int bq, int ws, bool mx) {
  return 2 * (bq * 128 + (mx ? bq * 4 : 0)) + ws * bp * 128;
}
constexpr int PG_LDS_MAX = 163840;
}  // namespace

struct PgArgs {
  void* out;
  const bf16_t* res;     // optional residual (bf16 [M][N_out], may alias out)
  float* ws;             // split-K slabs [tiles][splits][BP * BQ + BQ]
  unsigned* cnt;         // [tiles] arrival tickets, zero between launches
  const uint8_t* x;      // [M][K] bf16 or e4m3
  const uint8_t* W;      // [rows][K] bf16 or e4m3
  const float* xs;       // fp8: [M] per-token scales
  const float* wsc;      // fp8: [rows] per-row scales
  const uint8_t* xe;     // MX activations: E8M0 block scales, [K / 128][M] dwords (mx_scale_off)
  uint8_t* oq;           // MX output (SwiGLU): e4m3 [M][N_out] + E8M0 (mx_scale_off layout)
  uint8_t* oe;
  uint32_t kbytes;       // bytes per row of x and W
  int M, N_out, half_rows, K;
  int m_tiles, n_tiles, kt, splits, group_m, nwg;
  int prio;              // wave priority: 0 = s_setprio 1 around every MFMA section, 1 = waves 4-7 at 1 for the
                         // whole loop (MI355X_MICROARCH.md "static priority for the younger half"), 2 = none
  float eps;
  int row_slabs;         // split-K: 1 = every slice stores a row-major slab ([splits][M][wrows], then the RMS row
                         // sums [splits][M]) and k8s_pgemm_reduce (all CUs) combines them -- no last-arriver tail
};

template <int FP, int FQ, int EPI, bool FP8, bool RMS, bool MX = false, bool MXO = false, int WS = 2>
__global__ void __launch_bounds__(512) pgemm_kernel(PgArgs a) {
  constexpr int BP = 64 * FP, BQ = 128 * FQ;         // weight rows, tokens per tile
  constexpr int RP = BP / 2, RQ = BQ / 2;            // rows per PA / QB region
  constexpr int GP = RP / 64, GQ = RQ / 64;          // 16-byte DMA instructions per thread per region
  constexpr int GS = MX ? 1 : 0;                     // MX: one 4-byte scale LDS-DMA per wave with QB0
  constexpr int SCH = BQ / 8;                        // MX: scale dwords (token rows) per wave
  // LDS: x ring [2][QB0 | QB1 | MX scales], then the weight ring [WS][PA0 | PA1]
  constexpr int XSTAGE = BQ * 128 + (MX ? BQ * 4 : 0), WSTAGE = BP * 128, WOFF = 2 * XSTAGE;
  constexpr int OFF_QB0 = 0, OFF_QB1 = RQ * 128, OFF_SC = BQ * 128, OFF_PA0 = 0, OFF_PA1 = RP * 128;
  constexpr int RING = pg_lds_ring(BP, BQ, WS, MX);
  constexpr int NA = 2 * FP, NB = 2 * FQ;            // fragments per wave along P / Q
  constexpr int SLAB = BP * BQ + BQ;
  // counted waits (see phase()): j = 0 waits for PA1(t), j = 1 for QB0 / QB1 / PA0 of k-tile t + 1
  constexpr int STEADY0 = pg_steady<GP, GQ, GS, WS>(0), STEADY1 = pg_steady<GP, GQ, GS, WS>(1);
  static_assert(GP >= 1 && GQ >= 1 && WS >= 2 && WS <= 4 && STEADY0 <= 40 && STEADY1 <= 40, "tile shape");
  static_assert(RING <= PG_LDS_MAX && 64 + BQ * 4 <= RING, "LDS");
  static_assert(!(FP8 && RMS), "fp8 activations are quantized before the GEMM");
  static_assert(!MX || FP8, "MX: e4m3 activations");
  static_assert(!MXO || (EPI == PG_SWIGLU && FP8 && FP % 2 == 0), "MX output: SwiGLU fragment pairs");
  static_assert(SCH <= 64, "scale dwords per wave");
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the launch stub
  __shared__ __attribute__((aligned(16))) char lds[RING];
  // after the main loop only (the ring is dead then: every wave has passed the re-aligning barrier)
  unsigned* flag = reinterpret_cast<unsigned*>(lds);
  float* rss = reinterpret_cast<float*>(lds + 64);   // [BQ] row sums of squares

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int li = lane & 15, g = lane >> 4;
  const bool late = __builtin_amdgcn_readfirstlane(tid) >= 256;   // waves 4-7, provably wave-uniform

  // ---- block -> (tile, k-slice): XCD-aware bijective remap, grouped tile order
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
  const int kt0 = (int)((long long)slice * a.kt / a.splits);
  const int n = (int)((long long)(slice + 1) * a.kt / a.splits) - kt0;

  // ---- per-thread DMA sources (byte offsets from the operand bases; the host checks < 4 GiB)
  uint32_t oq0[GQ], oq1[GQ], op0[GP], op1[GP], osc = 0;
  if constexpr (MX)   // token row wid * SCH + lane of the tile, k-tile kt0: [K / 128][M] scale dwords
    osc = ((uint32_t)kt0 * (uint32_t)a.M + (uint32_t)min(mt * BQ + wid * SCH + min(lane, SCH - 1), a.M - 1)) * 4u;
#pragma unroll
  for (int i = 0; i < GQ; ++i) {
    const int p = i * 512 + tid, r = p >> 3, c = (p & 7) ^ ((r >> 1) & 7);
    const int w = r / (BQ / 8), q = r % (BQ / 8);
    const int m0 = mt * BQ + w * (BQ / 4) + q;
    const uint32_t col = (uint32_t)(c * 16 + kt0 * 128);
    oq0[i] = (uint32_t)min(m0, a.M - 1) * a.kbytes + col;
    oq1[i] = (uint32_t)min(m0 + BQ / 8, a.M - 1) * a.kbytes + col;
  }
#pragma unroll
  for (int i = 0; i < GP; ++i) {
    const int p = i * 512 + tid, r = p >> 3, c = (p & 7) ^ ((r >> 1) & 7);
    const int w = r / (BP / 4), q = r % (BP / 4);
    const uint32_t col = (uint32_t)(c * 16 + kt0 * 128);
    int r0, r1;
    if constexpr (EPI == PG_SWIGLU) {   // each wave's a0 half = gate rows, a1 half = the matching up rows
      const int f = min(nt * (BP / 2) + w * (BP / 4) + q, a.N_out - 1);
      r0 = f;
      r1 = a.half_rows + f;
    } else {
      r0 = min(nt * BP + w * (BP / 2) + q, a.N_out - 1);
      r1 = min(nt * BP + w * (BP / 2) + BP / 4 + q, a.N_out - 1);
    }
    op0[i] = (uint32_t)r0 * a.kbytes + col;
    op1[i] = (uint32_t)r1 * a.kbytes + col;
  }

  auto dma = [&](const uint8_t* src, const uint32_t* off, char* dst, auto G_) {
    constexpr int G = decltype(G_)::value;
#pragma unroll
    for (int i = 0; i < G; ++i)
      __builtin_amdgcn_global_load_lds(src + off[i], (__attribute__((address_space(3))) void*)(dst + i * 8192), 16,
                                       0, 0);
  };
  auto xstage = [&](int u) { return lds + (u & 1) * XSTAGE; };
  auto wstage = [&](int u) { return lds + WOFF + (WS == 2 ? (u & 1) : (int)((unsigned)u % (unsigned)WS)) * WSTAGE; };
  // issue region y of local k-tile u: x regions into x stage u & 1, weight regions into weight stage u % WS
  auto issue = [&](auto Y, int u) {
    constexpr int y = decltype(Y)::value;
    char* dst = ((y & 1) ? wstage(u) : xstage(u)) + wid * 1024 +
                (y == 0 ? OFF_QB0 : y == 1 ? OFF_PA0 : y == 2 ? OFF_QB1 : OFF_PA1);
    const uint32_t kb = (uint32_t)u * 128u;
    if constexpr (y == 0) {
      dma(a.x + kb, oq0, dst, std::integral_constant<int, GQ>{});
      if constexpr (MX) {
        if (lane < SCH)
          __builtin_amdgcn_global_load_lds(a.xe + (osc + (uint32_t)u * (uint32_t)a.M * 4u),   // saddr + 32-bit voffset
                                           (__attribute__((address_space(3))) void*)(xstage(u) + OFF_SC +
                                                                                     wid * SCH * 4),
                                           4, 0, 0);
      }
    }
    if constexpr (y == 1) dma(a.W + kb, op0, dst, std::integral_constant<int, GP>{});
    if constexpr (y == 2) dma(a.x + kb, oq1, dst, std::integral_constant<int, GQ>{});
    if constexpr (y == 3) dma(a.W + kb, op1, dst, std::integral_constant<int, GP>{});
  };
  using Y0 = std::integral_constant<int, 0>;
  using Y1 = std::integral_constant<int, 1>;
  using Y2 = std::integral_constant<int, 2>;
  using Y3 = std::integral_constant<int, 3>;

  // ---- fragment read offsets inside a region: row li of a 16-row fragment, swizzled 16-byte chunk
  const int swz = li >> 1;
  int lo[2];
#pragma unroll
  // lane (li, g): bf16 k32 step h = chunk 4 h + g; fp8 (one 16x16x128 step) chunks g and 4 + g, the scaled MFMA's
  // operand layout (k 16 g.. in bytes 0-15, 64 + 16 g.. in bytes 16-31; tools/experiments/mx_scale_probe.hip)
  for (int h = 0; h < 2; ++h) lo[h] = li * 128 + (((4 * h + g) ^ swz) << 4);
  const int pbase = wr * (BP / 4) * 128, qbase = wc * (BQ / 8) * 128;

  // operand registers: bf16 [k32 step][fragment]; fp8 [fragment] x two 16-byte halves
  using frag_t = typename std::conditional<FP8, pg_i32x8, bf16x8>::type;
  frag_t Ar[FP8 ? 1 : 2][FP], B0r[FP8 ? 1 : 2][FQ], B1r[FP8 ? 1 : 2][FQ];
  f32x4 acc[NA][NB];
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ss[FQ];
#pragma unroll
  for (int f = 0; f < FQ; ++f) ss[f] = 0.f;
  // MX: this lane's B scales (block g of its token row) for the 2 * FQ x fragments of the current k-tile, packed
  // one byte each into ONE register (byte h * FQ + f; the MFMA's op_sel picks it) -- the kernel sits at the VGPR
  // limit, and four separate registers spilled inside the main loop (scratch loads there drain the LDS-DMA ring)
  static_assert(!MX || FQ <= 2, "MX: 2 * FQ scale bytes per register");
  int scp = 0x7f7f7f7f;

  auto read_frags = [&](const char* rb, frag_t* d0, frag_t* d1, auto NF_) {
    constexpr int NF = decltype(NF_)::value;
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const char* p = rb + f * 16 * 128;
      if constexpr (FP8) {
        const pg_i32x4 lo4 = *reinterpret_cast<const pg_i32x4*>(p + lo[0]);
        const pg_i32x4 hi4 = *reinterpret_cast<const pg_i32x4*>(p + lo[1]);
        d0[f] = pg_i32x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
      } else {
        d0[f] = *reinterpret_cast<const bf16x8*>(p + lo[0]);
        d1[f] = *reinterpret_cast<const bf16x8*>(p + lo[1]);
      }
    }
  };
  using NFP = std::integral_constant<int, FP>;
  using NFQ = std::integral_constant<int, FQ>;

  auto mma = [&](auto AH, auto BH) {
    constexpr int ah = decltype(AH)::value, bh = decltype(BH)::value;
#pragma unroll
    for (int kk = 0; kk < (FP8 ? 1 : 2); ++kk)
#pragma unroll
      for (int fp = 0; fp < FP; ++fp)
#pragma unroll
        for (int fq = 0; fq < FQ; ++fq) {
          f32x4& c = acc[ah * FP + fp][bh * FQ + fq];
          if constexpr (FP8) {
            if (fq == 0)
              c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(Ar[0][fp], bh ? B1r[0][fq] : B0r[0][fq], c, 0, 0, 0,
                                                                   0x7f7f7f7f, bh * FQ, scp);
            else
              c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(Ar[0][fp], bh ? B1r[0][fq] : B0r[0][fq], c, 0, 0, 0,
                                                                   0x7f7f7f7f, (bh * FQ + 1) & 3, scp);
          } else {
            c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(Ar[kk][fp], bh ? B1r[kk][fq] : B0r[kk][fq], c, 0, 0, 0);
          }
        }
  };
  auto squares = [&](auto BH) {   // RMS prologue: this wave's x fragments of half bh
    if constexpr (RMS) {
      constexpr int bh = decltype(BH)::value;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int fq = 0; fq < FQ; ++fq) {
          const bf16x8 v = bh ? B1r[kk][fq] : B0r[kk][fq];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bf16x2 v2 = {v[2 * e], v[2 * e + 1]};
            ss[fq] = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, ss[fq], false);
          }
        }
    }
  };

  // one phase of local k-tile t (J = 0 / 1): phase 0 reads QB0 + QB1 + PA0 and runs quadrants (a0, b0), (a0, b1);
  // phase 1 reads PA1 and runs (a1, b1), (a1, b0)
  auto phase = [&](auto J, int t) {
    constexpr int j = decltype(J)::value;
    const char* sb = xstage(t);
    const char* wb = wstage(t);
    if constexpr (j == 0) {
      read_frags(sb + OFF_QB0 + qbase, B0r[0], B0r[FP8 ? 0 : 1], NFQ{});
      read_frags(sb + OFF_QB1 + qbase, B1r[0], B1r[FP8 ? 0 : 1], NFQ{});
      read_frags(wb + OFF_PA0 + pbase, Ar[0], Ar[FP8 ? 0 : 1], NFP{});
      if constexpr (MX) {   // both halves' scales now: the region is refilled in phase 1
        const int* scl = reinterpret_cast<const int*>(sb + OFF_SC);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int f = 0; f < FQ; ++f) {
            const uint32_t byte = ((uint32_t)scl[wc * (BQ / 4) + h * (BQ / 8) + f * 16 + li] >> (8 * g)) & 0xffu;
            scp = (int)(((uint32_t)scp & ~(0xffu << (8 * (h * FQ + f)))) | (byte << (8 * (h * FQ + f))));
          }
      }
      if (t + WS - 1 < n) {
        issue(Y1{}, t + WS - 1);
        issue(Y3{}, t + WS - 1);
      }
    } else {
      read_frags(wb + OFF_PA1 + pbase, Ar[0], Ar[FP8 ? 0 : 1], NFP{});
      if (t + 2 < n) {
        issue(Y0{}, t + 2);
        issue(Y2{}, t + 2);
      }
    }
    if (t >= 2 && t + WS < n) {
      pg_vmcnt<j == 0 ? STEADY0 : STEADY1>();
    } else {
      pg_vm_wait(pg_window<GP, GQ, GS, WS>(pg_wait_target<WS>(j, t), pg_issue_end(j, t), n));
    }
    pg_sync_reads();
    __builtin_amdgcn_sched_barrier(0);
    if (a.prio == 0) __builtin_amdgcn_s_setprio(1);
    if constexpr (j == 0) {
      mma(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
      mma(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{});
      if (wr == 0) squares(std::integral_constant<int, 0>{});
    } else {
      mma(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{});
      mma(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{});
      if (wr == 1) squares(std::integral_constant<int, 1>{});
    }
    if (a.prio == 0) __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    pg_barrier();
  };

  // ---- prologue: the sequence positions before k-tile 0's phase 0 (WS = 2: k-tile 0 whole and k-tile 1 except
  // PA1, which k-tile 0's phase 0 issues), in sequence order
#pragma unroll
  for (int s = -4 * WS - 4; s < 0; ++s) {
    const int u = pg_seq_tile<WS>(s), k = s - 4 * pg_floor4(s);
    if (u < 0 || u >= n) continue;
    if (k == 0) issue(Y1{}, u);
    else if (k == 1) issue(Y3{}, u);
    else if (k == 2) issue(Y0{}, u);
    else issue(Y2{}, u);
  }
  pg_vm_wait(pg_window<GP, GQ, GS, WS>(pg_wait_target<WS>(1, -1), -1, n));
  pg_barrier();
  if (late) __builtin_amdgcn_s_barrier();   // stagger waves 4-7 by one barrier (wave-uniform branch)
  if (a.prio == 1 && late) __builtin_amdgcn_s_setprio(1);

  for (int t = 0; t < n; ++t) {
    phase(std::integral_constant<int, 0>{}, t);
    phase(std::integral_constant<int, 1>{}, t);
  }
  if (!late) __builtin_amdgcn_s_barrier();  // re-align the two wave groups
  if (a.prio == 1) __builtin_amdgcn_s_setprio(0);
  pg_vmcnt<0>();

  // ---- RMS: row sums of squares of this slice -> rss[token row of the tile]
  if constexpr (RMS) {
#pragma unroll
    for (int f = 0; f < FQ; ++f) {
      ss[f] += __shfl_xor(ss[f], 16, WAVE);
      ss[f] += __shfl_xor(ss[f], 32, WAVE);
    }
    if (g == 0) {
#pragma unroll
      for (int f = 0; f < FQ; ++f) rss[wc * (BQ / 4) + wr * (BQ / 8) + f * 16 + li] = ss[f];
    }
    __syncthreads();
  }

  // ---- split-K, row-major slabs: this slice's raw sums go where the reduce kernel reads them; done
  if (a.splits > 1 && a.row_slabs) {
    const long long wrows = EPI == PG_SWIGLU ? 2LL * a.N_out : (long long)a.N_out;
    float* sl = a.ws + (size_t)slice * a.M * wrows;
#pragma unroll
    for (int bq = 0; bq < NB; ++bq) {
      const int bh = bq / FQ, fq = bq % FQ;
      const int m = mt * BQ + wc * (BQ / 4) + bh * (BQ / 8) + fq * 16 + li;
      if (m >= a.M) continue;
      float* row = sl + (size_t)m * wrows;
      if constexpr (EPI == PG_SWIGLU) {
#pragma unroll
        for (int fp = 0; fp < FP; ++fp) {
          const int f0 = nt * (BP / 2) + wr * (BP / 4) + fp * 16 + 4 * g;
          if (f0 >= a.N_out) continue;
          *reinterpret_cast<f32x4*>(row + f0) = acc[fp][bq];
          *reinterpret_cast<f32x4*>(row + a.N_out + f0) = acc[FP + fp][bq];
        }
      } else {
#pragma unroll
        for (int ap = 0; ap < NA; ++ap) {
          const int ah = ap / FP, fp = ap % FP;
          const int n0 = nt * BP + wr * (BP / 2) + ah * (BP / 4) + fp * 16 + 4 * g;
          if (n0 < a.N_out) *reinterpret_cast<f32x4*>(row + n0) = acc[ap][bq];
        }
      }
    }
    if constexpr (RMS) {   // one n-tile per m-tile publishes the slice's row sums of squares
      if (nt == 0 && tid < BQ && mt * BQ + tid < a.M)
        a.ws[(size_t)a.splits * a.M * wrows + (size_t)slice * a.M + mt * BQ + tid] = rss[tid];
    }
    return;
  }

  // ---- split-K: publish this slice; the last arriving slice of the tile reduces every slab in order
  if (a.splits > 1) {
    float* base = a.ws + (size_t)tile * a.splits * SLAB;
    float* slab = base + (size_t)slice * SLAB;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
        *reinterpret_cast<f32x4*>(slab + ((size_t)((wid * NA + i) * NB + j) * 64 + lane) * 4) = acc[i][j];
    if (RMS && tid < BQ) slab[BP * BQ + tid] = rss[tid];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned old = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned last = old == (unsigned)(a.splits - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        a.cnt[tile] = 0u;
      }
      *flag = last;
    }
    __syncthreads();
    if (*flag == 0u) return;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < a.splits; ++s) {
      const float* sl = base + (size_t)s * SLAB;
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          acc[i][j] += *reinterpret_cast<const f32x4*>(sl + ((size_t)((wid * NA + i) * NB + j) * 64 + lane) * 4);
    }
    if constexpr (RMS) {
      __syncthreads();
      if (tid < BQ) {
        float t = 0.f;
        for (int s = 0; s < a.splits; ++s) t += base[(size_t)s * SLAB + BP * BQ + tid];
        rss[tid] = t;
      }
      __syncthreads();
    }
  }

  // ---- epilogue: lane holds out[token li of fragment bq][features 4 g .. 4 g + 3 of fragment ap]
#pragma unroll
  for (int bq = 0; bq < NB; ++bq) {
    const int bh = bq / FQ, fq = bq % FQ;
    const int mloc = wc * (BQ / 4) + bh * (BQ / 8) + fq * 16 + li;
    const int m = mt * BQ + mloc;
    if (m >= a.M) continue;
    float sx = 1.f;
    if constexpr (FP8 && !MX) sx = a.xs[m];
    if constexpr (RMS) sx = rsqrtf(rss[mloc] / (float)a.K + a.eps);
    if constexpr (MXO) {   // 32-feature blocks = fragment pairs (2 b, 2 b + 1); the block's lanes share li
#pragma unroll
      for (int b = 0; b < FP / 2; ++b) {
        const int nb = nt * (BP / 2) + wr * (BP / 4) + b * 32;
        if (nb >= a.N_out) continue;   // N_out % 32 == 0: whole blocks
        float v[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fp = 2 * b + h, f0 = nb + 16 * h + 4 * g;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float gt = acc[fp][bq][i] * sx * a.wsc[f0 + i], up = acc[FP + fp][bq][i] * sx * a.wsc[a.half_rows + f0 + i];
            v[4 * h + i] = bf_round(pg_silu(gt) * up);
          }
        }
        float amax = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
        amax = fmaxf(amax, __shfl_xor(amax, 16, WAVE));
        amax = fmaxf(amax, __shfl_xor(amax, 32, WAVE));
        const uint32_t e = mx_e8m0(amax);
        const float inv = mx_inv_scale(e);
        uint8_t* orow = a.oq + (size_t)m * a.N_out;
        *reinterpret_cast<uint32_t*>(orow + nb + 4 * g) = mx_pack4(v[0], v[1], v[2], v[3], inv);
        *reinterpret_cast<uint32_t*>(orow + nb + 16 + 4 * g) = mx_pack4(v[4], v[5], v[6], v[7], inv);
        if (g == 0) a.oe[mx_scale_off(m, nb >> 5, a.M)] = (uint8_t)e;
      }
    } else if constexpr (EPI == PG_SWIGLU) {
#pragma unroll
      for (int fp = 0; fp < FP; ++fp) {
        const int f0 = nt * (BP / 2) + wr * (BP / 4) + fp * 16 + 4 * g;
        if (f0 >= a.N_out) continue;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          float gt = acc[fp][bq][i] * sx, up = acc[FP + fp][bq][i] * sx;
          if constexpr (FP8) {
            gt *= a.wsc[f0 + i];
            up *= a.wsc[a.half_rows + f0 + i];
          }
          v[i] = pg_silu(gt) * up;
        }
        const pg_u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
        *reinterpret_cast<pg_u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)m * a.N_out + f0) = o;
      }
    } else {
#pragma unroll
      for (int ap = 0; ap < NA; ++ap) {
        const int ah = ap / FP, fp = ap % FP;
        const int n0 = nt * BP + wr * (BP / 2) + ah * (BP / 4) + fp * 16 + 4 * g;
        if (n0 >= a.N_out) continue;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = acc[ap][bq][i] * sx * (FP8 ? a.wsc[n0 + i] : 1.f);
        if constexpr (EPI == PG_F32) {
          *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.out) + (size_t)m * a.N_out + n0) =
              f32x4{v[0], v[1], v[2], v[3]};
        } else {
          if (a.res != nullptr) {
            const pg_u32x2 rr = *reinterpret_cast<const pg_u32x2*>(a.res + (size_t)m * a.N_out + n0);
            v[0] += lo_bf(rr[0]);
            v[1] += hi_bf(rr[0]);
            v[2] += lo_bf(rr[1]);
            v[3] += hi_bf(rr[1]);
          }
          const pg_u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
          *reinterpret_cast<pg_u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (size_t)m * a.N_out + n0) = o;
        }
      }
    }
  }
#endif
}

}  // namespace k8sllm

using namespace k8sllm;

namespace {
struct PgCfg {
  int fp, fq, ws;
};
// tile configurations: BP = 64 FP weight rows x BQ = 128 FQ tokens, WS weight-ring stages.  (3-4-stage rings at the
// smaller tiles never beat configs 0-3: profiles/pgemm_weight_ring_r6.txt)
constexpr PgCfg kPgCfgs[] = {
    {4, 2, 2},   // 0: 256 x 256
    {2, 2, 2},   // 1: 128 x 256
    {4, 1, 2},   // 2: 256 x 128
    {2, 1, 2},   // 3: 128 x 128
    {4, 2, 3},   // 4: 256 x 256, three weight stages (all 160 KiB of LDS; MX activations: two)
};
// the weight-ring depth a config runs with: its own where the LDS holds it, else two
constexpr int pg_ws(const PgCfg& c, bool mx) {
  return pg_lds_ring(64 * c.fp, 128 * c.fq, c.ws, mx) <= PG_LDS_MAX ? c.ws : 2;
}
constexpr int kPgNumCfgs = sizeof(kPgCfgs) / sizeof(kPgCfgs[0]);

template <int C, int EPI, bool FP8, bool RMS, bool MX = false, bool MXO = false>
int pg_launch(const PgArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((pgemm_kernel<kPgCfgs[C].fp, kPgCfgs[C].fq, EPI, FP8, RMS, MX, MXO, pg_ws(kPgCfgs[C], MX)>),
                     dim3(a.nwg), dim3(512), 0, s, a);
  return (int)hipGetLastError();
}

template <int C, bool MX>
int pg_epi_f8(const PgArgs& a, int epi, bool mxo, hipStream_t s) {
  if (mxo) return epi == PG_SWIGLU ? pg_launch<C, PG_SWIGLU, true, false, MX, true>(a, s) : -2;
  switch (epi) {
    case PG_BF16: return pg_launch<C, PG_BF16, true, false, MX>(a, s);
    case PG_F32: return pg_launch<C, PG_F32, true, false, MX>(a, s);
    case PG_SWIGLU: return pg_launch<C, PG_SWIGLU, true, false, MX>(a, s);
  }
  return -2;
}

template <int C, bool FP8>
int pg_epi(const PgArgs& a, int epi, int rms, hipStream_t s) {
  if constexpr (FP8) {
    const bool mxo = a.oq != nullptr;
    return a.xe != nullptr ? pg_epi_f8<C, true>(a, epi, mxo, s) : pg_epi_f8<C, false>(a, epi, mxo, s);
  } else {
    if (rms) {
      switch (epi) {
        case PG_BF16: return pg_launch<C, PG_BF16, false, true>(a, s);
        case PG_F32: return pg_launch<C, PG_F32, false, true>(a, s);
        case PG_SWIGLU: return pg_launch<C, PG_SWIGLU, false, true>(a, s);
      }
    } else {
      switch (epi) {
        case PG_BF16: return pg_launch<C, PG_BF16, false, false>(a, s);
        case PG_F32: return pg_launch<C, PG_F32, false, false>(a, s);
        case PG_SWIGLU: return pg_launch<C, PG_SWIGLU, false, false>(a, s);
      }
    }
  }
  return -2;
}

template <bool FP8, int C = 0>
int pg_cfg(const PgArgs& a, int cfg, int epi, int rms, hipStream_t s) {
  if constexpr (C < kPgNumCfgs) {
    if (cfg == C) return pg_epi<C, FP8>(a, epi, rms, s);
    return pg_cfg<FP8, C + 1>(a, cfg, epi, rms, s);
  } else {
    return -4;
  }
}

struct PgGeom {
  int m_tiles, n_tiles, tiles, kt;
};
PgGeom pg_geom(int M, int N_out, int K, int epi, int fp8, int cfg) {
  const int bp = 64 * kPgCfgs[cfg].fp, bq = 128 * kPgCfgs[cfg].fq;
  const int feat = epi == PG_SWIGLU ? bp / 2 : bp;
  PgGeom g;
  g.m_tiles = (M + bq - 1) / bq;
  g.n_tiles = (N_out + feat - 1) / feat;
  g.tiles = g.m_tiles * g.n_tiles;
  g.kt = K * (fp8 ? 1 : 2) / 128;
  return g;
}
}  // namespace

// Wave-priority mode of the main loop (PgArgs::prio): K8S_PGEMM_PRIO at load, k8s_pgemm_set_prio for A/B probes.
static int g_pg_prio = [] { const char* e = getenv("K8S_PGEMM_PRIO"); return e ? atoi(e) : 0; }();
extern "C" int k8s_pgemm_set_prio(int mode) {
  const int old = g_pg_prio;
  if (mode >= 0 && mode <= 2) g_pg_prio = mode;
  return old;
}

// Split-K combine: 1 (default) = row-major slabs + k8s_pgemm_reduce over every CU (one launch more, no cache-wide
// fence, no single-CU tail); 0 = the last arriving slice of each tile sums the tile's slabs (fragment order) in the
// same launch, after agent-scope release / acquire fences (an L2 write-back per arriving workgroup and an L2
// invalidate per reducer).  Bit-identical results (same slice order, same epilogue arithmetic).  Measured on the
// default bench (245-row chunks, the down projection at 8 splits): prefill 53.8-53.9 -> 46.9 ms per decision on one
// box, 46.8 either way on others (profiles/bench_r4_pgemm_rowslab_ab.txt).  K8S_PGEMM_ROWSLAB at load,
// k8s_pgemm_set_row_slabs for A/B probes.
static int g_pg_row_slabs = [] { const char* e = getenv("K8S_PGEMM_ROWSLAB"); return e ? atoi(e) : 1; }();
extern "C" int k8s_pgemm_set_row_slabs(int on) {
  const int old = g_pg_row_slabs;
  if (on >= 0) g_pg_row_slabs = on ? 1 : 0;
  return old;
}
extern "C" int k8s_pgemm_reduce(void* out, const void* res, const float* slab, int splits, int M, int N_out, int K,
                                int epi, int rms, float eps, const float* xs, const float* wsc, void* oq, void* oe,
                                hipStream_t s);

extern "C" int k8s_pgemm_num_configs() { return kPgNumCfgs; }

extern "C" int k8s_pgemm_config(int cfg, int* bp, int* bq, int* lds_bytes) {
  if (cfg < 0 || cfg >= kPgNumCfgs) return -1;
  *bp = 64 * kPgCfgs[cfg].fp;
  *bq = 128 * kPgCfgs[cfg].fq;
  *lds_bytes = pg_lds_ring(*bp, *bq, kPgCfgs[cfg].ws, false);
  return 0;
}

// Launch facts of a (cfg, splits) plan: workgroups, fp32 slab elements, ticket count (0 without split-K).
extern "C" int k8s_pgemm_plan(int M, int N_out, int K, int epi, int fp8, int cfg, int splits, int* nwg,
                              long long* ws_elems, int* tickets) {
  if (cfg < 0 || cfg >= kPgNumCfgs || M <= 0 || N_out <= 0 || K <= 0 || splits < 1) return -1;
  if ((K * (fp8 ? 1 : 2)) % 128 != 0 || N_out % 4 != 0) return -1;
  const PgGeom g = pg_geom(M, N_out, K, epi, fp8, cfg);
  if (splits > g.kt) return -1;
  const int bp = 64 * kPgCfgs[cfg].fp, bq = 128 * kPgCfgs[cfg].fq;
  *nwg = g.tiles * splits;
  *ws_elems = splits > 1 ? (long long)g.tiles * splits * (bp * bq + bq) : 0;
  *tickets = splits > 1 ? g.tiles : 0;
  return 0;
}

// out[M, N_out] = epi(x[M, K] . W^T).  fp8 = 1: x / W are e4m3 bytes with per-row scales xs / wsc; fp8 = 3: x is
// MX e4m3 with its E8M0 block scales in xs (bytes, mx_scale_off layout), W e4m3 with row scales wsc.  SwiGLU: W holds
// 2 * N_out rows ([gate; up]); oq / oe (fp8): the output as MX e4m3 [M][N_out] + E8M0 (mx_scale_off layout) (out unused).
// res: bf16 residual added in the bf16 epilogue (may alias out).  rms: bf16 RMS prologue (out scaled by 1 / rms(x
// row); the norm gamma is folded into W).
extern "C" int k8s_pgemm(void* out, float* ws, unsigned* tickets, const void* x, const void* W, const float* xs,
                         const float* wsc, int M, int N_out, int K, int epi, int fp8, int cfg, int splits,
                         int group_m, const void* res, int rms, float eps, void* oq, void* oe, hipStream_t stream) {
  if (fp8 < 0 || fp8 > 3 || fp8 == 2) return -1;
  const bool mx = fp8 == 3;
  if (oq != nullptr && (oe == nullptr || !fp8 || epi != PG_SWIGLU || N_out % 128 != 0)) return -7;
  fp8 = fp8 ? 1 : 0;
  int nwg, nt;
  long long nws;
  if (k8s_pgemm_plan(M, N_out, K, epi, fp8, cfg, splits, &nwg, &nws, &nt) != 0) return -1;
  if (splits > 1 && (ws == nullptr || tickets == nullptr)) return -3;
  const long long kbytes = (long long)K * (fp8 ? 1 : 2);
  const long long wrows = epi == PG_SWIGLU ? 2LL * N_out : (long long)N_out;
  if (wrows * kbytes >= (1LL << 32) || (long long)M * kbytes >= (1LL << 32)) return -5;   // 32-bit DMA offsets
  if (fp8 && (xs == nullptr || wsc == nullptr)) return -3;
  if (res != nullptr && epi != PG_BF16) return -6;
  if (rms && fp8) return -6;
  const PgGeom g = pg_geom(M, N_out, K, epi, fp8, cfg);
  PgArgs a;
  a.out = out;
  a.res = static_cast<const bf16_t*>(res);
  a.ws = ws;
  a.cnt = tickets;
  a.x = static_cast<const uint8_t*>(x);
  a.W = static_cast<const uint8_t*>(W);
  a.xs = xs;
  a.wsc = wsc;
  a.xe = mx ? reinterpret_cast<const uint8_t*>(xs) : nullptr;
  a.oq = static_cast<uint8_t*>(oq);
  a.oe = static_cast<uint8_t*>(oe);
  a.kbytes = (uint32_t)kbytes;
  a.M = M;
  a.N_out = N_out;
  a.half_rows = epi == PG_SWIGLU ? N_out : 0;
  a.K = K;
  a.m_tiles = g.m_tiles;
  a.n_tiles = g.n_tiles;
  a.kt = g.kt;
  a.splits = splits;
  a.group_m = group_m > 0 ? group_m : 1;
  a.nwg = nwg;
  a.prio = g_pg_prio;
  a.eps = eps;
  a.row_slabs = splits > 1 && g_pg_row_slabs;
  const int rc = fp8 ? pg_cfg<true>(a, cfg, epi, 0, stream) : pg_cfg<false>(a, cfg, epi, rms, stream);
  if (rc != 0 || !a.row_slabs) return rc;
  return k8s_pgemm_reduce(out, res, ws, splits, M, N_out, K, epi, rms, eps, (fp8 && !mx) ? xs : nullptr,
                          fp8 ? wsc : nullptr, oq, oe, stream);
}
