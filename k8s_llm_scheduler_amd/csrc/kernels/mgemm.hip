// K3 / K8 / K9(+K10) / K11 / K15: hand-written MFMA GEMM for projections with more than 2 rows
// (prefill chunks, batched decode), bf16 or OCP-e4m3 weights, fp32 accumulate (gfx950).
//
//     out[M, N] = epi( x[M, K] . W[N, K]^T )        epi: bf16 | fp32 | SwiGLU (silu(g) * u)
//
// Design (MI355X-first, not a library tile recompiled):
//  * swapped orientation C^T = W . x^T on v_mfma_f32_16x16x32_bf16 (fp8: _16x16x32_fp8_fp8): the
//    A operand is 16 weight rows, the B operand 16 activation rows, both K-contiguous, so both are
//    staged the same way and every lane ends with 4 CONSECUTIVE output columns of one row
//    (one 8-byte bf16 / 16-byte fp32 store, and gate/up pairs side by side for SwiGLU).
//  * both operands move HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4): no VGPR staging, an
//    S-deep ring of 128-byte-wide k-steps (64 bf16 or 128 e4m3 per row), counted `s_waitcnt
//    vmcnt` so S-2 k-steps stay in flight across each raw s_barrier (MI355X_MICROARCH: LDS-DMA
//    stays in flight across barriers; __syncthreads would drain it).
//  * the LDS image is lane-linear (DMA destination = base + 16 * lane); the XOR swizzle that makes
//    the fragment reads (16 rows x one 16-byte column, ds_read_b128) conflict-free is applied on the
//    per-lane GLOBAL source address: 16-byte chunk c of row r lives at slot c ^ ((r >> 1) & 7).
//  * block -> tile mapping is XCD-aware (blocks b, b+8, .. share an XCD and get a contiguous
//    logical range), with the k-slices of one tile adjacent, then the m-tiles of one n-tile:
//    the weights a tile streams are re-read by its neighbours from the same L2.
//  * split-K for small grids (TP = 8 shapes: N = 1280, K = 8192): every slice writes an fp32 slab
//    in fragment order with write-through (sc1) 16-byte buffer stores, waits for them, and counts its
//    arrival with one relaxed device-scope ticket add; the last arriving slice of a tile reads all
//    slabs back with sc1 loads (fixed order), reduces them and applies the epilogue in the same launch
//    (no memset, no second kernel, no cache-wide fence; the ticket is reset by the reducer).  Measured
//    against the round-4 form (plain stores + agent-scope release / acquire fences, K8S_MGEMM_FENCED=1):
//    batch-64 decode 30.68 -> 30.46 ms/step bf16, 18.73 -> 18.30 fp8 (profiles/mgemm_fence_ab_r5.txt).
//  * fp8: activations are quantized per token (fp8.hip), weights per row; the epilogue applies
//    sx[m] * sw[n].  Non-scaled fp8 MFMA runs at the bf16 rate but halves the staged bytes.
//  * MX activations (host mode fp8 = 3): x is OCP MX e4m3 -- one E8M0 scale per 32 values of a row (fp8.hip), as
//    the SwiGLU epilogue below and the attention kernels write it -- and the MFMA is the block-scaled
//    v_mfma_scale_f32_16x16x128_f8f6f4: lane (li, g) holds k 16 g.. and 64 + 16 g.. of its row and passes the scale
//    byte of block g as its B scale (the weights' per-row scale stays in the epilogue, unit A scales).  The
//    scale bytes ride the x ring: one 4-byte LDS-DMA per (row, 128-value subtile) per k-step.  Twice the MFMA rate
//    of the non-scaled fp8 form, and no per-token absmax pass anywhere.
//  * MX output (SwiGLU epilogue, mx_out): the h = silu(g) * u values of 32 consecutive features of a row sit in
//    the lanes of one 16-lane column group of two adjacent fragments (the configurations whose per-wave feature
//    span is a multiple of 32), or of one fragment in each of two neighbouring waves (16 features per wave: the
//    row absmax goes through LDS, one barrier): a shuffle max gives the block's E8M0 scale and every lane stores
//    its e4m3 bytes -- the down projection's input is produced already quantized.
#include <cstdlib>

#include "common.h"

namespace k8sllm {

namespace {
enum { MG_BF16 = 0, MG_F32 = 1, MG_SWIGLU = 2 };

typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) int i32x4;

__device__ __forceinline__ float mg_silu(float g) { return g / (1.f + __expf(-g)); }

template <int N>
__device__ __forceinline__ void mg_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most `after` k-steps of LPS loads each are still in flight (after <= A)
template <int LPS, int A>
__device__ __forceinline__ void mg_wait_after(int after) {
  if constexpr (A == 0) {
    mg_vmcnt<0>();
  } else {
    if (after >= A) mg_vmcnt<A * LPS>();
    else mg_wait_after<LPS, A - 1>(after);
  }
}
// Raw barrier that leaves LDS-DMA (vmcnt) in flight.  The lgkmcnt(0) retires this wave's LDS reads
// first: a buffer is refilled right after the barrier, and an LDS read still in flight at the barrier
// (the compiler may sink its consuming MFMA past it) could otherwise return the new bytes (WAR).
__device__ __forceinline__ void mg_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
}  // namespace

struct MgArgs {
  void* out;
  float* ws;             // partial slabs: [tiles][cmax][BM * BN] fp32 (fragment order)
  unsigned* cnt;         // [tiles] arrival tickets, zero between launches
  const uint8_t* x;      // [M][K] bf16 or e4m3
  const uint8_t* W;      // [rows][K] bf16 or e4m3
  const float* xs;       // fp8 activations: [M] per-token activation scales
  const float* wsc;      // fp8: [rows] per-row weight scales
  const uint8_t* xe;     // MX activations: E8M0 block scales, [K / 128][M] dwords (mx_scale_off)
  uint8_t* oq;           // MX output (SwiGLU): e4m3 [M][N_out] ...
  uint8_t* oe;           // ... and its E8M0 block scales, mx_scale_off layout (bf16 out not written)
  long long kbytes;      // bytes per row of W (and of x)
  long long xkbytes;     // bytes per row of x
  long long total;       // tiles * T work items (one item = one tile x one 128-byte k-step)
  int M, N_out, half_rows;
  int m_tiles, T;        // T: 128-byte k-steps over the whole K
  int nwg, cmax;         // workgroups; most workgroups sharing one tile
  const bf16_t* res;     // optional residual (bf16 [M][N_out], may alias out): out = acc + res  (bf16 epilogue)
  int rms;               // 1: RMSNorm prologue -- out scaled by 1 / rms(x row) (the gamma is folded into W)
  float eps;
  int rms_mfma;          // bf16 rows: the row sums of squares from x . x^T on the MFMA (1) or v_dot2 (0)
  int fenced;            // split tiles: 1 = plain slab stores + agent-scope release / acquire fences (round-4 form)
};

// Wave layout: WM x WN waves own (BM / WM) x (BN / WN) output sub-tiles; WK waves share each
// sub-tile and take every WK-th k32 step of a stage (intra-workgroup split-K, reduced through LDS
// at the end of the segment).  RB: bytes of one row per k-step (128 / 256 / 512): wider k-steps
// read longer contiguous runs of every weight row.
template <int RB>
__device__ __forceinline__ int mg_swz_rb(int r) {
  // 16-byte chunks of 16 consecutive rows read at one column land on 16 distinct bank slots
  return RB == 64 ? ((r >> 2) & 3) : RB == 128 ? ((r >> 1) & 7) : (r & 15);
}

template <int BM, int BN, int WM, int WN, int WK, int RB, int S, int EPI, bool FP8, bool MX = false, bool MXO = false>
__global__ void __launch_bounds__(64 * WM * WN * WK) mgemm_kernel(MgArgs a) {
  constexpr int NW = WM * WN * WK;
  constexpr int FM = BM / (WM * 16), FN = BN / (WN * 16);
  static_assert(FM >= 1 && FN >= 1 && BM % (WM * 16) == 0 && BN % (WN * 16) == 0, "tile / wave split");
  static_assert(EPI != MG_SWIGLU || FN % 2 == 0, "SwiGLU pairs gate and up fragments");
  static_assert(S >= 2 && S <= 8, "ring depth");
  static_assert(WN == 1 || WN == 2 || WN == 4, "the RMS prologue splits a fragment's 4 dot2 over WN waves");
  static_assert(RB == 64 || RB == 128 || RB == 256 || RB == 512, "row bytes per k-step");
  static_assert(!MX || FP8, "MX: e4m3 activations with E8M0 block scales");
  static_assert(!MXO || (EPI == MG_SWIGLU && ((FN / 2) % 2 == 0 || (FN == 2 && WN % 2 == 0 && WK == 1))) ||
                    (EPI == MG_BF16 && FN % 2 == 0),
                "MX output: SwiGLU with 32-feature spans per wave or wave pair, or the residual epilogue");
  constexpr int XRB = RB;                            // x row bytes per k-step
  constexpr int CPR = RB / 16, XCPR = XRB / 16;      // 16-byte chunks per staged W / x row
  constexpr int KS = FP8 ? RB / 32 : RB / 64;        // k32 MFMA steps per k-step (RB = 64: one)
  static_assert(KS % WK == 0, "k32 steps split evenly over WK waves");
  constexpr int KS4 = RB / 128;                      // MX: 128-value subtiles per k-step, one scaled MFMA each
  static_assert(!MX || (KS4 >= 1 && KS4 % WK == 0), "MX: subtiles split evenly over WK waves");
  constexpr int SD = MX ? BM * KS4 : 0;              // MX: scale dwords per stage (row r, subtile d: r * KS4 + d)
  static_assert(SD % NW == 0, "scale dwords per wave");
  constexpr int WREG = BN * RB, XREG = BM * XRB, STAGE_B = BN * RB + BM * XRB + SD * 4;
  static_assert((BN * CPR) % NW == 0 && (BM * XCPR) % NW == 0, "chunks per wave");
  constexpr int WCH = BN * CPR / NW, XCH = BM * XCPR / NW;  // 16-byte chunks per wave per stage
  constexpr int SCH = SD / NW;                              // MX: scale dwords per wave per stage
  constexpr int WI = (WCH + 63) / 64, XI = (XCH + 63) / 64, SI = (SCH + 63) / 64, LPS = WI + XI + SI;
  static_assert((S - 2) * LPS <= 63, "vmcnt range");
  static_assert(WK == 1 || (WK - 1) * FN * FM * 64 * 16 * WM * WN <= S * STAGE_B, "LDS reduction space");
#if defined(__HIP_DEVICE_COMPILE__)  // the host pass only needs the launch stub (its lambdas use device builtins)
  constexpr int XPAIR = (MXO && EPI == MG_SWIGLU && FN == 2) ? WN * BM : 0;   // wave-pair MX absmax exchange
  __shared__ __attribute__((aligned(16))) char lds[S * STAGE_B + 16 + WK * WN * BM * 4 + XPAIR * 4];
  unsigned* flag = reinterpret_cast<unsigned*>(lds + S * STAGE_B);
  float* rss = reinterpret_cast<float*>(lds + S * STAGE_B + 16);   // [WK * WN][BM] row sums of squares
  float* xpair = rss + WK * WN * BM;                                 // [WN][BM] (wave-pair MX output)

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wk = wid % WK, wt = wid / WK;           // k-share, output sub-tile
  const int wm = wt / WN, wn = wt % WN;
  const int li = lane & 15, g = lane >> 4;

  // ---- block -> logical workgroup, XCD-aware and bijective for any grid size; logical workgroup
  // w streams the work items [w * total / nwg, (w + 1) * total / nwg)
  const int bid = blockIdx.x, q8 = a.nwg >> 3, r8 = a.nwg & 7, xcd = bid & 7, loc = bid >> 3;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  const long long it0 = (long long)lid * a.total / a.nwg, it1 = (long long)(lid + 1) * a.total / a.nwg;
  const int T = a.T;

  // fragment rows of this lane inside the stage images
  int arow[FN];
#pragma unroll
  for (int f = 0; f < FN; ++f) {
    if (EPI == MG_SWIGLU) {
      const int half = f / (FN / 2), ff = f % (FN / 2);
      arow[f] = half * (BN / 2) + wn * (BN / 2 / WN) + ff * 16 + li;
    } else {
      arow[f] = wn * (BN / WN) + f * 16 + li;
    }
  }
  const int brow0 = wm * (BM / WM) + li;

  bool first_segment = true;
  for (long long it = it0; it < it1;) {
    const int tile = (int)(it / T);
    const int kb = (int)(it - (long long)tile * T);
    const int ke = (int)min((long long)T, kb + (it1 - it));
    it += ke - kb;
    const int mt = tile % a.m_tiles, nt = tile / a.m_tiles;
    if (!first_segment) mg_barrier();  // every wave is done with the ring (and the reduction space)
    first_segment = false;

    // per-lane DMA sources as 32-bit offsets from the operand bases (swizzle on the source,
    // lane-linear LDS destination); the host checks that every operand spans < 4 GiB
    const uint8_t* wseg = a.W + (long long)kb * RB;
    const uint8_t* xseg = a.x + (long long)kb * XRB;
    const uint8_t* eseg = MX ? a.xe + (long long)kb * KS4 * a.M * 4 : nullptr;   // [K / 128][M] scale dwords
    uint32_t woff[WI], xoff[XI], soff[SI > 0 ? SI : 1];
#pragma unroll
    for (int i = 0; i < WI; ++i) {
      const int p = wid * WCH + min(i * 64 + lane, WCH - 1);
      const int r = p / CPR, c = (p % CPR) ^ mg_swz_rb<RB>(p / CPR);
      int grow;
      if (EPI == MG_SWIGLU) {
        const int f = min(nt * (BN / 2) + (r % (BN / 2)), a.N_out - 1);
        grow = r < BN / 2 ? f : a.half_rows + f;
      } else {
        grow = min(nt * BN + r, a.N_out - 1);
      }
      woff[i] = (uint32_t)grow * (uint32_t)a.kbytes + (uint32_t)(c * 16);
    }
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const int p = wid * XCH + min(i * 64 + lane, XCH - 1);
      const int r = p / XCPR, c = (p % XCPR) ^ mg_swz_rb<XRB>(p / XCPR);
      xoff[i] = (uint32_t)min(mt * BM + r, a.M - 1) * (uint32_t)a.xkbytes + (uint32_t)(c * 16);
    }
#pragma unroll
    for (int i = 0; i < SI; ++i) {   // MX: the 4 scale bytes of (row r, subtile d) of a k-step
      const int p = wid * SCH + min(i * 64 + lane, SCH - 1);
      const int r = p / KS4, d = p % KS4;
      soff[i] = ((uint32_t)d * (uint32_t)a.M + (uint32_t)min(mt * BM + r, a.M - 1)) * 4u;
    }

    auto issue = [&](int t, int stage) {
      char* sb = lds + stage * STAGE_B;
      const uint8_t* wb = wseg + (long long)t * RB;
      const uint8_t* xb = xseg + (long long)t * XRB;
#pragma unroll
      for (int i = 0; i < WI; ++i) {
        if (WCH % 64 == 0 || i * 64 + lane < WCH)
          __builtin_amdgcn_global_load_lds(wb + woff[i],
                                           (__attribute__((address_space(3))) void*)(sb + (wid * WCH + i * 64) * 16),
                                           16, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < XI; ++i) {
        if (XCH % 64 == 0 || i * 64 + lane < XCH)
          __builtin_amdgcn_global_load_lds(
              xb + xoff[i], (__attribute__((address_space(3))) void*)(sb + WREG + (wid * XCH + i * 64) * 16), 16, 0,
              0);
      }
      if constexpr (MX) {
        const uint8_t* eb = eseg + (long long)t * KS4 * a.M * 4;
#pragma unroll
        for (int i = 0; i < SI; ++i) {
          if (SCH % 64 == 0 || i * 64 + lane < SCH)
            __builtin_amdgcn_global_load_lds(
                eb + soff[i], (__attribute__((address_space(3))) void*)(sb + WREG + XREG + (wid * SCH + i * 64) * 4),
                4, 0, 0);
        }
      }
    };

    f32x4 acc[FN][FM];
#pragma unroll
    for (int f = 0; f < FN; ++f)
#pragma unroll
      for (int j = 0; j < FM; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    float ss[FM];   // RMS prologue: this lane's share of sum(x^2) of its fragment rows
#pragma unroll
    for (int j = 0; j < FM; ++j) ss[j] = 0.f;
    f32x4 accsq[FM];   // RMS prologue on the MFMA: x . x^T per row fragment (diagonal = sums of squares)
#pragma unroll
    for (int j = 0; j < FM; ++j) accsq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool rms_mfma = MX || a.rms_mfma != 0;
    const bool do_rms = (!FP8 || MX) && a.rms != 0;   // MX: the squares of the dequantized e4m3 values

    auto compute = [&](int stage) {
      const char* wb = lds + stage * STAGE_B;
      const char* xb = wb + WREG;
#pragma unroll
      for (int q = 0; q < KS / WK; ++q) {
        const int kk = q * WK + wk;
        if constexpr (!FP8) {
          const int c = kk * 4 + g;
          bf16x8 af[FN], bfr[FM];
#pragma unroll
          for (int f = 0; f < FN; ++f)
            af[f] = *reinterpret_cast<const bf16x8*>(wb + arow[f] * RB + ((c ^ mg_swz_rb<RB>(arow[f])) << 4));
#pragma unroll
          for (int j = 0; j < FM; ++j) {
            const int r = brow0 + j * 16;
            bfr[j] = *reinterpret_cast<const bf16x8*>(xb + r * XRB + ((c ^ mg_swz_rb<XRB>(r)) << 4));
          }
#pragma unroll
          for (int f = 0; f < FN; ++f)
#pragma unroll
            for (int j = 0; j < FM; ++j)
              acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[f], bfr[j], acc[f][j], 0, 0, 0);
          if (do_rms && rms_mfma) {
            // one more MFMA per x fragment, x . x^T (diagonal = the rows' sums of squares); a scalar branch
            // (readfirstlane), since an MFMA ignores EXEC.  In the weight-streaming regime the MFMA pipe is idle
            // enough that this costs less than v_dot2 squares in every k-step (or a norm launch).  Fragment j in
            // wave wn = j % WN of the row block: the extra MFMAs spread over the waves that share x
            const int wn_u = __builtin_amdgcn_readfirstlane(wn);
#pragma unroll
            for (int j = 0; j < FM; ++j)
              if (j % WN == wn_u) accsq[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], bfr[j], accsq[j], 0, 0, 0);
          } else if (do_rms) {   // the WN waves of a row block hold the same x fragments: each squares 1/WN of them
#pragma unroll
            for (int j = 0; j < FM; ++j)
#pragma unroll
              for (int e = 0; e < 4; ++e) {   // v_dot2_f32_bf16: two squares per instruction
                if (WN == 1 || e % WN == wn % 4) {
                  const bf16x2 v2 = {bfr[j][2 * e], bfr[j][2 * e + 1]};
                  ss[j] = __builtin_amdgcn_fdot2_f32_bf16(v2, v2, ss[j], false);
                }
              }
          }
        } else if constexpr (MX) {
          if (q < KS4 / WK) {
            // operand layout of the 16x16x128 f8f6f4 MFMA (measured, tools/experiments/mx_scale_probe.hip): lane
            // (li, g) holds k = 16 g .. +16 in bytes 0-15 and k = 64 + 16 g .. +16 in bytes 16-31, and the scale of
            // 32-value block b of row li is lane li + 16 b's -- so chunks 8 kk4 + g and 8 kk4 + 4 + g in natural k
            // order, and lane g passes the scale byte of block g
            const int kk4 = q * WK + wk, c0 = kk4 * 8 + g;
            const int* sl = reinterpret_cast<const int*>(xb + XREG);
            i32x8 af[FN], bx[FM];
            int sc[FM];
            auto frag32 = [&](const char* rowp, int row) {
              const i32x4 lo4 = *reinterpret_cast<const i32x4*>(rowp + ((c0 ^ mg_swz_rb<RB>(row)) << 4));
              const i32x4 hi4 = *reinterpret_cast<const i32x4*>(rowp + (((c0 + 4) ^ mg_swz_rb<RB>(row)) << 4));
              return i32x8{lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            };
#pragma unroll
            for (int f = 0; f < FN; ++f) af[f] = frag32(wb + arow[f] * RB, arow[f]);
#pragma unroll
            for (int j = 0; j < FM; ++j) {
              const int r = brow0 + j * 16;
              bx[j] = frag32(xb + r * RB, r);
              sc[j] = sl[r * KS4 + kk4] >> (8 * g);   // this lane's block scale in byte 0 (op_sel 0)
              // RMS prologue on MX rows: one more MFMA, x . x^T of the fragment with both scale operands = the
              // block scales -- its diagonal is the rows' sums of squares of the dequantized values (the VALU
              // form, 16 conversions + 32 FMAs per lane and subtile, was the bottleneck); wave wn = 0 of a row block.
              // The condition must be a scalar branch: an MFMA ignores EXEC, so a lane-masked "if" would still
              // accumulate in every wave (readfirstlane makes wn provably wave-uniform)
              if (do_rms && __builtin_amdgcn_readfirstlane(wn) == 0)
                accsq[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(bx[j], bx[j], accsq[j], 0, 0, 0, sc[j], 0,
                                                                            sc[j]);
            }
#pragma unroll
            for (int f = 0; f < FN; ++f)
#pragma unroll
              for (int j = 0; j < FM; ++j)
                acc[f][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[f], bx[j], acc[f][j], 0, 0, 0,
                                                                             0x7f7f7f7f, 0, sc[j]);
          }
        } else {
          const int c = kk * 2 + (g >> 1), hb = (g & 1) * 8;
          long af[FN], bfr[FM];
#pragma unroll
          for (int f = 0; f < FN; ++f)
            af[f] = *reinterpret_cast<const long*>(wb + arow[f] * RB + ((c ^ mg_swz_rb<RB>(arow[f])) << 4) + hb);
#pragma unroll
          for (int j = 0; j < FM; ++j) {
            const int r = brow0 + j * 16;
            bfr[j] = *reinterpret_cast<const long*>(xb + r * RB + ((c ^ mg_swz_rb<RB>(r)) << 4) + hb);
          }
#pragma unroll
          for (int f = 0; f < FN; ++f)
#pragma unroll
            for (int j = 0; j < FM; ++j)
              acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(af[f], bfr[j], acc[f][j], 0, 0, 0);
        }
      }
    };

    // ---- K loop over this segment: S-1 k-steps issued ahead; wait for the oldest, barrier,
    // refill the buffer everyone finished with, compute
    const int n = ke - kb;
#pragma unroll
    for (int t = 0; t < S - 1; ++t)
      if (t < n) issue(t, t);
    int stage = 0, fill = S - 1;
    for (int t = 0; t < n; ++t) {
      // k-steps issued after step t that may stay in flight
      mg_wait_after<LPS, S - 2>(min(S - 2, n - 1 - t));
      mg_barrier();  // step t landed for every wave; every wave finished reading the buffer refilled now
      if (t + S - 1 < n) issue(t + S - 1, fill);
      compute(stage);
      stage = stage + 1 == S ? 0 : stage + 1;
      fill = fill + 1 == S ? 0 : fill + 1;
    }

    // ---- intra-workgroup split-K: the WK waves of a sub-tile add up through LDS (fixed order)
    if constexpr (WK > 1) {
      mg_barrier();  // every wave's last fragment reads are done; no DMA is in flight
      float* red = reinterpret_cast<float*>(lds);
      if (wk > 0) {
#pragma unroll
        for (int f = 0; f < FN; ++f)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            *reinterpret_cast<f32x4*>(red + ((((wk - 1) * WM * WN + wt) * FN + f) * FM + j) * 256 + lane * 4) =
                acc[f][j];
      }
      mg_barrier();
      if (wk == 0) {
#pragma unroll
        for (int k2 = 1; k2 < WK; ++k2)
#pragma unroll
          for (int f = 0; f < FN; ++f)
#pragma unroll
            for (int j = 0; j < FM; ++j)
              acc[f][j] += *reinterpret_cast<const f32x4*>(red + ((((k2 - 1) * WM * WN + wt) * FN + f) * FM + j) * 256 +
                                                           lane * 4);
      }
    }

    // ---- RMS prologue: row sums of squares over this segment's k-steps -> rss[wk][row]
    if (do_rms && rms_mfma) {   // the diagonal of x . x^T: C[4 g + i][li] with 4 g + i == li
#pragma unroll
      for (int j = 0; j < FM; ++j) ss[j] = (g == (li >> 2)) ? accsq[j][li & 3] : 0.f;
    }
    if (do_rms) {
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        ss[j] += __shfl_xor(ss[j], 16, WAVE);
        ss[j] += __shfl_xor(ss[j], 32, WAVE);
      }
      if (g == 0) {
#pragma unroll
        for (int j = 0; j < FM; ++j) rss[(wk * WN + wn) * BM + wm * (BM / WM) + j * 16 + li] = ss[j];
      }
      mg_barrier();
      if (threadIdx.x < BM) {
        float t = 0.f;
#pragma unroll
        for (int k2 = 0; k2 < WK * WN; ++k2) t += rss[k2 * BM + threadIdx.x];
        rss[threadIdx.x] = t;   // row total of this segment (own thread reads / writes only)
      }
    }

    // ---- a tile shared by several workgroups: publish this partial tile; the last arriver reduces
    const long long i_first = (long long)tile * T;
    const int w_first = (int)(((i_first + 1) * a.nwg - 1) / a.total);
    const int w_last = (int)(((i_first + T) * a.nwg - 1) / a.total);
    const int nc = w_last - w_first + 1;
    constexpr int SLAB = BM * BN + BM;   // partial tile + row sums of squares
    if (nc > 1 && !a.fenced) {
      // the sgemv.hip protocol, no cache-wide fences (an agent-scope release / acquire costs an L2 write-back /
      // invalidate per arriving workgroup on this chip): device-coherent slab stores, every wave waits for its own
      // stores, one relaxed device-scope ticket add per workgroup, device-coherent slab loads by the last arriver
      float* base = a.ws + (long long)tile * a.cmax * SLAB;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
      const int sbase = (lid - w_first) * SLAB * 4;   // this workgroup's slab, bytes from base
      constexpr int MG_SC1 = 16;                       // buffer-op cache policy sc1: write-through, coherent at L2
      if (do_rms && threadIdx.x < BM)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, rss[threadIdx.x]), rs,
                                              sbase + (BM * BN + threadIdx.x) * 4, 0, MG_SC1);
      if (wk == 0) {
#pragma unroll
        for (int f = 0; f < FN; ++f)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[f][j]), rs,
                                                   sbase + ((((wt * FN + f) * FM + j) * 64 + lane) * 4) * 4, 0, MG_SC1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's slab stores have landed
      __syncthreads();
      if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned last = old == (unsigned)(nc - 1);
        if (last) __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
        *flag = last;
      }
      __syncthreads();
      if (*flag == 0u) continue;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");   // (compiler ordering: the loads stay below the add)
      if (wk == 0) {   // fixed summation order over ALL slabs (own included)
#pragma unroll
        for (int f = 0; f < FN; ++f)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s2 = 0; s2 < nc; ++s2) {
#pragma unroll
          for (int f = 0; f < FN; ++f)
#pragma unroll
            for (int j = 0; j < FM; ++j)
              acc[f][j] += __builtin_bit_cast(
                  f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                             rs, (s2 * SLAB + (((wt * FN + f) * FM + j) * 64 + lane) * 4) * 4, 0, MG_SC1));
        }
      }
      if (do_rms && threadIdx.x < BM) {
        float t = 0.f;
        for (int s2 = 0; s2 < nc; ++s2)
          t += __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rs, (s2 * SLAB + BM * BN + threadIdx.x) * 4, 0, MG_SC1));
        rss[threadIdx.x] = t;
      }
    } else if (nc > 1) {
      float* base = a.ws + (long long)tile * a.cmax * SLAB;
      float* slab = base + (long long)(lid - w_first) * SLAB;
      if (do_rms && threadIdx.x < BM) slab[BM * BN + threadIdx.x] = rss[threadIdx.x];
      if (wk == 0) {
#pragma unroll
        for (int f = 0; f < FN; ++f)
#pragma unroll
          for (int j = 0; j < FM; ++j)
            *reinterpret_cast<f32x4*>(slab + (((wt * FN + f) * FM + j) * 64 + lane) * 4) = acc[f][j];
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned old = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned last = old == (unsigned)(nc - 1);
        if (last) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          a.cnt[tile] = 0u;  // ready for the next launch
        }
        *flag = last;
      }
      __syncthreads();
      if (*flag == 0u) continue;
      // fixed summation order over ALL slabs (own included): the result does not depend on which
      // workgroup arrived last
      if (wk == 0) {
#pragma unroll
        for (int f = 0; f < FN; ++f)
#pragma unroll
          for (int j = 0; j < FM; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s2 = 0; s2 < nc; ++s2) {
          const float* sl = base + (long long)s2 * SLAB;
#pragma unroll
          for (int f = 0; f < FN; ++f)
#pragma unroll
            for (int j = 0; j < FM; ++j) {
              const f32x4 v = *reinterpret_cast<const f32x4*>(sl + (((wt * FN + f) * FM + j) * 64 + lane) * 4);
              acc[f][j] += v;
            }
        }
      }
      if (do_rms) {
        if (threadIdx.x < BM) {
          float t = 0.f;
          for (int s2 = 0; s2 < nc; ++s2) t += base[(long long)s2 * SLAB + BM * BN + threadIdx.x];
          rss[threadIdx.x] = t;
        }
      }
    }
    if (do_rms) mg_barrier();   // row totals visible to every wave's epilogue
    if (wk != 0) continue;

    if constexpr (MXO && EPI == MG_SWIGLU && FN == 2) {
      // MX output, 16 SwiGLU features per wave: a 32-feature block is waves wn and wn ^ 1 (same rows); each wave
      // parks its rows' absmax in LDS, one barrier, then both take the pair's max
      float v[FM][4], am[FM];
      const int n0 = nt * (BN / 2) + wn * 16 + 4 * g;
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = min(mt * BM + wm * (BM / WM) + j * 16 + li, a.M - 1);
        float sxx = MX ? 1.f : a.xs[m];
        if (do_rms) sxx = rsqrtf(rss[wm * (BM / WM) + j * 16 + li] / (float)a.xkbytes + a.eps);
        am[j] = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[j][i] = 0.f;
          if (n0 < a.N_out) {
            const float gt = acc[0][j][i] * sxx * a.wsc[n0 + i], up = acc[1][j][i] * sxx * a.wsc[a.half_rows + n0 + i];
            v[j][i] = bf_round(mg_silu(gt) * up);
          }
          am[j] = fmaxf(am[j], fabsf(v[j][i]));
        }
        am[j] = fmaxf(am[j], __shfl_xor(am[j], 16, WAVE));
        am[j] = fmaxf(am[j], __shfl_xor(am[j], 32, WAVE));
        xpair[wn * BM + wm * (BM / WM) + j * 16 + li] = am[j];
      }
      mg_barrier();
#pragma unroll
      for (int j = 0; j < FM; ++j) {
        const int m = mt * BM + wm * (BM / WM) + j * 16 + li;
        if (m >= a.M || n0 >= a.N_out) continue;   // N_out % 32 == 0: a wave pair is in or out together
        const float amax = fmaxf(am[j], xpair[(wn ^ 1) * BM + wm * (BM / WM) + j * 16 + li]);
        const uint32_t e = mx_e8m0(amax);
        *reinterpret_cast<uint32_t*>(a.oq + (long long)m * a.N_out + n0) =
            mx_pack4(v[j][0], v[j][1], v[j][2], v[j][3], mx_inv_scale(e));
        if (g == 0 && (wn & 1) == 0) a.oe[mx_scale_off(m, n0 >> 5, a.M)] = (uint8_t)e;
      }
      continue;
    }

    // ---- epilogue: lane holds out[m = brow][n = 4 g + i], i < 4, of every fragment pair
#pragma unroll
    for (int j = 0; j < FM; ++j) {
      const int m = mt * BM + wm * (BM / WM) + j * 16 + li;
      if (m >= a.M) continue;
      float sx = (FP8 && !MX) ? a.xs[m] : 1.f;
      if (do_rms) sx = rsqrtf(rss[wm * (BM / WM) + j * 16 + li] / (float)(MX ? a.xkbytes : (a.xkbytes >> 1)) + a.eps);
      if constexpr (MXO && EPI == MG_SWIGLU && FN != 2) {   // 32-feature blocks = fragment pairs (2 b, 2 b + 1)
#pragma unroll
        for (int b = 0; b < FN / 4; ++b) {
          const int nb = nt * (BN / 2) + wn * (BN / 2 / WN) + b * 32;   // first feature of the block
          if (nb >= a.N_out) continue;                                   // N_out % 32 == 0: whole blocks only
          float v[8];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int f = 2 * b + h, n0 = nb + h * 16 + 4 * g;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              float gt = acc[f][j][i] * sx * a.wsc[n0 + i], up = acc[f + FN / 2][j][i] * sx * a.wsc[a.half_rows + n0 + i];
              v[4 * h + i] = bf_round(mg_silu(gt) * up);
            }
          }
          float amax = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
          amax = fmaxf(amax, __shfl_xor(amax, 16, WAVE));
          amax = fmaxf(amax, __shfl_xor(amax, 32, WAVE));
          const uint32_t e = mx_e8m0(amax);
          const float inv = mx_inv_scale(e);
          uint8_t* orow = a.oq + (long long)m * a.N_out;
          *reinterpret_cast<uint32_t*>(orow + nb + 4 * g) = mx_pack4(v[0], v[1], v[2], v[3], inv);
          *reinterpret_cast<uint32_t*>(orow + nb + 16 + 4 * g) = mx_pack4(v[4], v[5], v[6], v[7], inv);
          if (g == 0) a.oe[mx_scale_off(m, nb >> 5, a.M)] = (uint8_t)e;
        }
      } else if constexpr (MXO && EPI == MG_BF16) {
        // residual epilogue + its MX copy: out = acc + res (bf16, the residual stream) and the same values as MX
        // e4m3 -- the next pre-norm projection's input (its RMS statistics are that GEMM's prologue)
#pragma unroll
        for (int b = 0; b < FN / 2; ++b) {
          const int nb = nt * BN + wn * (BN / WN) + b * 32;
          if (nb >= a.N_out) continue;   // N_out % 128 == 0: whole blocks
          float v[8];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int f = 2 * b + h, n0 = nb + 16 * h + 4 * g;
            const u32x2 rr = *reinterpret_cast<const u32x2*>(a.res + (long long)m * a.N_out + n0);
            float t[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) t[i] = acc[f][j][i] * sx * a.wsc[n0 + i];
            t[0] += lo_bf(rr[0]);
            t[1] += hi_bf(rr[0]);
            t[2] += lo_bf(rr[1]);
            t[3] += hi_bf(rr[1]);
            const u32x2 o = {pack_bf2(t[0], t[1]), pack_bf2(t[2], t[3])};
            *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (long long)m * a.N_out + n0) = o;
            v[4 * h] = lo_bf(o[0]);
            v[4 * h + 1] = hi_bf(o[0]);
            v[4 * h + 2] = lo_bf(o[1]);
            v[4 * h + 3] = hi_bf(o[1]);
          }
          float amax = 0.f;
#pragma unroll
          for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
          amax = fmaxf(amax, __shfl_xor(amax, 16, WAVE));
          amax = fmaxf(amax, __shfl_xor(amax, 32, WAVE));
          const uint32_t e = mx_e8m0(amax);
          const float inv = mx_inv_scale(e);
          uint8_t* orow = a.oq + (long long)m * a.N_out;
          *reinterpret_cast<uint32_t*>(orow + nb + 4 * g) = mx_pack4(v[0], v[1], v[2], v[3], inv);
          *reinterpret_cast<uint32_t*>(orow + nb + 16 + 4 * g) = mx_pack4(v[4], v[5], v[6], v[7], inv);
          if (g == 0) a.oe[mx_scale_off(m, nb >> 5, a.M)] = (uint8_t)e;
        }
      } else if constexpr (EPI == MG_SWIGLU) {
#pragma unroll
        for (int f = 0; f < FN / 2; ++f) {
          const int n0 = nt * (BN / 2) + wn * (BN / 2 / WN) + f * 16 + 4 * g;
          if (n0 >= a.N_out) continue;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float gt = acc[f][j][i] * sx, up = acc[f + FN / 2][j][i] * sx;
            if (FP8) { gt *= a.wsc[n0 + i]; up *= a.wsc[a.half_rows + n0 + i]; }
            v[i] = mg_silu(gt) * up;
          }
          u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
          *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (long long)m * a.N_out + n0) = o;
        }
      } else {
#pragma unroll
        for (int f = 0; f < FN; ++f) {
          const int n0 = nt * BN + wn * (BN / WN) + f * 16 + 4 * g;
          if (n0 >= a.N_out) continue;
          float v[4];
#pragma unroll
          for (int i = 0; i < 4; ++i) v[i] = acc[f][j][i] * sx * (FP8 ? a.wsc[n0 + i] : 1.f);
          if constexpr (EPI == MG_F32) {
            *reinterpret_cast<f32x4*>(reinterpret_cast<float*>(a.out) + (long long)m * a.N_out + n0) =
                f32x4{v[0], v[1], v[2], v[3]};
          } else {
            if (a.res != nullptr) {   // residual stream: out = acc + res, one rounding
              const u32x2 rr = *reinterpret_cast<const u32x2*>(a.res + (long long)m * a.N_out + n0);
              v[0] += lo_bf(rr[0]);
              v[1] += hi_bf(rr[0]);
              v[2] += lo_bf(rr[1]);
              v[3] += hi_bf(rr[1]);
            }
            u32x2 o = {pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3])};
            *reinterpret_cast<u32x2*>(reinterpret_cast<bf16_t*>(a.out) + (long long)m * a.N_out + n0) = o;
          }
        }
      }
    }
  }
#endif
}

}  // namespace k8sllm

using namespace k8sllm;

namespace {

// Tile configurations (BM x BN, waves WM x WN, ring depth S).  Index = config id of the host API.
struct MgCfg {
  int bm, bn, wm, wn, wk, rb, s;
};
constexpr MgCfg kMgCfgs[] = {
    // --- weight streaming (batched decode): small tiles, many workgroups; wk waves share a tile
    {16, 16, 1, 1, 4, 512, 4},    //  0  (no SwiGLU)
    {16, 32, 1, 1, 4, 512, 4},    //  1
    {16, 32, 1, 2, 2, 512, 4},    //  2  (no SwiGLU)
    {16, 64, 1, 2, 2, 256, 4},    //  3
    {16, 64, 1, 4, 1, 256, 5},    //  4  (no SwiGLU)
    {16, 128, 1, 4, 1, 128, 6},   //  5
    {32, 32, 1, 1, 4, 512, 3},    //  6
    {32, 32, 2, 1, 2, 512, 3},    //  7
    {32, 64, 1, 2, 2, 256, 4},    //  8
    {32, 128, 1, 4, 1, 128, 6},   //  9
    {64, 32, 1, 1, 4, 256, 4},    // 10
    {64, 32, 2, 1, 2, 256, 4},    // 11
    {64, 64, 2, 2, 1, 256, 4},    // 12
    {64, 128, 1, 4, 1, 128, 5},   // 13
    {64, 64, 2, 2, 1, 128, 7},    // 14
    // --- larger M (prefill chunks): MFMA-dense tiles
    {128, 128, 2, 2, 1, 128, 3},  // 15
    {128, 64, 2, 2, 1, 128, 4},   // 16
    {256, 128, 2, 2, 1, 128, 3},  // 17
    {256, 64, 4, 1, 1, 128, 3},   // 18
    {128, 256, 2, 4, 1, 128, 3},  // 19  8 waves
    {256, 256, 2, 4, 1, 128, 2},  // 20  8 waves
    {64, 128, 2, 4, 1, 128, 3},   // 21  8 waves
    {128, 128, 2, 4, 1, 128, 3},  // 22  8 waves
    {128, 64, 2, 2, 2, 256, 3},   // 23  k-shared waves, 8 waves
    // --- prefill with 32-wide k-steps: the 128 KiB ring holds 4 stages, 3 in flight
    {256, 256, 2, 4, 1, 64, 4},   // 24  8 waves
    {256, 128, 2, 2, 1, 64, 5},   // 25
    {128, 256, 2, 4, 1, 64, 6},   // 26  8 waves
    {256, 128, 2, 4, 1, 64, 5},   // 27  8 waves
    // --- 64-row weight-streaming tiles: 4-deep rings of 128-byte k-steps
    {64, 32, 2, 1, 2, 128, 4},    // 28
    {64, 64, 2, 2, 1, 128, 4},    // 29
    {64, 128, 1, 4, 1, 128, 4},   // 30
    {64, 64, 2, 2, 2, 128, 4},    // 31  8 waves, k-shared
    // --- weight-streaming tiles whose waves span whole 32-feature SwiGLU blocks (the MX-output epilogue)
    {64, 64, 2, 1, 2, 256, 4},    // 32
    {32, 64, 1, 1, 4, 512, 3},    // 33
    {64, 128, 2, 2, 1, 128, 6},   // 34
    {16, 64, 1, 1, 4, 512, 3},    // 35
    {128, 64, 2, 1, 2, 256, 3},   // 36
};
constexpr int kMgNumCfgs = sizeof(kMgCfgs) / sizeof(kMgCfgs[0]);

// LDS bytes of config c in mode (0 bf16, 1 fp8 x and W, 3 MX: fp8 W, MX x)
constexpr int mg_lds_bytes(const MgCfg c, int mode) {
  return c.s * (c.bn * c.rb + c.bm * c.rb + (mode == 3 ? c.bm * (c.rb / 32) : 0)) + 16 + c.wk * c.wn * c.bm * 4;
}
// MX activations: 128-value subtiles split evenly over the k-sharing waves, scale dwords evenly over all waves
constexpr bool mg_mx_cfg(int c) {
  return kMgCfgs[c].rb >= 128 && (kMgCfgs[c].rb / 128) % kMgCfgs[c].wk == 0 &&
         (kMgCfgs[c].bm * (kMgCfgs[c].rb / 128)) % (kMgCfgs[c].wm * kMgCfgs[c].wn * kMgCfgs[c].wk) == 0 &&
         mg_lds_bytes(kMgCfgs[c], 3) <= 160 * 1024;
}
// SwiGLU with MX output: every wave's feature span is whole 32-feature blocks
constexpr bool mg_mxo_cfg(int c) {
  return (kMgCfgs[c].bn / (kMgCfgs[c].wn * 16)) % 4 == 0 ||
         (kMgCfgs[c].bn / (kMgCfgs[c].wn * 16) == 2 && kMgCfgs[c].wn % 2 == 0 && kMgCfgs[c].wk == 1);
}

// residual epilogue with MX output: fragment pairs per wave
constexpr bool mg_mxr_cfg(int c) { return (kMgCfgs[c].bn / (kMgCfgs[c].wn * 16)) % 2 == 0; }

template <int C, int EPI, bool FP8, bool MX, bool MXO>
int mg_launch(const MgArgs& a, int grid, hipStream_t s) {
  constexpr bool ok = (EPI != MG_SWIGLU || (kMgCfgs[C].bn / (kMgCfgs[C].wn * 16)) % 2 == 0) &&
                      (!MX || mg_mx_cfg(C)) &&
                      (!MXO || (EPI == MG_SWIGLU && mg_mxo_cfg(C)) || (EPI == MG_BF16 && mg_mxr_cfg(C)));
  if constexpr (!ok) {
    return -2;
  } else {
    hipLaunchKernelGGL((mgemm_kernel<kMgCfgs[C].bm, kMgCfgs[C].bn, kMgCfgs[C].wm, kMgCfgs[C].wn, kMgCfgs[C].wk,
                                      kMgCfgs[C].rb, kMgCfgs[C].s, EPI, FP8, MX, MXO>),
                       dim3(grid), dim3(64 * kMgCfgs[C].wm * kMgCfgs[C].wn * kMgCfgs[C].wk), 0, s, a);
    return (int)hipGetLastError();
  }
}

template <int C, bool FP8, bool MX>
int mg_epi(const MgArgs& a, int grid, int epi, bool mxo, hipStream_t s) {
  if constexpr (FP8) {   // MX output: the SwiGLU / residual epilogues of the fp8 and MX modes
    if (mxo) {
      if (epi == MG_SWIGLU) return mg_launch<C, MG_SWIGLU, FP8, MX, true>(a, grid, s);
      if (epi == MG_BF16) return mg_launch<C, MG_BF16, FP8, MX, true>(a, grid, s);
      return -2;
    }
  }
  switch (epi) {
    case MG_BF16: return mg_launch<C, MG_BF16, FP8, MX, false>(a, grid, s);
    case MG_F32: return mg_launch<C, MG_F32, FP8, MX, false>(a, grid, s);
    case MG_SWIGLU: return mg_launch<C, MG_SWIGLU, FP8, MX, false>(a, grid, s);
  }
  return -2;
}

template <bool FP8, bool MX, int C = 0>
int mg_cfg(const MgArgs& a, int grid, int cfg, int epi, bool mxo, hipStream_t s) {
  if constexpr (C < kMgNumCfgs) {
    if (cfg == C) return mg_epi<C, FP8, MX>(a, grid, epi, mxo, s);
    return mg_cfg<FP8, MX, C + 1>(a, grid, cfg, epi, mxo, s);
  } else {
    return -4;
  }
}

}  // namespace

extern "C" int k8s_mgemm_num_configs() { return kMgNumCfgs; }

namespace {
constexpr bool mg_mx_ok(int c) { return c < kMgNumCfgs && mg_mx_cfg(c); }
template <int C = 0>
bool mg_mx_valid(int cfg) {
  if constexpr (C < kMgNumCfgs) return cfg == C ? mg_mx_ok(C) : mg_mx_valid<C + 1>(cfg);
  else return false;
}
template <int C = 0>
bool mg_mxo_valid(int cfg) {
  if constexpr (C < kMgNumCfgs) return cfg == C ? mg_mxo_cfg(C) : mg_mxo_valid<C + 1>(cfg);
  else return false;
}
bool mg_mxr_valid(int cfg) { return cfg >= 0 && cfg < kMgNumCfgs && (kMgCfgs[cfg].bn / (kMgCfgs[cfg].wn * 16)) % 2 == 0; }
}  // namespace

// LDS bytes of a config in a mode (0 bf16, 1 fp8, 3 MX activations; 2 is not a mode); -1: the config is not built for
// that mode.  Mode 4: 0 if the config's SwiGLU epilogue can write MX output, else -1; mode 5: the same for the residual
// epilogue.
extern "C" int k8s_mgemm_lds_bytes(int cfg, int mode) {
  if (cfg < 0 || cfg >= kMgNumCfgs || mode < 0 || mode > 5 || mode == 2) return -1;
  if (mode == 4) return mg_mxo_valid(cfg) ? 0 : -1;
  if (mode == 5) return mg_mxr_valid(cfg) ? 0 : -1;
  const int b = mg_lds_bytes(kMgCfgs[cfg], mode);
  if (mode == 3 && !mg_mx_valid(cfg)) return -1;
  return b;
}

// (bm, bn) of a config: the Python planner sizes grids from them.
extern "C" int k8s_mgemm_config(int cfg, int* bm, int* bn, int* threads, int* lds_bytes, int* swiglu, int* rb) {
  if (cfg < 0 || cfg >= kMgNumCfgs) return -1;
  const MgCfg c = kMgCfgs[cfg];
  *bm = c.bm;
  *bn = c.bn;
  *threads = 64 * c.wm * c.wn * c.wk;
  *lds_bytes = c.s * (c.bm + c.bn) * c.rb + 16 + c.wk * c.wn * c.bm * 4;
  *swiglu = (c.bn / (c.wn * 16)) % 2 == 0;
  *rb = c.rb;
  return 0;
}

namespace {
struct MgGeom {
  long long tiles, T, total;
};
MgGeom mg_geom(int M, int N_out, int K, int epi, int fp8, int cfg) {
  const MgCfg c = kMgCfgs[cfg];
  const int feat = epi == MG_SWIGLU ? c.bn / 2 : c.bn;
  MgGeom g;
  g.tiles = (long long)((N_out + feat - 1) / feat) * ((M + c.bm - 1) / c.bm);
  g.T = (long long)K * (fp8 ? 1 : 2) / c.rb;
  g.total = g.tiles * g.T;
  return g;
}
}  // namespace

// Plan facts for a launch of `nwg` workgroups: the tile count, the most workgroups sharing one tile
// (cmax), the fp32 slab workspace (elements) and the ticket count.  Returns -1 for bad arguments.
extern "C" int k8s_mgemm_plan_info(int M, int N_out, int K, int epi, int fp8, int cfg, int nwg, long long* tiles,
                                   int* cmax, long long* ws_elems) {
  if (cfg < 0 || cfg >= kMgNumCfgs || M <= 0 || N_out <= 0 || K <= 0 || nwg <= 0) return -1;
  const MgGeom g = mg_geom(M, N_out, K, epi, fp8, cfg);
  if (g.T <= 0 || (long long)K * (fp8 ? 1 : 2) % kMgCfgs[cfg].rb != 0 || nwg > g.total) return -1;
  int cm = 1;
  for (long long t = 0; t < g.tiles; ++t) {
    const long long f = ((t * g.T + 1) * nwg - 1) / g.total, l = (((t + 1) * g.T) * nwg - 1) / g.total;
    if (l - f + 1 > cm) cm = (int)(l - f + 1);
  }
  *tiles = g.tiles;
  *cmax = cm;
  *ws_elems = cm > 1 ? g.tiles * cm * (kMgCfgs[cfg].bm * kMgCfgs[cfg].bn + kMgCfgs[cfg].bm) : 0;
  return 0;
}

// out[M, N_out] = epi(x[M, K] . W^T) with `nwg` workgroups streaming equal shares of the
// (tile, k-step) items.  fp8 = 1: x / W are e4m3 bytes with per-row scales xs / wsc; fp8 = 3 (MX): W e4m3 with row
// scales wsc, x MX e4m3 with its E8M0 block scales in xs (bytes, mx_scale_off layout).  oq / oe (fp8 = 1 or 3, SwiGLU): the
// output is written as MX e4m3 [M][N_out] + E8M0 (mx_scale_off layout) instead of bf16 (out unused).
// SwiGLU: W holds 2 * N_out rows ([gate; up]); out has N_out columns.
extern "C" int k8s_mgemm(void* out, float* ws, unsigned* tickets, const void* x, const void* W, const float* xs,
                         const float* wsc, int M, int N_out, int K, int epi, int fp8, int cfg, int nwg, int cmax,
                         const void* res, int rms, float eps, void* oq, void* oe, int fenced, hipStream_t stream) {
  if (cfg < 0 || cfg >= kMgNumCfgs || M <= 0 || N_out <= 0 || K <= 0 || nwg <= 0 || cmax < 1) return -1;
  if (N_out % 4 != 0) return -1;
  if (fp8 < 0 || fp8 > 3 || fp8 == 2) return -1;
  const bool mx = fp8 == 3, mxo = oq != nullptr;
  if (mxo && (oe == nullptr || (fp8 != 1 && fp8 != 3) || N_out % 128 != 0 ||
              !(epi == MG_SWIGLU ? mg_mxo_valid(cfg) : (epi == MG_BF16 && res != nullptr && mg_mxr_valid(cfg)))))
    return -7;
  if (mx && (K % 128 != 0 || !mg_mx_valid(cfg))) return -7;
  const long long kbytes = (long long)K * (fp8 ? 1 : 2), xkbytes = kbytes;
  if (kbytes % kMgCfgs[cfg].rb != 0) return -1;
  const MgGeom g = mg_geom(M, N_out, K, epi, fp8, cfg);
  if (nwg > g.total) return -1;
  if (cmax > 1 && (ws == nullptr || tickets == nullptr)) return -3;
  const long long wrows = epi == MG_SWIGLU ? 2LL * N_out : (long long)N_out;
  if (wrows * kbytes >= (1LL << 32) || (long long)M * xkbytes >= (1LL << 32)) return -5;  // 32-bit DMA offsets
  if ((fp8 == 1 || fp8 == 3) && (xs == nullptr || wsc == nullptr)) return -3;
  if (res != nullptr && epi != MG_BF16) return -6;   // residual epilogue: bf16 output only
  if (rms && fp8 == 1) return -6;   // per-token e4m3 activations carry 1 / rms in their scales (MX rows: prologue)
  MgArgs a;
  a.res = static_cast<const bf16_t*>(res);
  a.rms = rms;
  a.eps = eps;
  // RMS prologue on the MFMA for the wide projections (>= 8192 output features: the 70B TP = 1 / 2 QKV, gate/up),
  // v_dot2 squares for the narrow ones, where the extra MFMA is as large as the tile's own work (one TP = 8 rank:
  // batch-64 decode 7.66 ms/step with v_dot2, 7.78 with the MFMA; TP = 1: 31.98 -> 30.72, profiles/rms_mfma_ab_r5.txt).
  // K8S_RMS_MFMA = 0 / 1 forces one form.
  static const int rms_mfma_env = [] { const char* e = getenv("K8S_RMS_MFMA"); return e ? atoi(e) : -1; }();
  a.rms_mfma = rms_mfma_env >= 0 ? rms_mfma_env : (N_out >= 8192 ? 1 : 0);
  a.fenced = fenced;   // (ops.mgemm: K8S_MGEMM_FENCED, or per call in the fenced-vs-fence-free test)
  a.out = out;
  a.ws = ws;
  a.cnt = tickets;
  a.x = static_cast<const uint8_t*>(x);
  a.W = static_cast<const uint8_t*>(W);
  a.xs = xs;
  a.wsc = wsc;
  a.xe = mx ? reinterpret_cast<const uint8_t*>(xs) : nullptr;
  a.oq = static_cast<uint8_t*>(oq);
  a.oe = static_cast<uint8_t*>(oe);
  a.kbytes = kbytes;
  a.xkbytes = xkbytes;
  a.total = g.total;
  a.M = M;
  a.N_out = N_out;
  a.half_rows = epi == MG_SWIGLU ? N_out : 0;
  a.m_tiles = (M + kMgCfgs[cfg].bm - 1) / kMgCfgs[cfg].bm;
  a.T = (int)g.T;
  a.nwg = nwg;
  a.cmax = cmax;
  if (mx) return mg_cfg<true, true>(a, nwg, cfg, epi, mxo, stream);
  return fp8 ? mg_cfg<true, false>(a, nwg, cfg, epi, mxo, stream) : mg_cfg<false, false>(a, nwg, cfg, epi, false, stream);
}
