// Activation-resident GEMM for 17-64 decode rows (VERDICT r4 "next round" item 3; SURVEY K3/K8/K9/K11 at batched
// decode): out[M, N] = epi(x[M, K] . W[N, K]^T), bf16 weights streamed exactly once at the weight-streaming rate.
//
// Why not mgemm at these rows: its ring stages x together with W every k-step (at 64 rows x is as large as a 64-wide
// W tile), so only ~24 KiB of weights are in flight per CU and the 64-row QKV / O stream at 2.8-3.7 TB/s.  Here:
//  * K is cut into slabs of KSL (2048) elements; a workgroup owns ONE slab and a contiguous range of BN-row weight
//    tiles.  Its 8 waves hold the slab's activations in REGISTERS for the whole launch (wave w: 16-row block
//    w % RBLK, every KP-th 32-element k-chunk, KP = 8 / RBLK) -- loaded once, never restaged;
//  * the weights alone stream through an LDS ring of NSTG 8 KiB stages (BN = 32 rows x 256 B per k-step, one 1 KiB
//    LDS-DMA per wave per stage, source-side XOR swizzle, counted vmcnt, raw barriers): ~(NSTG - 1) x 8 KiB of
//    weights in flight per CU, across tile boundaries (the next tile's weights load under this tile's tail);
//  * v_mfma_f32_16x16x32_bf16 with W as the A operand (16 output features) and the resident x as B (16 rows); the
//    KP k-parts of a row block are added through LDS at the end of a tile in a fixed order, and each (slab, tile)
//    stores fp32 partials; xgemm_finalize_kernel sums the slabs in slab order and applies the epilogue (bf16 / fp32
//    / SwiGLU / + residual / x 1/rms with the norm gamma folded into W).  Deterministic.
// The row sums of squares for the RMS epilogue come from the resident x (first workgroup of every slab).
#include "common.h"

namespace k8sllm {

namespace {
constexpr int XG_BN = 32;                 // weight rows per tile (granularity of the plans)
constexpr int XG_RB = 256;                // bytes of one weight row per k-step (128 bf16)
constexpr int XG_NT = 512;
enum { XG_BF16 = 0, XG_F32 = 1, XG_SWIGLU = 2 };

__device__ __forceinline__ void xg_barrier() {   // raw barrier: LDS-DMA stays in flight (mgemm.hip mg_barrier)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
__device__ __forceinline__ void xg_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ int xg_swz(int r) { return r & 15; }
}  // namespace

struct XgArgs {
  const bf16_t* x;     // [M][K]
  const bf16_t* W;     // [Nw][K]
  float* ws;           // [nslab][M][Nw] partials
  float* rss;          // [nslab][4 k-parts][M] row sums of squares (rms epilogue; unused parts zero), may be null
  int M, Nw, K, nslab, gps, ntiles;
};

// RBLK: 16-row blocks of x (2: M <= 32, 4: M <= 64).  NSTG: ring stages.  KSL: k elements per slab.  BN: weight rows
// per tile (32 or 64: one or two 1 KiB LDS-DMAs per wave per stage).
template <int RBLK, int NSTG, int KSL, int BN>
__global__ void __launch_bounds__(XG_NT) xgemm_kernel(XgArgs a) {
  constexpr int KP = 8 / RBLK;                 // k-parts (waves per row block)
  constexpr int KT = KSL / 128;                // k-steps per slab
  constexpr int SUB = 4 / KP;                  // k32 sub-steps per k-step and wave
  constexpr int FB = BN / 16;                  // 16-feature blocks per tile
  constexpr int DPW = BN / 32;                 // LDS-DMAs per wave per stage
  constexpr int XG_STAGE = BN * XG_RB;
  static_assert(KP * SUB == 4 && NSTG >= 3 && NSTG * XG_STAGE <= 128 * 1024 && (BN == 32 || BN == 64), "geometry");
  __shared__ __attribute__((aligned(16))) char lds[NSTG * XG_STAGE + 3 * RBLK * FB * 64 * 16];
  float* red = reinterpret_cast<float*>(lds + NSTG * XG_STAGE);   // [KP - 1][RBLK][FB][64 lanes][4]
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rblk = wid % RBLK, kp = wid / RBLK;
  const int li = lane & 15, g4 = lane >> 4;
  // slab and tile range: the workgroups of one slab share its activations (an XCD's L2 when nslab divides 8)
  const int s = blockIdx.x % a.nslab, grp = blockIdx.x / a.nslab;
  const int t0 = (int)(((long long)grp * a.ntiles) / a.gps), t1 = (int)(((long long)(grp + 1) * a.ntiles) / a.gps);
  const int k0 = s * KSL, klen = min(KSL, a.K - k0), kt = klen >> 7;   // k-steps of this slab (<= KT)
  const long long kb = (long long)a.K * 2;   // bytes per row

  // ---- the slab's activations, resident: wave (rblk, kp) holds row rblk*16 + li, k-chunks kk = kp + KP*i of every
  // k-step (8 bf16 per lane at k = k0 + 128 t + 32 kk + 8 g4)
  const int xrow = rblk * 16 + li;
  bf16x8 xf[KT][SUB];
  float ss = 0.f;
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int i = 0; i < SUB; ++i) {
      const int kk = kp + KP * i;
      bf16x8 v = {};
      if (t < kt && xrow < a.M)
        v = *reinterpret_cast<const bf16x8*>(a.x + (size_t)xrow * a.K + k0 + 128 * t + 32 * kk + 8 * g4);
      xf[t][i] = v;
    }
  if (a.rss != nullptr && grp == 0) {   // sum of squares of this slab's rows (one workgroup per slab)
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int i = 0; i < SUB; ++i)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float v = (float)xf[t][i][e];
          ss += v * v;
        }
    ss += __shfl_xor(ss, 16, WAVE);
    ss += __shfl_xor(ss, 32, WAVE);   // lanes li, li+16, li+32, li+48: the same row
  }

  // ---- the weight stream: global k-step j of this workgroup = (tile t0 + j / kt, k-step j % kt)
  const int nsteps = (t1 - t0) * kt;
  // this wave's KiBs of a stage: KiB q = DPW wid + d holds rows 4 q .. 4 q + 3 (lane: row 4 q + lane / 16, stage
  // chunk lane % 16, which holds row chunk (lane % 16) ^ swz(row): the swizzle is applied to the SOURCE address)
  const char* wbase[DPW];
#pragma unroll
  for (int d = 0; d < DPW; ++d) {
    const int drow = 4 * (DPW * wid + d) + (lane >> 4);
    wbase[d] = reinterpret_cast<const char*>(a.W) + (size_t)drow * kb + (size_t)k0 * 2 + ((lane & 15) ^ xg_swz(drow)) * 16;
  }
  auto issue = [&](int j) {
    const int tile = t0 + j / kt, t = j - (j / kt) * kt;
#pragma unroll
    for (int d = 0; d < DPW; ++d) {
      const char* src = wbase[d] + (size_t)tile * BN * kb + (size_t)t * XG_RB;
      __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(lds + (j % NSTG) * XG_STAGE +
                                                                                       (DPW * wid + d) * 1024), 16, 0, 0);
    }
  };
#pragma unroll
  for (int j = 0; j < NSTG - 1; ++j)
    if (j < nsteps) issue(j);

  // A-operand rows of this lane in a stage image (FB 16-feature blocks)
  int arow[FB], aswz[FB];
#pragma unroll
  for (int f = 0; f < FB; ++f) {
    arow[f] = f * 16 + li;
    aswz[f] = xg_swz(arow[f]);
  }
  int j = 0;
  for (int tile = t0; tile < t1; ++tile) {
    f32x4 acc[FB];
#pragma unroll
    for (int f = 0; f < FB; ++f) acc[f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      if (t < kt) {
        // step j landed for every wave (steady state: NSTG - 2 younger stages of ONE load per wave in flight)
        if (nsteps - 1 - j >= NSTG - 2) xg_vmcnt<(NSTG - 2) * DPW>();
        else xg_vmcnt<0>();
        xg_barrier();                                    // ...and every wave is done reading stage j - 1
        if (j + NSTG - 1 < nsteps) issue(j + NSTG - 1);  // refill the stage read at step j - 1
        const char* st = lds + (j % NSTG) * XG_STAGE;
#pragma unroll
        for (int i = 0; i < SUB; ++i) {
          const int c = (kp + KP * i) * 4 + g4;         // 16-byte chunk of the 256-byte row
#pragma unroll
          for (int f = 0; f < FB; ++f) {
            const bf16x8 af = *reinterpret_cast<const bf16x8*>(st + arow[f] * XG_RB + ((c ^ aswz[f]) << 4));
            acc[f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, xf[t][i], acc[f], 0, 0, 0);
          }
        }
        ++j;
      }
    }
    // ---- k-parts of a row block added in a fixed order, fp32 partials of (slab, tile)
    if constexpr (KP > 1) {
      if (kp > 0) {
#pragma unroll
        for (int f = 0; f < FB; ++f)
          *reinterpret_cast<f32x4*>(red + ((((kp - 1) * RBLK + rblk) * FB + f) * 64 + lane) * 4) = acc[f];
      }
      xg_barrier();
      if (kp == 0) {
#pragma unroll
        for (int q = 1; q < KP; ++q)
#pragma unroll
          for (int f = 0; f < FB; ++f)
            acc[f] += *reinterpret_cast<const f32x4*>(red + ((((q - 1) * RBLK + rblk) * FB + f) * 64 + lane) * 4);
      }
    }
    if (kp == 0 && xrow < a.M) {
      // lane: x row xrow, output features f*16 + 4 g4 .. + 3 of the tile
#pragma unroll
      for (int f = 0; f < FB; ++f)
        *reinterpret_cast<f32x4*>(a.ws + ((size_t)s * a.M + xrow) * a.Nw + tile * BN + f * 16 + 4 * g4) = acc[f];
    }
    if constexpr (KP > 1) xg_barrier();   // the reduction space is free for the next tile
  }
  if (a.rss != nullptr && grp == 0 && g4 == 0 && xrow < a.M)   // this wave's k-chunks of the row: slot kp
    a.rss[((size_t)s * 4 + kp) * a.M + xrow] = ss;
}

// Sum the slabs (slab order) and apply the epilogue.  out [M][N]; res [M][N] (bf16 epilogue, may alias out).
template <int EPI, bool RES, bool RMS>
__global__ void __launch_bounds__(256) xgemm_finalize_kernel(void* __restrict__ out, const float* __restrict__ ws,
                                                             const float* __restrict__ rss, const bf16_t* res, int M,
                                                             int N, int Nw, int K, int nslab, float eps) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  const int m = i / N, n = i - m * N;
  float v = 0.f, u = 0.f;
  for (int s = 0; s < nslab; ++s) {
    const float* p = ws + ((size_t)s * M + m) * Nw;
    v += p[n];
    if (EPI == XG_SWIGLU) u += p[N + n];
  }
  if (RMS) {
    float t = 0.f;
    for (int s = 0; s < 4 * nslab; ++s) t += rss[(size_t)s * M + m];   // (slab, k-part) order
    const float inv = rsqrtf(t / (float)K + eps);
    v *= inv;
    u *= inv;
  }
  if (EPI == XG_F32) {
    reinterpret_cast<float*>(out)[i] = v;
  } else if (EPI == XG_SWIGLU) {
    reinterpret_cast<bf16_t*>(out)[i] = f2bf(v / (1.f + __expf(-v)) * u);
  } else {
    if (RES) v += bf2f(res[i]);
    reinterpret_cast<bf16_t*>(out)[i] = f2bf(v);
  }
}

}  // namespace k8sllm

using namespace k8sllm;

namespace {
int xg_cus() {
  static const int v = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return v;
}
constexpr int XG_KSL = 2048;
// ring depth / tile width (K8S_XGEMM_CFG = "<stages>,<rows>"; defaults 12 stages of 32 rows)
struct XgCfg {
  int nstg, bn, fin;
};
XgCfg xg_cfg() {
  static const XgCfg c = [] {
    XgCfg r{12, 32, 1};
    if (const char* e = getenv("K8S_XGEMM_CFG")) sscanf(e, "%d,%d,%d", &r.nstg, &r.bn, &r.fin);
    return r;
  }();
  return c;
}
}  // namespace

// Plan: (nslab, groups per slab, workspace floats, rss floats); rc < 0 when the shape is not taken.
extern "C" int k8s_xgemm_plan(int M, int N, int K, int epi, int rms, int* nslab, int* gps, long long* ws_floats,
                              long long* rss_floats) {
  if (M < 1 || M > 64 || N <= 0 || K % 128 != 0 || K <= 0) return -1;
  const int Nw = epi == XG_SWIGLU ? 2 * N : N;
  const int bn = xg_cfg().bn;
  if (Nw % bn != 0 || (epi == XG_SWIGLU && N % bn != 0)) return -2;
  const int ns = (K + XG_KSL - 1) / XG_KSL;
  const int ntiles = Nw / bn;
  // at most one workgroup per CU in all (a second round would double the time), at most one per tile
  int g = xg_cus() / ns;
  if (g > ntiles) g = ntiles;
  if (g < 1) g = 1;
  *nslab = ns;
  *gps = g;
  *ws_floats = (long long)ns * M * Nw;
  *rss_floats = rms ? (long long)ns * 4 * M : 0;
  return 0;
}

// out [M, N] (bf16; fp32 for epi 1), x [M, K], W [Nw, K] bf16 (SwiGLU: [gate; up] rows), res optional (bf16 epilogue),
// ws: plan's workspace floats, rss: plan's rss floats (zeroed by this call when rms), eps: rms epsilon.
extern "C" int k8s_xgemm(void* out, void* ws, void* rss, const void* x, const void* W, const void* res, int M, int N,
                         int K, int epi, int rms, float eps, hipStream_t stream) {
  int ns, gps;
  long long wf, rf;
  const int rc = k8s_xgemm_plan(M, N, K, epi, rms, &ns, &gps, &wf, &rf);
  if (rc != 0) return rc;
  if (ws == nullptr || (rms && rss == nullptr)) return -3;
  if (res != nullptr && (epi != XG_BF16 || rms)) return -4;
  const int Nw = epi == XG_SWIGLU ? 2 * N : N;
  const XgCfg cf = xg_cfg();
  XgArgs a{static_cast<const bf16_t*>(x), static_cast<const bf16_t*>(W), static_cast<float*>(ws),
           rms ? static_cast<float*>(rss) : nullptr, M, Nw, K, ns, gps, Nw / cf.bn};
  if (rms) (void)hipMemsetAsync(rss, 0, (size_t)rf * 4, stream);
  const int grid = ns * gps;
#define XK(R, S, B) xgemm_kernel<R, S, XG_KSL, B><<<grid, XG_NT, 0, stream>>>(a)
#define XKR(S, B) if (M <= 32) XK(2, S, B); else XK(4, S, B)
  if (cf.bn == 64) { if (cf.nstg <= 4) { XKR(4, 64); } else { XKR(7, 64); } }
  else if (cf.nstg <= 6) { XKR(6, 32); }
  else if (cf.nstg >= 14) { XKR(14, 32); }
  else { XKR(12, 32); }
#undef XKR
#undef XK
  if (!cf.fin) return (int)hipGetLastError();   // (tuning: kernel alone)
  const int total = M * N, blocks = (total + 255) / 256;
  const float* rp = static_cast<const float*>(rss);
  const bf16_t* rr = static_cast<const bf16_t*>(res);
  const float* wp = static_cast<const float*>(ws);
#define XF(E, R, S) \
  xgemm_finalize_kernel<E, R, S><<<blocks, 256, 0, stream>>>(out, wp, rp, rr, M, N, Nw, K, ns, eps)
  if (epi == XG_F32) { if (rms) XF(XG_F32, false, true); else XF(XG_F32, false, false); }
  else if (epi == XG_SWIGLU) { if (rms) XF(XG_SWIGLU, false, true); else XF(XG_SWIGLU, false, false); }
  else if (rms) XF(XG_BF16, false, true);
  else if (res != nullptr) XF(XG_BF16, true, false);
  else XF(XG_BF16, false, false);
#undef XF
  return (int)hipGetLastError();
}
