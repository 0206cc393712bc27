// Probe: does one persistent launch that runs a chain of decode GEMVs (grid barriers between them, the next
// projection's first weights requested BEFORE the barrier wait) beat the same GEMVs as separate graph-captured
// launches?  This measures the cost model behind VERDICT r3 item 2 (one launch per decode layer) on the chip instead
// of the price-list estimate in docs/PERF.md.  Not used by the engine.
//
// Both modes run the same code: out_p[n] = sum_k W_p[n][k] * x_p[k], one wave per row at a time (rows gw, gw + nw, ..
// over all waves of the grid), 16-byte non-temporal weight loads through a buffer resource (chunks past K read 0
// without traffic), v_dot2_f32_bf16 against x staged in LDS, the next row's weights in flight while the current one
// is reduced.  x and out are fp32 (device-coherent 4-byte stores / device-scope loads, so a later phase of the SAME
// launch on another XCD reads them correctly); x is converted to bf16 while it is staged.
//
// Persistent mode: grid = one workgroup per CU (the LDS pad forbids two), phase p waits until every workgroup has
// arrived from phase p - 1 (a relaxed device-scope counter, polled by one lane with s_sleep, bounded by s_memrealtime:
// a wait that exceeds ~20 ms sets *err and proceeds, so a grid that is not co-resident cannot hang the GPU), and the
// last arrival of the last phase re-arms the counter.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -shared -fPIC -I k8s_llm_scheduler_amd/csrc/kernels \
//       tools/experiments/chain.hip -o tools/experiments/chain.so
#include "common.h"

using namespace k8sllm;

namespace {

constexpr int CH_NT = 256;      // threads per workgroup (4 waves)
constexpr int CH_CMAX = 16;     // 16-byte chunks per lane per row: K <= 8192
constexpr int CH_MAXPH = 32;
constexpr int CH_SC1 = 16;      // buffer-op cache policy: device scope
#ifndef CH_PRE2
#define CH_PRE2 0               // 1: two rows per wave requested before the barrier wait (and the loop issues after math)
#endif

struct ChPhase {
  const bf16_t* W;
  const float* x;
  float* out;
  int N, K;
};
struct ChArgs {
  ChPhase ph[CH_MAXPH];
  int nph;
  int persistent;
  unsigned* cnt;
  unsigned* err;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t ch_rsrc(const void* p, long long bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)min(bytes, 0x7fffffffLL), 0x00020000);
}

__global__ void __launch_bounds__(CH_NT) chain_kernel(ChArgs a) {
  __shared__ __attribute__((aligned(16))) u32x4 xs[CH_CMAX * 64];   // 16 KiB: x of one phase as bf16
  __shared__ char pad[96 * 1024];                                    // one workgroup per CU
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  pad[tid] = 0;   // (the pad is used below under a condition no launch meets, so it stays allocated)
  const int gw = blockIdx.x * (CH_NT / 64) + wid, nw = gridDim.x * (CH_NT / 64);
  constexpr unsigned OOB = 0x80000000u;

  for (int p = 0; p < a.nph; ++p) {
    const ChPhase ph = a.ph[p];
    const int C = ph.K / 512;
    const auto rw = ch_rsrc(ph.W, (long long)ph.N * ph.K * 2);
    auto load_row = [&](u32x4 (&w)[CH_CMAX], int r) {
#pragma unroll
      for (int i = 0; i < CH_CMAX; ++i) {
        const unsigned off = (i < C && r < ph.N) ? (unsigned)r * ph.K * 2 + (unsigned)(i * 64 + lane) * 16 : OOB;
        w[i] = __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 2);
      }
    };
    // the first PRE rows' weights go out before the wait for the previous phase (they do not depend on it)
    u32x4 w0[CH_CMAX], w1[CH_CMAX];
    load_row(w0, gw);
    if (CH_PRE2) load_row(w1, gw + nw);
    asm volatile("" ::: "memory");
    if (a.persistent && p > 0) {
      if (tid == 0) {
        const unsigned target = (unsigned)p * gridDim.x;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(a.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {   // ~20 ms at 100 MHz
            __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
          }
        }
      }
      __syncthreads();
    }
    // x -> LDS as bf16 (device-scope loads: written by other workgroups of this launch); past K: zeros
    {
      const auto rx = ch_rsrc(ph.x, (long long)ph.K * 4);
      for (int c = tid; c < CH_CMAX * 64; c += CH_NT) {
        u32x4 o = u32x4{0u, 0u, 0u, 0u};
        if (c * 8 < ph.K) {
          const u32x4 lo = __builtin_amdgcn_raw_buffer_load_b128(rx, c * 32, 0, CH_SC1);
          const u32x4 hi = __builtin_amdgcn_raw_buffer_load_b128(rx, c * 32 + 16, 0, CH_SC1);
          o = u32x4{pack_bf2(__uint_as_float(lo[0]), __uint_as_float(lo[1])),
                    pack_bf2(__uint_as_float(lo[2]), __uint_as_float(lo[3])),
                    pack_bf2(__uint_as_float(hi[0]), __uint_as_float(hi[1])),
                    pack_bf2(__uint_as_float(hi[2]), __uint_as_float(hi[3]))};
        }
        xs[c] = o;
      }
    }
    __syncthreads();
    auto dot_row = [&](const u32x4 (&w)[CH_CMAX], int r) {
      float acc = 0.f;
#pragma unroll
      for (int i = 0; i < CH_CMAX; ++i) {
        const u32x4 xv = xs[i * 64 + lane];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, w[i][e]), __builtin_bit_cast(bf16x2, xv[e]),
                                                acc, false);
      }
      acc = wave_sum(acc);
      if (lane == 0) __hip_atomic_store(ph.out + r, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    // two rows per trip so both register sets are static; a row's loads are in flight while the other is reduced
    for (int r = gw; r < ph.N; r += 2 * nw) {
      if (!CH_PRE2) {
        load_row(w1, r + nw);
        asm volatile("" ::: "memory");
      }
      dot_row(w0, r);
      if (CH_PRE2) {
        load_row(w0, r + 2 * nw);
        asm volatile("" ::: "memory");
      }
      if (r + nw >= ph.N) break;
      if (!CH_PRE2) {
        load_row(w0, r + 2 * nw);
        asm volatile("" ::: "memory");
      }
      dot_row(w1, r + nw);
      if (CH_PRE2) {
        load_row(w1, r + 3 * nw);
        asm volatile("" ::: "memory");
      }
    }
    if (a.nph > CH_MAXPH) ph.out[tid] = (float)pad[(tid * 7) & 1023];
    if (a.persistent) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's output stores have landed
      __syncthreads();                                     // (and every wave is done reading xs)
      if (tid == 0) {
        const unsigned prev = __hip_atomic_fetch_add(a.cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (p == a.nph - 1 && prev == (unsigned)a.nph * gridDim.x - 1)   // the last arrival: re-arm
          __hip_atomic_store(a.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      __syncthreads();
    }
  }
}

}  // namespace

// phases: W, x, out pointers and N, K per phase (K a multiple of 512, <= 8192).  persistent: one launch over all
// phases (grid = CUs); otherwise one launch per phase.  cnt / err: zeroed u32 each.
extern "C" int chain_run(const void* const* Ws, const void* const* xs, void* const* outs, const int* Ns,
                         const int* Ks, int nph, int persistent, int grid, unsigned* cnt, unsigned* err,
                         hipStream_t stream) {
  if (nph < 1 || nph > CH_MAXPH || grid < 1) return -1;
  for (int p = 0; p < nph; ++p)
    if (Ks[p] % 512 || Ks[p] > 8192 || Ns[p] < 1) return -2;
  ChArgs a{};
  a.persistent = persistent;
  a.cnt = cnt;
  a.err = err;
  if (persistent) {
    a.nph = nph;
    for (int p = 0; p < nph; ++p)
      a.ph[p] = ChPhase{(const bf16_t*)Ws[p], (const float*)xs[p], (float*)outs[p], Ns[p], Ks[p]};
    chain_kernel<<<grid, CH_NT, 0, stream>>>(a);
  } else {
    a.nph = 1;
    for (int p = 0; p < nph; ++p) {
      a.ph[0] = ChPhase{(const bf16_t*)Ws[p], (const float*)xs[p], (float*)outs[p], Ns[p], Ks[p]};
      chain_kernel<<<grid, CH_NT, 0, stream>>>(a);
    }
  }
  return (int)hipGetLastError();
}

extern "C" int chain_cus() {
  int dev = 0, n = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return -1;
  return n;
}
