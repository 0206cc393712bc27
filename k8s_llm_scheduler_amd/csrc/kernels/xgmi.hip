// One-shot all-reduce / all-gather over xGMI peer memory (MI355X node, one process per GPU).
//
// Decode-time tensor-parallel collectives are tiny (B x 8192 bf16 = 16 KiB per all-reduce at B = 1,
// 160 of them per token at TP = 8) and therefore pure latency.  A ring (RCCL) needs 2(W-1) dependent
// hops; here every rank PUSHES its whole contribution straight into every peer's receive buffer
// (xGMI is point-to-point: all 7 peers are one hop away, one link each), raises one flag per
// (workgroup, peer), waits for the peers' flags, and reduces the W contributions from its own HBM.
// One kernel, one fabric crossing + one flag crossing.
//
// Memory: each rank owns one IPC region (hipExtMallocWithFlags(..., hipDeviceMallocUncached), so no
// L2 holds stale copies of bytes another GPU wrote), mapped into every peer process:
//   [flags: 2 x XG_MAX_BLOCKS x 8 u32][flagged data: 2 slots x W x slot_bytes][LL data: 2 slots x W x slot_bytes]
//   [two-shot data: 2 phases x 2 slots x W x slot_bytes]
// The LL rows are a region of their own: an LL reader accepts a word whose tag equals its epoch, and
// raw payload bytes left by the flagged kernels could otherwise carry that tag by chance.
// Protocol per workgroup b of call k (epoch e = per-workgroup counter, identical on every rank since
// all ranks issue the same sequence of calls with the same fixed grid):
//   1. stores of its chunk into slot (e & 1), source row `rank`, of every peer   (sc0 sc1, 16 B)
//   2. s_waitcnt vmcnt(0) in every wave, barrier, then lane p stores flag[b][rank] = e at peer p
//   3. lane p polls the local flag[b][p] until it reaches e (>= : a fast peer may already be at e+1)
//   4. barrier, then sc0 sc1 loads of the W rows, fp32 sum in rank order 0..W-1 (bit-identical on
//      every rank), one bf16 rounding.
// Two slots suffice: a peer can only write slot (e+1)&1 after seeing our flag e, which we raise after
// our previous kernel (that read slot (e+1)&1) has completed in stream order.
// Polls are bounded (~timeout); a timeout sets *err and the kernel drains instead of hanging.
#include "common.h"

namespace k8sllm {

constexpr int XG_MAX_WORLD = 8;
constexpr int XG_MAX_BLOCKS = 64;
constexpr int XG_THREADS = 256;
constexpr long long XG_FLAG1_BYTES = XG_MAX_BLOCKS * XG_MAX_WORLD * 4;  // one flag array
constexpr long long XG_FLAG_BYTES = 2 * XG_FLAG1_BYTES;                  // + the two-shot phase-2 flags
constexpr int XG_SYS = 1 | 16;  // buffer-op aux: sc0 | sc1 (system coherence)

struct XgArgs {
  char* base[XG_MAX_WORLD];  // IPC region of every rank (own included), mapped here
  uint32_t* counters;        // [XG_MAX_BLOCKS] private epoch per workgroup
  uint32_t* err;             // set non-zero on a poll timeout
  const char* in;
  char* out;
  const char* res;           // optional bf16 residual added to the sum (AR + residual add, K14 + K2)
  long long bytes;           // payload bytes per rank (multiple of 16)
  long long slot_bytes;      // capacity of one (slot, source) row
  int rank, world;
  long long timeout_ticks;   // s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t xg_rsrc(const char* p, long long n) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)n, 0x00020000);
}

__device__ __forceinline__ uint32_t xg_epoch(const XgArgs& a) {
  __shared__ uint32_t s_e;
  if (threadIdx.x == 0) {
    uint32_t e = a.counters[blockIdx.x] + 1;
    a.counters[blockIdx.x] = e;
    s_e = e;
  }
  __syncthreads();
  return s_e;
}

// Steps 2 + 3: signal every peer, wait for every peer (flag array `which`: 0, or 1 = two-shot phase 2).
__device__ __forceinline__ void xg_handshake(const XgArgs& a, uint32_t e, int which = 0) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int p = threadIdx.x;
  if (p < a.world && p != a.rank) {
    const int fo = which * (XG_MAX_BLOCKS * XG_MAX_WORLD) + blockIdx.x * XG_MAX_WORLD;
    uint32_t* remote = reinterpret_cast<uint32_t*>(a.base[p]) + fo + a.rank;
    __hip_atomic_store(remote, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* local = reinterpret_cast<uint32_t*>(a.base[a.rank]) + fo + p;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(local, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
        __hip_atomic_fetch_or(a.err, 1u << p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// Step 1: push this rank's bytes [v*16] to row `rank` of slot (e&1) at every peer.
__device__ __forceinline__ void xg_push(const XgArgs& a, uint32_t e) {
  const long long nvec = a.bytes >> 4;
  const long long row = XG_FLAG_BYTES + ((long long)(e & 1) * a.world + a.rank) * a.slot_bytes;
  const u32x4* in = reinterpret_cast<const u32x4*>(a.in);
  for (int p = 0; p < a.world; ++p) {
    if (p == a.rank) continue;
    const auto rs = xg_rsrc(a.base[p] + row, a.slot_bytes);
    for (long long v = (long long)blockIdx.x * XG_THREADS + threadIdx.x; v < nvec; v += (long long)gridDim.x * XG_THREADS)
      __builtin_amdgcn_raw_buffer_store_b128(in[v], rs, (int)(v << 4), 0, XG_SYS);
  }
}

template <int W>
__global__ __launch_bounds__(XG_THREADS) void xg_allreduce_bf16_kernel(XgArgs a) {
  const uint32_t e = xg_epoch(a);
  xg_push(a, e);
  xg_handshake(a, e);
  const long long nvec = a.bytes >> 4;
  const long long slot0 = XG_FLAG_BYTES + (long long)(e & 1) * W * a.slot_bytes;
  const u32x4* in = reinterpret_cast<const u32x4*>(a.in);
  u32x4* out = reinterpret_cast<u32x4*>(a.out);
  for (long long v = (long long)blockIdx.x * XG_THREADS + threadIdx.x; v < nvec; v += (long long)gridDim.x * XG_THREADS) {
    // All W rows are loaded unconditionally (own row is stale, then replaced by a select) so the
    // loads issue back to back instead of behind W branches.
    const u32x4 mine = in[v];
    u32x4 rows[W];
#pragma unroll
    for (int t = 0; t < W; ++t)
      rows[t] = __builtin_amdgcn_raw_buffer_load_b128(xg_rsrc(a.base[a.rank] + slot0 + t * a.slot_bytes, a.slot_bytes),
                                                      (int)(v << 4), 0, XG_SYS);
#pragma unroll
    for (int t = 0; t < W; ++t)
      if (t == a.rank) rows[t] = mine;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) { acc[2 * j] = 0.f; acc[2 * j + 1] = 0.f; }
#pragma unroll
    for (int t = 0; t < W; ++t) {
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc[2 * j] += lo_bf(rows[t][j]); acc[2 * j + 1] += hi_bf(rows[t][j]); }
    }
    if (a.res != nullptr) {
      const u32x4 rv = reinterpret_cast<const u32x4*>(a.res)[v];
#pragma unroll
      for (int j = 0; j < 4; ++j) { acc[2 * j] += lo_bf(rv[j]); acc[2 * j + 1] += hi_bf(rv[j]); }
    }
    u32x4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = pack_bf2(acc[2 * j], acc[2 * j + 1]);
    out[v] = r;
  }
}

// LL ("low-latency") all-reduce for decode-size messages: the flag travels WITH the data.  Every
// 4-byte word (two bf16) is pushed as one 8-byte store {word, epoch} into row `rank` of slot (e & 1)
// at every peer; a reader polls each peer's 8-byte word until its high half equals e, so there is
// no separate flag store, no workgroup barrier and no second fabric crossing between the data and
// its readiness.  8-byte stores arrive untorn (MI355X_MICROARCH.md visibility notes).  The rows
// hold 2x the payload bytes.  Slot reuse is safe for the same reason as in the flagged kernel.
template <int W>
__global__ __launch_bounds__(XG_THREADS) void xg_allreduce_ll_kernel(XgArgs a) {
  typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
  const uint32_t e = xg_epoch(a);
  const long long nwords = a.bytes >> 2;
  const long long ll0 = XG_FLAG_BYTES + 2LL * W * a.slot_bytes;  // the LL region
  const long long my_row = ll0 + ((long long)(e & 1) * W + a.rank) * a.slot_bytes;
  const long long slot0 = ll0 + (long long)(e & 1) * W * a.slot_bytes;
  const uint32_t* in = reinterpret_cast<const uint32_t*>(a.in);
  uint32_t* out = reinterpret_cast<uint32_t*>(a.out);
  const long long stride = (long long)gridDim.x * XG_THREADS;
  for (long long v = (long long)blockIdx.x * XG_THREADS + threadIdx.x; v < nwords; v += stride) {
    const uint32_t mine = in[v];
    const u32x2 word = u32x2{mine, e};
#pragma unroll
    for (int p = 0; p < W; ++p) {
      if (p == a.rank) continue;
      __builtin_amdgcn_raw_buffer_store_b64(word, xg_rsrc(a.base[p] + my_row, a.slot_bytes), (int)(v << 3), 0, XG_SYS);
    }
  }
  for (long long v = (long long)blockIdx.x * XG_THREADS + threadIdx.x; v < nwords; v += stride) {
    uint32_t d[W];
    u32x2 w[W];
#pragma unroll
    for (int t = 0; t < W; ++t)
      if (t != a.rank)
        w[t] = __builtin_amdgcn_raw_buffer_load_b64(xg_rsrc(a.base[a.rank] + slot0 + t * a.slot_bytes, a.slot_bytes),
                                                    (int)(v << 3), 0, XG_SYS);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll
    for (int t = 0; t < W; ++t) {
      if (t == a.rank) {
        d[t] = in[v];
        continue;
      }
      while (w[t].y != e) {
        __builtin_amdgcn_s_sleep(1);
        if ((long long)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout_ticks) {
          __hip_atomic_fetch_or(a.err, 1u << t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        w[t] = __builtin_amdgcn_raw_buffer_load_b64(xg_rsrc(a.base[a.rank] + slot0 + t * a.slot_bytes, a.slot_bytes),
                                                    (int)(v << 3), 0, XG_SYS);
      }
      d[t] = w[t].x;
    }
    float lo = 0.f, hi = 0.f;
#pragma unroll
    for (int t = 0; t < W; ++t) {  // fixed rank order: bit-identical on every rank
      lo += lo_bf(d[t]);
      hi += hi_bf(d[t]);
    }
    if (a.res != nullptr) {
      const uint32_t rr = reinterpret_cast<const uint32_t*>(a.res)[v];
      lo += lo_bf(rr);
      hi += hi_bf(rr);
    }
    out[v] = pack_bf2(lo, hi);
  }
}

// Two-shot all-reduce (reduce-scatter + all-gather) for large messages: the payload is cut into W
// shards; every rank pushes shard p of its contribution to peer p only (phase 1), reduces its OWN shard
// from the W contributions (fixed rank order, + residual, one rounding: the same bits as the one-shot
// kernel), then pushes the reduced shard to every peer (phase 2) and gathers theirs.  Each link carries
// 2 x bytes / W instead of the one-shot's full `bytes`, spread over all W - 1 links at once.  Workgroup
// b moves the same vector range of every shard in both phases, so per-workgroup flags suffice.
template <int W>
__global__ __launch_bounds__(XG_THREADS) void xg_allreduce_2shot_kernel(XgArgs a) {
  const uint32_t e = xg_epoch(a);
  const long long nvec = a.bytes >> 4, seg = (nvec + W - 1) / W;
  const long long ts0 = XG_FLAG_BYTES + 4LL * W * a.slot_bytes;           // two-shot region
  const long long p1 = ts0 + (long long)(e & 1) * W * a.slot_bytes;         // phase-1 rows (slot e & 1)
  const long long p2 = ts0 + 2LL * W * a.slot_bytes + (long long)(e & 1) * W * a.slot_bytes;
  const u32x4* in = reinterpret_cast<const u32x4*>(a.in);
  u32x4* out = reinterpret_cast<u32x4*>(a.out);
  const long long v0 = (long long)blockIdx.x * XG_THREADS + threadIdx.x, vs = (long long)gridDim.x * XG_THREADS;
  auto shard_len = [&](int t) -> long long { return max(0LL, min(seg, nvec - t * seg)); };
  // phase 1: shard p of my contribution -> row `rank` of peer p's phase-1 slot
  for (int p = 0; p < W; ++p) {
    if (p == a.rank) continue;
    const auto rs = xg_rsrc(a.base[p] + p1 + (long long)a.rank * a.slot_bytes, a.slot_bytes);
    const long long n = shard_len(p);
    for (long long v = v0; v < n; v += vs)
      __builtin_amdgcn_raw_buffer_store_b128(in[p * seg + v], rs, (int)(v << 4), 0, XG_SYS);
  }
  xg_handshake(a, e, 0);
  // reduce my shard; keep it and push it to every peer's phase-2 slot
  {
    const long long n = shard_len(a.rank), base = a.rank * seg;
    for (long long v = v0; v < n; v += vs) {
      u32x4 rows[W];
#pragma unroll
      for (int t = 0; t < W; ++t)
        rows[t] = __builtin_amdgcn_raw_buffer_load_b128(
            xg_rsrc(a.base[a.rank] + p1 + (long long)t * a.slot_bytes, a.slot_bytes), (int)(v << 4), 0, XG_SYS);
      const u32x4 mine = in[base + v];
#pragma unroll
      for (int t = 0; t < W; ++t)
        if (t == a.rank) rows[t] = mine;
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll
      for (int t = 0; t < W; ++t) {
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[2 * j] += lo_bf(rows[t][j]); acc[2 * j + 1] += hi_bf(rows[t][j]); }
      }
      if (a.res != nullptr) {
        const u32x4 rv = reinterpret_cast<const u32x4*>(a.res)[base + v];
#pragma unroll
        for (int j = 0; j < 4; ++j) { acc[2 * j] += lo_bf(rv[j]); acc[2 * j + 1] += hi_bf(rv[j]); }
      }
      u32x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) r[j] = pack_bf2(acc[2 * j], acc[2 * j + 1]);
      out[base + v] = r;
#pragma unroll
      for (int p = 0; p < W; ++p) {
        if (p == a.rank) continue;
        __builtin_amdgcn_raw_buffer_store_b128(
            r, xg_rsrc(a.base[p] + p2 + (long long)a.rank * a.slot_bytes, a.slot_bytes), (int)(v << 4), 0, XG_SYS);
      }
    }
  }
  xg_handshake(a, e, 1);
  // phase 2: gather every peer's reduced shard
  for (int t = 0; t < W; ++t) {
    if (t == a.rank) continue;
    const auto rs = xg_rsrc(a.base[a.rank] + p2 + (long long)t * a.slot_bytes, a.slot_bytes);
    const long long n = shard_len(t);
    for (long long v = v0; v < n; v += vs) out[t * seg + v] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(v << 4), 0, XG_SYS);
  }
}

// out[t * bytes ...] = contribution of rank t (shard-major), any dtype.
__global__ __launch_bounds__(XG_THREADS) void xg_allgather_kernel(XgArgs a) {
  const uint32_t e = xg_epoch(a);
  xg_push(a, e);
  xg_handshake(a, e);
  const long long nvec = a.bytes >> 4;
  const long long slot0 = XG_FLAG_BYTES + (long long)(e & 1) * a.world * a.slot_bytes;
  const u32x4* in = reinterpret_cast<const u32x4*>(a.in);
  for (int t = 0; t < a.world; ++t) {
    u32x4* out = reinterpret_cast<u32x4*>(a.out + t * a.bytes);
    const auto rs = xg_rsrc(a.base[a.rank] + slot0 + t * a.slot_bytes, a.slot_bytes);
    const u32x4* src = t == a.rank ? in : nullptr;
    for (long long v = (long long)blockIdx.x * XG_THREADS + threadIdx.x; v < nvec; v += (long long)gridDim.x * XG_THREADS)
      out[v] = src ? src[v] : __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(v << 4), 0, XG_SYS);
  }
}

}  // namespace k8sllm

using namespace k8sllm;

extern "C" long long k8s_xgmi_flag_bytes() { return XG_FLAG_BYTES; }
extern "C" int k8s_xgmi_max_blocks() { return XG_MAX_BLOCKS; }

static int xg_fill(XgArgs& a, void* const* bases, uint32_t* counters, uint32_t* err, const void* in, void* out,
                   long long bytes, long long slot_bytes, int rank, int world, long long timeout_ticks) {
  if (world < 2 || world > XG_MAX_WORLD || rank < 0 || rank >= world) return -1;
  if (bytes <= 0 || bytes > slot_bytes || (bytes & 15) || ((uintptr_t)in & 15) || ((uintptr_t)out & 15)) return -2;
  if (XG_FLAG_BYTES + 8LL * world * slot_bytes > 0x7fffffffLL) return -3;
  for (int i = 0; i < XG_MAX_WORLD; ++i) a.base[i] = i < world ? static_cast<char*>(bases[i]) : nullptr;
  a.counters = counters; a.err = err;
  a.in = static_cast<const char*>(in); a.out = static_cast<char*>(out); a.res = nullptr;
  a.bytes = bytes; a.slot_bytes = slot_bytes; a.rank = rank; a.world = world; a.timeout_ticks = timeout_ticks;
  return 0;
}

extern "C" int k8s_xgmi_allreduce_bf16(void* const* bases, uint32_t* counters, uint32_t* err, const void* in,
                                       void* out, long long bytes, long long slot_bytes, int rank, int world,
                                       int blocks, long long timeout_ticks, const void* residual, hipStream_t s) {
  XgArgs a;
  if (int rc = xg_fill(a, bases, counters, err, in, out, bytes, slot_bytes, rank, world, timeout_ticks)) return rc;
  if ((uintptr_t)residual & 15) return -2;
  a.res = static_cast<const char*>(residual);
  if (blocks < 1 || blocks > XG_MAX_BLOCKS) return -4;
  switch (world) {
    case 2: xg_allreduce_bf16_kernel<2><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 4: xg_allreduce_bf16_kernel<4><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 8: xg_allreduce_bf16_kernel<8><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 3: xg_allreduce_bf16_kernel<3><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 5: xg_allreduce_bf16_kernel<5><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 6: xg_allreduce_bf16_kernel<6><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 7: xg_allreduce_bf16_kernel<7><<<blocks, XG_THREADS, 0, s>>>(a); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int k8s_xgmi_allreduce_ll_bf16(void* const* bases, uint32_t* counters, uint32_t* err, const void* in,
                                          void* out, long long bytes, long long slot_bytes, int rank, int world,
                                          int blocks, long long timeout_ticks, const void* residual, hipStream_t s) {
  XgArgs a;
  if (2 * bytes > slot_bytes) return -2;  // LL rows carry a flag word per data word
  if (int rc = xg_fill(a, bases, counters, err, in, out, bytes, slot_bytes, rank, world, timeout_ticks)) return rc;
  if ((uintptr_t)residual & 3) return -2;
  a.res = static_cast<const char*>(residual);
  if (blocks < 1 || blocks > XG_MAX_BLOCKS) return -4;
  switch (world) {
    case 2: xg_allreduce_ll_kernel<2><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 4: xg_allreduce_ll_kernel<4><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 8: xg_allreduce_ll_kernel<8><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 3: xg_allreduce_ll_kernel<3><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 5: xg_allreduce_ll_kernel<5><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 6: xg_allreduce_ll_kernel<6><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 7: xg_allreduce_ll_kernel<7><<<blocks, XG_THREADS, 0, s>>>(a); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int k8s_xgmi_allreduce_2shot_bf16(void* const* bases, uint32_t* counters, uint32_t* err, const void* in,
                                             void* out, long long bytes, long long slot_bytes, int rank, int world,
                                             int blocks, long long timeout_ticks, const void* residual,
                                             hipStream_t s) {
  XgArgs a;
  // shards of ceil(bytes / 16 / world) vectors must fit one row
  if (bytes <= 0 || (bytes & 15) || ((bytes / 16 + world - 1) / world) * 16 > slot_bytes) return -2;
  if (int rc = xg_fill(a, bases, counters, err, in, out, 16, slot_bytes, rank, world, timeout_ticks)) return rc;
  a.bytes = bytes;
  if ((uintptr_t)residual & 15) return -2;
  a.res = static_cast<const char*>(residual);
  if (blocks < 1 || blocks > XG_MAX_BLOCKS) return -4;
  switch (world) {
    case 2: xg_allreduce_2shot_kernel<2><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 4: xg_allreduce_2shot_kernel<4><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 8: xg_allreduce_2shot_kernel<8><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 3: xg_allreduce_2shot_kernel<3><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 5: xg_allreduce_2shot_kernel<5><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 6: xg_allreduce_2shot_kernel<6><<<blocks, XG_THREADS, 0, s>>>(a); break;
    case 7: xg_allreduce_2shot_kernel<7><<<blocks, XG_THREADS, 0, s>>>(a); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}

extern "C" int k8s_xgmi_allgather(void* const* bases, uint32_t* counters, uint32_t* err, const void* in, void* out,
                                  long long bytes, long long slot_bytes, int rank, int world, int blocks,
                                  long long timeout_ticks, hipStream_t s) {
  XgArgs a;
  if (int rc = xg_fill(a, bases, counters, err, in, out, bytes, slot_bytes, rank, world, timeout_ticks)) return rc;
  if (blocks < 1 || blocks > XG_MAX_BLOCKS) return -4;
  xg_allgather_kernel<<<blocks, XG_THREADS, 0, s>>>(a);
  return (int)hipGetLastError();
}
