// MFMA shape probe: does v_mfma_f32_32x32x16_bf16 beat v_mfma_f32_16x16x32_bf16 at the big-tile
// GEMM's wave tile?  Both variants run pgemm's geometry -- 512-thread workgroups, one per CU, waves 2 (P) x 4 (Q), a
// 128 x 64 output tile per wave, 64-deep k-tiles read from an XOR-swizzled LDS image with ds_read_b128 -- over the
// SAME LDS bytes (no global traffic: the loop is MFMA + LDS only), on random bf16 data, and report TFLOP/s.
//   16x16x32: per k-tile 2 k32 steps x (8 A + 4 B fragment reads, 32 MFMAs)
//   32x32x16: per k-tile 4 k16 steps x (4 A + 2 B fragment reads, 8 MFMAs)
// Same LDS bytes per MAC at this wave tile (24 x 1 KiB fragment reads per wave and k-tile either way), same
// accumulator registers (128), so the difference is the MFMA pipe itself and how each shape's reads interleave with it.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mfma_shape_probe tools/experiments/mfma_shape_probe.hip
//   /tmp/mfma_shape_probe [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int ROWS = 256, KT = 64;                 // LDS image: A [256][64] + B [256][64] bf16 = 64 KiB
__device__ __forceinline__ int slot(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }

template <bool BIG>
__global__ void __launch_bounds__(512) probe(const uint16_t* __restrict__ src, float* __restrict__ out, int iters) {
  __shared__ __attribute__((aligned(16))) char lds[2 * ROWS * KT * 2 + 20480];   // > 80 KiB: one workgroup per CU
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 2, wc = wid & 3;
  for (int i = tid; i < 2 * ROWS * 8; i += 512) {   // fill both images (16-byte chunks), swizzled
    const int img = i / (ROWS * 8), r = (i / 8) % ROWS, c = i % 8;
    *reinterpret_cast<uint4*>(lds + img * ROWS * 128 + slot(r, c)) =
        *reinterpret_cast<const uint4*>(src + ((size_t)blockIdx.x * 2 * ROWS * 8 + i) * 8);
  }
  __syncthreads();
  const char* A = lds;
  const char* B = lds + ROWS * 128;
  float sum = 0.f;
  if constexpr (!BIG) {
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int li = lane & 15, g = lane >> 4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 a[8], b[4];
#pragma unroll
        for (int f = 0; f < 8; ++f) a[f] = *reinterpret_cast<const bf16x8*>(A + slot(wr * 128 + f * 16 + li, kk * 4 + g));
#pragma unroll
        for (int f = 0; f < 4; ++f) b[f] = *reinterpret_cast<const bf16x8*>(B + slot(wc * 64 + f * 16 + li, kk * 4 + g));
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
  } else {
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;
    const int li = lane & 31, h = lane >> 5;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bf16x8 a[4], b[2];
#pragma unroll
        for (int f = 0; f < 4; ++f) a[f] = *reinterpret_cast<const bf16x8*>(A + slot(wr * 128 + f * 32 + li, kk * 2 + h));
#pragma unroll
        for (int f = 0; f < 2; ++f) b[f] = *reinterpret_cast<const bf16x8*>(B + slot(wc * 64 + f * 32 + li, kk * 2 + h));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) sum += acc[i][j][e];
  }
  out[blockIdx.x * 512 + tid] = sum;
}

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));        \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus;
  const size_t n = (size_t)grid * 2 * ROWS * KT;
  std::vector<uint16_t> h(n);
  uint32_t s = 12345;
  for (auto& v : h) {   // random bf16: random sign and mantissa, |v| in [2^-7, 2)
    s = s * 1664525u + 1013904223u;
    v = (uint16_t)(((s >> 31) << 15) | ((120u + ((s >> 20) & 7u)) << 7) | ((s >> 8) & 0x7f));
  }
  uint16_t* d_src;
  float* d_out;
  CK(hipMalloc(&d_src, n * 2));
  CK(hipMalloc(&d_out, (size_t)grid * 512 * 4));
  CK(hipMemcpy(d_src, h.data(), n * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double flop = 2.0 * 128 * 64 * KT * 8 /*waves*/ * (double)iters * grid;
  for (int rep = 0; rep < 3; ++rep) {
    for (int big = 0; big < 2; ++big) {
      // warm-up, then timed
      if (big) probe<true><<<grid, 512>>>(d_src, d_out, 64); else probe<false><<<grid, 512>>>(d_src, d_out, 64);
      CK(hipEventRecord(e0));
      if (big) probe<true><<<grid, 512>>>(d_src, d_out, iters); else probe<false><<<grid, 512>>>(d_src, d_out, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("rep %d %-10s %8.3f ms  %7.1f TFLOP/s\n", rep, big ? "32x32x16" : "16x16x32", ms, flop / ms / 1e9);
    }
  }
  CK(hipGetLastError());
  return 0;
}
