// Issue rate of v_mfma_scale_f32_16x16x128_f8f6f4 with unit (inline-constant) scales vs block scales held in a
// VGPR: one wave per SIMD (one 256-thread workgroup per CU, every CU), 8 independent accumulators, ITERS rounds;
// reports TFLOP/s over the whole chip for each form.  Question: does pgemm's MX mode lose its ~10 % to the MFMA itself
// (a register scale operand) or to the staging around it?
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/experiments/mx_mfma_rate_probe.bin tools/experiments/mx_mfma_rate_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int MODE>   // 0: constant unit scales, 1: VGPR scales (same value for all), 2: VGPR scales, op_sel varied
__global__ void __launch_bounds__(256) rate(float* out, int iters, int seed) {
  const int lane = threadIdx.x & 63;
  i32x8 a, b;
  for (int r = 0; r < 8; ++r) {
    a[r] = 0x38383838 ^ (lane * 7 + r + seed);
    b[r] = 0x30303030 ^ (lane * 5 + r);
  }
  int sc = 0x7f7f7f7f ^ ((lane & 1) * seed);   // seed = 0 at run time: unit scales, but not a constant
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (MODE == 0)
        acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, 0x7f7f7f7f, 0, 0x7f7f7f7f);
      else if constexpr (MODE == 1)
        acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, 0x7f7f7f7f, 0, sc);
      else if (j % 2 == 0)
        acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, 0x7f7f7f7f, 0, sc);
      else
        acc[j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc[j], 0, 0, 0, 0x7f7f7f7f, 1, sc);
    }
  }
  float s = 0.f;
  for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int n_cu = 0;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  float* d;
  (void)hipMalloc(&d, (size_t)n_cu * 256 * sizeof(float));
  const int iters = 20000;
  const char* names[3] = {"constant unit scales", "VGPR scales", "VGPR scales, op_sel varied"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t t0, t1;
      (void)hipEventCreate(&t0);
      (void)hipEventCreate(&t1);
      (void)hipEventRecord(t0);
      if (mode == 0) hipLaunchKernelGGL(rate<0>, dim3(n_cu), dim3(256), 0, 0, d, iters, 0);
      if (mode == 1) hipLaunchKernelGGL(rate<1>, dim3(n_cu), dim3(256), 0, 0, d, iters, 0);
      if (mode == 2) hipLaunchKernelGGL(rate<2>, dim3(n_cu), dim3(256), 0, 0, d, iters, 0);
      (void)hipEventRecord(t1);
      (void)hipEventSynchronize(t1);
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, t0, t1);
      const double flop = 2.0 * 16 * 16 * 128 * 8.0 * iters * 4.0 * n_cu;   // 4 waves per CU
      if (rep) printf("%-30s %8.3f ms  %7.1f TFLOP/s\n", names[mode], ms, flop / (ms * 1e-3) / 1e12);
    }
  }
  (void)hipFree(d);
  return 0;
}
