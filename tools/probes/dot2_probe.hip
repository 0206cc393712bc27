// Probe: semantics of __builtin_amdgcn_fdot2_f32_bf16 on gfx950 vs explicit fp32 FMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
__global__ void k(const uint32_t* a, const uint32_t* b, float* out) {
  int i = threadIdx.x;
  out[i * 2] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2, a[i]), __builtin_bit_cast(bf16x2, b[i]), 0.5f, false);
  float al = __uint_as_float(a[i] << 16), ah = __uint_as_float(a[i] & 0xffff0000u);
  float bl = __uint_as_float(b[i] << 16), bh = __uint_as_float(b[i] & 0xffff0000u);
  out[i * 2 + 1] = al * bl + ah * bh + 0.5f;
}
static uint16_t bf(float f) { uint32_t u; memcpy(&u, &f, 4); return u >> 16; }
int main() {
  const int n = 8;
  uint32_t ha[n], hb[n];
  float vals[] = {1.f, 2.f, -3.f, 0.25f, 1.5f, -7.f, 100.f, 0.125f};
  for (int i = 0; i < n; ++i) { ha[i] = bf(vals[i]) | (bf(vals[(i + 1) % n]) << 16); hb[i] = bf(vals[(i + 3) % n]) | (bf(2.f) << 16); }
  uint32_t *da, *db; float* dout;
  hipMalloc(&da, sizeof ha); hipMalloc(&db, sizeof hb); hipMalloc(&dout, 2 * n * sizeof(float));
  hipMemcpy(da, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(db, hb, sizeof hb, hipMemcpyHostToDevice);
  k<<<1, n>>>(da, db, dout);
  float ho[2 * n]; hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n; ++i) { printf("dot2=%g fma=%g\n", ho[2 * i], ho[2 * i + 1]); bad += ho[2*i] != ho[2*i+1]; }
  printf(bad ? "DOT2_MISMATCH\n" : "DOT2_OK\n");
  return 0;
}
