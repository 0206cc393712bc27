// Prints where v_mfma_f32_4x4x4bf16_1k reads A / B and writes D: A = 1 only in lane LA item KA, B = 1 everywhere,
// so D is nonzero exactly in the lanes/items of the block and row that lane LA's A value feeds.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe(float* out, int la, int ka, int lb, int kb) {
  const int l = threadIdx.x;
  bf16x4 a, b;
  for (int e = 0; e < 4; ++e) {
    a[e] = (__bf16)((l == la && e == ka) ? 1.f : 0.f);
    b[e] = (__bf16)((lb < 0 || (l == lb && e == kb)) ? 1.f : 0.f);
  }
  if (lb >= 0)
    for (int e = 0; e < 4; ++e) a[e] = (__bf16)1.f;   // second mode: A = 1, B one-hot
  f32x4 d = {0.f, 0.f, 0.f, 0.f};
  d = __builtin_amdgcn_mfma_f32_4x4x4bf16_1k(a, b, d, 0, 0, 0);
  for (int e = 0; e < 4; ++e) out[l * 4 + e] = d[e];
}

int main() {
  float* o;
  float h[256];
  (void)hipMalloc(&o, 1024);
  const int cases[][4] = {{0, 0, -1, 0}, {1, 0, -1, 0}, {4, 0, -1, 0}, {16, 0, -1, 0}, {5, 2, -1, 0},
                          {0, 0, 0, 0}, {1, 0, 1, 0}, {4, 0, 4, 0}, {16, 0, 16, 0}, {6, 3, 6, 3}};
  for (auto& c : cases) {
    probe<<<1, 64>>>(o, c[0], c[1], c[2], c[3]);
    (void)hipMemcpy(h, o, 1024, hipMemcpyDeviceToHost);
    printf(c[2] < 0 ? "A one-hot lane %d item %d -> D nonzero at:" : "B one-hot lane %d item %d -> D nonzero at:",
           c[2] < 0 ? c[0] : c[2], c[2] < 0 ? c[1] : c[3]);
    for (int i = 0; i < 256; ++i)
      if (h[i] != 0.f) printf(" (lane %d item %d)", i / 4, i % 4);
    printf("\n");
  }
  return 0;
}
