// Scale-operand mapping of v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3), measured instead of assumed: which
// lane's scale byte applies to which (lane, byte) of the A / B operand registers, and which output element a B byte
// lands in.  Trial p (0..2047) puts 1.0 at byte p % 32 of lane p / 32 of one operand (all other bytes 0; the other
// operand all 1.0) and gives lane L the scale 2^(L - 32) (E8M0 byte 95 + L, the other operand unit scales), so every
// non-zero output is 2^(Ls - 32) where Ls is the lane whose scale applied.  Prints, per operand, whether every byte
// of lane L took lane L's scale, and the output column (token) of each B lane.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/mx_scale_probe tools/experiments/mx_scale_probe.hip && /tmp/mx_scale_probe
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void __launch_bounds__(64) probe(float* __restrict__ out) {
  const int lane = threadIdx.x, p = blockIdx.x & 2047, side = blockIdx.x >> 11;   // side 0: B one-hot, 1: A
  const int hot_lane = p / 32, hot_byte = p % 32;
  int ones[8], hot[8];
  for (int r = 0; r < 8; ++r) {
    ones[r] = 0x38383838;   // four e4m3 1.0
    hot[r] = 0;
  }
  if (lane == hot_lane) hot[hot_byte / 4] = 0x38 << (8 * (hot_byte % 4));
  const i32x8 one_v = {ones[0], ones[1], ones[2], ones[3], ones[4], ones[5], ones[6], ones[7]};
  const i32x8 hot_v = {hot[0], hot[1], hot[2], hot[3], hot[4], hot[5], hot[6], hot[7]};
  const int e = 95 + lane;
  const int sc = e | (e << 8) | (e << 16) | (e << 24);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (side == 0)
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(one_v, hot_v, acc, 0, 0, 0, 0x7f7f7f7f, 0, sc);
  else
    acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(hot_v, one_v, acc, 0, 0, 0, sc, 0, 0x7f7f7f7f);
  for (int r = 0; r < 4; ++r) out[(size_t)blockIdx.x * 256 + (4 * (lane >> 4) + r) * 16 + (lane & 15)] = acc[r];
}

int main() {
  float* d;
  hipMalloc(&d, 4096 * 256 * sizeof(float));
  hipLaunchKernelGGL(probe, dim3(4096), dim3(64), 0, 0, d);
  std::vector<float> h(4096 * 256);
  hipMemcpy(h.data(), d, h.size() * sizeof(float), hipMemcpyDeviceToHost);
  for (int side = 0; side < 2; ++side) {
    int own = 0, other = 0, bad = 0;
    int col_of_lane[64];
    for (int i = 0; i < 64; ++i) col_of_lane[i] = -1;
    for (int p = 0; p < 2048; ++p) {
      const float* o = &h[(size_t)(side * 2048 + p) * 256];
      int nz = 0, ls = -1, col = -1, row = -1;
      for (int i = 0; i < 256; ++i)
        if (o[i] != 0.f) {
          ++nz;
          ls = (int)std::lround(std::log2(o[i])) + 32;
          row = i / 16;
          col = i % 16;
        }
      if (nz != 16) {
        ++bad;
        if (bad < 5) printf("side %d p %d: %d non-zero outputs\n", side, p, nz);
        continue;
      }
      if (ls == p / 32) ++own;
      else {
        ++other;
        if (other < 9) printf("side %s lane %d byte %d took lane %d's scale\n", side ? "A" : "B", p / 32, p % 32, ls);
      }
      if (side == 0) col_of_lane[p / 32] = col;
      (void)row;
    }
    // the layout the kernels assume: bytes 0-15 of lane (li, g) are k = 16 g.., bytes 16-31 k = 64 + 16 g.., and
    // block b = k / 32 of row li takes lane li + 16 b's scale
    int match = 0;
    for (int p = 0; p < 2048; ++p) {
      const float* o = &h[(size_t)(side * 2048 + p) * 256];
      const int L = p / 32, j = p % 32, g = L / 16, li = L % 16;
      const int k = (j < 16 ? 16 * g + j : 64 + 16 * g + (j - 16));
      int ls = -1;
      for (int i = 0; i < 256; ++i)
        if (o[i] != 0.f) ls = (int)std::lround(std::log2(o[i])) + 32;
      match += ls == li + 16 * (k / 32);
    }
    printf("%s operand: %d of 2048 bytes follow the assumed k layout / scale lanes\n", side ? "A" : "B", match);
    printf("%s operand: %d bytes took their own lane's scale, %d another lane's, %d trials malformed\n",
           side ? "A" : "B", own, other, bad);
    if (side == 0) {
      printf("B lane -> output column:");
      for (int i = 0; i < 64; ++i) printf(" %d", col_of_lane[i]);
      printf("\n");
    }
  }
  hipFree(d);
  return 0;
}
