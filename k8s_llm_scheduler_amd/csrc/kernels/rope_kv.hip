// K4 + K5: rotary embedding (llama3-scaled table precomputed on the host) fused with the
// paged KV-cache write.  Input is the QKV projection output
// [T, (nq + 2*nkv) * D]; q is rotated into q_out [T, nq, D]; k is rotated and v copied into the
// paged caches [num_slots, nkv, D] at the token's slot (slot = block * block_size + offset).
//
// Two addressing modes:
//   prefill: positions[T], slot_mapping[T] given (slot < 0 -> token's KV is not stored)
//   decode : context_lens[T] and block_tables[T, max_blocks] given; the token is the last one of
//            its sequence: pos = ctx - 1, slot from the block table.  This keeps a decode step
//            free of host-computed metadata so it can be replayed from a hipGraph.
// Rotation is "rotate-half" (HF Llama): x' = x*cos + rotate_half(x)*sin, pairs (i, i + D/2).
#include "common.h"

#define K8S_CHK_THIS_UNIT 2

namespace k8sllm {

__global__ void __launch_bounds__(256) rope_kv_kernel(
    bf16_t* __restrict__ q_out, bf16_t* __restrict__ k_cache, bf16_t* __restrict__ v_cache,
    const bf16_t* __restrict__ qkv, const float* __restrict__ cos_sin, const int* __restrict__ positions,
    const int* __restrict__ slot_mapping, const int* __restrict__ context_lens, const int* __restrict__ block_tables,
    int max_blocks, int block_size, int nq, int nkv, int D) {
  const int t = blockIdx.x;
  int pos, slot;
  if (positions != nullptr) {
    pos = positions[t];
    slot = slot_mapping[t];
    if (slot >= 0) K8S_CHECK_RANGE(slot, 0, K8S_CHK_SLOT, -1);   // (checked builds: a bad slot is not written)
  } else {
    int ctx = context_lens[t];
    if (ctx <= 0) return;  // padded batch row
    K8S_CHECK_MAX(ctx, max_blocks * block_size, K8S_CHK_CTX);
    pos = ctx - 1;
    int blk = block_tables[(size_t)t * max_blocks + pos / block_size];
    K8S_CHECK_RANGE(blk, 0, K8S_CHK_BLOCK, 0);
    slot = blk * block_size + pos % block_size;
  }
  const int half = D >> 1;
  const int q4 = half >> 2;  // groups of 4 pairs per head
  const bf16_t* src = qkv + (size_t)t * (nq + 2 * nkv) * D;
  const float* cs = cos_sin + (size_t)pos * D;
  const int n_rot = (nq + nkv) * q4;
  for (int it = threadIdx.x; it < n_rot; it += blockDim.x) {
    const int h = it / q4, g = it - h * q4;
    const int i0 = g * 4;
    const bf16_t* xh = src + (size_t)h * D;
    const uint2 a = *reinterpret_cast<const uint2*>(xh + i0);
    const uint2 b = *reinterpret_cast<const uint2*>(xh + i0 + half);
    const float4 c = *reinterpret_cast<const float4*>(cs + i0);
    const float4 s = *reinterpret_cast<const float4*>(cs + half + i0);
    float x1[4] = {lo_bf(a.x), hi_bf(a.x), lo_bf(a.y), hi_bf(a.y)};
    float x2[4] = {lo_bf(b.x), hi_bf(b.x), lo_bf(b.y), hi_bf(b.y)};
    float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {s.x, s.y, s.z, s.w};
    float y1[4], y2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      y1[j] = x1[j] * cc[j] - x2[j] * ss[j];
      y2[j] = x2[j] * cc[j] + x1[j] * ss[j];
    }
    const uint2 o1 = make_uint2(pack_bf2(y1[0], y1[1]), pack_bf2(y1[2], y1[3]));
    const uint2 o2 = make_uint2(pack_bf2(y2[0], y2[1]), pack_bf2(y2[2], y2[3]));
    bf16_t* dst;
    if (h < nq) {
      dst = q_out + ((size_t)t * nq + h) * D;
    } else {
      if (slot < 0) continue;
      dst = k_cache + ((size_t)slot * nkv + (h - nq)) * D;
    }
    *reinterpret_cast<uint2*>(dst + i0) = o1;
    *reinterpret_cast<uint2*>(dst + i0 + half) = o2;
  }
  if (slot < 0) return;
  // v: plain 16-byte copies
  const int v8 = D >> 3;
  const u32x4* vs = reinterpret_cast<const u32x4*>(src + (size_t)(nq + nkv) * D);
  u32x4* vd = reinterpret_cast<u32x4*>(v_cache + (size_t)slot * nkv * D);
  for (int it = threadIdx.x; it < nkv * v8; it += blockDim.x) vd[it] = vs[it];
}

}  // namespace k8sllm

using namespace k8sllm;

K8S_CHECK_UNIT(rope_kv)

extern "C" int k8s_rope_kv_write(void* q_out, void* k_cache, void* v_cache, const void* qkv, const float* cos_sin,
                                 const int* positions, const int* slot_mapping, const int* context_lens,
                                 const int* block_tables, int max_blocks, int block_size, int T, int nq, int nkv,
                                 int D, hipStream_t stream) {
  if (T <= 0) return 0;
  if (D % 8 != 0) return -1;
  if (positions == nullptr && (context_lens == nullptr || block_tables == nullptr)) return -2;
  rope_kv_kernel<<<T, 256, 0, stream>>>((bf16_t*)q_out, (bf16_t*)k_cache, (bf16_t*)v_cache, (const bf16_t*)qkv,
                                        cos_sin, positions, slot_mapping, context_lens, block_tables, max_blocks,
                                        block_size, nq, nkv, D);
  return (int)hipGetLastError();
}
