// K4: fused rotary embedding + paged KV-cache write.
//
// Input is the fused QKV GEMM output [T, (nq + 2 nkv) * D].  One workgroup per
// token; each lane handles 8 rotary pairs (element i and i + D/2, the Llama
// "rotate_half" convention) with 16-B loads/stores.  Q is rotated in place (the
// attention kernels read it with the QKV row stride, so there is no extra copy),
// K is rotated and written straight into the paged cache, V is copied into the
// paged cache.  The cos/sin table is precomputed on the host (llama3 rope
// scaling included) as fp32 [max_pos, D] = [cos(D/2) | sin(D/2)], so the kernel
// does no transcendental math (Appendix B "Element-wise": trig tables on host).
//
// Cache layouts: K [num_blocks, n_kv_heads, block_size, D] (token rows) and V
// [num_blocks, n_kv_heads, D, block_size] (TRANSPOSED: dim rows), so one (block,
// head) tile of either is a contiguous block_size*D*2-byte run and both MFMA
// operands of the attention kernels load straight from it: K rows are the A
// operand of QK^T, V^T rows (consecutive tokens of one dim) the B operand of PV.
#include "ft_common.h"

namespace ft {

// KV8: fp8 (e4m3) caches, same layouts with 1-byte elements (ft_common.h fp8x*)
template <int D, bool KV8>
__global__ __launch_bounds__(256) void rope_kv_kernel(uint16_t* __restrict__ qkv, int qkv_stride,
                                                      const int* __restrict__ positions,
                                                      const float* __restrict__ cos_sin,
                                                      const int* __restrict__ slot_mapping,
                                                      void* __restrict__ k_cache,
                                                      void* __restrict__ v_cache, int nq,
                                                      int nkv, int block_size, int cos_rows,
                                                      int num_slots) {
  constexpr int HALF = D / 2;
  constexpr int CPH = HALF / 8;  // 8-pair chunks per head
  const int t = blockIdx.x;
  const int pos = FT_CHECK_IDX(positions[t], cos_rows, kCkPosition, t);
  int slot = slot_mapping[t];
  if (slot >= 0) slot = FT_CHECK_IDX(slot, num_slots, kCkSlot, t);
  uint16_t* row = qkv + (size_t)t * qkv_stride;
  const float* cs = cos_sin + (size_t)pos * D;

  const int n_rot = (nq + nkv) * CPH;
  for (int item = threadIdx.x; item < n_rot; item += blockDim.x) {
    const int head = item / CPH;
    const int c = item - head * CPH;
    uint16_t* hp = row + head * D;  // q heads then k heads are contiguous
    uint4* p1 = reinterpret_cast<uint4*>(hp + c * 8);
    uint4* p2 = reinterpret_cast<uint4*>(hp + HALF + c * 8);
    float x1[8], x2[8], co[8], si[8];
    load8(*p1, x1);
    load8(*p2, x2);
    const float4* c4 = reinterpret_cast<const float4*>(cs + c * 8);
    const float4* s4 = reinterpret_cast<const float4*>(cs + HALF + c * 8);
    float4 ca = c4[0], cb = c4[1], sa = s4[0], sb = s4[1];
    co[0] = ca.x; co[1] = ca.y; co[2] = ca.z; co[3] = ca.w;
    co[4] = cb.x; co[5] = cb.y; co[6] = cb.z; co[7] = cb.w;
    si[0] = sa.x; si[1] = sa.y; si[2] = sa.z; si[3] = sa.w;
    si[4] = sb.x; si[5] = sb.y; si[6] = sb.z; si[7] = sb.w;
    float y1[8], y2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      y1[j] = x1[j] * co[j] - x2[j] * si[j];
      y2[j] = x2[j] * co[j] + x1[j] * si[j];
    }
    const uint4 o1 = store8(y1), o2 = store8(y2);
    if (head < nq) {
      *p1 = o1;
      *p2 = o2;
    } else if (slot >= 0) {
      const int kh = head - nq;
      const int blk = slot / block_size, off = slot - blk * block_size;
      const size_t e = (((size_t)blk * nkv + kh) * block_size + off) * D;
      if constexpr (KV8) {
        uint8_t* kp = reinterpret_cast<uint8_t*>(k_cache) + e;
        reinterpret_cast<uint2*>(kp + c * 8)[0] = fp8x8_pack(y1);
        reinterpret_cast<uint2*>(kp + HALF + c * 8)[0] = fp8x8_pack(y2);
      } else {
        uint16_t* kp = reinterpret_cast<uint16_t*>(k_cache) + e;
        reinterpret_cast<uint4*>(kp + c * 8)[0] = o1;
        reinterpret_cast<uint4*>(kp + HALF + c * 8)[0] = o2;
      }
    }
  }
  if (slot >= 0) {
    const int blk = slot / block_size, off = slot - blk * block_size;
    const int nv = nkv * (D / 8);
    const uint4* vsrc = reinterpret_cast<const uint4*>(row + (nq + nkv) * D);
    for (int item = threadIdx.x; item < nv; item += blockDim.x) {
      const int kh = item / (D / 8), c = item - kh * (D / 8);
      // V blocks are transposed ([D][block_size]): dims c*8.. of this token
      const size_t e = (((size_t)blk * nkv + kh) * D + c * 8) * block_size + off;
      const uint4 v = vsrc[item];
      if constexpr (KV8) {
        float f[8];
        load8(v, f);
        const uint2 q8 = fp8x8_pack(f);
        uint8_t* vp = reinterpret_cast<uint8_t*>(v_cache) + e;
#pragma unroll
        for (int j = 0; j < 8; ++j) vp[j * block_size] = (uint8_t)(((j < 4 ? q8.x : q8.y) >> (8 * (j & 3))) & 0xffu);
      } else {
        uint16_t* vp = reinterpret_cast<uint16_t*>(v_cache) + e;
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          vp[(2 * j) * block_size] = (uint16_t)(w[j] & 0xffffu);
          vp[(2 * j + 1) * block_size] = (uint16_t)(w[j] >> 16);
        }
      }
    }
  }
}

}  // namespace ft

extern "C" int ft_rope_kv_write(void* qkv, int qkv_stride, const int* positions,
                                const float* cos_sin, const int* slot_mapping, void* k_cache,
                                void* v_cache, int tokens, int nq, int nkv, int head_dim,
                                int block_size, int cos_rows, int num_slots, int kv8,
                                hipStream_t stream) {
  if (tokens <= 0) return 0;
  dim3 grid(tokens), block(256);
#define FT_ROPE(DD, K8)                                                                     \
  hipLaunchKernelGGL((ft::rope_kv_kernel<DD, K8>), grid, block, 0, stream, (uint16_t*)qkv,  \
                     qkv_stride, positions, cos_sin, slot_mapping, k_cache, v_cache, nq, nkv, \
                     block_size, cos_rows, num_slots)
  if (head_dim == 128) {
    if (kv8) FT_ROPE(128, true); else FT_ROPE(128, false);
  } else if (head_dim == 64) {
    if (kv8) FT_ROPE(64, true); else FT_ROPE(64, false);
  } else {
    return -1;
  }
#undef FT_ROPE
  return static_cast<int>(hipGetLastError());
}

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(rope_kv)
