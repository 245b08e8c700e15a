// Shared device helpers for the FastTalk MI355X (gfx950 / CDNA4) kernels.
//
// Conventions used by every kernel in csrc/kernels:
//   * wave64: lane = threadIdx.x & 63, block sizes are multiples of 64.
//   * bf16 tensors are moved 16 B per lane (8 elements, `uint4`) and widened to
//     fp32 with a shift (bf16 is the top half of an fp32), accumulation is fp32.
//   * every launcher takes the hipStream_t of the caller so the launch can be
//     captured into a hipGraph (no allocation / sync inside launchers).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ft {

constexpr int kWave = 64;

using bf16_raw = uint16_t;

__device__ __forceinline__ float bf16_to_f32(uint16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

// round-to-nearest-even fp32 -> bf16 (NaN stays NaN): a plain cast, which hipcc
// lowers to the hardware v_cvt_pk_bf16_f32 (one VALU op for two values) -- the
// integer-rounding form this replaces cost ~6 VALU ops per value in every epilogue
// and in the attention kernels' P conversion (guide: MI355X_MICROARCH.md,
// Correctness boundaries, f32 -> bf16 row)
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  return __builtin_bit_cast(uint16_t, static_cast<__bf16>(f));
}

typedef __bf16 ft_bf16x2_t __attribute__((ext_vector_type(2)));

// unpack a 32-bit word holding two bf16 (low element first)
__device__ __forceinline__ void unpack2(uint32_t w, float& lo, float& hi) {
  lo = __uint_as_float(w << 16);
  hi = __uint_as_float(w & 0xffff0000u);
}

__device__ __forceinline__ uint32_t pack2(float lo, float hi) {
  const ft_bf16x2_t v = {static_cast<__bf16>(lo), static_cast<__bf16>(hi)};
  return __builtin_bit_cast(uint32_t, v);
}

// 8 x bf16 <-> 8 x fp32
__device__ __forceinline__ void load8(const uint4& v, float (&f)[8]) {
  unpack2(v.x, f[0], f[1]);
  unpack2(v.y, f[2], f[3]);
  unpack2(v.z, f[4], f[5]);
  unpack2(v.w, f[6], f[7]);
}

__device__ __forceinline__ uint4 store8(const float (&f)[8]) {
  uint4 v;
  v.x = pack2(f[0], f[1]);
  v.y = pack2(f[2], f[3]);
  v.z = pack2(f[4], f[5]);
  v.w = pack2(f[6], f[7]);
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// reduce within aligned groups of `W` lanes (W power of two <= 64)
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int W>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int o = W / 2; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// reduce over the 4 lanes {l, l^16, l^32, l^48} (the k groups of an MFMA 16x16
// C-layout column): gfx950 VALU lane swaps -- v_permlane16_swap exchanges the odd
// rows of one copy with the even rows of the other (the xor-16 partners),
// v_permlane32_swap the wave halves (xor 32) -- instead of ds_bpermute round trips,
// which put two waited LDS latencies on an attention tile's critical path
__device__ __forceinline__ float kgroups_max(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const unsigned v = __float_as_uint(x);
  const auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

__device__ __forceinline__ float kgroups_sum(float x) {
  const unsigned u = __float_as_uint(x);
  const auto r16 = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  x = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
  const unsigned v = __float_as_uint(x);
  const auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

inline int ceil_div(int a, int b) { return (a + b - 1) / b; }

}  // namespace ft

#define FT_HIP_CHECK(expr)                                                   \
  do {                                                                       \
    hipError_t _e = (expr);                                                  \
    if (_e != hipSuccess) return static_cast<int>(_e);                       \
  } while (0)
