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

// fp8 KV cache (OCP e4m3, torch.float8_e4m3fn; ENGINE_KV_CACHE_DTYPE=fp8).  Stored
// value = x at a per-tensor scale of 1 (vLLM's uncalibrated default), clamped to the
// format's +-448 first: gfx950's v_cvt_pk_fp8_f32 turns an out-of-range value into
// NaN, not the max (bench/probes/fp8_cvt_check.py, measured).  Reads widen straight
// to bf16 MFMA operands with v_cvt_scalef32_pk_bf16_fp8 (2 values per op; its scale
// operand is exact for powers of two only -- probe -- so it stays 1).
constexpr float kFp8Max = 448.f;

__device__ __forceinline__ uint32_t fp8x4_pack(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -kFp8Max), kFp8Max);
  b = fminf(fmaxf(b, -kFp8Max), kFp8Max);
  c = fminf(fmaxf(c, -kFp8Max), kFp8Max);
  d = fminf(fmaxf(d, -kFp8Max), kFp8Max);
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  w = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
  return (uint32_t)w;
}

// 8 fp32 -> 8 fp8 (low element first)
__device__ __forceinline__ uint2 fp8x8_pack(const float (&f)[8]) {
  return make_uint2(fp8x4_pack(f[0], f[1], f[2], f[3]), fp8x4_pack(f[4], f[5], f[6], f[7]));
}

// 4 fp8 (one word, low byte first) -> 4 bf16 (two words)
__device__ __forceinline__ uint2 fp8x4_to_bf16(uint32_t w) {
  const ft_bf16x2_t lo = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.f, false);
  const ft_bf16x2_t hi = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.f, true);
  return make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
}

// 8 fp8 -> 8 bf16 (a 16-B MFMA fragment)
__device__ __forceinline__ uint4 fp8x8_to_bf16(uint32_t w0, uint32_t w1) {
  const uint2 a = fp8x4_to_bf16(w0), b = fp8x4_to_bf16(w1);
  return make_uint4(a.x, a.y, b.x, b.y);
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

// ---------------------------------------------------------------------------------
// Checked kernel build (SURVEY §5 "bounds checks in debug builds"): ops/build.py
// --checked compiles every kernel with -DFT_KERNEL_CHECKS=1 into _C_checked.so,
// loaded when FT_KERNEL_CHECKS=1.  Index-taking kernels route block-table entries,
// KV slots, rotary positions and token ids through ft_check_idx: an out-of-range
// value is counted in a device error word (first violation: code + context + value,
// and one printf per wave), then clamped to 0 so the kernel does not fault -- no
// trap; the runner reads the word after every step and fails it loudly
// (engine/runner.py, KernelCheckError).  Each translation unit holds its own copy of
// the word pointer and the limits (kernels are not compiled -fgpu-rdc); the host sets
// them through ft_check_hook_<unit> (FT_CHECK_HOOK at the end of each unit).  In the
// release build all of this compiles to nothing.
// ---------------------------------------------------------------------------------
namespace ft {
enum FtCheckCode : int {
  kCkBlockTable = 1,   // paged attention: block-table entry >= num_blocks
  kCkSlot = 2,         // KV write: slot >= num_blocks * block_size
  kCkPosition = 3,     // RoPE: position >= rows of the cos/sin table
  kCkTokenId = 4,      // embedding: input id >= vocab
  kCkSampled = 5,      // sampler: sampled id >= vocab
  kCkCopyBlock = 6,    // KV copy / swap: block id >= num_blocks
};
}  // namespace ft

#if defined(FT_KERNEL_CHECKS) && FT_KERNEL_CHECKS
namespace ft {
// [0] violations, [1] code of the first, [2] its context (row / token), [3] its value
static __device__ uint32_t* ft_check_word;

__device__ __noinline__ static void ft_check_fail(int code, int ctx, int value) {
  uint32_t* w = ft_check_word;
  if (w == nullptr) return;
  if (atomicAdd(w, 1u) == 0u) {
    w[1] = static_cast<uint32_t>(code);
    w[2] = static_cast<uint32_t>(ctx);
    w[3] = static_cast<uint32_t>(value);
    printf("[ft-check] kernel bounds violation: code %d ctx %d value %d (block %d thread %d)\n",
           code, ctx, value, (int)blockIdx.x, (int)threadIdx.x);
  }
}

// value if 0 <= value < limit (a limit <= 0 is unknown: unchecked), else report and 0
__device__ __forceinline__ int ft_check_idx(int value, long limit, int code, int ctx) {
  if (limit > 0 && (value < 0 || (long)value >= limit)) {
    ft_check_fail(code, ctx, value);
    return 0;
  }
  return value;
}
}  // namespace ft
#define FT_CHECK_IDX(v, lim, code, ctx) ::ft::ft_check_idx((v), (lim), (code), (ctx))
#define FT_CHECK_HOOK(NAME)                                                                  \
  extern "C" int ft_check_hook_##NAME(uint32_t* word) {                                     \
    return static_cast<int>(                                                                \
        hipMemcpyToSymbol(HIP_SYMBOL(::ft::ft_check_word), &word, sizeof(word)));           \
  }
#else
#define FT_CHECK_IDX(v, lim, code, ctx) (v)
#define FT_CHECK_HOOK(NAME)
#endif
