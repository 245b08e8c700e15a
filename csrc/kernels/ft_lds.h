// LDS-DMA + inline-asm LDS read helpers shared by the MFMA kernels that stage
// operands with global_load_lds_dwordx4 (attn_prefill.hip, packed_gemm.hip).
#pragma once
#include "ft_common.h"

#include <type_traits>

namespace ft {

// LDS reads in inline asm: with LDS-DMA (global_load_lds) in flight hipcc cannot
// tell a ds_read from the DMA's destination and waits vmcnt(0) before every LDS
// read, draining the prefetch.  These reads are invisible to its waitcnt pass, so
// the kernel orders them itself: lgkm_wait<N>() (N reads may stay outstanding)
// followed by dep() on each value it is about to consume.
__device__ __forceinline__ uint32_t lds_off(const void* p) {
  return (uint32_t)reinterpret_cast<uintptr_t>(p);
}
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ds_read16(uint32_t a) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return __builtin_bit_cast(uint4, v);
}
__device__ __forceinline__ uint2 ds_read8(uint32_t a) {
  u32x2_t v;
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
  return __builtin_bit_cast(uint2, v);
}
// LDS store in inline asm, ordered with the asm reads above ("memory": the compiler
// keeps it between the surrounding waits and barriers)
__device__ __forceinline__ void ds_write16(uint32_t a, const uint4& v) {
  const u32x4_t w = __builtin_bit_cast(u32x4_t, v);
  asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(w) : "memory");
}
// the same with a compile-time immediate offset (the ds_read offset field, 0..65535):
// per-lane base addresses computed once, per-fragment displacements as immediates
template <int OFF>
__device__ __forceinline__ uint4 ds_read16o(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds_read offset field");
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return __builtin_bit_cast(uint4, v);
}
template <int OFF>
__device__ __forceinline__ uint2 ds_read8o(uint32_t a) {
  static_assert(OFF >= 0 && OFF < 65536, "ds_read offset field");
  u32x2_t v;
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return __builtin_bit_cast(uint2, v);
}
// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// global_load_lds_dwordx4 in inline asm (guide idiom): M0 = the wave-uniform LDS
// destination, lanes land at M0 + 16 * lane.  hipcc's waitcnt pass does not see it
// (it would otherwise treat the address VGPRs as pending and wait vmcnt(0) at their
// reuse); the kernel waits for it with explicit counted vmcnt.
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

// the same with the non-temporal policy (streamed-once data: decode K/V)
__device__ __forceinline__ void glds16nt(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds_dst))
      : "memory");
}

template <int N>
__device__ __forceinline__ void lgkm_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void dep(uint4& v) {
  u32x4_t t = __builtin_bit_cast(u32x4_t, v);
  asm volatile("" : "+v"(t));
  v = __builtin_bit_cast(uint4, t);
}
__device__ __forceinline__ void dep(uint2& v) {
  u32x2_t t = __builtin_bit_cast(u32x2_t, v);
  asm volatile("" : "+v"(t));
  v = __builtin_bit_cast(uint2, t);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

}  // namespace ft
