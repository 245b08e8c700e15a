// Streaming-read ceiling probe (diagnostic, not part of the package): how fast
// can a plain kernel read N bytes of cold HBM at the decode-GEMM / KV sizes?
// Each thread keeps U 16-B non-temporal loads in flight per iteration over a
// grid-stride loop and folds them into one value (stored once, vector store).
// Built by bench/bw_read.py with hipcc into bench/libbwk.so, called via ctypes.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void stream_read(const u32x4* __restrict__ p, size_t n16,
                                                   unsigned* __restrict__ out) {
  const size_t stride = (size_t)gridDim.x * 256;
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  unsigned acc = 0;
  for (; i + (U - 1) * stride < n16; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < n16; i += stride) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[(size_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// Contiguous-chunk variant: block b reads its own contiguous [b*chunk, (b+1)*chunk)
// range (like a GEMM workgroup streaming its weight tiles), U loads in flight.
template <int U>
__global__ __launch_bounds__(256) void chunk_read(const u32x4* __restrict__ p, size_t n16,
                                                  unsigned* __restrict__ out) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x;
  const size_t beg = (size_t)blockIdx.x * per;
  const size_t end = beg + per < n16 ? beg + per : n16;
  unsigned acc = 0;
  size_t i = beg + threadIdx.x;
  for (; i + (U - 1) * 256 < end; i += U * 256) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(p + i + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i < end; i += 256) {
    u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[(size_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

extern "C" int bw_read(const void* p, size_t nbytes, void* out, int blocks, int unroll, int mode,
                       hipStream_t stream) {
  const size_t n16 = nbytes / 16;
#define L(K, UU)                                                                              \
  if (unroll == UU) {                                                                         \
    hipLaunchKernelGGL((K<UU>), dim3(blocks), dim3(256), 0, stream, (const u32x4*)p, n16,     \
                       (unsigned*)out);                                                       \
    return (int)hipGetLastError();                                                            \
  }
  if (mode == 0) {
    L(stream_read, 1) L(stream_read, 2) L(stream_read, 4) L(stream_read, 8) L(stream_read, 16)
  } else {
    L(chunk_read, 1) L(chunk_read, 2) L(chunk_read, 4) L(chunk_read, 8) L(chunk_read, 16)
  }
#undef L
  return -1;
}
