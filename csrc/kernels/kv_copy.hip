// K13: batched KV block copy (copy-on-write of a shared prefix block, and the
// device half of host swap-in).  One workgroup row per (src, dst) pair, 16-B
// lane copies of both K and V caches; pairs are int32 [n, 2] on the device so
// the copy list never needs a host sync.
#include "ft_common.h"

namespace ft {

__global__ __launch_bounds__(256) void kv_block_copy_kernel(uint4* __restrict__ k_cache,
                                                            uint4* __restrict__ v_cache,
                                                            const int* __restrict__ pairs,
                                                            long vec_per_block, int num_blocks) {
  const int p = blockIdx.y;
  const long src = FT_CHECK_IDX(pairs[2 * p], num_blocks, kCkCopyBlock, p);
  const long dst = FT_CHECK_IDX(pairs[2 * p + 1], num_blocks, kCkCopyBlock, p);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < vec_per_block; i += gridDim.x * 256L) {
    k_cache[dst * vec_per_block + i] = k_cache[src * vec_per_block + i];
    v_cache[dst * vec_per_block + i] = v_cache[src * vec_per_block + i];
  }
}

}  // namespace ft

extern "C" int ft_kv_block_copy(void* k_cache, void* v_cache, const int* src_dst, int num_pairs,
                                long block_elems, int num_blocks, hipStream_t stream) {
  if (num_pairs <= 0) return 0;
  const long vec = block_elems / 8;
  int gx = (int)((vec + 255) / 256);
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(ft::kv_block_copy_kernel, dim3(gx, num_pairs), dim3(256), 0, stream,
                     (uint4*)k_cache, (uint4*)v_cache, src_dst, vec, num_blocks);
  return static_cast<int>(hipGetLastError());
}

// E6/K13 host swap (vLLM --swap-space): the blocks of a preempted sequence are
// gathered from all 2L layer caches into a contiguous device staging buffer
// [n][2L][block] in ONE launch, so the host side is one DMA per block instead
// of 2L strided copies; swap-in is the reverse scatter.  ptrs: device array of
// the 2L cache base pointers (k0, v0, k1, v1, ...); ids: device int32 [n].
namespace ft {

__global__ __launch_bounds__(256) void kv_swap_kernel(const uint64_t* __restrict__ ptrs,
                                                      const int* __restrict__ ids,
                                                      uint4* __restrict__ staging,
                                                      long vec_per_block, int ncache,
                                                      int to_staging, int num_blocks) {
  const int c = blockIdx.y, p = blockIdx.z;
  uint4* cache = reinterpret_cast<uint4*>(ptrs[c]) +
                 (long)FT_CHECK_IDX(ids[p], num_blocks, kCkCopyBlock, p) * vec_per_block;
  uint4* st = staging + ((long)p * ncache + c) * vec_per_block;
  if (to_staging) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < vec_per_block; i += gridDim.x * 256L)
      st[i] = cache[i];
  } else {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < vec_per_block; i += gridDim.x * 256L)
      cache[i] = st[i];
  }
}

}  // namespace ft

extern "C" int ft_kv_swap(const uint64_t* ptrs_dev, int ncache, const int* ids_dev, int n,
                          void* staging, long block_elems, int to_staging, int num_blocks,
                          hipStream_t stream) {
  if (n <= 0) return 0;
  if (block_elems % 8 != 0 || ncache <= 0 || ncache > 65535 || n > 65535) return -1;
  const long vec = block_elems / 8;
  int gx = (int)((vec + 255) / 256);
  if (gx > 16) gx = 16;
  hipLaunchKernelGGL(ft::kv_swap_kernel, dim3(gx, ncache, n), dim3(256), 0, stream, ptrs_dev,
                     ids_dev, (uint4*)staging, vec, ncache, to_staging, num_blocks);
  return static_cast<int>(hipGetLastError());
}

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(kv_copy)
