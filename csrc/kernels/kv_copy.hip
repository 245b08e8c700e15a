// K13: batched KV block copy (copy-on-write of a shared prefix block, and the
// device half of host swap-in).  One workgroup row per (src, dst) pair, 16-B
// lane copies of both K and V caches; pairs are int32 [n, 2] on the device so
// the copy list never needs a host sync.
#include "ft_common.h"

namespace ft {

__global__ __launch_bounds__(256) void kv_block_copy_kernel(uint4* __restrict__ k_cache,
                                                            uint4* __restrict__ v_cache,
                                                            const int* __restrict__ pairs,
                                                            long vec_per_block) {
  const int p = blockIdx.y;
  const long src = pairs[2 * p], dst = pairs[2 * p + 1];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < vec_per_block; i += gridDim.x * 256L) {
    k_cache[dst * vec_per_block + i] = k_cache[src * vec_per_block + i];
    v_cache[dst * vec_per_block + i] = v_cache[src * vec_per_block + i];
  }
}

}  // namespace ft

extern "C" int ft_kv_block_copy(void* k_cache, void* v_cache, const int* src_dst, int num_pairs,
                                long block_elems, hipStream_t stream) {
  if (num_pairs <= 0) return 0;
  const long vec = block_elems / 8;
  int gx = (int)((vec + 255) / 256);
  if (gx > 64) gx = 64;
  hipLaunchKernelGGL(ft::kv_block_copy_kernel, dim3(gx, num_pairs), dim3(256), 0, stream,
                     (uint4*)k_cache, (uint4*)v_cache, src_dst, vec);
  return static_cast<int>(hipGetLastError());
}
