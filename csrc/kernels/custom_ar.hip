// X1/X2: one-shot all-reduce over xGMI peer mappings for the
// decode-size activations of tensor parallelism ([tokens, hidden] bf16, a few
// hundred KiB to a few MiB).
//
// Why not only RCCL: a ring all-reduce crosses one xGMI link per step and pays
// 2(W-1) latency-bound hops; at decode sizes the step is latency, not bandwidth.
// One-shot: every rank publishes its input in an IPC-shared buffer, then every
// rank reads all W inputs directly over its 7 xGMI links at once and sums them.
//
// Protocol (one kernel, graph-safe: no host-side argument changes between replays):
//   * each rank owns one uncached (hipDeviceMallocUncached) region
//       [epoch u32 | error u32 | arrived u32 | signal[8] u32 | staging[2][max_bytes]]
//     mapped into every peer with hipIpcOpenMemHandle;
//   * every block reads the epoch (= counter + 1), copies its slice of x into
//     my staging[epoch & 1] and counts itself in `arrived`;
//   * block 0 waits for all blocks of this rank (grid <= 128 blocks, always
//     co-resident), resets `arrived`, bumps the counter for the next call and
//     stores `epoch` into signal[my_rank] of every rank (system-scope release);
//   * every block waits until all ranks' signals in MY region reach `epoch`
//     (system-scope acquire, bounded spin), then sums the W staging slots.
//   Staging is double buffered by epoch parity: a rank can be at most one call
//   ahead of the slowest peer (it must see that peer's signal for the current
//   call first), so the slot it overwrites was consumed two calls ago.
//   * a wait beyond the spin budget sets the error word instead of hanging the
//     GPU; the host checks it and falls back to RCCL.
#include "ft_common.h"

namespace ft {

struct ArLayout {
  static constexpr size_t kCounter = 0;     // u32 epoch counter (this rank)
  static constexpr size_t kError = 4;       // u32 error flag
  static constexpr size_t kArrived = 8;     // u32 blocks of this rank done with staging
  static constexpr size_t kSignal = 64;     // u32 signal[8] (written by all ranks)
  static constexpr size_t kStaging = 4096;  // staging[2][max_bytes]
};

__device__ __forceinline__ uint32_t* ar_u32(uint8_t* base, size_t off) {
  return reinterpret_cast<uint32_t*>(base + off);
}

__device__ __forceinline__ bool ar_wait_ge(uint32_t* p, uint32_t target, uint32_t budget,
                                           int scope_system) {
  uint32_t spins = 0;
  while ((scope_system ? __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)
                       : __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) < target) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > budget) return false;
  }
  return true;
}

template <int W>
__global__ __launch_bounds__(256) void ar_oneshot_kernel(uint16_t* __restrict__ out,
                                                         const uint16_t* __restrict__ x,
                                                         const uint64_t* __restrict__ peers,
                                                         int rank, size_t max_bytes, int n8,
                                                         uint32_t spin_budget) {
  uint8_t* mine = reinterpret_cast<uint8_t*>(peers[rank]);
  __shared__ uint32_t s_epoch;
  __shared__ int s_ok;
  if (threadIdx.x == 0)
    s_epoch = __hip_atomic_load(ar_u32(mine, ArLayout::kCounter), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const uint32_t epoch = s_epoch;
  const size_t slot = ArLayout::kStaging + (epoch & 1) * max_bytes;

  // 1. publish my slice
  uint4* stage = reinterpret_cast<uint4*>(mine + slot);
  const uint4* src = reinterpret_cast<const uint4*>(x);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x)
    stage[i] = src[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ar_u32(mine, ArLayout::kArrived), 1u, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    if (blockIdx.x == 0) {
      // 2. all of this rank's blocks published: bump the counter, signal everyone
      ok = ar_wait_ge(ar_u32(mine, ArLayout::kArrived), gridDim.x, spin_budget, 0);
      __hip_atomic_store(ar_u32(mine, ArLayout::kArrived), 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ar_u32(mine, ArLayout::kCounter), epoch, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      for (int r = 0; r < W; ++r) {
        uint8_t* peer = reinterpret_cast<uint8_t*>(peers[r]);
        __hip_atomic_store(ar_u32(peer, ArLayout::kSignal) + rank, epoch, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    // 3. wait until every rank has published this call's slice
    uint32_t* sig = ar_u32(mine, ArLayout::kSignal);
    for (int r = 0; r < W && ok; ++r) ok = ar_wait_ge(sig + r, epoch, spin_budget, 1);
    if (!ok)
      __hip_atomic_store(ar_u32(mine, ArLayout::kError), 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    s_ok = ok;
  }
  __syncthreads();
  if (!s_ok) return;

  // 4. sum the W published slices (read once each, straight from every peer's HBM)
  const uint4* in[W];
#pragma unroll
  for (int r = 0; r < W; ++r)
    in[r] = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(peers[r]) + slot);
  uint4* dst = reinterpret_cast<uint4*>(out);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    float acc[8];
    load8(in[0][i], acc);
#pragma unroll
    for (int r = 1; r < W; ++r) {
      float v[8];
      load8(in[r][i], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    dst[i] = store8(acc);
  }
}

}  // namespace ft

extern "C" size_t ft_ar_header_bytes() { return ft::ArLayout::kStaging; }

extern "C" int ft_ar_alloc(size_t bytes, void** ptr) {
  FT_HIP_CHECK(hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached));
  FT_HIP_CHECK(hipMemset(*ptr, 0, bytes));
  FT_HIP_CHECK(hipDeviceSynchronize());
  return 0;
}

extern "C" int ft_ar_free(void* ptr) { return static_cast<int>(hipFree(ptr)); }

extern "C" int ft_ar_ipc_handle(void* ptr, char* out64) {
  hipIpcMemHandle_t h;
  FT_HIP_CHECK(hipIpcGetMemHandle(&h, ptr));
  static_assert(sizeof(h) <= 64, "ipc handle size");
  for (size_t i = 0; i < sizeof(h); ++i) out64[i] = reinterpret_cast<const char*>(&h)[i];
  return 0;
}

extern "C" int ft_ar_ipc_open(const char* in64, void** ptr) {
  hipIpcMemHandle_t h;
  for (size_t i = 0; i < sizeof(h); ++i) reinterpret_cast<char*>(&h)[i] = in64[i];
  FT_HIP_CHECK(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
  return 0;
}

extern "C" int ft_ar_ipc_close(void* ptr) { return static_cast<int>(hipIpcCloseMemHandle(ptr)); }

extern "C" int ft_ar_read_error(void* mine, int* err) {
  uint32_t v = 0;
  FT_HIP_CHECK(hipMemcpy(&v, reinterpret_cast<uint8_t*>(mine) + ft::ArLayout::kError, 4,
                         hipMemcpyDeviceToHost));
  *err = (int)v;
  return 0;
}

// x (bf16, n elements, n % 8 == 0, n*2 <= max_bytes) is summed over the W
// ranks into out (may alias x).  peers: device array of W region base pointers.
extern "C" int ft_ar_allreduce(void* out, const void* x, long n, const uint64_t* peers_dev,
                               int rank, int world, size_t max_bytes, unsigned spin_budget,
                               hipStream_t stream) {
  if (n <= 0) return 0;
  if (n % 8 != 0 || (size_t)n * 2 > max_bytes) return -1;
  const int n8 = (int)(n / 8);
  const int blocks = (int)std::min<long>(ft::ceil_div(n8, 256), 64);
#define FT_AR_CASE(WW)                                                                       \
  case WW:                                                                                   \
    hipLaunchKernelGGL((ft::ar_oneshot_kernel<WW>), dim3(blocks), dim3(256), 0, stream,      \
                       (uint16_t*)out, (const uint16_t*)x, peers_dev, rank, max_bytes, n8,   \
                       spin_budget);                                                         \
    break;
  switch (world) {
    FT_AR_CASE(2)
    FT_AR_CASE(4)
    FT_AR_CASE(8)
    default:
      return -2;
  }
#undef FT_AR_CASE
  return static_cast<int>(hipGetLastError());
}
