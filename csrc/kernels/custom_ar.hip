// X1/X2/X4: all-reduce and all-gather over xGMI peer mappings for
// the decode-size activations of tensor parallelism ([tokens, hidden] bf16, a few
// hundred KiB to a few MiB) and the vocab-sharded logits.
//
// Why not only RCCL: a ring all-reduce crosses one xGMI link per step and pays
// 2(W-1) latency-bound hops; at decode sizes the step is latency, not bandwidth.
//   one-shot: every rank publishes its input in an IPC-shared buffer, then every
//     rank reads all W inputs directly over its 7 xGMI links at once and sums
//     them.  Remote bytes read per rank: (W-1) * n.
//   two-shot: reduce-scatter + all-gather through the same buffers -- rank r sums
//     chunk r of all W inputs in place (its own staging), a second barrier, then
//     every rank copies the W reduced chunks.  Remote bytes per rank:
//     2 (W-1)/W * n, at the price of a second cross-rank barrier; the host picks
//     it above a size crossover (custom_allreduce.py).
//   all-gather: publish, one barrier, read the W shards interleaved into rows.
//
// Protocol (one kernel per collective, graph-safe: no host-side argument changes
// between replays):
//   * each rank owns one uncached (hipDeviceMallocUncached) region
//       [epoch | error | arrived[2] | signal[2][8] | staging[2][max_bytes]]
//     mapped into every peer with hipIpcOpenMemHandle;
//   * every block reads the epoch (= counter + 1) and this rank's error word;
//     a rank whose error word is set skips every later collective at once
//     (sticky: the host sees it and switches the group to RCCL);
//   * barrier b: every block counts itself in arrived[b]; block 0 waits for all
//     blocks of this rank (grid <= 128 blocks, always co-resident), resets the
//     count, (b == 0: bumps the counter for the next call) and stores `epoch` into
//     signal[b][my_rank] of every rank (system-scope release); every block then
//     waits until all W signals[b] in MY region reach `epoch` (system-scope
//     acquire, bounded spin).
//   Staging is double buffered by epoch parity: a rank can be at most one call
//   ahead of the slowest peer (it must see that peer's first-barrier signal for
//   the current call first), so the slot it overwrites was consumed two calls ago.
//   * a wait beyond the spin budget sets the error word and the kernel returns
//     with `out` NOT reduced; ar_export_error (captured at the end of every decode
//     step) folds the W error words into a device flag the runner copies to the
//     host with the sampled ids, so the step's tokens are discarded, never emitted.
#include "ft_common.h"

namespace ft {

struct ArLayout {
  static constexpr size_t kCounter = 0;     // u32 epoch counter (this rank)
  static constexpr size_t kError = 4;       // u32 error flag (sticky)
  static constexpr size_t kArrived = 8;     // u32 arrived[2]: blocks of this rank at barrier b
  static constexpr size_t kSignal = 64;     // u32 signal[2][8] (written by all ranks)
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

// Block-uniform start of a collective: epoch of this call, or 0 if this rank has
// already failed (then the caller returns without touching out).
__device__ __forceinline__ uint32_t ar_begin(uint8_t* mine, uint32_t* s_word) {
  if (threadIdx.x == 0) {
    const uint32_t err = __hip_atomic_load(ar_u32(mine, ArLayout::kError), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
    *s_word = err ? 0u
                  : __hip_atomic_load(ar_u32(mine, ArLayout::kCounter), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT) + 1;
  }
  __syncthreads();
  return *s_word;
}

// Cross-rank barrier b (0 or 1) after this block's stores; returns block-uniform ok.
template <int W>
__device__ bool ar_barrier(uint8_t* mine, const uint64_t* __restrict__ peers, int rank,
                           uint32_t epoch, int b, uint32_t budget, int* s_ok) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* arrived = ar_u32(mine, ArLayout::kArrived) + b;
    __hip_atomic_fetch_add(arrived, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    if (blockIdx.x == 0) {
      ok = ar_wait_ge(arrived, gridDim.x, budget, 0);
      __hip_atomic_store(arrived, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (b == 0)
        __hip_atomic_store(ar_u32(mine, ArLayout::kCounter), epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      __threadfence_system();
      if (ok) {
        for (int r = 0; r < W; ++r) {
          uint8_t* peer = reinterpret_cast<uint8_t*>(peers[r]);
          __hip_atomic_store(ar_u32(peer, ArLayout::kSignal) + 8 * b + rank, epoch,
                             __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
    uint32_t* sig = ar_u32(mine, ArLayout::kSignal) + 8 * b;
    for (int r = 0; r < W && ok; ++r) ok = ar_wait_ge(sig + r, epoch, budget, 1);
    if (!ok)
      __hip_atomic_store(ar_u32(mine, ArLayout::kError), 1u, __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

__device__ __forceinline__ void ar_publish(uint8_t* mine, size_t slot, const uint16_t* x, int n8) {
  uint4* stage = reinterpret_cast<uint4*>(mine + slot);
  const uint4* src = reinterpret_cast<const uint4*>(x);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x)
    stage[i] = src[i];
}

template <int W>
__device__ __forceinline__ void ar_sum_range(uint4* dst, const uint64_t* __restrict__ peers,
                                             size_t slot, int lo, int hi) {
  const uint4* in[W];
#pragma unroll
  for (int r = 0; r < W; ++r)
    in[r] = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(peers[r]) + slot);
  for (int i = lo + blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += gridDim.x * blockDim.x) {
    uint4 raw[W];
#pragma unroll
    for (int r = 0; r < W; ++r) raw[r] = in[r][i];  // W loads in flight before the adds
    float acc[8];
    load8(raw[0], acc);
#pragma unroll
    for (int r = 1; r < W; ++r) {
      float v[8];
      load8(raw[r], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    dst[i] = store8(acc);
  }
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
  const uint32_t epoch = ar_begin(mine, &s_epoch);
  if (epoch == 0) return;
  const size_t slot = ArLayout::kStaging + (epoch & 1) * max_bytes;
  ar_publish(mine, slot, x, n8);
  if (!ar_barrier<W>(mine, peers, rank, epoch, 0, spin_budget, &s_ok)) return;
  ar_sum_range<W>(reinterpret_cast<uint4*>(out), peers, slot, 0, n8);
}

template <int W>
__global__ __launch_bounds__(256) void ar_twoshot_kernel(uint16_t* __restrict__ out,
                                                         const uint16_t* __restrict__ x,
                                                         const uint64_t* __restrict__ peers,
                                                         int rank, size_t max_bytes, int n8,
                                                         uint32_t spin_budget) {
  uint8_t* mine = reinterpret_cast<uint8_t*>(peers[rank]);
  __shared__ uint32_t s_epoch;
  __shared__ int s_ok;
  const uint32_t epoch = ar_begin(mine, &s_epoch);
  if (epoch == 0) return;
  const size_t slot = ArLayout::kStaging + (epoch & 1) * max_bytes;
  ar_publish(mine, slot, x, n8);
  if (!ar_barrier<W>(mine, peers, rank, epoch, 0, spin_budget, &s_ok)) return;
  // reduce-scatter: chunk `rank` of every input, summed into MY staging in place
  // (peers only read their own chunk index from my staging in this phase)
  const int lo = (int)((long)rank * n8 / W), hi = (int)((long)(rank + 1) * n8 / W);
  ar_sum_range<W>(reinterpret_cast<uint4*>(mine + slot), peers, slot, lo, hi);
  if (!ar_barrier<W>(mine, peers, rank, epoch, 1, spin_budget, &s_ok)) return;
  // all-gather of the W reduced chunks
  uint4* dst = reinterpret_cast<uint4*>(out);
#pragma unroll
  for (int r = 0; r < W; ++r) {
    const uint4* src =
        reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(peers[r]) + slot);
    const int a = (int)((long)r * n8 / W), e = (int)((long)(r + 1) * n8 / W);
    for (int i = a + blockIdx.x * blockDim.x + threadIdx.x; i < e; i += gridDim.x * blockDim.x)
      dst[i] = src[i];
  }
}

// out[row, r * row8 + c] (in uint4 units, W * row8 per row) = shard of rank r.
template <int W>
__global__ __launch_bounds__(256) void ar_allgather_kernel(uint16_t* __restrict__ out,
                                                           const uint16_t* __restrict__ x,
                                                           const uint64_t* __restrict__ peers,
                                                           int rank, size_t max_bytes, int n8,
                                                           int row8, uint32_t spin_budget) {
  uint8_t* mine = reinterpret_cast<uint8_t*>(peers[rank]);
  __shared__ uint32_t s_epoch;
  __shared__ int s_ok;
  uint4* dst = reinterpret_cast<uint4*>(out);
  const uint32_t epoch = ar_begin(mine, &s_epoch);
  bool ok = epoch != 0;
  const size_t slot = ArLayout::kStaging + (epoch & 1) * max_bytes;
  if (ok) {
    ar_publish(mine, slot, x, n8);
    ok = ar_barrier<W>(mine, peers, rank, epoch, 0, spin_budget, &s_ok);
  }
  if (!ok) {  // failed: zeros (finite logits; the host discards the step anyway)
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8 * W; i += gridDim.x * blockDim.x)
      dst[i] = make_uint4(0u, 0u, 0u, 0u);
    return;
  }
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int row = i / row8, c = i - row * row8;
    uint4 v[W];
#pragma unroll
    for (int r = 0; r < W; ++r)
      v[r] = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(peers[r]) + slot)[i];
#pragma unroll
    for (int r = 0; r < W; ++r) dst[((size_t)row * W + r) * row8 + c] = v[r];
  }
}

// X1/X2 fused with the residual add + RMSNorm that follows every row-parallel
// projection (o, down) -- one launch instead of slab_store -> all-reduce ->
// add+RMSNorm:
//   publish  this rank's partial rows as bf16: its split-K fp32 slabs summed
//            (ws != null, the projection's own epilogue format) or a bf16 block x;
//   barrier  (one, as the one-shot all-reduce);
//   rows     strided over the blocks: the W partials summed in rank order (fp32,
//            identical on every rank, rounded to bf16 like the all-reduce's output)
//            + residual -> residual (bf16) and
//            out = rmsnorm(residual) * w, both rounded like row_add_rmsnorm_kernel.
// A timed-out barrier leaves residual / out untouched and the error word set
// (the step is discarded by the runner, as for every custom collective).
template <int W, int VPT>
__global__ __launch_bounds__(256) void ar_add_rmsnorm_kernel(
    uint16_t* __restrict__ out, int out_stride, uint16_t* __restrict__ residual,
    const uint16_t* __restrict__ weight, float eps, const float* __restrict__ ws, int splits,
    const uint16_t* __restrict__ x, int x_stride, int rows, int hidden,
    const uint64_t* __restrict__ peers, int rank, size_t max_bytes, uint32_t spin_budget) {
  uint8_t* mine = reinterpret_cast<uint8_t*>(peers[rank]);
  __shared__ uint32_t s_epoch;
  __shared__ int s_ok;
  __shared__ float red[4];
  const uint32_t epoch = ar_begin(mine, &s_epoch);
  if (epoch == 0) return;
  const size_t slot = ArLayout::kStaging + (epoch & 1) * max_bytes;
  const int h8 = hidden / 8;
  const int n8 = rows * h8;
  uint4* stage = reinterpret_cast<uint4*>(mine + slot);
  const size_t slab = (size_t)rows * hidden;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += gridDim.x * blockDim.x) {
    const int row = i / h8, c = (i - row * h8) * 8;
    float v[8];
    if (ws != nullptr) {
      const float* p = ws + (size_t)row * hidden + c;
      float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
      for (int sp = 1; sp < splits; ++sp) {
        const float4 a2 = reinterpret_cast<const float4*>(p + sp * slab)[0];
        const float4 b2 = reinterpret_cast<const float4*>(p + sp * slab)[1];
        a.x += a2.x; a.y += a2.y; a.z += a2.z; a.w += a2.w;
        b.x += b2.x; b.y += b2.y; b.z += b2.z; b.w += b2.w;
      }
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
      load8(*reinterpret_cast<const uint4*>(x + (size_t)row * x_stride + c), v);
    }
    stage[i] = store8(v);
  }
  if (!ar_barrier<W>(mine, peers, rank, epoch, 0, spin_budget, &s_ok)) return;
  const uint4* in[W];
#pragma unroll
  for (int r = 0; r < W; ++r)
    in[r] = reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(peers[r]) + slot);
  // Two passes per row, each column block in its own (non-unrolled) iteration, so at
  // most W peer loads are in flight per thread and nothing is live across blocks:
  // hoisting all VPT * W loads took 256 VGPRs + 82 AGPRs at W = 8, VPT = 4 (one wave
  // per SIMD: every spinning block held a whole CU, and ranks sharing one GPU starved
  // the one still computing).  Pass 1 writes the new residual; pass 2 re-reads this
  // thread's own stores (same thread, no fence) for the normalised output.
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * hidden);
    float ss = 0.f;
#pragma unroll 1
    for (int c = 0; c < VPT; ++c) {
      const int e = row * h8 + c * 256 + threadIdx.x;
      uint4 raw[W];
#pragma unroll
      for (int r = 0; r < W; ++r) raw[r] = in[r][e];   // W peer loads in flight
      float v[8];
      load8(raw[0], v);
#pragma unroll
      for (int r = 1; r < W; ++r) {
        float t[8];
        load8(raw[r], t);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] += t[j];
      }
      // the reduced partial is rounded to bf16 first, exactly as the separate
      // all-reduce would store it: fused, unfused and RCCL-fallback TP steps (and the
      // retried steps after a collective fault) produce the same bits
      float rv[8];
      load8(store8(v), v);
      load8(rr[c * 256 + threadIdx.x], rv);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += rv[j];
      const uint4 rb = store8(v);
      rr[c * 256 + threadIdx.x] = rb;
      load8(rb, v);   // continue from the bf16-rounded residual
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += v[j] * v[j];
    }
    ss = wave_sum(ss);
    __syncthreads();
    if (lane_id() == 0) red[wave_id()] = ss;
    __syncthreads();
    const float inv = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)hidden + eps);
    uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * out_stride);
#pragma unroll 1
    for (int c = 0; c < VPT; ++c) {
      float v[8], wf[8];
      load8(rr[c * 256 + threadIdx.x], v);
      load8(*reinterpret_cast<const uint4*>(weight + (c * 256 + threadIdx.x) * 8), wf);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf16_to_f32(f32_to_bf16(v[j] * inv)) * wf[j];
      orow[c * 256 + threadIdx.x] = store8(v);
    }
  }
}

// dst[0] = OR of the W ranks' error words (one lane; captured in the decode graph).
__global__ void ar_export_error_kernel(int* __restrict__ dst, const uint64_t* __restrict__ peers,
                                       int world) {
  if (threadIdx.x != 0) return;
  uint32_t e = 0;
  for (int r = 0; r < world; ++r)
    e |= __hip_atomic_load(ar_u32(reinterpret_cast<uint8_t*>(peers[r]), ArLayout::kError),
                           __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  dst[0] = (int)e;
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

// Grid cap of every collective (all loops are grid-strided).  128 by default; ranks
// that share ONE device (tests / rehearsals) lower it so the W-1 kernels that spin
// while a peer is still computing leave that peer CUs to compute on.
static int g_ar_max_blocks = 128;

extern "C" void ft_ar_set_max_blocks(int n) { g_ar_max_blocks = std::max(1, std::min(n, 128)); }

static int ar_blocks(int n8) {
  return (int)std::min<long>(ft::ceil_div(n8, 256), g_ar_max_blocks);
}

// x (bf16, n elements, n % 8 == 0, n*2 <= max_bytes) is summed over the W
// ranks into out (may alias x).  peers: device array of W region base pointers.
extern "C" int ft_ar_allreduce(void* out, const void* x, long n, const uint64_t* peers_dev,
                               int rank, int world, size_t max_bytes, unsigned spin_budget,
                               int two_shot, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n % 8 != 0 || (size_t)n * 2 > max_bytes) return -1;
  const int n8 = (int)(n / 8);
  const int blocks = ar_blocks(n8);
#define FT_AR_CASE(WW)                                                                       \
  case WW:                                                                                   \
    if (two_shot)                                                                            \
      hipLaunchKernelGGL((ft::ar_twoshot_kernel<WW>), dim3(blocks), dim3(256), 0, stream,    \
                         (uint16_t*)out, (const uint16_t*)x, peers_dev, rank, max_bytes, n8, \
                         spin_budget);                                                       \
    else                                                                                     \
      hipLaunchKernelGGL((ft::ar_oneshot_kernel<WW>), dim3(blocks), dim3(256), 0, stream,    \
                         (uint16_t*)out, (const uint16_t*)x, peers_dev, rank, max_bytes, n8, \
                         spin_budget);                                                       \
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

// x: [rows, row_elems] bf16 shard of this rank; out: [rows, world * row_elems].
extern "C" int ft_ar_allgather(void* out, const void* x, long rows, long row_elems,
                               const uint64_t* peers_dev, int rank, int world, size_t max_bytes,
                               unsigned spin_budget, hipStream_t stream) {
  const long n = rows * row_elems;
  if (n <= 0) return 0;
  if (row_elems % 8 != 0 || (size_t)n * 2 > max_bytes) return -1;
  const int n8 = (int)(n / 8), row8 = (int)(row_elems / 8);
  const int blocks = ar_blocks(n8);
#define FT_AG_CASE(WW)                                                                           \
  case WW:                                                                                       \
    hipLaunchKernelGGL((ft::ar_allgather_kernel<WW>), dim3(blocks), dim3(256), 0, stream,        \
                       (uint16_t*)out, (const uint16_t*)x, peers_dev, rank, max_bytes, n8, row8, \
                       spin_budget);                                                             \
    break;
  switch (world) {
    FT_AG_CASE(2)
    FT_AG_CASE(4)
    FT_AG_CASE(8)
    default:
      return -2;
  }
#undef FT_AG_CASE
  return static_cast<int>(hipGetLastError());
}

// residual [rows, hidden] += sum over ranks of this rank's partial (fp32 split-K slabs
// ws[splits][rows][hidden], or bf16 x [rows, x_stride]); out = rmsnorm(residual) * w.
// hidden % 2048 == 0 (<= 8192), rows * hidden * 2 <= max_bytes.
extern "C" int ft_ar_add_rmsnorm(void* out, int out_stride, void* residual, const void* weight,
                                 float eps, const float* ws, int splits, const void* x,
                                 int x_stride, long rows, long hidden, const uint64_t* peers_dev,
                                 int rank, int world, size_t max_bytes, unsigned spin_budget,
                                 hipStream_t stream) {
  if (rows <= 0) return 0;
  if (hidden % 2048 != 0 || hidden > 8192) return -3;
  if ((size_t)(rows * hidden) * 2 > max_bytes) return -1;
  if ((ws == nullptr) == (x == nullptr) || (ws != nullptr && splits < 1)) return -4;
  const int blocks = (int)std::min<long>(rows, g_ar_max_blocks);
  const int vpt = (int)(hidden / 2048);
#define FT_ARN(WW, VV)                                                                         \
  if (world == WW && vpt == VV) {                                                              \
    hipLaunchKernelGGL((ft::ar_add_rmsnorm_kernel<WW, VV>), dim3(blocks), dim3(256), 0, stream,\
                       (uint16_t*)out, out_stride, (uint16_t*)residual, (const uint16_t*)weight,\
                       eps, ws, splits, (const uint16_t*)x, x_stride, (int)rows, (int)hidden,   \
                       peers_dev, rank, max_bytes, spin_budget);                               \
    return static_cast<int>(hipGetLastError());                                                \
  }
#define FT_ARN_W(WW) FT_ARN(WW, 1) FT_ARN(WW, 2) FT_ARN(WW, 3) FT_ARN(WW, 4)
  FT_ARN_W(2)
  FT_ARN_W(4)
  FT_ARN_W(8)
#undef FT_ARN_W
#undef FT_ARN
  return -2;
}

extern "C" int ft_ar_export_error(int* dst, const uint64_t* peers_dev, int world,
                                  hipStream_t stream) {
  hipLaunchKernelGGL(ft::ar_export_error_kernel, dim3(1), dim3(64), 0, stream, dst, peers_dev,
                     world);
  return static_cast<int>(hipGetLastError());
}
