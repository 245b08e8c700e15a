// K12: fused sampler -- constrained-decoding mask, temperature, top-k, top-p
// (nucleus) and the draw, one workgroup per sequence.  SURVEY.md §2.4 K12.
//
// No sort: top-k and top-p thresholds are found with a 4-pass MSB radix select
// over the order-preserving uint32 image of the logits (8 bits per pass,
// 256-bin LDS histograms; counts for top-k, probability mass for top-p), then
// the draw is a Gumbel-max over the surviving tokens with a counter-based RNG
// (splitmix64 of seed, step, token id), so the sampler is deterministic per
// (seed, step), needs no host round trip and can live inside the captured
// decode graph.  temperature == 0 is the greedy argmax fast path (one pass).
// The optional allow-bitmask (1 bit per vocab id) implements the token-mask
// FSM of JSON-constrained tool calls (E19).
#include "ft_common.h"

namespace ft {

constexpr int kSampThreads = 1024;
constexpr int kSampWaves = kSampThreads / 64;

__device__ __forceinline__ uint32_t f2key(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

template <typename T>
__device__ __forceinline__ float load_logit(const T* p, long i);
template <>
__device__ __forceinline__ float load_logit<float>(const float* p, long i) { return p[i]; }
template <>
__device__ __forceinline__ float load_logit<uint16_t>(const uint16_t* p, long i) {
  return bf16_to_f32(p[i]);
}

struct SampShared {
  float hist_f[256];
  int hist_i[256];
  float wred[kSampWaves];
  int wredi[kSampWaves];
  uint32_t wkey[kSampWaves];
  int sel_bin;
  float sel_rem_f;
  int sel_rem_i;
};

// block-wide max of (value, index) preferring the lower index on ties
__device__ __forceinline__ void block_argmax(float& v, int& idx, SampShared& sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(v, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ov > v || (ov == v && oi < idx)) {
      v = ov;
      idx = oi;
    }
  }
  if (lane_id() == 0) {
    sh.wred[wave_id()] = v;
    sh.wredi[wave_id()] = idx;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    v = threadIdx.x < kSampWaves ? sh.wred[threadIdx.x] : -INFINITY;
    idx = threadIdx.x < kSampWaves ? sh.wredi[threadIdx.x] : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(v, o, 64);
      const int oi = __shfl_xor(idx, o, 64);
      if (ov > v || (ov == v && oi < idx)) {
        v = ov;
        idx = oi;
      }
    }
    if (threadIdx.x == 0) {
      sh.wred[0] = v;
      sh.wredi[0] = idx;
    }
  }
  __syncthreads();
  v = sh.wred[0];
  idx = sh.wredi[0];
  __syncthreads();
}

__device__ __forceinline__ float block_sum(float v, SampShared& sh) {
  v = wave_sum(v);
  if (lane_id() == 0) sh.wred[wave_id()] = v;
  __syncthreads();
  if (threadIdx.x < 64) {
    v = threadIdx.x < kSampWaves ? sh.wred[threadIdx.x] : 0.f;
    v = wave_sum(v);
    if (threadIdx.x == 0) sh.wred[0] = v;
  }
  __syncthreads();
  v = sh.wred[0];
  __syncthreads();
  return v;
}

// Given a 256-bin histogram (counts or mass), walk bins from the top (255) and
// select the bin where the running total first reaches `rem`.  Threads 0..255
// participate: an inclusive scan over descending bins.
template <typename V>
__device__ __forceinline__ void select_bin(V* hist, V rem, SampShared& sh, int* out_bin,
                                           V* out_rem) {
  const int t = threadIdx.x;
  V val = (t < 256) ? hist[255 - t] : V(0);
  // wave inclusive scan
  V inc = val;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const V y = __shfl_up(inc, o, 64);
    if (lane_id() >= o) inc += y;
  }
  __shared__ V wtot[4];
  if (t < 256 && lane_id() == 63) wtot[wave_id()] = inc;
  __syncthreads();
  if (t < 256) {
    V off = V(0);
    for (int w = 0; w < wave_id(); ++w) off += wtot[w];
    inc += off;
    const V exc = inc - val;
    // the first descending bin whose inclusive total reaches rem
    const bool hit = (inc >= rem) && (exc < rem);
    if (hit) {
      *out_bin = 255 - t;
      *out_rem = rem - exc;
    }
  }
  __syncthreads();
}

template <typename T>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(
    int* __restrict__ out_tokens, const T* __restrict__ logits, long logit_stride, int vocab,
    const float* __restrict__ temperature, const float* __restrict__ top_p,
    const int* __restrict__ top_k, const long long* __restrict__ seeds,
    const int* __restrict__ steps, const uint32_t* __restrict__ allow_mask, int mask_words) {
  __shared__ SampShared sh;
  const int row = blockIdx.x;
  const T* x = logits + (long)row * logit_stride;
  const uint32_t* mrow = allow_mask ? allow_mask + (long)row * mask_words : nullptr;
  auto masked = [&](int i) -> bool { return mrow && !((mrow[i >> 5] >> (i & 31)) & 1u); };

  // ---- pass 1: max / argmax --------------------------------------------------------
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int i = threadIdx.x; i < vocab; i += kSampThreads) {
    float v = load_logit<T>(x, i);
    if (masked(i)) v = -INFINITY;
    if (v > best) {
      best = v;
      besti = i;
    }
  }
  block_argmax(best, besti, sh);
  const float temp = temperature[row];
  if (temp <= 0.f || best == -INFINITY) {
    if (threadIdx.x == 0) out_tokens[row] = (besti == 0x7fffffff) ? 0 : besti;
    return;
  }
  const float inv_t = 1.f / temp;
  const float M = best;

  // ---- top-k threshold (radix select on count) ----------------------------------------
  uint32_t thr = 0u;  // keep keys >= thr
  const int k = top_k[row];
  if (k > 0 && k < vocab) {
    uint32_t prefix = 0u, pmask = 0u;
    int rem = k;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      if (threadIdx.x < 256) sh.hist_i[threadIdx.x] = 0;
      __syncthreads();
      for (int i = threadIdx.x; i < vocab; i += kSampThreads) {
        if (masked(i)) continue;
        const uint32_t key = f2key(load_logit<T>(x, i));
        if ((key & pmask) == prefix) atomicAdd(&sh.hist_i[(key >> shift) & 255u], 1);
      }
      __syncthreads();
      select_bin<int>(sh.hist_i, rem, sh, &sh.sel_bin, &sh.sel_rem_i);
      const int bin = sh.sel_bin;
      rem = sh.sel_rem_i;
      prefix |= (uint32_t)bin << shift;
      pmask |= 255u << shift;
      __syncthreads();
    }
    thr = prefix;
  }

  // ---- top-p threshold (radix select on probability mass) ----------------------------
  const float tp = top_p[row];
  if (tp < 1.f) {
    float tot = 0.f;
    for (int i = threadIdx.x; i < vocab; i += kSampThreads) {
      if (masked(i)) continue;
      const float v = load_logit<T>(x, i);
      if (f2key(v) >= thr) tot += __expf((v - M) * inv_t);
    }
    tot = block_sum(tot, sh);
    float rem = tp * tot;
    uint32_t prefix = 0u, pmask = 0u;
    for (int pass = 0; pass < 4; ++pass) {
      const int shift = 24 - 8 * pass;
      if (threadIdx.x < 256) sh.hist_f[threadIdx.x] = 0.f;
      __syncthreads();
      for (int i = threadIdx.x; i < vocab; i += kSampThreads) {
        if (masked(i)) continue;
        const float v = load_logit<T>(x, i);
        const uint32_t key = f2key(v);
        if (key >= thr && (key & pmask) == prefix)
          atomicAdd(&sh.hist_f[(key >> shift) & 255u], __expf((v - M) * inv_t));
      }
      __syncthreads();
      sh.sel_bin = -1;
      __syncthreads();
      select_bin<float>(sh.hist_f, rem, sh, &sh.sel_bin, &sh.sel_rem_f);
      int bin = sh.sel_bin;
      if (bin < 0) {
        // rounding: rem slightly above the histogram total -> take the lowest
        // non-empty bin so the whole remaining mass is kept
        bin = 0;
        if (threadIdx.x == 0) {
          for (int j = 0; j < 256; ++j)
            if (sh.hist_f[j] > 0.f) { sh.sel_bin = j; break; }
        }
        __syncthreads();
        bin = sh.sel_bin < 0 ? 0 : sh.sel_bin;
        rem = 0.f;
      } else {
        rem = sh.sel_rem_f;
      }
      prefix |= (uint32_t)bin << shift;
      pmask |= 255u << shift;
      __syncthreads();
    }
    if (prefix > thr) thr = prefix;
  }

  // ---- Gumbel-max draw over survivors --------------------------------------------------
  const uint64_t s0 = splitmix64((uint64_t)seeds[row] ^ (0x632BE59BD9B4E019ull * (uint64_t)(steps[row] + 1)));
  float gbest = -INFINITY;
  int gi = 0x7fffffff;
  for (int i = threadIdx.x; i < vocab; i += kSampThreads) {
    if (masked(i)) continue;
    const float v = load_logit<T>(x, i);
    if (f2key(v) < thr) continue;
    const uint64_t h = splitmix64(s0 + (uint64_t)i);
    const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);  // (0,1)
    const float g = -__logf(-__logf(u));
    const float sc = (v - M) * inv_t + g;
    if (sc > gbest) {
      gbest = sc;
      gi = i;
    }
  }
  block_argmax(gbest, gi, sh);
  if (threadIdx.x == 0) out_tokens[row] = (gi == 0x7fffffff) ? besti : gi;
}

}  // namespace ft

extern "C" int ft_sample(int* out_tokens, const void* logits, int logits_is_bf16, long logit_stride,
                         int batch, int vocab, const float* temperature, const float* top_p,
                         const int* top_k, const long long* seeds, const int* steps,
                         const uint32_t* allow_mask, int mask_words, hipStream_t stream) {
  if (batch <= 0) return 0;
  dim3 grid(batch), block(ft::kSampThreads);
  if (logits_is_bf16) {
    hipLaunchKernelGGL(ft::sample_kernel<uint16_t>, grid, block, 0, stream, out_tokens,
                       (const uint16_t*)logits, logit_stride, vocab, temperature, top_p, top_k,
                       seeds, steps, allow_mask, mask_words);
  } else {
    hipLaunchKernelGGL(ft::sample_kernel<float>, grid, block, 0, stream, out_tokens,
                       (const float*)logits, logit_stride, vocab, temperature, top_p, top_k,
                       seeds, steps, allow_mask, mask_words);
  }
  return static_cast<int>(hipGetLastError());
}
