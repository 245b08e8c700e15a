// K12: fused sampler -- constrained-decoding mask, temperature, top-k, top-p
// (nucleus) and the draw; one 1024-thread workgroup per sequence.
// SURVEY.md §2.4 K12.
//
// Design (measured: the first version, a 4-pass radix select with LDS-atomic
// histograms, spent 410 us per 50-row step because every logit of a row lands
// in one or two MSB bins -> fully serialised LDS atomics):
//   * every pass streams the row (<= 131072 ids, 256 KiB bf16, L2-resident after
//     the first pass) with 16-B lane loads as ordered 16-bit keys (bf16 bits
//     made monotonic); a register-cached variant spilled (128-VGPR cap at 1024
//     threads) and was slower.
//   * greedy: one pass, argmax (lowest id on ties).
//   * top-k: 4-ary search on the 16-bit key (count >= k), 8 passes (was a
//     16-pass bisection).
//   * sampling: inverse CDF in a fixed (thread, slot) order -- one exp pass
//     gives per-thread masses, a block scan locates the thread holding the
//     target mass, that thread walks its 16 chunks.
//   * top-p: exact rejection -- a drawn token s is accepted iff the mass of
//     strictly more likely kept tokens is < top_p * Z (i.e. s is in the
//     nucleus); accepted draws are distributed exactly as the renormalised
//     nucleus.  Acceptance >= top_p per round, 8 rounds max; if all miss
//     (<= (1 - top_p)^8), the nucleus threshold is found by a 4-ary search on
//     the key and the draw repeats restricted to it -- exact in every case.
//     Each round costs one pass.
//   * RNG: splitmix64(seed, step, round) -> one uniform per round per row, so
//     sampling is reproducible per (seed, step) and graph-capturable.
//   * allow-bitmask (1 bit / vocab id) implements the JSON token FSM (E19).
#include "ft_common.h"

namespace ft {

constexpr int kSampThreads = 1024;
constexpr int kSampWaves = kSampThreads / 64;
constexpr int kSlots = 128;  // keys per lane -> vocab <= 131072
constexpr uint32_t kNegInfKey = 0x007Fu;  // ordered key of bf16 -inf (0xFF80)

__device__ __forceinline__ uint32_t bf16_to_key(uint32_t b) {
  return (b & 0x8000u) ? (~b & 0xFFFFu) : (b | 0x8000u);
}
__device__ __forceinline__ float key_to_f32(uint32_t k) {
  const uint32_t b = (k & 0x8000u) ? (k & 0x7FFFu) : (~k & 0xFFFFu);
  return __uint_as_float(b << 16);
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct SampShared {
  float f[kSampWaves];
  int i[kSampWaves];
  uint32_t u[kSampWaves];
  float scan[kSampWaves];
  int i3[3][kSampWaves];
  int winner;
  int found;
};

__device__ __forceinline__ float block_sum_f(float v, SampShared& sh) {
  v = wave_sum(v);
  __syncthreads();
  if (lane_id() == 0) sh.f[wave_id()] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) t += sh.f[w];
  return t;
}

__device__ __forceinline__ int block_sum_i(int v, SampShared& sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if (lane_id() == 0) sh.i[wave_id()] = v;
  __syncthreads();
  int t = 0;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) t += sh.i[w];
  return t;
}

// three block sums behind one pair of barriers
__device__ __forceinline__ void block_sum_i3(int& a, int& b, int& c, SampShared& sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
    c += __shfl_xor(c, o, 64);
  }
  __syncthreads();
  if (lane_id() == 0) {
    sh.i3[0][wave_id()] = a;
    sh.i3[1][wave_id()] = b;
    sh.i3[2][wave_id()] = c;
  }
  __syncthreads();
  a = b = c = 0;
#pragma unroll
  for (int w = 0; w < kSampWaves; ++w) {
    a += sh.i3[0][w];
    b += sh.i3[1][w];
    c += sh.i3[2][w];
  }
}

// max key, lowest index on ties
__device__ __forceinline__ void block_argmax_key(uint32_t& k, int& idx, SampShared& sh) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t ok = __shfl_xor(k, o, 64);
    const int oi = __shfl_xor(idx, o, 64);
    if (ok > k || (ok == k && oi < idx)) {
      k = ok;
      idx = oi;
    }
  }
  __syncthreads();
  if (lane_id() == 0) {
    sh.u[wave_id()] = k;
    sh.i[wave_id()] = idx;
  }
  __syncthreads();
  k = sh.u[0];
  idx = sh.i[0];
#pragma unroll
  for (int w = 1; w < kSampWaves; ++w) {
    if (sh.u[w] > k || (sh.u[w] == k && sh.i[w] < idx)) {
      k = sh.u[w];
      idx = sh.i[w];
    }
  }
}


// 8 consecutive ids starting at `base` (multiple of 8) as ordered keys; masked
// or out-of-range ids get the key of -inf
template <typename T>
__device__ __forceinline__ void load_keys8(const T* x, const uint32_t* mrow, int base, int vocab,
                                           uint32_t (&key)[8]) {
  if (base >= vocab) {
#pragma unroll
    for (int j = 0; j < 8; ++j) key[j] = kNegInfKey;
    return;
  }
  uint32_t bits[8];
  if constexpr (sizeof(T) == 2) {
    const uint4 v = *reinterpret_cast<const uint4*>(x + base);
    bits[0] = v.x & 0xFFFFu; bits[1] = v.x >> 16; bits[2] = v.y & 0xFFFFu; bits[3] = v.y >> 16;
    bits[4] = v.z & 0xFFFFu; bits[5] = v.z >> 16; bits[6] = v.w & 0xFFFFu; bits[7] = v.w >> 16;
  } else {
    const float4 a = *reinterpret_cast<const float4*>(x + base);
    const float4 c = *reinterpret_cast<const float4*>(x + base + 4);
    bits[0] = f32_to_bf16(a.x); bits[1] = f32_to_bf16(a.y); bits[2] = f32_to_bf16(a.z);
    bits[3] = f32_to_bf16(a.w); bits[4] = f32_to_bf16(c.x); bits[5] = f32_to_bf16(c.y);
    bits[6] = f32_to_bf16(c.z); bits[7] = f32_to_bf16(c.w);
  }
  const uint32_t mb = mrow ? (mrow[base >> 5] >> (base & 31)) : 0xFFu;
#pragma unroll
  for (int j = 0; j < 8; ++j) key[j] = ((mb >> j) & 1u) ? bf16_to_key(bits[j]) : kNegInfKey;
}

constexpr int kChunks = kSlots / 8;  // 16 chunks of 8 ids per lane

template <typename T>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(
    int* __restrict__ out_tokens, const T* __restrict__ logits, long logit_stride, int vocab,
    const float* __restrict__ temperature, const float* __restrict__ top_p,
    const int* __restrict__ top_k, const long long* __restrict__ seeds,
    const int* __restrict__ steps, const uint32_t* __restrict__ allow_mask, int mask_words) {
  __shared__ SampShared sh;
  __shared__ float chunk_mass[kChunks * kSampThreads];  // 64 KiB
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const T* x = logits + (long)row * logit_stride;
  const uint32_t* mrow = allow_mask ? allow_mask + (long)row * mask_words : nullptr;
  auto chunk_base = [&](int c) { return (tid + c * kSampThreads) * 8; };

  // ---- pass 1: argmax (exact on fp32 input, bf16 keys otherwise) ----------------------
  uint32_t bestk = 0u;
  int besti = 0x7fffffff;
  if constexpr (sizeof(T) == 4) {
    uint32_t best32 = 0u;
#pragma unroll 4
    for (int c = 0; c < kChunks; ++c) {
      const int base = chunk_base(c);
      if (base >= vocab) continue;
      const uint32_t mb = mrow ? (mrow[base >> 5] >> (base & 31)) : 0xFFu;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t u = __float_as_uint(x[base + j]);
        const uint32_t k32 = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        if (((mb >> j) & 1u) && k32 > best32) {
          best32 = k32;
          besti = base + j;
        }
      }
    }
    block_argmax_key(best32, besti, sh);
    const uint32_t bits = (best32 & 0x80000000u) ? (best32 & 0x7fffffffu) : ~best32;
    bestk = bf16_to_key(f32_to_bf16(__uint_as_float(bits)));
  } else {
#pragma unroll 4
    for (int c = 0; c < kChunks; ++c) {
      uint32_t key[8];
      load_keys8<T>(x, mrow, chunk_base(c), vocab, key);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (key[j] > bestk) {
          bestk = key[j];
          besti = chunk_base(c) + j;
        }
    }
    block_argmax_key(bestk, besti, sh);
  }
  const float temp = temperature[row];
  if (temp <= 0.f || besti == 0x7fffffff || bestk <= kNegInfKey) {
    if (tid == 0) out_tokens[row] = (besti == 0x7fffffff) ? 0 : besti;
    return;
  }
  const float M = key_to_f32(bestk);
  const float cexp = 1.4426950408889634f / temp;  // exp(z) = exp2((x - M) * cexp)

  // ---- top-k: 4-ary search on the 16-bit key (2 bits per pass, 8 passes) -------------
  // invariant: count(key >= lo) >= k and the answer -- the largest t with
  // count(key >= t) >= k -- lies in [lo, lo + 4 << shift)
  uint32_t thr = kNegInfKey + 1u;  // keep keys >= thr (drops masked / -inf)
  const int k = top_k[row];
  if (k > 0 && k < vocab) {
    uint32_t lo = 0u;
    for (int shift = 14; shift >= 0; shift -= 2) {
      const uint32_t t1 = lo + (1u << shift), t2 = lo + (2u << shift), t3 = lo + (3u << shift);
      int c1 = 0, c2 = 0, c3 = 0;
#pragma unroll 8
      for (int c = 0; c < kChunks; ++c) {
        uint32_t key[8];
        load_keys8<T>(x, mrow, chunk_base(c), vocab, key);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          c1 += key[j] >= t1 ? 1 : 0;
          c2 += key[j] >= t2 ? 1 : 0;
          c3 += key[j] >= t3 ? 1 : 0;
        }
      }
      block_sum_i3(c1, c2, c3, sh);
      lo = (c3 >= k) ? t3 : (c2 >= k) ? t2 : (c1 >= k) ? t1 : lo;
    }
    if (lo > thr) thr = lo;
  }

  // ---- per-chunk masses of kept tokens (LDS), per-thread totals -------------------------
  float mass = 0.f, excl = 0.f, Z = 0.f;
  auto masses = [&](uint32_t th) {
    mass = 0.f;
#pragma unroll 8
    for (int c = 0; c < kChunks; ++c) {
      uint32_t key[8];
      load_keys8<T>(x, mrow, chunk_base(c), vocab, key);
      float cm = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) cm += key[j] >= th ? exp2f((key_to_f32(key[j]) - M) * cexp) : 0.f;
      chunk_mass[c * kSampThreads + tid] = cm;
      mass += cm;
    }
    // block exclusive scan of per-thread masses
    float incl = mass;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float y = __shfl_up(incl, o, 64);
      if (lane_id() >= o) incl += y;
    }
    __syncthreads();
    if (lane_id() == 63) sh.scan[wave_id()] = incl;
    __syncthreads();
    float wbase = 0.f;
    Z = 0.f;
#pragma unroll
    for (int w = 0; w < kSampWaves; ++w) {
      const float t = sh.scan[w];
      if (w < wave_id()) wbase += t;
      Z += t;
    }
    excl = wbase + incl - mass;
  };
  masses(thr);

  const float tp = top_p[row];
  const uint64_t s0 =
      splitmix64((uint64_t)seeds[row] ^ (0x632BE59BD9B4E019ull * (uint64_t)(steps[row] + 1)));
  int chosen = -1;
  const int rounds = (tp < 1.f) ? 8 : 1;
  // inverse CDF over the kept ids (key >= th) whose chunk masses masses(th) left
  auto draw = [&](uint32_t th, float u) -> int {
    const float target = u * Z;
    __syncthreads();
    if (tid == 0) sh.found = 0;
    __syncthreads();
    // the thread whose [excl, excl + mass) holds the target walks its chunks
    const bool mine = (target >= excl && target < excl + mass) ||
                      (tid == kSampThreads - 1 && target >= excl + mass && mass > 0.f);
    if (mine) {
      // locate the chunk from the LDS chunk masses, then the id inside it
      float acc = excl;
      int cc = -1, lastc = -1;
      for (int c = 0; c < kChunks; ++c) {
        const float cm = chunk_mass[c * kSampThreads + tid];
        if (cm > 0.f) {
          lastc = c;
          if (acc + cm > target) {
            cc = c;
            break;
          }
          acc += cm;
        }
      }
      if (cc < 0) {
        cc = lastc;
        acc = target;  // rounding tail: take the last kept id of the last chunk
      }
      int pick = -1;
      if (cc >= 0) {
        uint32_t key[8];
        load_keys8<T>(x, mrow, chunk_base(cc), vocab, key);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (key[j] >= th) {
            const float pj = exp2f((key_to_f32(key[j]) - M) * cexp);
            pick = chunk_base(cc) + j;
            if (acc + pj > target) break;
            acc += pj;
          }
        }
      }
      if (pick >= 0 && atomicCAS(&sh.found, 0, 1) == 0) sh.winner = pick;
    }
    __syncthreads();
    return sh.found ? sh.winner : besti;
  };
  for (int r = 0; r < rounds; ++r) {
    const uint64_t h = splitmix64(s0 + (uint64_t)r * 0xD1B54A32D192ED03ull);
    const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
    const int s = draw(thr, u);
    if (tp >= 1.f) {
      chosen = s;
      break;
    }
    // nucleus membership: mass of strictly more likely kept tokens < top_p * Z
    uint32_t ks;
    {
      uint32_t key[8];
      load_keys8<T>(x, mrow, s & ~7, vocab, key);
      ks = key[s & 7];
    }
    float above = 0.f;
#pragma unroll 8
    for (int c = 0; c < kChunks; ++c) {
      uint32_t key[8];
      load_keys8<T>(x, mrow, chunk_base(c), vocab, key);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        above += (key[j] > ks && key[j] >= thr) ? exp2f((key_to_f32(key[j]) - M) * cexp) : 0.f;
    }
    above = block_sum_f(above, sh);
    if (above < tp * Z) {
      chosen = s;
      break;
    }
  }
  if (chosen < 0) {
    // every rejection round missed (probability <= (1 - top_p)^8): draw exactly from
    // the nucleus instead of falling back to the argmax.  Nucleus = kept ids with
    // key >= t*, t* = the smallest key t whose strictly-more-likely mass
    // f(t) = mass(key > t) is < top_p * Z; 4-ary search, 3 masses per pass.
    const float tgt = tp * Z;
    uint32_t lo = 0u;   // invariant: f(lo) >= tgt (f(0) = Z)
    for (int shift = 14; shift >= 0; shift -= 2) {
      const uint32_t t1 = lo + (1u << shift), t2 = lo + (2u << shift), t3 = lo + (3u << shift);
      float f1 = 0.f, f2 = 0.f, f3 = 0.f;
#pragma unroll 8
      for (int c = 0; c < kChunks; ++c) {
        uint32_t key[8];
        load_keys8<T>(x, mrow, chunk_base(c), vocab, key);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (key[j] >= thr && key[j] > t1) {
            const float pj = exp2f((key_to_f32(key[j]) - M) * cexp);
            f1 += pj;
            f2 += key[j] > t2 ? pj : 0.f;
            f3 += key[j] > t3 ? pj : 0.f;
          }
        }
      }
      f1 = block_sum_f(f1, sh);
      f2 = block_sum_f(f2, sh);
      f3 = block_sum_f(f3, sh);
      lo = (f3 >= tgt) ? t3 : (f2 >= tgt) ? t2 : (f1 >= tgt) ? t1 : lo;
    }
    const uint32_t tstar = lo + 1u;
    masses(tstar > thr ? tstar : thr);
    const uint64_t h = splitmix64(s0 + 8ull * 0xD1B54A32D192ED03ull);
    chosen = draw(tstar > thr ? tstar : thr, ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f));
  }
  if (tid == 0) out_tokens[row] = chosen;
}

}  // namespace ft

extern "C" int ft_sample(int* out_tokens, const void* logits, int logits_is_bf16, long logit_stride,
                         int batch, int vocab, const float* temperature, const float* top_p,
                         const int* top_k, const long long* seeds, const int* steps,
                         const uint32_t* allow_mask, int mask_words, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (vocab > ft::kSlots * ft::kSampThreads) return -3;
  if (vocab % 8 != 0 || logit_stride % 8 != 0) return -4;
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
