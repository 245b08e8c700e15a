// K12: fused sampler -- constrained-decoding mask, temperature, top-k, top-p
// (nucleus) and the draw.  SURVEY.md §2.4 K12.
//
// Rows without top-k (greedy, temperature, top-p: the serving default) take the
// multi-workgroup path further down (samp_*_kernel: 32 vocabulary slices per row,
// 28.6 vs 84.6 us for top-p at 50 rows, profiles/sampler_probe_r02.log); top-k
// rows and the rare rows whose nucleus candidates were all rejected run the
// one-workgroup-per-row kernel described here.
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

// multi-workgroup sampler (samp_*_kernel below)
constexpr int kSlices = 32;
constexpr int kSlThreads = 256;
// top-k rows with k <= kTopkMax take the multi-workgroup top-k path: each slice
// keeps its own top-k candidates (the global top-k is a subset of their union)
constexpr int kTopkMax = 64;
constexpr int kTopkKept = 256;   // kept set (top-k + ties) the merge kernel holds
static_assert(kTopkKept <= kSlThreads, "one merge thread per kept rank");
// per-row fp32 scratch: slice stats [kSlices][4] (M_p, Z_p, key, id) | M, Z |
// cand (key, id) x kCand | above [kSlices][kCand] | flag | top-k candidate counts
// [kSlices] | top-k candidates [kSlices][kTopkMax] (key, id)
// kCand inverse-CDF candidates per top-p row: all rejected with probability <= (1 - top_p)^kCand
// (1e-4 at top_p 0.9), so the one-workgroup fallback -- a ~30 us tail the whole sampler launch
// waits for -- almost never runs (with 2 candidates: 1% of rows, ~40% of 50-row steps)
constexpr int kCand = 4;
constexpr int kWsStats = 0, kWsMZ = 4 * kSlices, kWsCand = kWsMZ + 2, kWsAbove = kWsCand + 2 * kCand,
              kWsFlag = kWsAbove + kCand * kSlices, kWsTkCnt = kWsFlag + 1,
              kWsTk = kWsTkCnt + kSlices, kWsRow = kWsTk + 2 * kSlices * kTopkMax;

template <typename T>
__global__ __launch_bounds__(kSampThreads) void sample_kernel(
    int* __restrict__ out_tokens, const T* __restrict__ logits, long logit_stride, int vocab,
    const float* __restrict__ temperature, const float* __restrict__ top_p,
    const int* __restrict__ top_k, const long long* __restrict__ seeds,
    const int* __restrict__ steps, const uint32_t* __restrict__ allow_mask, int mask_words,
    const int* __restrict__ flags, int flag_stride) {
  __shared__ SampShared sh;
  __shared__ float chunk_mass[kChunks * kSampThreads];  // 64 KiB
  const int row = blockIdx.x;
  // multi-workgroup path (flags != null): 0 = row already sampled there, 1 = both of
  // its candidates were rejected (run here on fresh uniforms, rounds kCand..), 2 = top-k row
  int fl = flags ? flags[(long)row * flag_stride] : 2;
  if (fl == 0) return;
  if (fl == 3) {
    // accept step of the multi-workgroup path: candidate r is in the nucleus iff the
    // mass strictly above it (samp_above_kernel, per slice) is < top_p * Z
    if (threadIdx.x == 0) {
      const float* wr = reinterpret_cast<const float*>(flags) + (long)row * flag_stride - kWsFlag;
      float a[kCand] = {};
      for (int p = 0; p < kSlices; ++p) {
#pragma unroll
        for (int c = 0; c < kCand; ++c) a[c] += wr[kWsAbove + kCand * p + c];
      }
      const float lim = top_p[row] * wr[kWsMZ + 1];
      int res = 1;
#pragma unroll
      for (int c = 0; c < kCand; ++c) {
        if (res && a[c] < lim) {   // the first accepted candidate is the sample
          out_tokens[row] = FT_CHECK_IDX(__float_as_int(wr[kWsCand + 2 * c + 1]), vocab, kCkSampled, row);
          res = 0;
        }
      }
      sh.winner = res;
    }
    __syncthreads();
    fl = sh.winner;
    __syncthreads();
    if (fl == 0) return;
  }
  const int r0 = fl == 1 ? kCand : 0;
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
    if (tid == 0) out_tokens[row] = FT_CHECK_IDX((besti == 0x7fffffff) ? 0 : besti, vocab, kCkSampled, row);
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
    const uint64_t h = splitmix64(s0 + (uint64_t)(r + r0) * 0xD1B54A32D192ED03ull);
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
    const uint64_t h = splitmix64(s0 + (uint64_t)(8 + r0) * 0xD1B54A32D192ED03ull);
    chosen = draw(tstar > thr ? tstar : thr, ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f));
  }
  if (tid == 0) out_tokens[row] = FT_CHECK_IDX(chosen, vocab, kCkSampled, row);
}

// ---------------------------------------------------------------------------
// Multi-workgroup path for the rows without top-k (the serving default: greedy,
// or temperature + top-p).  One 1024-thread workgroup per row is VALU bound on a
// single CU (every pass is 128k exp2 / compares): 97 us per 50-row step.  Here
// the vocabulary is cut into kSlices slices, each streamed by its own workgroup:
//   K1 slice stats     (rows x kSlices): argmax key / id, and the slice's mass
//                      Z_p = sum exp2((x - M_p) c) relative to its own max M_p
//   K2 draw            (rows): M, Z = sum Z_p 2^((M_p - M) c); greedy rows end
//                      here; kCand inverse-CDF candidates (uniforms u0..u3 of the
//                      same splitmix64 stream): slice by the prefix of the Z_p,
//                      then the id inside that slice (one pass over 1/kSlices)
//   K3 above-mass      (rows x kSlices): per slice, the mass of ids strictly more
//                      likely than each candidate
//   accept             (sample_kernel's first step, rows): candidate r is in the
//                      nucleus iff its above-mass < top_p * Z; the first accepted
//                      one is the sample
// A row whose kCand candidates are all rejected (probability (1 - top_p)^kCand) is
// finished by the one-workgroup kernel on uniforms kCand.. (independent of u0..u3,
// so the mixture is exactly the renormalised nucleus); top-k rows go there too.


__device__ __forceinline__ int slice_len(int vocab) {
  return ((vocab + kSlices * 8 - 1) / (kSlices * 8)) * 8;
}

__device__ __forceinline__ bool topk_row(const int* top_k, int row, int vocab) {
  const int k = top_k[row];
  return k > 0 && k < vocab;
}

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// max over the workgroup (<= 16 waves), s: >= waves ints of LDS
__device__ __forceinline__ uint32_t wave_max_u32_wg(uint32_t v, int* s) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  __syncthreads();
  if (lane_id() == 0) s[wave_id()] = (int)v;
  __syncthreads();
  uint32_t m = 0u;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) m = max(m, (uint32_t)s[w]);
  return m;
}

// top-k rows the multi-workgroup path samples (greedy rows stay on the argmax path)
__device__ __forceinline__ bool mw_topk_row(const int* top_k, const float* temperature, int row,
                                            int vocab) {
  return topk_row(top_k, row, vocab) && top_k[row] <= kTopkMax && temperature[row] > 0.f;
}

// largest t with count(key >= t) >= kk over NK register keys per thread of the
// workgroup (4-ary search on the 16-bit key, 3 counts per pass); kk >= 1
template <int NK>
__device__ __forceinline__ uint32_t wg_kth_key(const uint32_t (&key)[NK], int kk, int* s3) {
  uint32_t t = 0u;
#pragma unroll 1
  for (int shift = 14; shift >= 0; shift -= 2) {
    int c[3] = {0, 0, 0};
#pragma unroll
    for (int j = 0; j < NK; ++j)
#pragma unroll
      for (int q = 0; q < 3; ++q) c[q] += key[j] >= t + ((uint32_t)(q + 1) << shift) ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 3; ++q) c[q] = wave_sum_int(c[q]);
    __syncthreads();
    if (lane_id() == 0)
#pragma unroll
      for (int q = 0; q < 3; ++q) s3[3 * wave_id() + q] = c[q];
    __syncthreads();
    const int nw = blockDim.x >> 6;
    uint32_t nt = t;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      int tot = 0;
      for (int w = 0; w < nw; ++w) tot += s3[3 * w + q];
      if (tot >= kk) nt = t + ((uint32_t)(q + 1) << shift);
    }
    t = nt;
  }
  return t;
}

// (key desc, id asc) argmax over a small workgroup (<= 16 waves) via LDS
__device__ __forceinline__ void wg_argmax(uint32_t& k, int& idx, uint32_t* su, int* si) {
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
    su[wave_id()] = k;
    si[wave_id()] = idx;
  }
  __syncthreads();
  const int nw = blockDim.x >> 6;
  k = su[0];
  idx = si[0];
  for (int w = 1; w < nw; ++w)
    if (su[w] > k || (su[w] == k && si[w] < idx)) {
      k = su[w];
      idx = si[w];
    }
}

__device__ __forceinline__ float wg_sum(float v, float* sf) {
  v = wave_sum(v);
  __syncthreads();
  if (lane_id() == 0) sf[wave_id()] = v;
  __syncthreads();
  float t = 0.f;
  const int nw = blockDim.x >> 6;
  for (int w = 0; w < nw; ++w) t += sf[w];
  return t;
}

template <typename T>
__global__ __launch_bounds__(kSlThreads) void samp_stats_kernel(
    const T* __restrict__ logits, long stride, int vocab, const float* __restrict__ temperature,
    const int* __restrict__ top_k, const uint32_t* __restrict__ allow_mask, int mask_words,
    float* __restrict__ ws) {
  __shared__ uint32_t su[kSlThreads / 64];
  __shared__ int si[kSlThreads / 64];
  __shared__ float sf[kSlThreads / 64];
  __shared__ int s3[3 * (kSlThreads / 64)];
  __shared__ int s_n;
  __shared__ uint32_t s_ck[kTopkMax];
  __shared__ int s_ci[kTopkMax];
  const int row = blockIdx.y, p = blockIdx.x;
  const T* x = logits + (long)row * stride;
  const uint32_t* mrow = allow_mask ? allow_mask + (long)row * mask_words : nullptr;
  const int S = slice_len(vocab);
  const int beg = p * S, end = min(vocab, beg + S);
  if (mw_topk_row(top_k, temperature, row, vocab)) {
    // this slice's top-k candidates: every id whose key is >= the slice's own k-th
    // largest key (ties included); the global k-th largest key is never below it
    static_assert(kSlThreads * 16 >= 4096, "two 8-id chunks per thread cover a slice");
    uint32_t key[16];
    {
      uint32_t a[8], b[8];
      const int b0 = beg + threadIdx.x * 8, b1 = b0 + kSlThreads * 8;
      load_keys8<T>(x, mrow, b0 < end ? b0 : vocab, vocab, a);
      load_keys8<T>(x, mrow, b1 < end ? b1 : vocab, vocab, b);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        key[j] = a[j];
        key[8 + j] = b[j];
      }
    }
    int nv = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) nv += key[j] > kNegInfKey ? 1 : 0;
    nv = wave_sum_int(nv);
    if (lane_id() == 0) s3[wave_id()] = nv;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    int valid = 0;
    for (int w = 0; w < kSlThreads / 64; ++w) valid += s3[w];
    const int kk = min(top_k[row], valid);
    int* cnt = reinterpret_cast<int*>(ws + (long)row * kWsRow + kWsTkCnt);
    if (kk == 0) {
      if (threadIdx.x == 0) cnt[p] = 0;
      return;
    }
    const uint32_t th = max(wg_kth_key<16>(key, kk, s3), kNegInfKey + 1u);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (key[j] >= th) {
        const int slot = atomicAdd(&s_n, 1);
        if (slot < kTopkMax) {
          s_ck[slot] = key[j];
          s_ci[slot] = beg + threadIdx.x * 8 + (j & 7) + (j >> 3) * kSlThreads * 8;
        }
      }
    __syncthreads();
    const int n = s_n;
    float* cand = ws + (long)row * kWsRow + kWsTk + 2 * kTopkMax * p;
    if (threadIdx.x < min(n, kTopkMax)) {
      cand[2 * threadIdx.x] = __uint_as_float(s_ck[threadIdx.x]);
      cand[2 * threadIdx.x + 1] = __int_as_float(s_ci[threadIdx.x]);
    }
    if (threadIdx.x == 0) cnt[p] = n <= kTopkMax ? n : -1;   // -1: ties overflow, one-WG path
    return;
  }
  if (topk_row(top_k, row, vocab)) return;
  // argmax: exact on fp32 input (32-bit ordered keys, masked ids excluded), bf16 keys
  // otherwise -- the same rule as sample_kernel's pass 1
  uint32_t best = 0u;
  int besti = 0x7fffffff;
  for (int base = beg + threadIdx.x * 8; base < end; base += kSlThreads * 8) {
    if constexpr (sizeof(T) == 4) {
      const uint32_t mb = mrow ? (mrow[base >> 5] >> (base & 31)) : 0xFFu;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t u = __float_as_uint(x[base + j]);
        const uint32_t k32 = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
        if (((mb >> j) & 1u) && k32 > best) {
          best = k32;
          besti = base + j;
        }
      }
    } else {
      uint32_t key[8];
      load_keys8<T>(x, mrow, base, vocab, key);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (key[j] > best) {
          best = key[j];
          besti = base + j;
        }
    }
  }
  wg_argmax(best, besti, su, si);
  uint32_t bestk = best;
  if constexpr (sizeof(T) == 4) {
    const uint32_t bits = (best & 0x80000000u) ? (best & 0x7fffffffu) : ~best;
    bestk = best ? bf16_to_key(f32_to_bf16(__uint_as_float(bits))) : 0u;
  }
  float* st = ws + (long)row * kWsRow + kWsStats + 4 * p;
  const float temp = temperature[row];
  float Mp = -INFINITY, Zp = 0.f;
  if (temp > 0.f && besti != 0x7fffffff && bestk > kNegInfKey) {
    Mp = key_to_f32(bestk);
    const float cexp = 1.4426950408889634f / temp;
    float z = 0.f;
    for (int base = beg + threadIdx.x * 8; base < end; base += kSlThreads * 8) {
      uint32_t key[8];
      load_keys8<T>(x, mrow, base, vocab, key);
#pragma unroll
      for (int j = 0; j < 8; ++j) z += key[j] > kNegInfKey ? exp2f((key_to_f32(key[j]) - Mp) * cexp) : 0.f;
    }
    Zp = wg_sum(z, sf);
  }
  if (threadIdx.x == 0) {
    st[0] = Mp;
    st[1] = Zp;
    st[2] = __uint_as_float(best);   // 32-bit key (fp32 input) or 16-bit key
    st[3] = __int_as_float(besti);
  }
}

template <typename T>
__global__ __launch_bounds__(kSampThreads) void samp_draw_kernel(
    int* __restrict__ out_tokens, const T* __restrict__ logits, long stride, int vocab,
    const float* __restrict__ temperature, const float* __restrict__ top_p,
    const int* __restrict__ top_k, const long long* __restrict__ seeds,
    const int* __restrict__ steps, const uint32_t* __restrict__ allow_mask, int mask_words,
    float* __restrict__ ws) {
  static_assert(kSlices <= 64, "one lane per slice");
  // top-p rows: candidate r is searched by threads [r * per, (r + 1) * per), per = kSampThreads /
  // kCand; without a nucleus only candidate 0 is drawn, by the whole workgroup
  __shared__ float s_scan[kSampThreads / 64];
  __shared__ float s_M, s_cexp, s_tgt[kCand];
  __shared__ int s_ps[kCand], s_done, s_last[kCand], s_found[kCand];
  const int row = blockIdx.x, tid = threadIdx.x, lane = lane_id();
  float* wr = ws + (long)row * kWsRow;
  int* flag = reinterpret_cast<int*>(wr + kWsFlag);
  if (topk_row(top_k, row, vocab)) {
    // multi-workgroup top-k rows: samp_topk_kernel sets the flag; others: one-WG path
    if (tid == 0 && !mw_topk_row(top_k, temperature, row, vocab)) *flag = 2;
    return;
  }
  const float tp = top_p[row];
  if (wave_id() == 0) {
    // lane p: slice p's stats; argmax (key desc, id asc), global max, masses
    uint32_t k = 0u;
    int i = 0x7fffffff;
    float Mp = -INFINITY, Zp = 0.f;
    if (lane < kSlices) {
      const float4 st = *reinterpret_cast<const float4*>(wr + kWsStats + 4 * lane);
      Mp = st.x;
      Zp = st.y;
      k = __float_as_uint(st.z);
      i = __float_as_int(st.w);
    }
    uint32_t best = k;
    int besti = i;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint32_t ok = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(besti, o, 64);
      if (ok > best || (ok == best && oi < besti)) {
        best = ok;
        besti = oi;
      }
    }
    const float M = wave_max(Mp);
    uint32_t bestk = best;
    if constexpr (sizeof(T) == 4) {
      const uint32_t bits = (best & 0x80000000u) ? (best & 0x7fffffffu) : ~best;
      bestk = best ? bf16_to_key(f32_to_bf16(__uint_as_float(bits))) : 0u;
    }
    const float temp = temperature[row];
    const bool done = temp <= 0.f || besti == 0x7fffffff || bestk <= kNegInfKey;
    if (done) {
      if (lane == 0) {
        out_tokens[row] = FT_CHECK_IDX((besti == 0x7fffffff) ? 0 : besti, vocab, kCkSampled, row);
        *flag = 0;
        s_done = 1;
      }
    } else {
      const float cexp = 1.4426950408889634f / temp;
      const float zp = Mp == -INFINITY ? 0.f : Zp * exp2f((Mp - M) * cexp);
      float incl = zp;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const float y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      const float Z = __shfl(incl, 63, 64);
      const uint64_t lastmask = __builtin_amdgcn_ballot_w64(zp > 0.f);
      const int lastp = lastmask ? 63 - __builtin_clzll(lastmask) : 0;
      const uint64_t s0 =
          splitmix64((uint64_t)seeds[row] ^ (0x632BE59BD9B4E019ull * (uint64_t)(steps[row] + 1)));
#pragma unroll
      for (int r = 0; r < kCand; ++r) {
        const uint64_t h = splitmix64(s0 + (uint64_t)r * 0xD1B54A32D192ED03ull);
        const float u = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f);
        const float T0 = u * Z;
        // first slice whose inclusive prefix passes the target; rounding tail: the
        // last slice with mass, at its end
        const uint64_t hit = __builtin_amdgcn_ballot_w64(zp > 0.f && incl > T0);
        const int ps = hit ? __builtin_ctzll(hit) : lastp;
        const float base = __shfl(incl - zp, ps, 64);
        const float tgt = hit ? T0 - base : __shfl(zp, ps, 64);
        if (lane == 0) {
          s_ps[r] = ps;
          s_tgt[r] = tgt;
        }
      }
      if (lane == 0) {
        s_M = M;
        s_cexp = cexp;
        s_done = 0;
        wr[kWsMZ] = M;
        wr[kWsMZ + 1] = Z;
#pragma unroll
        for (int c = 0; c < kCand; ++c) {   // defined even if a search finds nothing
          wr[kWsCand + 2 * c] = __uint_as_float(bestk);
          wr[kWsCand + 2 * c + 1] = __int_as_float(besti);
        }
      }
    }
  }
  if (tid < kCand) {
    s_last[tid] = -1;
    s_found[tid] = 0;
  }
  __syncthreads();
  if (s_done) return;
  // inverse CDF inside the chosen slice, all candidates at once (kSampThreads / kCand each),
  // in (thread, chunk, id) order; the first chunk's keys stay in registers
  const int per = tp < 1.f ? kSampThreads / kCand : kSampThreads;
  const int r = tid / per, lt = tid - r * per, w = lt >> 6;
  float* scan = s_scan + r * (per >> 6);
  const float M = s_M, cexp = s_cexp, tgt = s_tgt[r];
  const int S = slice_len(vocab);
  const int beg = s_ps[r] * S, end = min(vocab, beg + S);
  const uint32_t* mrow = allow_mask ? allow_mask + (long)row * mask_words : nullptr;
  const T* x = logits + (long)row * stride;
  uint32_t k0[8];
  float mass = 0.f;
  {
    load_keys8<T>(x, mrow, beg + lt * 8 < end ? beg + lt * 8 : vocab, vocab, k0);
#pragma unroll
    for (int j = 0; j < 8; ++j) mass += k0[j] > kNegInfKey ? exp2f((key_to_f32(k0[j]) - M) * cexp) : 0.f;
    for (int b2 = beg + (lt + per) * 8; b2 < end; b2 += per * 8) {
      uint32_t key[8];
      load_keys8<T>(x, mrow, b2, vocab, key);
#pragma unroll
      for (int j = 0; j < 8; ++j) mass += key[j] > kNegInfKey ? exp2f((key_to_f32(key[j]) - M) * cexp) : 0.f;
    }
  }
  float incl = mass;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) scan[w] = incl;
  if (mass > 0.f) atomicMax(&s_last[r], lt);
  __syncthreads();
  float wbase = 0.f;
  for (int w2 = 0; w2 < w; ++w2) wbase += scan[w2];
  const float excl = wbase + incl - mass;
  const bool mine = mass > 0.f &&
                    ((tgt >= excl && tgt < excl + mass) || (lt == s_last[r] && tgt >= excl + mass));
  if (mine) {
    float a = excl;
    int pick = -1, lastk = -1;
    uint32_t pk = 0u, lastkey = 0u;
    auto walk = [&](const uint32_t (&key)[8], int base) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (pick < 0 && key[j] > kNegInfKey) {
          const float pj = exp2f((key_to_f32(key[j]) - M) * cexp);
          lastk = base + j;
          lastkey = key[j];
          if (a + pj > tgt) {
            pick = base + j;
            pk = key[j];
          }
          a += pj;
        }
      }
    };
    walk(k0, beg + lt * 8);
    for (int b2 = beg + (lt + per) * 8; pick < 0 && b2 < end; b2 += per * 8) {
      uint32_t key[8];
      load_keys8<T>(x, mrow, b2, vocab, key);
      walk(key, b2);
    }
    if (pick < 0) {   // rounding tail: this thread's last kept id
      pick = lastk;
      pk = lastkey;
    }
    if (pick >= 0 && atomicCAS(&s_found[r], 0, 1) == 0) {
      wr[kWsCand + 2 * r] = __uint_as_float(pk);
      wr[kWsCand + 2 * r + 1] = __int_as_float(pick);
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (tp >= 1.f) {   // no nucleus: the first draw is the sample
      out_tokens[row] = FT_CHECK_IDX(__float_as_int(wr[kWsCand + 1]), vocab, kCkSampled, row);
      *flag = 0;
    } else {
      *flag = 3;   // samp_above_kernel + the accept step decide
    }
  }
}

template <typename T>
__global__ __launch_bounds__(kSlThreads) void samp_above_kernel(
    const T* __restrict__ logits, long stride, int vocab, const float* __restrict__ temperature,
    const uint32_t* __restrict__ allow_mask, int mask_words, float* __restrict__ ws) {
  __shared__ float sf[kSlThreads / 64];
  const int row = blockIdx.y, p = blockIdx.x;
  float* wr = ws + (long)row * kWsRow;
  if (*reinterpret_cast<const int*>(wr + kWsFlag) != 3) return;
  const T* x = logits + (long)row * stride;
  const uint32_t* mrow = allow_mask ? allow_mask + (long)row * mask_words : nullptr;
  const float M = wr[kWsMZ];
  const float cexp = 1.4426950408889634f / temperature[row];
  uint32_t kc[kCand], kmin = 0xffffffffu;
#pragma unroll
  for (int c = 0; c < kCand; ++c) {
    kc[c] = __float_as_uint(wr[kWsCand + 2 * c]);
    kmin = min(kmin, kc[c]);
  }
  const int S = slice_len(vocab);
  const int beg = p * S, end = min(vocab, beg + S);
  float a[kCand] = {};
  for (int base = beg + threadIdx.x * 8; base < end; base += kSlThreads * 8) {
    uint32_t key[8];
    load_keys8<T>(x, mrow, base, vocab, key);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float e = key[j] > kmin ? exp2f((key_to_f32(key[j]) - M) * cexp) : 0.f;
#pragma unroll
      for (int c = 0; c < kCand; ++c) a[c] += key[j] > kc[c] ? e : 0.f;
    }
  }
#pragma unroll
  for (int c = 0; c < kCand; ++c) {
    a[c] = wg_sum(a[c], sf);
    if (threadIdx.x == 0) wr[kWsAbove + kCand * p + c] = a[c];
  }
}

// Top-k rows (k <= kTopkMax, temperature > 0), one workgroup per row: merge the
// slices' candidates, keep key >= t* (t* = largest key with count(key >= t*) >= k,
// the single-workgroup kernel's rule: ties at the threshold stay), then top-p over
// the kept ids (an id is in the nucleus iff the mass of strictly more likely kept
// ids is < top_p * Z) and one inverse-CDF draw in (key desc, id asc) order over a
// rank-ordered prefix sum -- deterministic whatever order the candidates were
// appended in.  Rows whose
// candidates or kept set overflow go to the one-workgroup kernel (flag 2).
__global__ __launch_bounds__(kSlThreads) void samp_topk_kernel(
    int* __restrict__ out_tokens, int vocab, const float* __restrict__ temperature,
    const float* __restrict__ top_p, const int* __restrict__ top_k,
    const long long* __restrict__ seeds, const int* __restrict__ steps, float* __restrict__ ws) {
  constexpr int NC = kSlices * kTopkMax / kSlThreads;   // candidates per thread
  __shared__ int s_off[kSlices + 1];
  __shared__ int s3[3 * (kSlThreads / 64)];
  __shared__ float sf[kSlThreads / 64];
  __shared__ int s_nk, s_bad, s_pick, s_last;
  __shared__ uint32_t s_k[kTopkKept];
  __shared__ int s_i[kTopkKept];
  __shared__ float s_e[kTopkKept];
  __shared__ float s_c[kTopkKept];
  const int row = blockIdx.x, tid = threadIdx.x;
  if (!mw_topk_row(top_k, temperature, row, vocab)) return;
  float* wr = ws + (long)row * kWsRow;
  int* flag = reinterpret_cast<int*>(wr + kWsFlag);
  const int* cnt = reinterpret_cast<const int*>(wr + kWsTkCnt);
  if (tid == 0) {
    int o = 0, bad = 0;
    for (int p = 0; p < kSlices; ++p) {
      s_off[p] = o;
      bad |= cnt[p] < 0;
      o += max(cnt[p], 0);
    }
    s_off[kSlices] = o;
    s_bad = bad;
    s_nk = 0;
    s_pick = -1;
    s_last = -1;
  }
  __syncthreads();
  if (s_bad) {
    if (tid == 0) *flag = 2;
    return;
  }
  const int C = s_off[kSlices];
  uint32_t key[NC];
  int id[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = tid + kSlThreads * j;
    key[j] = 0u;
    id[j] = 0;
    if (c < C) {
      int p = 0;
      while (s_off[p + 1] <= c) ++p;
      const float* e = wr + kWsTk + 2 * kTopkMax * p + 2 * (c - s_off[p]);
      key[j] = __float_as_uint(e[0]);
      id[j] = __float_as_int(e[1]);
    }
  }
  const int kk = min(top_k[row], C);
  if (kk == 0) {   // everything masked
    if (tid == 0) {
      out_tokens[row] = FT_CHECK_IDX(0, vocab, kCkSampled, row);
      *flag = 0;
    }
    return;
  }
  const uint32_t th = wg_kth_key<NC>(key, kk, s3);
#pragma unroll
  for (int j = 0; j < NC; ++j)
    if (key[j] >= th && key[j] > kNegInfKey) {
      const int slot = atomicAdd(&s_nk, 1);
      if (slot < kTopkKept) {
        s_k[slot] = key[j];
        s_i[slot] = id[j];
      }
    }
  __syncthreads();
  const int nk = s_nk;
  if (nk > kTopkKept) {
    if (tid == 0) *flag = 2;
    return;
  }
  const float cexp = 1.4426950408889634f / temperature[row];
  const uint32_t kmax = wave_max_u32_wg(tid < nk ? s_k[tid] : 0u, s3);
  const float M = key_to_f32(kmax);
  const float e = tid < nk ? exp2f((key_to_f32(s_k[tid]) - M) * cexp) : 0.f;
  if (tid < nk) s_e[tid] = e;
  const float Z = wg_sum(e, sf);   // (its barriers also publish s_e)
  const float tp = top_p[row];
  // strictly-more-likely mass and (key desc, id asc) rank of this thread's kept id
  float above = 0.f;
  int rank = 0;
  const uint32_t mk = tid < nk ? s_k[tid] : 0u;
  const int mi = tid < nk ? s_i[tid] : 0;
  for (int j = 0; j < nk; ++j) {
    const uint32_t kj = s_k[j];
    if (kj > mk) above += s_e[j];
    rank += (kj > mk || (kj == mk && s_i[j] < mi)) ? 1 : 0;
  }
  const bool member = tid < nk && (tp >= 1.f || above < tp * Z);
  __syncthreads();
  // nucleus masses in (key desc, id asc) rank order (the ranks are a permutation of
  // 0..nk-1), then ONE prefix sum over that order: the members' intervals
  // [cum, cum + e) tile [0, Zn) exactly and every sum has a fixed order, whatever
  // order the candidates were appended in (a seeded draw reproduces bit for bit)
  if (tid < nk) s_e[rank] = member ? e : 0.f;
  __syncthreads();
  float incl = tid < nk ? s_e[tid] : 0.f;   // the mass of rank tid, then its inclusive prefix
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float y = __shfl_up(incl, o, 64);
    if (lane_id() >= o) incl += y;
  }
  if (lane_id() == 63) sf[wave_id()] = incl;
  __syncthreads();
  float wbase = 0.f;
  for (int w = 0; w < wave_id(); ++w) wbase += sf[w];
  float Zn = 0.f;
  for (int w = 0; w < kSlThreads / 64; ++w) Zn += sf[w];
  float excl = __shfl_up(incl, 1, 64);
  if (lane_id() == 0) excl = 0.f;
  // the start of rank tid's interval; an interval ends where the next one starts, so
  // consecutive boundaries tile [0, Zn) with no gap or overlap under any rounding
  if (tid < nk) s_c[tid] = wbase + excl;
  __syncthreads();
  const float cum = member ? s_c[rank] : 0.f;
  const uint64_t s0 =
      splitmix64((uint64_t)seeds[row] ^ (0x632BE59BD9B4E019ull * (uint64_t)(steps[row] + 1)));
  const uint64_t h = splitmix64(s0);
  const float T = ((float)(h >> 40) + 0.5f) * (1.0f / 16777216.0f) * Zn;
  const float hi = rank + 1 < nk ? s_c[rank + 1] : Zn;   // the next rank's start
  if (member && e > 0.f && T >= cum && T < hi) s_pick = mi;
  if (member) atomicMax(&s_last, rank);   // rounding tail: the last-ranked member
  __syncthreads();
  if (s_pick < 0 && member && rank == s_last) s_pick = mi;
  __syncthreads();
  if (tid == 0) {
    out_tokens[row] = FT_CHECK_IDX(s_pick, vocab, kCkSampled, row);
    *flag = 0;
  }
}

}  // namespace ft

extern "C" int ft_sample_ws_floats() { return ft::kWsRow; }

extern "C" int ft_sample(int* out_tokens, const void* logits, int logits_is_bf16, long logit_stride,
                         int batch, int vocab, const float* temperature, const float* top_p,
                         const int* top_k, const long long* seeds, const int* steps,
                         const uint32_t* allow_mask, int mask_words, float* ws, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (vocab > ft::kSlots * ft::kSampThreads) return -3;
  if (vocab % 8 != 0 || logit_stride % 8 != 0) return -4;
  int* flags = nullptr;
  // ws (batch * ft_sample_ws_floats() fp32): the multi-workgroup path for every row
  // without top-k, then the one-workgroup kernel only for top-k and fallback rows
#define FT_SAMPLE_ALL(TT)                                                                       \
  {                                                                                             \
    const TT* lg = (const TT*)logits;                                                           \
    if (ws != nullptr) {                                                                        \
      hipLaunchKernelGGL(ft::samp_stats_kernel<TT>, dim3(ft::kSlices, batch), dim3(ft::kSlThreads),\
                         0, stream, lg, logit_stride, vocab, temperature, top_k, allow_mask,     \
                         mask_words, ws);                                                        \
      hipLaunchKernelGGL(ft::samp_draw_kernel<TT>, dim3(batch), dim3(ft::kSampThreads), 0, stream,\
                         out_tokens, lg, logit_stride, vocab, temperature, top_p, top_k, seeds,  \
                         steps, allow_mask, mask_words, ws);                                     \
      hipLaunchKernelGGL(ft::samp_above_kernel<TT>, dim3(ft::kSlices, batch), dim3(ft::kSlThreads),\
                         0, stream, lg, logit_stride, vocab, temperature, allow_mask, mask_words, \
                         ws);                                                                    \
      hipLaunchKernelGGL(ft::samp_topk_kernel, dim3(batch), dim3(ft::kSlThreads), 0, stream,     \
                         out_tokens, vocab, temperature, top_p, top_k, seeds, steps, ws);        \
      flags = reinterpret_cast<int*>(ws + ft::kWsFlag);                                          \
    }                                                                                            \
  }
  if (logits_is_bf16) FT_SAMPLE_ALL(uint16_t) else FT_SAMPLE_ALL(float)
#undef FT_SAMPLE_ALL
  dim3 grid(batch), block(ft::kSampThreads);
  if (logits_is_bf16) {
    hipLaunchKernelGGL(ft::sample_kernel<uint16_t>, grid, block, 0, stream, out_tokens,
                       (const uint16_t*)logits, logit_stride, vocab, temperature, top_p, top_k,
                       seeds, steps, allow_mask, mask_words, (const int*)flags, ft::kWsRow);
  } else {
    hipLaunchKernelGGL(ft::sample_kernel<float>, grid, block, 0, stream, out_tokens,
                       (const float*)logits, logit_stride, vocab, temperature, top_p, top_k,
                       seeds, steps, allow_mask, mask_words, (const int*)flags, ft::kWsRow);
  }
  return static_cast<int>(hipGetLastError());
}

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(sampling)
