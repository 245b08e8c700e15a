// K6: paged decode attention (one query token per sequence), split-K
// ("flash-decoding") with an optional combine kernel.  SURVEY.md §2.4 K6.
//
// Decode attention is an HBM stream over the KV cache (4 KiB per token per layer
// for Llama-3-8B); the kernel is designed around bytes in flight and a short
// dependent-latency chain per workgroup, not FLOPs:
//   * grid = (seq * kv_head, split).  Split s of a sequence of length L owns the
//     token range [s*P, (s+1)*P), P = roundup16(ceil(L / splits)): every sequence
//     is cut into `splits` near-equal partitions whatever its length, so the grid
//     depends only on (batch bucket, splits) and ONE hipGraph per batch bucket
//     covers every context length.  There is no upper bound on P (no LDS score
//     buffer): the host picks `splits` only to fill the chip.
//   * a workgroup computes all G = nq/nkv query heads of its kv head (GQA
//     packing: every K/V byte is read once per step).
//   * the 4 waves take interleaved 16-token tiles (one aligned piece of one KV
//     block each) and run an independent online softmax (exp2 domain).  The KV
//     offsets of a wave's next 64 tiles come from ONE block-table load (lane i
//     holds tile i's, read back with v_readlane), and the tiles are double
//     buffered in registers, so after the prologue every K/V round trip overlaps
//     the previous tile's math instead of following a block-table read.
//   * QK^T: 16 lanes share a token (8 head dims each); q stays packed bf16 and
//     the dot is v_dot2_f32_bf16 on the raw K words (no K unpacking); the
//     16-lane sum is 4 DPP adds (quad_perm, row_half_mirror, row_mirror), no
//     LDS traffic.  P.V accumulates fp32 in registers.
//   * the waves' (m, l, acc) merge through LDS; a partition that is the whole
//     sequence writes bf16 output directly, otherwise fp32 partials + (m, l) for
//     the combine kernel (launched only when splits > 1).
#include "ft_common.h"

namespace ft {

typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int decode_part(int L, int splits) {
  const int p = (L + splits - 1) / splits;
  return max(16, (p + 15) & ~15);
}

__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a),
                                         __builtin_bit_cast(bf16x2_t, b), c, false);
}

// sum over aligned groups of LPT (8 or 16) lanes; every lane gets the group sum
template <int LPT>
__device__ __forceinline__ float lane_group_sum(float v) {
  v += __builtin_amdgcn_update_dpp(0.f, v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0.f, v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0.f, v, 0x141, 0xf, 0xf, false);  // row_half_mirror
  if constexpr (LPT == 16) v += __builtin_amdgcn_update_dpp(0.f, v, 0x140, 0xf, 0xf, false);
  return v;
}

// reduce across the token groups of a wave (lanes differing above log2(LPT))
template <int LPT>
__device__ __forceinline__ float token_group_max(float v) {
#pragma unroll
  for (int o = LPT; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
template <int LPT>
__device__ __forceinline__ float token_group_sum(float v) {
#pragma unroll
  for (int o = LPT; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// one wave tile = 16 consecutive tokens = one aligned 16-token piece of one KV
// block (block_size is a power of two >= 16 and partitions start at multiples
// of 16), so a tile needs exactly one block-table entry.
template <int D, int G>
struct DecTile {
  static constexpr int LPT = D / 8;      // lanes per token
  static constexpr int TPW = 64 / LPT;   // tokens per wave instruction
  static constexpr int U = 16 / TPW;     // loads of K (and of V) per lane per tile
  uint4 k[U], v[U];
};

template <int D, int G>
__device__ __forceinline__ void dec_load_tile(DecTile<D, G>& t, const uint16_t* __restrict__ k_cache,
                                              const uint16_t* __restrict__ v_cache, size_t base,
                                              int valid_tokens, int ts, int c) {
  using T = DecTile<D, G>;
  // unconditional loads (slots past the end re-read the last valid token and
  // are masked in dec_consume_tile): a uniform load count lets the compiler
  // wait with exact vmcnt values instead of draining at a branch merge
#pragma unroll
  for (int u = 0; u < T::U; ++u) {
    const int tl = min(u * T::TPW + ts, valid_tokens - 1);
    const size_t off = base + (size_t)tl * D;
    t.k[u] = reinterpret_cast<const uint4*>(k_cache + off)[c];
    t.v[u] = reinterpret_cast<const uint4*>(v_cache + off)[c];
  }
}

template <int D, int G>
__device__ __forceinline__ void dec_consume_tile(const DecTile<D, G>& t, const uint4 (&qp)[G],
                                                 int valid_tokens, int ts, float scale_log2,
                                                 float (&m)[G], float (&l)[G], float (&acc)[G][8]) {
  using T = DecTile<D, G>;
  constexpr int U = T::U, LPT = T::LPT;
  float s[U][G];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const bool valid = u * T::TPW + ts < valid_tokens;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float d = dot2_bf16(t.k[u].x, qp[g].x, 0.f);
      d = dot2_bf16(t.k[u].y, qp[g].y, d);
      d = dot2_bf16(t.k[u].z, qp[g].z, d);
      d = dot2_bf16(t.k[u].w, qp[g].w, d);
      d = lane_group_sum<LPT>(d);
      s[u][g] = valid ? d * scale_log2 : -INFINITY;
    }
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    float tm = s[0][g];
#pragma unroll
    for (int u = 1; u < U; ++u) tm = fmaxf(tm, s[u][g]);
    tm = token_group_max<LPT>(tm);
    const float mn = fmaxf(m[g], tm);
    const float alpha = exp2f(m[g] - mn);
    m[g] = mn;
    l[g] *= alpha;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] *= alpha;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      s[u][g] = exp2f(s[u][g] - mn);
      l[g] += s[u][g];
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float vf[8];
    load8(t.v[u], vf);
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[g][j] += s[u][g] * vf[j];
  }
}

template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_kernel(
    uint16_t* __restrict__ out, int out_stride, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, const uint16_t* __restrict__ q, int q_stride,
    const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    int nkv, int bs_shift, int max_splits, float scale_log2) {
  using T = DecTile<D, G>;
  constexpr int LPT = T::LPT;
  __shared__ float s_acc[4][G][D];
  __shared__ float s_m[4][G], s_l[4][G];

  const int b = blockIdx.x / nkv;
  const int kvh = blockIdx.x - b * nkv;
  const int split = blockIdx.y;
  const int L = seq_lens[b];
  const int PART = decode_part(L, max_splits);
  const int start = split * PART;
  if (start >= L) return;
  const int n = min(L - start, PART);
  const int nsplit = (L + PART - 1) / PART;
  const int nq = nkv * G;
  const int bmask = (1 << bs_shift) - 1;

  const int lane = lane_id(), wave = wave_id();
  const int c = lane % LPT;       // 8-dim chunk owned by this lane
  const int ts = lane / LPT;      // token slot within a wave instruction

  uint4 qp[G];
#pragma unroll
  for (int g = 0; g < G; ++g)
    qp[g] = reinterpret_cast<const uint4*>(q + (size_t)b * q_stride + (kvh * G + g) * D)[c];

  const int* bt = block_tables + (size_t)b * bt_stride;
  const size_t head_off = (size_t)kvh * (bmask + 1) * D;
  const size_t blk_stride = (size_t)nkv * (bmask + 1) * D;

  float m[G], l[G], acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;
  }

  // this wave's tiles: i = 0.. with first token start + 16*(wave + 4 i).  The
  // KV-cache base offset of 64 consecutive tiles is fetched in ONE load (lane i
  // holds tile i's), so the K/V loads never wait on a block-table read.
  const int ntiles = (n + 15) >> 4;
  const int my_tiles = ntiles > wave ? (ntiles - wave + 3) >> 2 : 0;
  for (int c0 = 0; c0 < my_tiles; c0 += 64) {
    const int cnt = min(64, my_tiles - c0);
    size_t my_base = 0;
    if (lane < cnt) {
      const int tok = start + 16 * (wave + 4 * (c0 + lane));
      my_base = (size_t)bt[tok >> bs_shift] * blk_stride + head_off + (size_t)(tok & bmask) * D;
    }
    auto tile_base = [&](int i) -> size_t {
      const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)my_base, i);
      const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(my_base >> 32), i);
      return ((size_t)hi << 32) | lo;
    };
    auto tile_valid = [&](int i) { return n - 16 * (wave + 4 * (c0 + i)); };
    // double-buffered: tile i+1's K/V loads are in flight while tile i computes
    // (a prefetch index past the end re-loads the last tile: L2 hit, never consumed)
    auto ld = [&](DecTile<D, G>& t, int i) {
      const int j = min(i, cnt - 1);
      dec_load_tile<D, G>(t, k_cache, v_cache, tile_base(j), tile_valid(j), ts, c);
    };
    DecTile<D, G> ta, tb;
    ld(ta, 0);
    int i = 0;
    // sched_barrier(0) keeps each prefetch ahead of the math it overlaps
    for (; i + 1 < cnt; i += 2) {
      ld(tb, i + 1);
      __builtin_amdgcn_sched_barrier(0);
      dec_consume_tile<D, G>(ta, qp, tile_valid(i), ts, scale_log2, m, l, acc);
      __builtin_amdgcn_sched_barrier(0);
      ld(ta, i + 2);
      __builtin_amdgcn_sched_barrier(0);
      dec_consume_tile<D, G>(tb, qp, tile_valid(i + 1), ts, scale_log2, m, l, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (i < cnt) dec_consume_tile<D, G>(ta, qp, tile_valid(i), ts, scale_log2, m, l, acc);
  }

  // ---- merge token slots of the wave, then the 4 waves ---------------------------
#pragma unroll
  for (int g = 0; g < G; ++g) {
    l[g] = token_group_sum<LPT>(l[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = token_group_sum<LPT>(acc[g][j]);
  }
  if (lane < LPT) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_acc[wave][g][c * 8 + j] = acc[g][j];
      if (lane == 0) {
        s_m[wave][g] = m[g];
        s_l[wave][g] = l[g];
      }
    }
  }
  __syncthreads();

  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int g = i / D, d = i - g * D;
    float M = s_m[0][g];
#pragma unroll
    for (int w = 1; w < 4; ++w) M = fmaxf(M, s_m[w][g]);
    float num = 0.f, den = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float e = (s_l[w][g] > 0.f) ? exp2f(s_m[w][g] - M) : 0.f;
      num += e * s_acc[w][g][d];
      den += e * s_l[w][g];
    }
    const int h = kvh * G + g;
    if (nsplit == 1) {
      out[(size_t)b * out_stride + h * D + d] = f32_to_bf16(num / den);
    } else {
      const size_t o = ((size_t)b * nq + h) * max_splits + split;
      tmp_out[o * D + d] = num;
      if (d == 0) {
        tmp_ml[o * 2] = M;
        tmp_ml[o * 2 + 1] = den;
      }
    }
  }
}

// One workgroup per (sequence, q head): wave 0 turns the partitions' (m, l) into
// merge weights (lane s = partition s, wave-wide max / sum), then every thread
// sums its head dim over the partitions with 16 loads in flight (clamped
// indices, zero weights past the end) -- the merge is a handful of dependent
// round trips, not one per partition.
template <int D>
__global__ __launch_bounds__(D) void paged_decode_combine_kernel(
    uint16_t* __restrict__ out, int out_stride, const float* __restrict__ tmp_out,
    const float* __restrict__ tmp_ml, const int* __restrict__ seq_lens, int nq, int max_splits) {
  const int b = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  const int L = seq_lens[b];
  const int part = decode_part(L, max_splits);
  const int ns = (L + part - 1) / part;
  if (ns <= 1) return;
  __shared__ float s_w[64];
  const size_t base = ((size_t)b * nq + h) * max_splits;
  if (d < 64) {  // max_splits <= 64 (checked by the launcher)
    const float ms = d < ns ? tmp_ml[(base + d) * 2] : -INFINITY;
    const float ls = d < ns ? tmp_ml[(base + d) * 2 + 1] : 0.f;
    float M = ms;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    const float w = d < ns ? exp2f(ms - M) : 0.f;
    float den = w * ls;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) den += __shfl_xor(den, o, 64);
    s_w[d] = w / den;
  }
  __syncthreads();
  const float* src = tmp_out + base * D + d;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < ns; s0 += 16) {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = src[(size_t)min(s0 + u, ns - 1) * D];
#pragma unroll
    for (int u = 0; u < 16; ++u) acc[u & 3] += (s0 + u < ns ? s_w[s0 + u] : 0.f) * v[u];
  }
  out[(size_t)b * out_stride + h * D + d] = f32_to_bf16((acc[0] + acc[1]) + (acc[2] + acc[3]));
}

}  // namespace ft

// partitions are unbounded (online softmax): any splits >= 1 covers any length
extern "C" int ft_decode_partition_size() { return 1 << 30; }

extern "C" int ft_paged_decode_attention(void* out, int out_stride, float* tmp_out, float* tmp_ml,
                                         const void* q, int q_stride, const void* k_cache,
                                         const void* v_cache, const int* block_tables,
                                         int bt_stride, const int* seq_lens, int batch, int nq,
                                         int nkv, int head_dim, int block_size, int max_splits,
                                         float scale, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (nq % nkv != 0) return -1;
  if (max_splits < 1 || max_splits > 64) return -3;
  if (block_size < 16 || (block_size & (block_size - 1))) return -4;
  const int bs_shift = __builtin_ctz(block_size);
  const int G = nq / nkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(batch * nkv, max_splits), block(256);
#define FT_DEC_CASE(DD, GG)                                                                  \
  if (head_dim == DD && G == GG) {                                                               \
    hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG>), grid, block, 0, stream,            \
                       (uint16_t*)out, out_stride, tmp_out, tmp_ml, (const uint16_t*)q,          \
                       q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,             \
                       block_tables, bt_stride, seq_lens, nkv, bs_shift, max_splits, scale_log2); \
    if (max_splits > 1)                                                                          \
      hipLaunchKernelGGL((ft::paged_decode_combine_kernel<DD>), dim3(batch, nq), dim3(DD), 0,    \
                         stream, (uint16_t*)out, out_stride, tmp_out, tmp_ml, seq_lens, nq,      \
                         max_splits);                                                            \
    return static_cast<int>(hipGetLastError());                                                  \
  }
  FT_DEC_CASE(128, 1)
  FT_DEC_CASE(128, 2)
  FT_DEC_CASE(128, 3)
  FT_DEC_CASE(128, 4)
  FT_DEC_CASE(128, 8)
  FT_DEC_CASE(64, 1)
  FT_DEC_CASE(64, 2)
  FT_DEC_CASE(64, 4)
  FT_DEC_CASE(64, 8)
#undef FT_DEC_CASE
  return -2;
}
