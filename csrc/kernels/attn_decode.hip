// K6: paged decode attention (one query token per sequence) with split-K
// ("flash-decoding") and a combine kernel.  SURVEY.md §2.4 K6.
//
// Decode attention is an HBM stream over the KV cache (4 KiB per token per layer
// for Llama-3-8B), so the design goal is bytes in flight, not FLOPs:
//   * grid = (seq * kv_head, split); split s of a sequence of length L owns
//     the token range [s*P, (s+1)*P) with P = roundup16(ceil(L / splits)) <= 1024,
//     i.e. every sequence is cut into `splits` near-equal partitions whatever its
//     length, so the grid depends only on (batch bucket, splits) and ONE hipGraph
//     per batch bucket covers every context length up to max_model_len (an
//     earlier power-of-two split bucket forced lazy re-captures mid-serving).
//     A workgroup computes all G = nq/nkv query heads of its kv head against its
//     partition, so every K/V byte is read once per step (GQA packing).
//   * 4 waves; D/8 lanes share a token (16 lanes at D=128 -> 4 tokens per wave
//     instruction, 1 KiB per wave instruction), each lane owns 8 head dims and
//     keeps its 8*G query values in registers for the whole partition.
//   * U=4 token groups are issued back to back before any use so every lane has
//     4 independent 16-B loads in flight (the kernel is latency bound otherwise).
//   * scores live in LDS (fp32 [G][PART]); the softmax of a partition is a
//     wave reduction per head; P.V accumulates in registers and is reduced
//     over token slots with shuffles + one LDS pass.
//   * partitions write unnormalised fp32 partials + (max, sum); the combine
//     kernel rescales.  A sequence that fits one partition writes bf16 output
//     directly and the combine kernel skips it.
#include "ft_common.h"

namespace ft {

constexpr int kMaxPart = 1024;  // LDS score buffer per (head, partition)

__device__ __forceinline__ int decode_part(int L, int splits) {
  const int p = (L + splits - 1) / splits;
  return max(16, (p + 15) & ~15);
}

template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_kernel(
    uint16_t* __restrict__ out, int out_stride, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, const uint16_t* __restrict__ q, int q_stride,
    const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    int nkv, int block_size, int max_splits, float scale) {
  constexpr int LPT = D / 8;        // lanes per token
  constexpr int TPW = 64 / LPT;     // tokens per wave instruction
  constexpr int TPB = 4 * TPW;      // tokens per workgroup iteration
  constexpr int U = 4;              // iterations issued together
  __shared__ float s_p[G][kMaxPart];
  __shared__ float s_red[4][G][D];
  __shared__ float s_m[G], s_l[G];

  const int b = blockIdx.x / nkv;
  const int kvh = blockIdx.x - b * nkv;
  const int split = blockIdx.y;
  const int L = seq_lens[b];
  const int PART = decode_part(L, max_splits);
  const int start = split * PART;
  if (start >= L) return;
  const int n = min(min(L - start, PART), kMaxPart);  // host guarantees PART <= kMaxPart
  const int nsplit = (L + PART - 1) / PART;
  const int nq = nkv * G;

  const int lane = lane_id(), wave = wave_id();
  const int c = lane % LPT;        // dim chunk owned by this lane
  const int tslot = wave * TPW + lane / LPT;

  float qr[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint4 v = reinterpret_cast<const uint4*>(q + (size_t)b * q_stride + (kvh * G + g) * D)[c];
    load8(v, qr[g]);
#pragma unroll
    for (int j = 0; j < 8; ++j) qr[g][j] *= scale;
  }

  const int* bt = block_tables + (size_t)b * bt_stride;
  const size_t head_off = (size_t)kvh * block_size * D;
  const size_t blk_stride = (size_t)nkv * block_size * D;

  // ---- scores ---------------------------------------------------------------
  for (int base = 0; base < n; base += TPB * U) {
    uint4 kv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tl = base + u * TPB + tslot;
      if (tl < n) {
        const int tok = start + tl;
        const int blk = bt[tok / block_size];
        const int off = tok - (tok / block_size) * block_size;
        kv[u] = reinterpret_cast<const uint4*>(k_cache + blk * blk_stride + head_off +
                                               (size_t)off * D)[c];
      } else {
        kv[u] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float kf[8];
      load8(kv[u], kf);
      float dot[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s += kf[j] * qr[g][j];
        dot[g] = group_sum<LPT>(s);
      }
      const int tl = base + u * TPB + tslot;
      if (tl < n && c == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) s_p[g][tl] = dot[g];
      }
    }
  }
  __syncthreads();

  // ---- softmax per head (one wave per head) -----------------------------------
  for (int g = wave; g < G; g += 4) {
    float m = -INFINITY;
    for (int i = lane; i < n; i += 64) m = fmaxf(m, s_p[g][i]);
    m = wave_max(m);
    float l = 0.f;
    for (int i = lane; i < n; i += 64) {
      const float p = __expf(s_p[g][i] - m);
      s_p[g][i] = p;
      l += p;
    }
    l = wave_sum(l);
    if (lane == 0) {
      s_m[g] = m;
      s_l[g] = l;
    }
  }
  __syncthreads();

  // ---- P.V ---------------------------------------------------------------------
  float acc[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[g][j] = 0.f;

  for (int base = 0; base < n; base += TPB * U) {
    uint4 vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tl = base + u * TPB + tslot;
      if (tl < n) {
        const int tok = start + tl;
        const int blk = bt[tok / block_size];
        const int off = tok - (tok / block_size) * block_size;
        vv[u] = reinterpret_cast<const uint4*>(v_cache + blk * blk_stride + head_off +
                                               (size_t)off * D)[c];
      } else {
        vv[u] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int tl = base + u * TPB + tslot;
      if (tl < n) {
        float vf[8];
        load8(vv[u], vf);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const float p = s_p[g][tl];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[g][j] += p * vf[j];
        }
      }
    }
  }
  // reduce over the token slots of this wave (lanes that share chunk c)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = acc[g][j];
#pragma unroll
      for (int o = LPT; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
      acc[g][j] = v;
    }
  if (lane < LPT) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) s_red[wave][g][c * 8 + j] = acc[g][j];
  }
  __syncthreads();

  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int g = i / D, d = i - g * D;
    const float v = s_red[0][g][d] + s_red[1][g][d] + s_red[2][g][d] + s_red[3][g][d];
    const int h = kvh * G + g;
    if (nsplit == 1) {
      out[(size_t)b * out_stride + h * D + d] = f32_to_bf16(v / s_l[g]);
    } else {
      const size_t o = ((size_t)b * nq + h) * max_splits + split;
      tmp_out[o * D + d] = v;
      if (d == 0) {
        tmp_ml[o * 2] = s_m[g];
        tmp_ml[o * 2 + 1] = s_l[g];
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(D) void paged_decode_combine_kernel(
    uint16_t* __restrict__ out, int out_stride, const float* __restrict__ tmp_out,
    const float* __restrict__ tmp_ml, const int* __restrict__ seq_lens, int nq, int max_splits) {
  const int b = blockIdx.x, h = blockIdx.y, d = threadIdx.x;
  const int L = seq_lens[b];
  const int part = decode_part(L, max_splits);
  const int ns = (L + part - 1) / part;
  if (ns <= 1) return;
  const size_t base = ((size_t)b * nq + h) * max_splits;
  float M = -INFINITY;
  for (int s = 0; s < ns; ++s) M = fmaxf(M, tmp_ml[(base + s) * 2]);
  float den = 0.f, acc = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float w = __expf(tmp_ml[(base + s) * 2] - M);
    den += w * tmp_ml[(base + s) * 2 + 1];
    acc += w * tmp_out[(base + s) * D + d];
  }
  out[(size_t)b * out_stride + h * D + d] = f32_to_bf16(acc / den);
}

}  // namespace ft

// max tokens one decode partition may hold: splits must be >= ceil(max_len / this)
extern "C" int ft_decode_partition_size() { return ft::kMaxPart; }

extern "C" int ft_paged_decode_attention(void* out, int out_stride, float* tmp_out, float* tmp_ml,
                                         const void* q, int q_stride, const void* k_cache,
                                         const void* v_cache, const int* block_tables,
                                         int bt_stride, const int* seq_lens, int batch, int nq,
                                         int nkv, int head_dim, int block_size, int max_splits,
                                         float scale, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (nq % nkv != 0) return -1;
  if (max_splits < 1) return -3;
  const int G = nq / nkv;
  dim3 grid(batch * nkv, max_splits), block(256);
#define FT_DEC_CASE(DD, GG)                                                                   \
  if (head_dim == DD && G == GG) {                                                            \
    hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG>), grid, block, 0, stream,             \
                       (uint16_t*)out, out_stride, tmp_out, tmp_ml, (const uint16_t*)q,       \
                       q_stride, (const uint16_t*)k_cache, (const uint16_t*)v_cache,          \
                       block_tables, bt_stride, seq_lens, nkv, block_size, max_splits, scale); \
    if (max_splits > 1)                                                                       \
      hipLaunchKernelGGL((ft::paged_decode_combine_kernel<DD>), dim3(batch, nq), dim3(DD), 0, \
                         stream, (uint16_t*)out, out_stride, tmp_out, tmp_ml, seq_lens, nq,   \
                         max_splits);                                                         \
    return static_cast<int>(hipGetLastError());                                               \
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
