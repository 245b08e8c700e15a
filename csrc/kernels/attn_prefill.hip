// K5: varlen causal prefill attention over the paged KV cache (new tokens +
// cached prefix, i.e. multi-turn history reuse) on MFMA.  SURVEY.md §2.4 K5.
//
// Work decomposition (GQA-aware): a workgroup owns one (query tile, kv head).
// Its 64 MFMA rows are (token, q-head) pairs flattened token-major, row r ->
// token r / G, head r % G, so the G query heads that share a kv head share
// every K/V tile the workgroup stages (each K/V byte is read once per tile of
// 64/G query tokens).  4 waves x 16 rows.
//
// Per 64-token KV tile:
//   * K is staged row-major into LDS with a 16-B-chunk XOR swizzle
//     (chunk ^ (row & 15)) so the B-operand reads (16 different rows, same
//     column) are bank-conflict free (guide T2).
//   * V blocks are stored transposed in the cache ([D][block_size], see
//     rope_kv.hip), so the tile is staged as a [D][64 tok] image with whole
//     16-B copies, chunk c of dim row r at slot c ^ ((r >> 1) & 7) (the 16
//     rows one ds_read_b128 lane group touches land on 16 distinct bank
//     quads), and the PV B operand (k = 8 consecutive tokens, n = one head
//     dim) is one plain ds_read_b128 per MFMA.
//   * Pipelined staging (split STAGE_LOAD / STAGE_WRITE): the next tile's K and
//     V^T global loads are issued into registers before the current tile's
//     MFMAs and written to LDS after the barrier that retires them, so HBM/L2
//     latency hides behind the QK^T / softmax / PV work.
//   * S = Q K^T with v_mfma_f32_16x16x32_bf16 (Q fragments live in registers for
//     the whole kernel), causal + length mask, online softmax in the log2
//     domain, P goes through a per-wave LDS tile to become the A operand of
//     O += P V (16x16x32 again).  Running max/sum stay per lane; the sum is
//     reduced across the 16 lanes of a row group only once at the end.
#include "ft_common.h"

namespace ft {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_t as_frag(const uint4& v) {
  return __builtin_bit_cast(bf16x8_t, v);
}

constexpr int kPrefillBK = 64;   // kv tokens per tile
constexpr int kPStride = 72;     // per-wave P tile row stride

template <int D, int G>
__global__ __launch_bounds__(256) void prefill_attn_kernel(
    uint16_t* __restrict__ out, int out_stride, const uint16_t* __restrict__ q, int q_stride,
    const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    const int* __restrict__ q_start_loc, const int* __restrict__ tile_info, int nkv,
    int block_size, float scale_log2) {
  constexpr int NCH = D / 8;          // 16-B chunks per row
  constexpr int KC = D / 32;          // k-chunks of the QK^T product
  constexpr int ND = D / 16;          // 16-wide output column tiles
  constexpr int TQ = 64 / G;          // query tokens per tile
  constexpr int SWZ = (NCH >= 16) ? 15 : (NCH - 1);

  __shared__ __attribute__((aligned(16))) uint16_t Ks[kPrefillBK * D];
  __shared__ __attribute__((aligned(16))) uint16_t Vs[D * kPrefillBK];   // V^T [D][64 tok], swizzled
  __shared__ __attribute__((aligned(16))) uint16_t Ps[4][16 * kPStride];

  const int tile = blockIdx.x;
  const int kvh = blockIdx.y;
  const int b = tile_info[tile * 2];
  const int qs = tile_info[tile * 2 + 1];
  const int L = seq_lens[b];
  const int q0 = q_start_loc[b];
  const int qlen = q_start_loc[b + 1] - q0;
  const int ctx0 = L - qlen;  // position of the first new token
  const int ntok = min(TQ, qlen - qs);

  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, lg = lane >> 4;
  const int nq = nkv * G;

  // ---- Q fragments (A operand): row = lane & 15 of this wave's 16 rows ----------
  uint4 qa[KC];
  {
    const int r = wave * 16 + l15;
    const int tq = r / G, g = r - (r / G) * G;
    const bool valid = (r < TQ * G) && (tq < ntok);
    const uint16_t* qp = q + (size_t)(q0 + qs + (valid ? tq : 0)) * q_stride + (kvh * G + g) * D;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      qa[kc] = valid ? reinterpret_cast<const uint4*>(qp + kc * 32 + 8 * lg)[0]
                     : make_uint4(0, 0, 0, 0);
  }
  // query position of the 4 C-layout rows this lane holds
  int qpos[4];
  bool rvalid[4];
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = wave * 16 + lg * 4 + rr;
    const int tq = r / G;
    rvalid[rr] = (r < TQ * G) && (tq < ntok);
    qpos[rr] = ctx0 + qs + tq;
  }

  floatx4_t o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = floatx4_t{0.f, 0.f, 0.f, 0.f};
  float m_run[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  float l_run[4] = {0.f, 0.f, 0.f, 0.f};

  const int kv_end = min(L, ctx0 + qs + ntok);  // exclusive
  const int ntiles = (kv_end + kPrefillBK - 1) / kPrefillBK;
  const int* bt = block_tables + (size_t)b * bt_stride;
  const size_t head_off = (size_t)kvh * block_size * D;
  const size_t blk_stride = (size_t)nkv * block_size * D;
  const int bs_shift = __builtin_ctz(block_size);
  const int bmask = block_size - 1;
  // V^T staging: item = (block j of the tile, dim d, 8-token chunk cc), cc fastest,
  // so consecutive lanes read consecutive 16 B of one transposed block
  const int tb_shift = min(bs_shift, 6);          // log2 tokens of one block inside a tile
  const int cpr_shift = tb_shift - 3;             // log2 16-B chunks per block row
  constexpr int IT = kPrefillBK * NCH / 256;      // staged 16-B items per thread (K and V each)
  uint4 kreg[IT], vreg[IT];
  auto stage_load = [&](int kbase) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = threadIdx.x + it * 256;
      {  // K row t, chunk ch
        const int t = idx / NCH, ch = idx - (idx / NCH) * NCH;
        const int p = kbase + t;
        kreg[it] = make_uint4(0, 0, 0, 0);
        if (p < kv_end)
          kreg[it] = *reinterpret_cast<const uint4*>(k_cache + bt[p >> bs_shift] * blk_stride +
                                                     head_off + (size_t)(p & bmask) * D + ch * 8);
      }
      {  // V^T dim d, tokens t .. t+7
        const int cc = idx & ((1 << cpr_shift) - 1), rest = idx >> cpr_shift;
        const int d = rest % D, j = rest / D;
        const int p = kbase + (j << tb_shift) + cc * 8;
        vreg[it] = make_uint4(0, 0, 0, 0);
        if (p < kv_end)
          vreg[it] = *reinterpret_cast<const uint4*>(v_cache + bt[p >> bs_shift] * blk_stride +
                                                     head_off + (size_t)d * block_size + (p & bmask));
      }
    }
  };
  auto stage_write = [&]() {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int idx = threadIdx.x + it * 256;
      const int t = idx / NCH, ch = idx - (idx / NCH) * NCH;
      reinterpret_cast<uint4*>(Ks + t * D)[ch ^ (t & SWZ)] = kreg[it];
      const int cc = idx & ((1 << cpr_shift) - 1), rest = idx >> cpr_shift;
      const int d = rest % D, j = rest / D;
      const int c = ((j << tb_shift) >> 3) + cc;   // 16-B chunk (8 tokens) within the row
      reinterpret_cast<uint4*>(Vs + d * kPrefillBK)[c ^ ((d >> 1) & 7)] = vreg[it];
    }
  };

  if (ntiles > 0) {
    stage_load(0);
    stage_write();
  }
  __syncthreads();
  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * kPrefillBK;
    if (kt + 1 < ntiles) stage_load(kbase + kPrefillBK);  // in flight during this tile's math
    // ---- S = Q K^T -----------------------------------------------------------------
    floatx4_t s[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      s[n] = floatx4_t{0.f, 0.f, 0.f, 0.f};
      const int row = n * 16 + l15;
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        const int ch = kc * 4 + lg;
        const uint4 kb = reinterpret_cast<const uint4*>(Ks + row * D)[ch ^ (row & SWZ)];
        s[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(qa[kc]), as_frag(kb), s[n], 0, 0,
                                                        0);
      }
    }
    // ---- mask + online softmax (log2 domain) ---------------------------------------
    float alpha[4];
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      float mt = -INFINITY;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const int kp = kbase + n * 16 + l15;
        float v = s[n][rr] * scale_log2;
        if (!rvalid[rr] || kp > qpos[rr] || kp >= kv_end) v = -INFINITY;
        s[n][rr] = v;
        mt = fmaxf(mt, v);
      }
      mt = group_max<16>(mt);
      const float mn = fmaxf(m_run[rr], mt);
      const float base = (mn == -INFINITY) ? 0.f : mn;
      alpha[rr] = exp2f(m_run[rr] - base);
      m_run[rr] = mn;
      float ls = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n) {
        const float p = exp2f(s[n][rr] - base);
        s[n][rr] = p;
        ls += p;
      }
      l_run[rr] = l_run[rr] * alpha[rr] + ls;
    }
#pragma unroll
    for (int nd = 0; nd < ND; ++nd)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) o[nd][rr] *= alpha[rr];

    // ---- P (C layout) -> LDS -> A layout ------------------------------------------
    uint16_t* pw = Ps[wave];
#pragma unroll
    for (int n = 0; n < 4; ++n)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) pw[(lg * 4 + rr) * kPStride + n * 16 + l15] = f32_to_bf16(s[n][rr]);
    __syncthreads();

    // ---- O += P V ------------------------------------------------------------------
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const uint4 pa = *reinterpret_cast<const uint4*>(pw + l15 * kPStride + kc * 32 + 8 * lg);
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        // B operand: tokens kc*32 + 8 lg .. +8 of head dim nd*16 + l15
        const int row = nd * 16 + l15;
        const uint4 vb = reinterpret_cast<const uint4*>(Vs + row * kPrefillBK)[
            (kc * 4 + lg) ^ ((row >> 1) & 7)];
        o[nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(pa), as_frag(vb), o[nd], 0, 0, 0);
      }
    }
    __syncthreads();   // every wave is done with this tile's Ks / Vs / Ps
    if (kt + 1 < ntiles) {
      stage_write();
      __syncthreads();
    }
  }

  // ---- normalise + store -------------------------------------------------------------
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const float l = group_sum<16>(l_run[rr]);
    if (!rvalid[rr]) continue;
    const int r = wave * 16 + lg * 4 + rr;
    const int tq = r / G, g = r - (r / G) * G;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + (size_t)(q0 + qs + tq) * out_stride + (kvh * G + g) * D;
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) op[nd * 16 + l15] = f32_to_bf16(o[nd][rr] * inv);
  }
  (void)nq;
}

}  // namespace ft

extern "C" int ft_prefill_tile_tokens(int nq, int nkv) { return 64 / (nq / nkv); }

extern "C" int ft_prefill_attention(void* out, int out_stride, const void* q, int q_stride,
                                    const void* k_cache, const void* v_cache,
                                    const int* block_tables, int bt_stride, const int* seq_lens,
                                    const int* q_start_loc, const int* tile_info, int num_tiles,
                                    int nq, int nkv, int head_dim, int block_size, float scale,
                                    hipStream_t stream) {
  if (num_tiles <= 0) return 0;
  if (nq % nkv != 0) return -1;
  const int G = nq / nkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_tiles, nkv), block(256);
#define FT_PF_CASE(DD, GG)                                                                   \
  if (head_dim == DD && G == GG) {                                                           \
    hipLaunchKernelGGL((ft::prefill_attn_kernel<DD, GG>), grid, block, 0, stream,            \
                       (uint16_t*)out, out_stride, (const uint16_t*)q, q_stride,             \
                       (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables,     \
                       bt_stride, seq_lens, q_start_loc, tile_info, nkv, block_size,         \
                       scale_log2);                                                          \
    return static_cast<int>(hipGetLastError());                                              \
  }
  FT_PF_CASE(128, 1)
  FT_PF_CASE(128, 2)
  FT_PF_CASE(128, 3)
  FT_PF_CASE(128, 4)
  FT_PF_CASE(128, 8)
  FT_PF_CASE(64, 1)
  FT_PF_CASE(64, 2)
  FT_PF_CASE(64, 4)
  FT_PF_CASE(64, 8)
#undef FT_PF_CASE
  return -2;
}
