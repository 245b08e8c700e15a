// K6: paged decode attention (one query token per sequence) on MFMA, with a
// load-balanced flattened work partition.  SURVEY.md §2.4 K6.
//
// Decode attention is an HBM stream over the KV cache (4 KiB per token per layer
// for Llama-3-8B).  What bounds it on MI355X is bytes in flight per CU and how
// evenly the CUs are loaded, so the kernel is built around those two things:
//
// * Layout.  K blocks are [block_size tok][D] (row-major); V blocks are stored
//   TRANSPOSED, [D][block_size tok] (csrc/kernels/rope_kv.hip writes them so).
//   With that, every MFMA operand of a 16-token tile loads straight from HBM
//   into registers with no LDS round trip and no transposing read:
//     S[16 tok x 16 heads] = K[16 x D] . Qpad^T      v_mfma_f32_16x16x32_bf16
//        A = K rows (16 B per lane), B = the G query heads of the kv head (GQA
//        packed, padded to 16 columns), C lane (g, n) = tokens 4g..4g+3, head n
//     O[16 heads x D]     += P[16 x 16 tok] . V       v_mfma_f32_16x16x16_bf16
//        A = P: exactly the S C-layout (lane (g, n) = head n, tokens 4g..4g+3)
//        converted to bf16 in place; B = V^T rows: tokens 4g..4g+3 of dim n =
//        8 contiguous bytes of the transposed V block.
//   VALU work per tile is the online softmax of 4 values per lane (v3, the VALU
//   dot2 kernel this replaces, needed ~440 instructions and 247 VGPRs per wave
//   for the same tile; at 2 waves/SIMD the CUs were latency-starved).
// * Partition.  Every (sequence, kv head, 16-token tile) is flattened into one
//   index space of `total` tiles and the grid's waves (all resident) each take
//   an equal contiguous range, so every CU streams the same number of bytes
//   whatever the mix of context lengths (v3 gave each (sequence, kv head) a
//   workgroup: 400 workgroups on 256 CUs at the 50-session batch).  A wave walks
//   its range segment by segment ((b, h) pieces) with an R-deep register ring
//   (R-1 tiles in flight while one computes).  A segment that one wave covers
//   whole is written as bf16 at once; pieces of shared segments leave fp32
//   (acc, m, l) partials at slot = segment + wave (collision-free: consecutive
//   segments share at most one wave).
// * Combine in the same launch (counters != null): a wave that leaves a partial
//   stores it write-through (agent-scope atomic stores = sc1), drains its stores
//   and counts itself in the segment's counter; the wave that draws the last
//   ticket merges the segment's partials (sc1 loads) into bf16 and resets the
//   counter for the next call.  This is the guide's sc1 hand-off (§6 Guideline
//   16): no fences, correct for any wave -> XCD placement.  The partials are
//   stored dim-permuted so every lane writes / reads contiguous 8-B words, and
//   the last arriver batches all of a segment's partial loads (8 slots in
//   flight) -- the first version's element-wise sc1 round trips made it lose to
//   the separate combine kernel (12.3 vs 10.9 ms per decode step).  At one
//   workgroup per CU it matches or beats the combine kernel (85 vs 86 us at 50 x
//   1.5-3k, 177 vs 182 us at 64 x 4k) and saves a launch per layer: the engine
//   uses it unless FT_DECODE_FUSED_COMBINE=0.
#include "ft_common.h"

#include <stdlib.h>

#include <type_traits>

namespace ft {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short short4_t __attribute__((ext_vector_type(4)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));

constexpr int kDecMaxBatch = 1024;
// default: >= 128 tokens per wave (short contexts use fewer waves).  Swept on MI355X
// (profiles/attn_min_tiles_r04.log): 8 vs 4 is 14.6 vs 21.4 us at 1 x 4k, 12.5 vs
// 13.4 at 1 x 2k, 20.0 vs 21.2 at 8 x 2k, even at 50 x 3k, 0.8 us slower at 1 x 512
constexpr int kDecMinTiles = 8;
// deferred-rescale threshold (log2 units): p = exp2(score - reference max) stays <= 2^8,
// exact in fp32 and in bf16's range
constexpr float kDecRescaleThr = 8.f;

// s_pre[b] = sum_{b' < b} ceil(ceil(L_b' / 16) / per) (tiles, or pieces of `per` tiles,
// per kv head), b = 0..batch; wave-wide scan
__device__ __forceinline__ void dec_prefix(int* s_pre, const int* __restrict__ seq_lens, int batch,
                                           int per) {
  const int lane = lane_id();
  int run = 0;
  for (int b0 = 0; b0 < batch; b0 += 64) {
    const int b = b0 + lane;
    int x = b < batch ? (max(seq_lens[b], 0) + 15) >> 4 : 0;
    if (per > 1) x = (x + per - 1) / per;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (b < batch) s_pre[b + 1] = run + x;
    run += __shfl(x, 63, 64);
  }
  if (lane == 0) s_pre[0] = 0;
}

// waves the flattened partition uses: at least min_tiles 16-token tiles each (a
// launch argument: fewer, longer ranges mean fewer partials for the last arriver to
// merge -- the latency that dominates short batches)
__device__ __forceinline__ int dec_num_waves(int total, int nw_grid, int min_tiles) {
  return max(1, min(nw_grid, (total + min_tiles - 1) / min_tiles));
}

// one 16-token tile of one kv head in registers: K rows (A operand of QK^T, one
// uint4 per 32-deep k-step) and V^T rows (B operand of PV, 4 tokens per 16 dims)
template <int D>
struct MTile {
  uint4 k[D / 32];
  uint2 v[D / 16];
};

// One tile's loads as buffer loads: the wave-uniform tile bases become SGPR
// descriptors and each lane keeps ONE 32-bit byte offset per image; the K
// k-steps are immediate offsets and the V^T dim tiles' stride (16 rows of the
// transposed block) goes in soffset, so the ring costs no address VGPRs (with
// 64-bit flat addresses the R = 3 kernel needed 204 VGPRs: 2 waves / SIMD).
// aux 2 = nt: the step's KV (0.4-1 GB at 50-64 sessions) is read once and far
// exceeds the 256 MiB Infinity Cache (the bare stream ran 5-7 % faster with nt).
// a wave-uniform pointer the compiler can PROVE uniform (SGPR descriptor, no
// waterfall loop around each buffer op: the tile indices derive from wave_id())
__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
}

template <int D>
__device__ __forceinline__ void mt_load(MTile<D>& t, const uint16_t* __restrict__ k_cache,
                                        const uint16_t* __restrict__ v_cache, size_t kbase,
                                        size_t vbase, int koff_b, int voff_b, int vstep_b) {
  const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(k_cache + kbase), 0, 16 * D * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(v_cache + vbase), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int kc = 0; kc < D / 32; ++kc)
    t.k[kc] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(kr, koff_b + kc * 64, 0, 2));
#pragma unroll
  for (int nd = 0; nd < D / 16; ++nd)
    t.v[nd] = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(vr, voff_b, nd * vstep_b, 2));
}

// fp8 (e4m3) tile (KV8): 1-byte K rows and V^T rows.  Lane (g, n) loads 16
// consecutive dims of K row n per 64-dim pair of k-steps (dims 64 p + 16 g + [0, 16):
// the first 8 feed k-step 2p, the next 8 k-step 2p+1 -- the Q fragments use the same
// dim permutation, so S is unchanged) and 4 tokens of each V^T dim row; both widen
// to bf16 fragments in registers (ft_common.h fp8x8_to_bf16).  Half the bytes of
// the bf16 tile per token.
template <int D>
struct MTile8 {
  uint4 k[D / 64];
  uint32_t v[D / 16];
};

template <int D>
__device__ __forceinline__ void mt_load8(MTile8<D>& t, const uint8_t* __restrict__ k_cache,
                                         const uint8_t* __restrict__ v_cache, size_t kbase,
                                         size_t vbase, int koff_b, int voff_b, int vstep_b) {
  const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(k_cache + kbase), 0, 16 * D, 0x00020000);
  const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
      uniform_ptr(v_cache + vbase), 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int p = 0; p < D / 64; ++p)
    t.k[p] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(kr, koff_b + p * 64, 0, 2));
#pragma unroll
  for (int nd = 0; nd < D / 16; ++nd)
    t.v[nd] = __builtin_amdgcn_raw_buffer_load_b32(vr, voff_b, nd * vstep_b, 2);
}

// End of a wave's piece of segment (b, h): the whole segment -> bf16 output;
// otherwise an fp32 (acc, m, l) partial at slot segment + wave, and with FC the
// in-launch combine by the last arriving wave (see the header comment).
// whole: this wave covered the segment alone; otherwise its partial goes to slot
// `slot` and the segment's np partials sit at slots first .. first + np - 1.
template <int D, int G, int ND, bool FC>
__device__ __forceinline__ void dec_finish(floatx4_t (&o)[ND], float l_run, float m_run, int b, int h,
                                           bool whole, int slot_i, int first, int np, int nkv,
                                           uint16_t* __restrict__ out, int out_stride,
                                           float* __restrict__ tmp_out, float* __restrict__ tmp_ml,
                                           int* __restrict__ counters, int lane, int g, int n) {
  // head n's sum over the 4 token groups
  const float l_tot = kgroups_sum(l_run);
  // C-layout rows of O: lane (g, n) holds heads 4g+i, dim n (+16 nd)
  const int seg = b * nkv + h;
  if (whole) {   // the whole segment: final bf16 output
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      const int r = 4 * g + i4;
      const float lr = __shfl(l_tot, r & 15, 64);
      if (r < G) {
        const float inv = 1.f / lr;
        uint16_t* op = out + (size_t)b * out_stride + (h * G + r) * D + n;
#pragma unroll
        for (int nd = 0; nd < ND; ++nd) op[nd * 16] = f32_to_bf16(o[nd][i4] * inv);
      }
    }
  } else {
    const size_t slot = (size_t)slot_i;
#pragma unroll
    for (int i4 = 0; i4 < 4; ++i4) {
      const int r = 4 * g + i4;
      const float lr = __shfl(l_tot, r & 15, 64);
      const float mr = __shfl(m_run, r & 15, 64);
      if (r < G) {
        float* dst = tmp_out + (slot * G + r) * D + n;
        if (FC) {
          // write-through (read by another wave in this launch), dims permuted to
          // [n][nd] so each lane's ND values are contiguous: 8-B sc1 stores, and
          // (m, l) as one 8-B store
          uint64_t* dp = reinterpret_cast<uint64_t*>(tmp_out + (slot * G + r) * D + n * ND);
#pragma unroll
          for (int p2 = 0; p2 < ND / 2; ++p2) {
            const uint64_t v = (uint64_t)__float_as_uint(o[2 * p2][i4]) |
                               ((uint64_t)__float_as_uint(o[2 * p2 + 1][i4]) << 32);
            __hip_atomic_store(dp + p2, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
          if (n == 0) {
            const uint64_t ml = (uint64_t)__float_as_uint(mr) | ((uint64_t)__float_as_uint(lr) << 32);
            __hip_atomic_store(reinterpret_cast<uint64_t*>(tmp_ml + (slot * G + r) * 2), ml,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          }
        } else {
#pragma unroll
          for (int nd = 0; nd < ND; ++nd) dst[nd * 16] = o[nd][i4];
          if (n == 0) {
            tmp_ml[(slot * G + r) * 2] = mr;
            tmp_ml[(slot * G + r) * 2 + 1] = lr;
          }
        }
      }
    }
    if (FC) {
      // publish (every partial store of this wave retired), then take a ticket
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int prev = 0;
      if (lane == 0)
        prev = __hip_atomic_fetch_add(counters + seg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      prev = __shfl(prev, 0, 64);
      if (prev == np - 1) {   // last arriver: merge the np partials of this segment
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keep the loads below the ticket
        const size_t base = (size_t)first;
        uint16_t* op = out + (size_t)b * out_stride + h * G * D;
        // lane (r, c): head r, dims c + 16 nd of the permuted partials; the
        // partial slots are read in batches of 8 with every load of a batch in
        // flight at once (8-B sc1 loads; slots past np re-read the last one and
        // are masked), online-max merge
        for (int q4 = lane; q4 < G * 16; q4 += 64) {
          const int r = q4 >> 4, c = q4 & 15;
          float M = -INFINITY, den = 0.f, acc[ND];
#pragma unroll
          for (int nd = 0; nd < ND; ++nd) acc[nd] = 0.f;
          for (int k0 = 0; k0 < np; k0 += 8) {
            uint64_t mlv[8], ov[8][ND / 2];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const size_t sl = (base + min(k0 + k, np - 1)) * G + r;
              mlv[k] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(tmp_ml + sl * 2),
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              const uint64_t* sp = reinterpret_cast<const uint64_t*>(tmp_out + sl * D + c * ND);
#pragma unroll
              for (int p2 = 0; p2 < ND / 2; ++p2)
                ov[k][p2] = __hip_atomic_load(sp + p2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              if (k0 + k < np) {
                const float m = __uint_as_float((uint32_t)mlv[k]);
                const float l = __uint_as_float((uint32_t)(mlv[k] >> 32));
                const float mn = fmaxf(M, m);
                const float a = exp2f(M - mn), e = exp2f(m - mn);
                den = den * a + e * l;
#pragma unroll
                for (int p2 = 0; p2 < ND / 2; ++p2) {
                  acc[2 * p2] = acc[2 * p2] * a + e * __uint_as_float((uint32_t)ov[k][p2]);
                  acc[2 * p2 + 1] = acc[2 * p2 + 1] * a + e * __uint_as_float((uint32_t)(ov[k][p2] >> 32));
                }
                M = mn;
              }
            }
          }
          const float inv = 1.f / den;
#pragma unroll
          for (int nd = 0; nd < ND; ++nd) op[r * D + 16 * nd + c] = f32_to_bf16(acc[nd] * inv);
        }
        if (lane == 0)
          __hip_atomic_store(counters + seg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

template <int D, int G, int R, bool FC, int WPC, bool PIECE = false, bool KV8 = false>
__global__ __launch_bounds__(256, WPC) void paged_decode_kernel(
    uint16_t* __restrict__ out, int out_stride, float* __restrict__ tmp_out,
    float* __restrict__ tmp_ml, const uint16_t* __restrict__ q, int q_stride,
    uint16_t* __restrict__ k_cache, uint16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    int batch, int nkv, int bs_shift, float scale_log2, int* __restrict__ counters,
    int min_tiles, int piece, int slot_cap, int num_blocks) {
  static_assert(G >= 1 && G <= 16, "GQA group must fit the 16 MFMA columns");
  constexpr int KC = D / 32, ND = D / 16;
  // s_pre: tile prefix; s_pre + kDecMaxBatch + 1: piece prefix (piece mode)
  __shared__ int s_pre[2 * (kDecMaxBatch + 1)];
  int* s_pp = s_pre + kDecMaxBatch + 1;
  if (wave_id() == 0) dec_prefix(s_pre, seq_lens, batch, 1);
  if (PIECE && wave_id() == 1) dec_prefix(s_pp, seq_lens, batch, piece);
  __syncthreads();
  const int total = nkv * s_pre[batch];
  const int wpg = blockDim.x >> 6;   // waves per workgroup (FT_DECODE_WAVES sweeps 2 / 4)
  const int nw = PIECE ? gridDim.x * wpg : dec_num_waves(total, gridDim.x * wpg, min_tiles);
  const int w = wave_id() * gridDim.x + blockIdx.x;  // spreads low wave ids over CUs
  if (FC && blockIdx.x == 0) {
    // fused-combine mode has no combine kernel to define empty sequences' outputs
    // (the padded rows of a decode graph bucket): one thread per empty segment
    for (int seg = threadIdx.x; seg < batch * nkv; seg += blockDim.x) {
      const int b = seg / nkv;
      if (s_pre[b + 1] == s_pre[b]) {
        uint4* o = reinterpret_cast<uint4*>(out + (size_t)b * out_stride + (seg - b * nkv) * G * D);
        for (int i = 0; i < G * D / 8; ++i) o[i] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
  }
  if (total == 0 || w >= nw) return;

  const int lane = lane_id();
  const float thr_raw = kDecRescaleThr / scale_log2;   // the threshold in raw score units
  const int n = lane & 15;   // MFMA column (head) / row (token) / dim within a tile
  const int g = lane >> 4;   // k group
  const int bsz = 1 << bs_shift;
  const int bmask = bsz - 1;
  const size_t blk_stride = (size_t)nkv * bsz * D;
  // per-lane offsets inside a 16-token tile (element size EB)
  constexpr int EB = KV8 ? 1 : 2;
  // bytes: K row n, dims 8g.. (+32 kc); fp8: dims 16g.. (+64 p)
  const int koff_b = KV8 ? (n * D + 16 * g) : 2 * (n * D + 8 * g);
  const int voff_b = EB * (n * bsz + 4 * g);   // bytes: V^T row n (+16 nd), tokens 4g..4g+3
  const int vstep_b = EB * 16 * bsz;           // bytes between the V^T dim tiles
  using Tile = typename std::conditional<KV8, MTile8<D>, MTile<D>>::type;

  // tiles [t0, t0 + cnt) of segment (b, h), then dec_finish
  auto run = [&](int b, int h, int t0, int cnt, int nb, bool whole, int slot_i, int first, int np) {
    const int L = seq_lens[b];

    // Q^T fragments (B operand): lane (g, n) = head n of this kv head, dims 8g.. (+32 kc)
    uint4 qb[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) {
      // fp8 tiles: k-step kc covers dims 64 (kc / 2) + 16 g + 8 (kc & 1) (MTile8)
      const int d0 = KV8 ? 64 * (kc >> 1) + 16 * g + 8 * (kc & 1) : kc * 32 + 8 * g;
      qb[kc] = n < G ? *reinterpret_cast<const uint4*>(q + (size_t)b * q_stride + (h * G + n) * D + d0)
                     : make_uint4(0, 0, 0, 0);
    }
    floatx4_t o[ND];
#pragma unroll
    for (int nd = 0; nd < ND; ++nd) o[nd] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    float m_run = -INFINITY;   // reference max of head n, raw score units (uniform over g)
    float l_run = 0.f;         // this lane's share of the running sum of head n
    float nbias = 0.f;         // -m_run * scale_log2

    const int* bt = block_tables + (size_t)b * bt_stride;
    for (int c0 = 0; c0 < cnt; c0 += 64) {
      const int cc = min(64, cnt - c0);
      // lane i holds tile (t0 + c0 + i)'s block index and in-block token offset
      int my_blk = 0, my_off = 0;
      if (lane < cc) {
        const int tok = (t0 + c0 + lane) << 4;
        my_blk = FT_CHECK_IDX(bt[tok >> bs_shift], num_blocks, kCkBlockTable, b);
        my_off = tok & bmask;
      }
      auto ld = [&](Tile& t, int i) {
        const int j = min(i, cc - 1);  // past the end: re-load the last tile (never consumed)
        const size_t blk = (size_t)(uint32_t)__builtin_amdgcn_readlane(my_blk, j);
        const int off = __builtin_amdgcn_readlane(my_off, j);
        const size_t hb = blk * blk_stride + (size_t)h * bsz * D;
        if constexpr (KV8)
          mt_load8<D>(t, reinterpret_cast<const uint8_t*>(k_cache), reinterpret_cast<const uint8_t*>(v_cache),
                      hb + (size_t)off * D, hb + off, koff_b, voff_b, vstep_b);
        else
          mt_load<D>(t, k_cache, v_cache, hb + (size_t)off * D, hb + off, koff_b, voff_b, vstep_b);
      };
      auto consume = [&](Tile& t, int i) {
        const int valid = L - ((t0 + c0 + i) << 4);   // tokens of this tile inside the sequence
        floatx4_t s = floatx4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
          uint4 kf;
          if constexpr (KV8) {
            const uint4& w = t.k[kc >> 1];
            kf = (kc & 1) ? fp8x8_to_bf16(w.z, w.w) : fp8x8_to_bf16(w.x, w.y);
          } else {
            kf = t.k[kc];
          }
          s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, kf),
                                                      __builtin_bit_cast(bf16x8_t, qb[kc]), s, 0, 0, 0);
        }
        // only a sequence's last tile can be partial: a wave-uniform branch, so full
        // tiles carry no mask compares / selects
        if (valid < 16) {
#pragma unroll
          for (int i4 = 0; i4 < 4; ++i4)
            if (4 * g + i4 >= valid) s[i4] = -INFINITY;
        }
        float tm = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
        tm = kgroups_max(tm);   // over the 4 token groups of head n
        // deferred rescale (guide T13): the reference max m_run (raw score units) moves
        // only when some head's tile max passes it by more than kDecRescaleThr (log2
        // units), so p <= 2^thr and most tiles skip alpha, the O rescale and the l
        // rescale; the branch is wave-uniform
        if (__builtin_amdgcn_ballot_w64(tm > m_run + thr_raw) != 0) {
          const float mn = fmaxf(m_run, tm);
          const float alpha = __builtin_amdgcn_exp2f((m_run - mn) * scale_log2);  // -inf -> 0
          m_run = mn;
          l_run *= alpha;
          float a[4];
#pragma unroll
          for (int i4 = 0; i4 < 4; ++i4) a[i4] = __shfl(alpha, (4 * g + i4) & 15, 64);
#pragma unroll
          for (int nd = 0; nd < ND; ++nd)
#pragma unroll
            for (int i4 = 0; i4 < 4; ++i4) o[nd][i4] *= a[i4];
          nbias = -m_run * scale_log2;
        }
        float p[4];
#pragma unroll
        for (int i4 = 0; i4 < 4; ++i4) p[i4] = __builtin_amdgcn_exp2f(fmaf(s[i4], scale_log2, nbias));
        l_run += (p[0] + p[1]) + (p[2] + p[3]);
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t pw = {pack2(p[0], p[1]), pack2(p[2], p[3])};   // 2 x v_cvt_pk_bf16_f32
        const short4_t pa = __builtin_bit_cast(short4_t, pw);
#pragma unroll
        for (int nd = 0; nd < ND; ++nd) {
          uint2 vf;
          if constexpr (KV8) vf = fp8x4_to_bf16(t.v[nd]);
          else vf = t.v[nd];
          o[nd] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(pa, __builtin_bit_cast(short4_t, vf),
                                                           o[nd], 0, 0, 0);
        }
      };
      Tile ring[R];
#pragma unroll
      for (int r = 0; r + 1 < R; ++r) ld(ring[r], r);
      for (int i = 0; i < cc; i += R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          ld(ring[(r + R - 1) % R], i + r + R - 1);
          __builtin_amdgcn_sched_barrier(0);
          if (i + r < cc) consume(ring[r], i + r);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }

    dec_finish<D, G, ND, FC>(o, l_run, m_run * scale_log2, b, h, whole, slot_i, first, np, nkv, out,
                             out_stride, tmp_out, tmp_ml, counters, lane, g, n);
  };
  // b = last sequence with nkv * pre[b] <= f
  auto find_seq = [&](const int* pre, int f) {
    int lo = 0, hi = batch - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (nkv * pre[mid] <= f) lo = mid; else hi = mid - 1;
    }
    return lo;
  };

  if constexpr (PIECE) {
    // batch-invariant partition: segment (b, h) is cut into pieces of `piece` tiles
    // from its first token, whatever the rest of the batch; piece p of the flattened
    // piece space writes partial slot p and the segment's last arriver merges its
    // pieces in order, so a sequence's output depends on its own length only
    const int npieces = nkv * s_pp[batch];
    for (int p = w; p < npieces && p < slot_cap; p += nw) {
      const int b = find_seq(s_pp, p);
      const int npb = s_pp[b + 1] - s_pp[b];
      const int rel = p - nkv * s_pp[b];
      const int h = rel / npb, k = rel - h * npb;
      const int nb = s_pre[b + 1] - s_pre[b];
      const int t0 = k * piece;
      run(b, h, t0, min(piece, nb - t0), nb, npb == 1, p, p - k, npb);
    }
  } else {
  int f = (int)(((long long)w * total) / nw);
  const int f1 = (int)(((long long)(w + 1) * total) / nw);
  while (f < f1) {
    // segment (b, h) holding flattened tile f
    const int b = find_seq(s_pre, f);
    const int nb = s_pre[b + 1] - s_pre[b];
    const int rel = f - nkv * s_pre[b];
    const int h = rel / nb;
    const int t0 = rel - h * nb;
    const int cnt = min(f1 - f, nb - t0);
    // waves sharing the segment: the first and last whose tile range meets it
    const int S = nkv * s_pre[b] + h * nb, E = S + nb;
    const int wf = (int)(((long long)(S + 1) * nw - 1) / total);
    const int wl = (int)(((long long)E * nw - 1) / total);
    const int seg = b * nkv + h;
    run(b, h, t0, cnt, nb, t0 == 0 && cnt == nb, seg + w, seg + wf, wl - wf + 1);
    f += cnt;
  }
  }
}

// One workgroup per (sequence, kv head): merges the partials of a segment that
// several waves shared (slots segment + w, w = first..last wave of the segment).
template <int D, int G>
__global__ __launch_bounds__(256) void paged_decode_combine_kernel(
    uint16_t* __restrict__ out, int out_stride, const float* __restrict__ tmp_out,
    const float* __restrict__ tmp_ml, const int* __restrict__ seq_lens, int batch, int nkv,
    int nw_grid, int min_tiles) {
  __shared__ int s_pre[kDecMaxBatch + 1];
  __shared__ float s_M[G], s_den[G];
  if (wave_id() == 0) dec_prefix(s_pre, seq_lens, batch, 1);
  __syncthreads();
  const int total = nkv * s_pre[batch];
  const int nw = dec_num_waves(total, nw_grid, min_tiles);
  const int seg = blockIdx.x;
  const int b = seg / nkv, h = seg - b * nkv;
  const int nb = s_pre[b + 1] - s_pre[b];
  uint16_t* o = out + (size_t)b * out_stride + h * G * D;
  if (nb == 0) {  // empty sequence: define the output
    for (int i = threadIdx.x; i < G * D; i += blockDim.x) o[i] = 0;
    return;
  }
  const int S = nkv * s_pre[b] + h * nb, E = S + nb;
  const int wf = (int)(((long long)(S + 1) * nw - 1) / total);
  const int wl = (int)(((long long)E * nw - 1) / total);
  const int np = wl - wf + 1;
  if (np <= 1) return;  // one wave covered it and wrote bf16 directly
  const size_t base = (size_t)(seg + wf);
  const int lane = lane_id();
  for (int g = wave_id(); g < G; g += blockDim.x / 64) {
    float M = -INFINITY;
    for (int k = lane; k < np; k += 64) M = fmaxf(M, tmp_ml[((base + k) * G + g) * 2]);
    M = wave_max(M);
    float den = 0.f;
    for (int k = lane; k < np; k += 64)
      den += exp2f(tmp_ml[((base + k) * G + g) * 2] - M) * tmp_ml[((base + k) * G + g) * 2 + 1];
    den = wave_sum(den);
    if (lane == 0) {
      s_M[g] = M;
      s_den[g] = den;
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < G * D; i += blockDim.x) {
    const int g = i / D, d = i - g * D;
    const float M = s_M[g];
    float a0 = 0.f, a1 = 0.f;
    int k = 0;
    for (; k + 1 < np; k += 2) {
      const size_t s0 = (base + k) * G + g, s1 = (base + k + 1) * G + g;
      a0 += exp2f(tmp_ml[s0 * 2] - M) * tmp_out[s0 * D + d];
      a1 += exp2f(tmp_ml[s1 * 2] - M) * tmp_out[s1 * D + d];
    }
    if (k < np) {
      const size_t s0 = (base + k) * G + g;
      a0 += exp2f(tmp_ml[s0 * 2] - M) * tmp_out[s0 * D + d];
    }
    o[i] = f32_to_bf16((a0 + a1) / s_den[g]);
  }
}

}  // namespace ft

static int ft_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

// Workgroups per CU.  Fewer bytes in flight stream FASTER here: the bare load
// stream of this partition (bench/attn_diag.py SWEEP=1, 50 x 1.5-3k ragged, random
// blocks) ran 6.28 TB/s with one 4-wave workgroup per CU and one tile in flight
// per wave, 5.77 TB/s at 2 workgroups x 2 tiles, 4.77 TB/s at 4 x 3 -- ~8 MB in
// flight chip-wide is the sweet spot, more thrashes the HBM queues (the plain
// streaming-read ceiling, bench/bw_read.py, peaks at the same 8 MB).
// FT_DECODE_WPC (1-3) overrides for A/B runs.
static int dec_wg_per_cu() {
  static const int w = [] {
    const char* e = getenv("FT_DECODE_WPC");
    const int v = e ? atoi(e) : 1;
    return (v >= 1 && v <= 3) ? v : 1;
  }();
  return w;
}

// upper bound on the waves of the decode grid: the workspace holds batch * nkv +
// waves partial slots
extern "C" int ft_decode_waves() { return ft_num_cus() * 3 * 4; }
extern "C" int ft_decode_max_batch() { return ft::kDecMaxBatch; }

extern "C" int ft_paged_decode_attention(void* out, int out_stride, float* tmp_out, float* tmp_ml,
                                         const void* q, int q_stride, const void* k_cache,
                                         const void* v_cache, const int* block_tables,
                                         int bt_stride, const int* seq_lens, int batch, int nq,
                                         int nkv, int head_dim, int block_size, float scale,
                                         int* counters, int piece, int slot_cap,
                                         int num_blocks, int kv8, hipStream_t stream) {
  if (batch <= 0) return 0;
  if (nq % nkv != 0) return -1;
  if (piece < 0 || (piece > 0 && counters == nullptr)) return -6;  // pieces merge in-launch
  if (batch > ft::kDecMaxBatch) return -5;
  if (block_size < 16 || (block_size & (block_size - 1))) return -4;
  const int bs_shift = __builtin_ctz(block_size);
  const int G = nq / nkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  // register-ring depth (tiles per wave: R - 1 in flight); FT_DECODE_RING overrides
  // the default for the A/B sweeps (bench/attn_sweep.py)
  static const int ring = [] {
    const char* e = getenv("FT_DECODE_RING");
    const int r = e ? atoi(e) : 2;
    return (r >= 2 && r <= 4) ? r : 2;
  }();
  // minimum tiles per wave of the partition; FT_DECODE_MIN_TILES overrides (sweeps)
  static const int min_tiles_env = [] {
    const char* e = getenv("FT_DECODE_MIN_TILES");
    return e ? max(1, atoi(e)) : 0;
  }();
  const int min_tiles = min_tiles_env ? min_tiles_env : ft::kDecMinTiles;
  // 1 workgroup per CU, or the register-limited maximum for the ring depth
  const int wpc = min(dec_wg_per_cu(), ring == 2 ? 3 : 2);
  // waves per workgroup: 2 (one 128-thread workgroup per CU, 512 waves) -- engine A/B
  // at 50 x 3k: decode step 7.15-7.17 vs 7.29 ms with 4 waves, 8.71 with 1; the bare
  // kernel 130.7-135 vs 138-145 us at 64 x 4k (profiles/attn_waves_per_wg_r04.log).
  // FT_DECODE_WAVES (1 / 2 / 4) overrides for sweeps.
  static const int nwv = [] {
    const char* e = getenv("FT_DECODE_WAVES");
    const int v = e ? atoi(e) : 2;
    return (v == 1 || v == 2 || v == 4) ? v : 2;
  }();
  // ring depth of the fp8 path (FT_DECODE_RING8, 2 / 3).  bench/attn_fp8_bench.py,
  // 50 x 1.5-3k / 50 x 2.2-4.5k / 64 x 4k (profiles/attn_fp8_r06.log): 2 waves per
  // workgroup 68.7 / 98.6 / 131.5 us (ring 3), 4 waves 56.7 / 77.7 / 106.8 (ring 3) and
  // 55.3 / 74.4 / 102.6 (ring 2) -- against 84.8 / 120.1 / 170.6 us on bf16 caches
  static const int ring8 = [] {
    const char* e = getenv("FT_DECODE_RING8");
    const int r = e ? atoi(e) : 2;
    return (r == 2 || r == 3) ? r : 2;
  }();
  // waves per workgroup of the fp8 path (FT_DECODE_WAVES8, 2 / 4): the widening
  // conversions double the VALU work per byte, so the fp8 stream wants every SIMD
  static const int nwv8 = [] {
    const char* e = getenv("FT_DECODE_WAVES8");
    const int v = e ? atoi(e) : 4;
    return (v == 2 || v == 4) ? v : 4;
  }();
  // FT_DECODE_WPC8=2: two fp8 workgroups per CU -- measured 61.8 / 81.1 / 105.8 us against
  // 55.5 / 74.1 / 100.0 at one (profiles/attn_fp8_r06.log), kept for sweeps
  static const int wpc8 = [] {
    const char* e = getenv("FT_DECODE_WPC8");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  int nwg = 0;
#define FT_DEC_ARGS                                                                             \
  (uint16_t*)out, out_stride, tmp_out, tmp_ml, (const uint16_t*)q, q_stride, (uint16_t*)k_cache, \
      (uint16_t*)v_cache, block_tables, bt_stride, seq_lens, batch, nkv, bs_shift, scale_log2,   \
      counters, min_tiles, piece, slot_cap, num_blocks
#define FT_DEC_LAUNCH(DD, GG, RR, FCC)                                                  \
  if (wpc == 1)                                                                                \
    hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, RR, FCC, 1>), dim3(nwg), dim3(64 * nwv), \
                       0, stream, FT_DEC_ARGS);                                                \
  else                                                                                         \
    hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, RR, FCC, (RR == 2 ? 3 : 2)>),          \
                       dim3(nwg), dim3(64 * nwv), 0, stream, FT_DEC_ARGS)
#define FT_DEC_CASE(DD, GG, RR)                                                                \
  if (head_dim == DD && G == GG) {                                                             \
    nwg = ft_num_cus() * wpc;                                                                  \
    if (kv8) {  /* fp8 caches: one workgroup per CU, ring8 tiles deep */                       \
      nwg = ft_num_cus();                                                                      \
      if (piece > 0)                                                                           \
        hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, 2, true, 1, true, true>), dim3(nwg), \
                           dim3(256), 0, stream, FT_DEC_ARGS);                                 \
      else if (counters != nullptr && wpc8 == 2)                                               \
        hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, 2, true, 2, false, true>),          \
                           dim3(2 * nwg), dim3(64 * nwv8), 0, stream, FT_DEC_ARGS);              \
      else if (counters != nullptr && ring8 == 3)                                              \
        hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, 3, true, 1, false, true>), dim3(nwg), \
                           dim3(64 * nwv8), 0, stream, FT_DEC_ARGS);                            \
      else if (counters != nullptr)                                                            \
        hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, 2, true, 1, false, true>), dim3(nwg), \
                           dim3(64 * nwv8), 0, stream, FT_DEC_ARGS);                            \
      else {                                                                                   \
        hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, 2, false, 1, false, true>), dim3(nwg), \
                           dim3(64 * nwv8), 0, stream, FT_DEC_ARGS);                            \
        hipLaunchKernelGGL((ft::paged_decode_combine_kernel<DD, GG>), dim3(batch * nkv), dim3(256),\
                           0, stream, (uint16_t*)out, out_stride, tmp_out, tmp_ml, seq_lens, batch,\
                           nkv, nwg * nwv8, min_tiles);                                         \
      }                                                                                        \
      return static_cast<int>(hipGetLastError());                                              \
    }                                                                                          \
    if (piece > 0) {                                                                           \
      nwg = ft_num_cus();                                                                      \
      hipLaunchKernelGGL((ft::paged_decode_kernel<DD, GG, 2, true, 1, true>), dim3(nwg),      \
                         dim3(256), 0, stream, FT_DEC_ARGS);                                   \
    } else if (counters != nullptr) {                                                          \
      FT_DEC_LAUNCH(DD, GG, RR, true);                                                         \
    } else {                                                                                   \
      FT_DEC_LAUNCH(DD, GG, RR, false);                                                        \
      hipLaunchKernelGGL((ft::paged_decode_combine_kernel<DD, GG>), dim3(batch * nkv), dim3(256),\
                         0, stream, (uint16_t*)out, out_stride, tmp_out, tmp_ml, seq_lens, batch,\
                         nkv, nwg * nwv, min_tiles);                                             \
    }                                                                                            \
    return static_cast<int>(hipGetLastError());                                                  \
  }
  // ring 2 at one workgroup per CU: full kernel 86 vs 92 us (ring 3) at 50 x 1.5-3k,
  // 125 vs 128 us at 50 x 2.2-4.5k (bench/attn_diag.py, profiles/attn_decode_w1_r02.log)
  if (ring == 3 && !kv8) { FT_DEC_CASE(128, 4, 3) }
  if (ring == 4 && !kv8) { FT_DEC_CASE(128, 4, 4) }
  FT_DEC_CASE(128, 1, 2)
  FT_DEC_CASE(128, 2, 2)
  FT_DEC_CASE(128, 3, 2)
  FT_DEC_CASE(128, 4, 2)
  FT_DEC_CASE(128, 8, 2)
  FT_DEC_CASE(64, 1, 2)
  FT_DEC_CASE(64, 2, 2)
  FT_DEC_CASE(64, 4, 2)
  FT_DEC_CASE(64, 8, 2)
#undef FT_DEC_CASE
#undef FT_DEC_LAUNCH
#undef FT_DEC_ARGS
  return -2;
}

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(attn_decode)
