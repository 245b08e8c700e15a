// K5: varlen causal prefill attention over the paged KV cache (new tokens +
// cached prefix, i.e. multi-turn history reuse) on MFMA.  SURVEY.md §2.4 K5.
//
// Built for the serving regime of a voice chat: every turn prefills a short new
// chunk (tens of tokens) on top of a long cached history (thousands), so the
// kernel is a KV stream like decode, and what matters is reading each K/V byte
// ONCE per (sequence, kv head) and keeping bytes in flight.
//
// * Work: a workgroup owns (query block, kv head); its 256 MFMA rows are (token,
//   q-head) pairs flattened token-major (row r -> token r / G, head r % G), so
//   the G query heads of the kv head share every staged K/V tile and a block
//   holds 256 / G tokens (64 at GQA 4: a typical turn is one block).  8 waves x
//   2 m-tiles of 16 rows (512 threads, 2 waves per SIMD, one workgroup per CU).
// * Transposed formulation, everything lane-local:
//     S^T[64 kv x 16 q]  = K . Q^T      A = K rows from LDS, B = Q^T (registers)
//     O^T[D x 16 q]     += V^T . P^T    A = V^T rows from LDS, B = P^T = S^T's
//                                       C layout converted to bf16 in place
//   A lane owns one query column of each m-tile: its running max / sum / rescale
//   need no cross-lane traffic except one 4-lane max per tile, and P never goes
//   through LDS.  The PV k-slots of a lane are tokens {4g..4g+3, 16+4g..16+4g+3}
//   of each 32-token half (the S^T C layout); the V^T A operand uses the same
//   permutation (two 8-B reads of the V^T image).
// * Staging: K rows (16-B chunk XOR swizzle, conflict-free A reads) and V^T rows
//   (V blocks are stored transposed in the cache, [D][block_size], rope_kv.hip;
//   chunk c of dim row r at slot c ^ ((r >> 1) & 7)) in LDS, shared by the 8
//   waves.  Tiles stream by LDS-DMA (global_load_lds_dwordx4) into a 4-slot
//   ring: the swizzles are applied on the per-lane SOURCE address (the DMA's LDS
//   destination is lane-linear), tiles t+1..t+3 stay in flight while tile t
//   computes (counted vmcnt + raw s_barrier; a __syncthreads would drain the
//   DMA).  The block-table entries of the KV range are copied to LDS once, so
//   issuing a tile never waits on a table read.
// * Split-KV (flash-decoding for prefill): a chat turn prefills ~100 tokens over a
//   history of thousands, i.e. 2 query blocks per sequence -- a mixed step of ~10
//   prompts was 160 workgroups on 256 CUs, each streaming the whole history alone
//   (213 us per layer at the driver config, 0.25 PFLOP/s).  A work item is now
//   (query block, KV tile range): long ranges are split over several workgroups
//   (host plan, ops.build_prefill_tiles), each leaves fp32 (O, m, l) partials and
//   prefill_combine_kernel merges them; items covering the whole range still
//   write bf16 directly.
#include "ft_common.h"
#include "ft_lds.h"

namespace ft {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8_t as_frag(const uint4& v) {
  return __builtin_bit_cast(bf16x8_t, v);
}

constexpr int kPrefillBK = 64;   // kv tokens per tile
constexpr float kPrefillRescaleThr = 8.f;
constexpr int kPrefillRows = 256; // query rows (token x head) per workgroup
constexpr int kPrefillMaxBlocks = 4096;  // block-table entries staged in LDS (checked on the host)

// max / sum over aligned groups of 4 lanes that differ in bits 4..5 (the k groups):
// ft_common.h kgroups_max / kgroups_sum (VALU lane swaps)
__device__ __forceinline__ float kgroup_max(float v) { return kgroups_max(v); }
__device__ __forceinline__ float kgroup_sum(float v) { return kgroups_sum(v); }

// INV (batch-invariant mode): the deferred rescale is decided per query row (lane)
// instead of wave-wide, so a row's rounding never depends on the rows that share its
// wave -- which change with chunking and prefix-cache hits.
//
// KV8 (fp8 e4m3 caches): the LDS images stay bf16 -- the same swizzled layouts, so
// tile_math is unchanged -- but they are filled through registers: every thread
// loads one 16-B piece of fp8 K rows and one of V^T rows (16 elements each), widens
// them to bf16 (ft_common.h fp8x8_to_bf16) and writes two 16-B chunks at their
// swizzled slots.  Two tiles are in flight in registers (loaded two iterations ahead)
// over two LDS slots; one barrier per tile.
template <int D, int G, bool INV, bool KV8 = false>
__global__ __launch_bounds__(512, 1) void prefill_attn_kernel(
    uint16_t* __restrict__ out, int out_stride, const uint16_t* __restrict__ q, int q_stride,
    const uint16_t* __restrict__ k_cache, const uint16_t* __restrict__ v_cache,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ seq_lens,
    const int* __restrict__ q_start_loc, const int* __restrict__ tile_info, int nkv,
    int block_size, float scale_log2, float* __restrict__ part_o, float* __restrict__ part_ml,
    int num_blocks) {
  constexpr int NCH = D / 8;          // 16-B chunks per K row
  constexpr int KC = D / 32;          // k-steps of S^T = K Q^T
  constexpr int ND = D / 16;          // 16-row dim tiles of O^T
  constexpr int NW = 8;               // waves per workgroup
  constexpr int MT = kPrefillRows / (16 * NW);  // 16-query m-tiles per wave
  constexpr int QB = kPrefillRows / G;  // query tokens per workgroup
  constexpr int SWZ = (NCH >= 16) ? 15 : (NCH - 1);

  // one LDS array (guide §5 item 4a): [NSLOT slots][K image | V^T image], then the table
  constexpr int NSLOT = KV8 ? 2 : 4;
  constexpr int KIMG = kPrefillBK * D, VIMG = D * kPrefillBK;   // bf16 elements
  constexpr int SLOT = KIMG + VIMG;
  __shared__ __attribute__((aligned(16))) uint16_t smem[NSLOT * SLOT + 2 * kPrefillMaxBlocks];
  int* s_bt = reinterpret_cast<int*>(smem + NSLOT * SLOT);

  const int tile = blockIdx.x;
  const int kvh = blockIdx.y;
  // work item: (sequence, first query token, KV tile range lo << 16 | hi, partial slot)
  const int b = tile_info[tile * 4];
  const int qs = tile_info[tile * 4 + 1];
  const int krange = tile_info[tile * 4 + 2];
  const int pslot = tile_info[tile * 4 + 3];   // < 0: the item covers the whole range
  const int L = seq_lens[b];
  const int q0 = q_start_loc[b];
  const int qlen = q_start_loc[b + 1] - q0;
  const int ctx0 = L - qlen;  // position of the first new token
  const int ntok = min(QB, qlen - qs);

  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, lg = lane >> 4;

  // ---- Q^T fragments (B operand) + the query column each lane owns ----------------
  uint4 qb[MT][KC];
  int qpos[MT];   // position of this lane's query column (-1: padding row)
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int r = (wave * MT + m) * 16 + l15;
    const int tq = r / G, g = r - (r / G) * G;
    const bool valid = (r < QB * G) && (tq < ntok);
    qpos[m] = valid ? ctx0 + qs + tq : -1;
    const uint16_t* qp = q + (size_t)(q0 + qs + (valid ? tq : 0)) * q_stride + (kvh * G + g) * D;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc)
      qb[m][kc] = valid ? reinterpret_cast<const uint4*>(qp + kc * 32 + 8 * lg)[0]
                        : make_uint4(0, 0, 0, 0);
  }

  // retire the Q loads here, outside the tile loop: a compiler-inserted wait at
  // their first use inside the loop would be a vmcnt(0) that drains the K/V DMA
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) dep(qb[m][kc]);

  floatx4_t o[MT][ND];   // O^T: lane (l15 = query, lg) rows = dims 16 nd + 4 lg + i
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int i = 0; i < ND; ++i) o[m][i] = floatx4_t{0.f, 0.f, 0.f, 0.f};
  float m_run[MT], l_run[MT], nbias[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    m_run[m] = -INFINITY;
    l_run[m] = 0.f;
    nbias[m] = 0.f;
  }
  const float thr_raw = kPrefillRescaleThr / scale_log2;

  const int kv_end = min(L, ctx0 + qs + ntok);  // exclusive
  const int kt_lo = krange >> 16;
  const int ntiles = min((kv_end + kPrefillBK - 1) / kPrefillBK, krange & 0xffff);
  const int first_q = ctx0 + qs;                // lowest query position of the block
  const int* bt = block_tables + (size_t)b * bt_stride;
  const size_t head_off = (size_t)kvh * block_size * D;
  const size_t blk_stride = (size_t)nkv * block_size * D;
  const int bs_shift = __builtin_ctz(block_size);
  const int bmask = block_size - 1;
  const int nblk = (kv_end + block_size - 1) >> bs_shift;
  const uint32_t lds0 = lds_off(smem);
  // LDS-DMA of one tile into ring slot `slot`: 16 KiB K image + 16 KiB V^T image (D
  // = 128) = 32 wave-instructions of 1 KiB, 4 per wave.  Lanes past kv_end re-read
  // a valid chunk (finite data; those keys are masked, their P is 0).
  constexpr int KI = KIMG * 2 / 1024, VI = VIMG * 2 / 1024;   // 1-KiB pieces per image
  constexpr int PER_WAVE = (KI + VI) / NW;
  // Per-lane constants of this wave's DMA pieces, computed once (the per-tile issue
  // used to recompute every lane's row / chunk / block lookup: ~140 VALU per tile).
  //   K piece (TPP rows of one block: the block index is wave-uniform): lane -> row t
  //   of the piece, LDS slot sl; source chunk = sl ^ swizzle(t)
  //   V^T piece: lane -> dim d, LDS slot sl; source token chunk c = sl ^ swizzle(d)
  constexpr int KR = KI / NW, VR = VI / NW;    // K / V^T pieces per wave per tile
  static_assert(KR * NW == KI && VR * NW == VI, "pieces must split evenly over the waves");
  constexpr int TPP = 64 / NCH;                // K rows per 1-KiB piece (4 at D = 128)
  int k_lane[KR], v_lane[VR], v_tok[VR];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const int e = (wave + r * NW) * 64 + lane;   // 16-B element of the K image
    const int t = e / NCH, sl = e - t * NCH;
    k_lane[r] = (t & bmask) * D + (sl ^ (t & SWZ)) * 8;
  }
#pragma unroll
  for (int r = 0; r < VR; ++r) {
    const int e = (wave + r * NW) * 64 + lane;   // 16-B element of the V^T image
    const int d = e >> 3, sl = e & 7;
    v_lane[r] = d * block_size;
    v_tok[r] = (sl ^ ((d >> 1) & 7)) << 3;
  }
  auto issue_tile = [&](int kt, int slot) {
    const int kbase = kt * kPrefillBK;
    const uint32_t kimg = lds0 + slot * SLOT * 2, vimg = kimg + KIMG * 2;
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const int piece = wave + r * NW;
      // the piece's rows share one block; past kv_end the piece re-reads rows of the
      // last block (finite data; those keys are masked, their P is 0)
      const int tp = min(kbase + piece * TPP, kv_end - 1);
      const int blk = __builtin_amdgcn_readfirstlane(s_bt[tp >> bs_shift]);
      const uint16_t* src = k_cache + (size_t)blk * blk_stride + head_off +
                            (size_t)(kbase & bmask) * D + k_lane[r];
      glds16(src, kimg + piece * 1024);
    }
#pragma unroll
    for (int r = 0; r < VR; ++r) {
      const int p = min(kbase + v_tok[r], (kv_end - 1) & ~7);
      const uint16_t* src = v_cache + (size_t)s_bt[p >> bs_shift] * blk_stride + head_off +
                            v_lane[r] + (p & bmask);
      glds16(src, vimg + (wave + r * NW) * 1024);
    }
  };
  uint32_t koff[KC];
#pragma unroll
  for (int kc = 0; kc < KC; ++kc) koff[kc] = l15 * D * 2 + ((((kc * 4 + lg) ^ (l15 & SWZ))) << 4);
  uint32_t voff[2][2];
#pragma unroll
  for (int kc = 0; kc < 2; ++kc)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      voff[kc][h] = l15 * kPrefillBK * 2 + (((kc * 4 + h * 2 + (lg >> 1)) ^ ((l15 >> 1) & 7)) << 4) +
                    ((lg & 1) << 3);
  uint32_t kb = 0;   // LDS byte address of the current slot's K image (V^T image follows)

  auto tile_math = [&](int kt) {
    const int kbase = kt * kPrefillBK;
    // ---- S^T = K Q^T: lane (l15 = query of m-tile m, lg) holds kv 16 n + 4 lg + i ----
    floatx4_t s[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) s[m][n] = floatx4_t{0.f, 0.f, 0.f, 0.f};
    // K A-fragments: 4 reads per 16-kv n-tile, the next n-tile's in flight
    uint32_t ka[KC];
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) ka[kc] = kb + koff[kc];
    auto kread = [&](uint4 (&kf)[KC], int n) {
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        if (n == 0) kf[kc] = ds_read16o<0>(ka[kc]);
        else if (n == 1) kf[kc] = ds_read16o<32 * D>(ka[kc]);
        else if (n == 2) kf[kc] = ds_read16o<64 * D>(ka[kc]);
        else kf[kc] = ds_read16o<96 * D>(ka[kc]);
      }
    };
    uint4 kf[2][KC];
    kread(kf[0], 0);
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      if (n + 1 < 4) {
        kread(kf[(n + 1) & 1], n + 1);
        lgkm_wait<KC>();
      } else {
        lgkm_wait<0>();
      }
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) {
        dep(kf[n & 1][kc]);
#pragma unroll
        for (int m = 0; m < MT; ++m)
          s[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(kf[n & 1][kc]), as_frag(qb[m][kc]),
                                                             s[m][n], 0, 0, 0);
      }
    }
    const bool edge = kbase + kPrefillBK > kv_end || kbase + kPrefillBK - 1 > first_q;
    if (__builtin_expect(edge, 0)) {
      asm volatile("" ::: "memory");   // keep this a branch: if-converted, every tile paid the mask
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const int lim = min(qpos[m], kv_end - 1) - kbase - lg * 4;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (n * 16 + i > lim) s[m][n][i] = -INFINITY;
      }
    }
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      float mt = fmaxf(fmaxf(s[m][0][0], s[m][0][1]), fmaxf(s[m][0][2], s[m][0][3]));
#pragma unroll
      for (int n = 1; n < 4; ++n)
        mt = fmaxf(mt, fmaxf(fmaxf(s[m][n][0], s[m][n][1]), fmaxf(s[m][n][2], s[m][n][3])));
      mt = kgroup_max(mt);
      const bool up = mt > m_run[m] + thr_raw;
      if (INV ? up : __builtin_amdgcn_ballot_w64(up) != 0) {
        const float mn = fmaxf(m_run[m], mt);
        const float alpha = mn == -INFINITY ? 1.f : __builtin_amdgcn_exp2f((m_run[m] - mn) * scale_log2);
        m_run[m] = mn;
        nbias[m] = mn == -INFINITY ? 0.f : -mn * scale_log2;
        l_run[m] *= alpha;
#pragma unroll
        for (int nd = 0; nd < ND; ++nd)
#pragma unroll
          for (int i = 0; i < 4; ++i) o[m][nd][i] *= alpha;
      }
      float ls = 0.f;
#pragma unroll
      for (int n = 0; n < 4; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float p = __builtin_amdgcn_exp2f(fmaf(s[m][n][i], scale_log2, nbias[m]));
          s[m][n][i] = p;
          ls += p;
        }
      l_run[m] += ls;
    }

    // ---- O^T += V^T P^T: k-slots of lane (., lg) = tokens {4lg.., 16+4lg..} + 32 kc ----
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      uint4 pb[MT];
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const floatx4_t& lo = s[m][2 * kc];
        const floatx4_t& hi = s[m][2 * kc + 1];
        pb[m] = make_uint4(pack2(lo[0], lo[1]), pack2(lo[2], lo[3]), pack2(hi[0], hi[1]),
                           pack2(hi[2], hi[3]));
      }
      // V^T A-fragments: 2 reads per dim tile, the next tile's in flight
      const uint32_t va0 = kb + KIMG * 2 + voff[kc][0], va1 = kb + KIMG * 2 + voff[kc][1];
      auto vread = [&](uint2 (&vv)[2], int nd) {
        switch (nd) {   // constant after unrolling: the dim tile's displacement is an immediate
#define FT_VR(I) case I: vv[0] = ds_read8o<I * 32 * kPrefillBK>(va0); vv[1] = ds_read8o<I * 32 * kPrefillBK>(va1); break;
          FT_VR(0) FT_VR(1) FT_VR(2) FT_VR(3) FT_VR(4) FT_VR(5) FT_VR(6)
          default: vv[0] = ds_read8o<7 * 32 * kPrefillBK>(va0); vv[1] = ds_read8o<7 * 32 * kPrefillBK>(va1);
#undef FT_VR
        }
      };
      uint2 vv[2][2];
      vread(vv[0], 0);
#pragma unroll
      for (int nd = 0; nd < ND; ++nd) {
        if (nd + 1 < ND) {
          vread(vv[(nd + 1) & 1], nd + 1);
          lgkm_wait<2>();
        } else {
          lgkm_wait<0>();
        }
        dep(vv[nd & 1][0]);
        dep(vv[nd & 1][1]);
        const uint4 vf = make_uint4(vv[nd & 1][0].x, vv[nd & 1][0].y, vv[nd & 1][1].x,
                                    vv[nd & 1][1].y);
#pragma unroll
        for (int m = 0; m < MT; ++m)
          o[m][nd] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_frag(vf), as_frag(pb[m]),
                                                              o[m][nd], 0, 0, 0);
      }
    }
  };

  // block-table entries of the KV range (LDS reads never wait on the DMA's vmcnt)
  for (int i = threadIdx.x; i < nblk; i += blockDim.x)
    s_bt[i] = FT_CHECK_IDX(bt[i], num_blocks, kCkBlockTable, b);
  __syncthreads();

  if constexpr (KV8) {
    // ---- fp8 caches: register-staged tiles (see the comment above the kernel) ----
    constexpr int NP = kPrefillBK * D / 16;   // 16-B fp8 pieces per image (K and V^T alike)
    constexpr int KPR = D / 16;               // K pieces per row
    const int tid = threadIdx.x;
    const uint8_t* k8 = reinterpret_cast<const uint8_t*>(k_cache);
    const uint8_t* v8 = reinterpret_cast<const uint8_t*>(v_cache);
    auto load8t = [&](int kt, uint4& kr, uint4& vr) {
      const int kbase = kt * kPrefillBK;
      if (tid < NP) {
        const int t = tid / KPR, j = tid - (tid / KPR) * KPR;
        const int tok = min(kbase + t, kv_end - 1);   // past kv_end: a valid row (masked)
        kr = *reinterpret_cast<const uint4*>(k8 + (size_t)s_bt[tok >> bs_shift] * blk_stride + head_off +
                                             (size_t)(tok & bmask) * D + 16 * j);
        const int d = tid >> 2, c = tid & 3;          // V^T: dim d, tokens 16 c .. 16 c + 15
        const int p = min(kbase + 16 * c, (kv_end - 1) & ~15);
        vr = *reinterpret_cast<const uint4*>(v8 + (size_t)s_bt[p >> bs_shift] * blk_stride + head_off +
                                             (size_t)d * block_size + (p & bmask));
      }
    };
    auto store8t = [&](int slot, const uint4& kr, const uint4& vr) {
      if (tid < NP) {
        const uint32_t kimg = lds0 + slot * SLOT * 2, vimg = kimg + KIMG * 2;
        const int t = tid / KPR, j = tid - (tid / KPR) * KPR;
        const uint32_t kr0 = kimg + t * D * 2;
        ds_write16(kr0 + (((2 * j) ^ (t & SWZ)) << 4), fp8x8_to_bf16(kr.x, kr.y));
        ds_write16(kr0 + (((2 * j + 1) ^ (t & SWZ)) << 4), fp8x8_to_bf16(kr.z, kr.w));
        const int d = tid >> 2, c = tid & 3, sw = (d >> 1) & 7;
        const uint32_t vr0 = vimg + d * kPrefillBK * 2;
        ds_write16(vr0 + (((2 * c) ^ sw) << 4), fp8x8_to_bf16(vr.x, vr.y));
        ds_write16(vr0 + (((2 * c + 1) ^ sw) << 4), fp8x8_to_bf16(vr.z, vr.w));
      }
    };
    uint4 kr0 = make_uint4(0, 0, 0, 0), vr0 = kr0, kr1 = kr0, vr1 = kr0;
    // register set (kt - kt_lo) & 1 holds tile kt; LDS slot kt & 1
    if (kt_lo < ntiles) load8t(kt_lo, kr0, vr0);
    if (kt_lo + 1 < ntiles) load8t(kt_lo + 1, kr1, vr1);
    if (kt_lo < ntiles) store8t(kt_lo & 1, kr0, vr0);
    if (kt_lo + 2 < ntiles) load8t(kt_lo + 2, kr0, vr0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // one tile: math on slot kt & 1, then the next tile (registers `kn`, `vn`) into the
    // other slot -- last read at tile kt - 1, before the previous barrier -- and the
    // tile after next into the registers just freed
    auto step = [&](int kt, uint4& kn, uint4& vn) {
      kb = lds0 + (kt & 1) * SLOT * 2;
      tile_math(kt);
      if (kt + 1 < ntiles) store8t((kt + 1) & 1, kn, vn);
      if (kt + 3 < ntiles) load8t(kt + 3, kn, vn);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
    for (int kt = kt_lo; kt < ntiles; kt += 2) {
      step(kt, kr1, vr1);
      if (kt + 1 < ntiles) step(kt + 1, kr0, vr0);
    }
  } else {
#pragma unroll
  for (int t = 0; t < NSLOT - 1; ++t)
    if (kt_lo + t < ntiles) issue_tile(kt_lo + t, (kt_lo + t) % NSLOT);
  for (int kt = kt_lo; kt < ntiles; ++kt) {
    const int slot = kt % NSLOT;
    const int ahead = min(ntiles - 1 - kt, NSLOT - 1);   // tiles in flight behind tile kt
    if (kt + NSLOT - 1 < ntiles)
      issue_tile(kt + NSLOT - 1, (kt + NSLOT - 1) % NSLOT);  // slot of tile kt-1, retired
    if (ahead >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * PER_WAVE) : "memory");
    else if (ahead == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * PER_WAVE) : "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PER_WAVE) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // every wave's pieces of tile kt have landed
    kb = lds0 + slot * SLOT * 2;
    tile_math(kt);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();          // slot kt % NSLOT may be refilled
  }
  }

  // ---- normalise + store: lane (l15 = query, lg) writes dims 16 nd + 4 lg .. +3 -------
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const float l = kgroup_sum(l_run[m]);
    if (qpos[m] < 0) continue;
    const int r = (wave * MT + m) * 16 + l15;
    if (pslot >= 0) {   // split item: unnormalised fp32 O + (m, l) of row r
      float* po = part_o + (((size_t)pslot * nkv + kvh) * kPrefillRows + r) * D + 4 * lg;
#pragma unroll
      for (int nd = 0; nd < ND; ++nd)
        *reinterpret_cast<float4*>(po + nd * 16) = make_float4(o[m][nd][0], o[m][nd][1], o[m][nd][2], o[m][nd][3]);
      if (lg == 0)
        *reinterpret_cast<float2*>(part_ml + (((size_t)pslot * nkv + kvh) * kPrefillRows + r) * 2) =
            make_float2(m_run[m] == -INFINITY ? -INFINITY : m_run[m] * scale_log2, l);
      continue;
    }
    const int tq = r / G, g = r - (r / G) * G;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    uint16_t* op = out + (size_t)(q0 + qs + tq) * out_stride + (kvh * G + g) * D + 4 * lg;
#pragma unroll
    for (int nd = 0; nd < ND; ++nd)
      *reinterpret_cast<uint2*>(op + nd * 16) =
          make_uint2(pack2(o[m][nd][0] * inv, o[m][nd][1] * inv),
                     pack2(o[m][nd][2] * inv, o[m][nd][3] * inv));
  }
}

// Merges the split items of one (query block, kv head): combine entry = (sequence,
// first query token, first partial slot, number of splits).  One thread per (row,
// 4 dims): 256 / (D / 4) rows per workgroup, grid.z covers the 256 rows, so the
// merge is a wide parallel pass (a wave per row with dependent split loads was
// latency-bound at ~100 us).  Online-max merge, the next split's loads in flight.
template <int D, int G>
__global__ __launch_bounds__(256) void prefill_combine_kernel(
    uint16_t* __restrict__ out, int out_stride, const float* __restrict__ part_o,
    const float* __restrict__ part_ml, const int* __restrict__ q_start_loc,
    const int* __restrict__ combine, int nkv) {
  constexpr int QB = kPrefillRows / G;
  constexpr int CH = D / 4;                 // float4 chunks per row
  constexpr int RPB = 256 / CH;             // rows per workgroup
  const int c = blockIdx.x, kvh = blockIdx.y;
  const int b = combine[c * 4], qs = combine[c * 4 + 1], s0 = combine[c * 4 + 2], ns = combine[c * 4 + 3];
  const int q0 = q_start_loc[b];
  const int ntok = min(QB, q_start_loc[b + 1] - q0 - qs);
  const int r = blockIdx.z * RPB + threadIdx.x / CH;
  const int ch = threadIdx.x % CH;
  if (r >= ntok * G) return;
  const size_t stride = (size_t)nkv * kPrefillRows;          // rows between slots
  size_t row = ((size_t)s0 * nkv + kvh) * kPrefillRows + r;
  float M = -INFINITY, den = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  float2 ml = *reinterpret_cast<const float2*>(part_ml + row * 2);
  float4 v = *reinterpret_cast<const float4*>(part_o + row * D + 4 * ch);
  for (int k = 0; k < ns; ++k) {
    float2 ml_n = ml;
    float4 v_n = v;
    if (k + 1 < ns) {   // next split's loads before this one's math
      const size_t rn = row + stride;
      ml_n = *reinterpret_cast<const float2*>(part_ml + rn * 2);
      v_n = *reinterpret_cast<const float4*>(part_o + rn * D + 4 * ch);
    }
    if (ml.x != -INFINITY) {   // a split wholly above this row's position adds nothing
      const float mn = fmaxf(M, ml.x);
      const float a = exp2f(M - mn), e = exp2f(ml.x - mn);
      den = den * a + e * ml.y;
      acc.x = acc.x * a + e * v.x;
      acc.y = acc.y * a + e * v.y;
      acc.z = acc.z * a + e * v.z;
      acc.w = acc.w * a + e * v.w;
      M = mn;
    }
    ml = ml_n;
    v = v_n;
    row += stride;
  }
  const float inv = den > 0.f ? 1.f / den : 0.f;
  const int tq = r / G, g = r - (r / G) * G;
  *reinterpret_cast<uint2*>(out + (size_t)(q0 + qs + tq) * out_stride + (kvh * G + g) * D + 4 * ch) =
      make_uint2(pack2(acc.x * inv, acc.y * inv), pack2(acc.z * inv, acc.w * inv));
}

}  // namespace ft

extern "C" int ft_prefill_tile_tokens(int nq, int nkv) { return ft::kPrefillRows / (nq / nkv); }

extern "C" int ft_prefill_attention(void* out, int out_stride, const void* q, int q_stride,
                                    const void* k_cache, const void* v_cache,
                                    const int* block_tables, int bt_stride, const int* seq_lens,
                                    const int* q_start_loc, const int* tile_info, int num_tiles,
                                    int nq, int nkv, int head_dim, int block_size, float scale,
                                    float* part_o, float* part_ml, const int* combine,
                                    int num_combine, int invariant, int num_blocks, int kv8,
                                    hipStream_t stream) {
  if (num_tiles <= 0) return 0;
  if (nq % nkv != 0) return -1;
  if (num_combine > 0 && (part_o == nullptr || part_ml == nullptr || combine == nullptr)) return -3;
  const int G = nq / nkv;
  const float scale_log2 = scale * 1.4426950408889634f;
  dim3 grid(num_tiles, nkv), block(512);
#define FT_PF_CASE(DD, GG)                                                                   \
  if (head_dim == DD && G == GG) {                                                           \
    if (kv8 && invariant)                                                                    \
      hipLaunchKernelGGL((ft::prefill_attn_kernel<DD, GG, true, true>), grid, block, 0, stream, \
                         (uint16_t*)out, out_stride, (const uint16_t*)q, q_stride,           \
                         (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables,   \
                         bt_stride, seq_lens, q_start_loc, tile_info, nkv, block_size,       \
                         scale_log2, part_o, part_ml, num_blocks);                           \
    else if (kv8)                                                                            \
      hipLaunchKernelGGL((ft::prefill_attn_kernel<DD, GG, false, true>), grid, block, 0, stream, \
                         (uint16_t*)out, out_stride, (const uint16_t*)q, q_stride,           \
                         (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables,   \
                         bt_stride, seq_lens, q_start_loc, tile_info, nkv, block_size,       \
                         scale_log2, part_o, part_ml, num_blocks);                           \
    else if (invariant)                                                                      \
      hipLaunchKernelGGL((ft::prefill_attn_kernel<DD, GG, true>), grid, block, 0, stream,    \
                         (uint16_t*)out, out_stride, (const uint16_t*)q, q_stride,           \
                         (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables,   \
                         bt_stride, seq_lens, q_start_loc, tile_info, nkv, block_size,       \
                         scale_log2, part_o, part_ml, num_blocks);                           \
    else                                                                                     \
      hipLaunchKernelGGL((ft::prefill_attn_kernel<DD, GG, false>), grid, block, 0, stream,   \
                         (uint16_t*)out, out_stride, (const uint16_t*)q, q_stride,           \
                         (const uint16_t*)k_cache, (const uint16_t*)v_cache, block_tables,   \
                         bt_stride, seq_lens, q_start_loc, tile_info, nkv, block_size,       \
                         scale_log2, part_o, part_ml, num_blocks);                           \
    if (num_combine > 0)                                                                     \
      hipLaunchKernelGGL((ft::prefill_combine_kernel<DD, GG>),                               \
                         dim3(num_combine, nkv, ft::kPrefillRows / (256 / (DD / 4))),         \
                         dim3(256), 0, stream, (uint16_t*)out, out_stride, part_o, part_ml,  \
                         q_start_loc, combine, nkv);                                         \
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

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(attn_prefill)
