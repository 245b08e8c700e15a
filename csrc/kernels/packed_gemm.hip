// K3/K7/K8/K10/K11 above the decode row counts: y[M, N] = x[M, K] . W^T for
// M > 64 (prefill chunks, mixed steps, large decode batches) on the SAME packed
// MFMA-fragment weight image the decode kernels stream (skinny_gemm.hip,
// ops.pack_weight: [N/16][K/64][half][lane][8]), so the model keeps one copy of
// every weight (no row-major originals for a library GEMM).
//
// Tiling (guide §5 "standard MFMA GEMM main loop" with LDS-DMA staging):
//   * workgroup tile BM x BN, 8 waves as WM x WN, each wave MT x NT 16x16 tiles
//     (v_mfma_f32_16x16x32_bf16, fp32 accumulators), K in steps of 64;
//   * both operands go global -> LDS by global_load_lds_dwordx4 into an S-slot
//     ring (S-2 stages stay in flight across the one barrier per k-step; counted
//     vmcnt + raw s_barrier, never __syncthreads, which would drain the DMA);
//   * W: a 16-column x 64-k fragment block is 2 KiB contiguous in the packed
//     image, so every DMA instruction moves 1 KiB of consecutive bytes and the LDS
//     image is already in fragment order: lane l reads 16 B at l * 16 (one 1 KiB
//     contiguous ds_read_b128 per half, conflict-free);
//   * x: 8 rows x 128 B per DMA instruction into a [BM][64] image whose 16-B
//     chunk c of local row r sits at slot c ^ ((r >> 1) & 5) (swizzle applied on
//     the per-lane SOURCE address; conflict-free for the ds_read_b128 lane groups
//     of the A fragments, k = 16 g + 8 h + e as in the packed image);
//   * tiles are ordered m-fastest inside an n-block and remapped so consecutive
//     ids share an XCD: the m-blocks that read the same weight columns run
//     together and hit that XCD's L2;
//   * split-K over gridDim.y leaves fp32 slabs ws[s][M][N] for the row-wise
//     epilogue kernels (fused_epilogue.hip), like the decode GEMMs.
// Epilogues: bf16 store, fp32 slab store, or SiLU-mul of gate/up pairs (the
// gate_up image interleaves 16 gate rows with their 16 up rows,
// ops.interleave_gate_up(w, 1)): out[M, N/2] = silu(g) * u, no [M, 2I] round trip.
#include "ft_common.h"
#include "ft_lds.h"

namespace ft {

typedef __bf16 pg_bf16x8 __attribute__((ext_vector_type(8)));
typedef float pg_floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ pg_bf16x8 pg_frag(const uint4& v) {
  return __builtin_bit_cast(pg_bf16x8, v);
}

enum PgEpi { kPgStore = 0, kPgSlab = 1, kPgSilu = 2 };

template <int PW, int S>
__device__ __forceinline__ void pg_wait_ahead(int ahead) {
  // this wave's DMA groups are issued one stage at a time: leave `ahead` stages
  // (PW instructions each) in flight, retire everything older
  if (S >= 4 && ahead >= 2) {
    vm_wait<(S >= 4 ? 2 * PW : 0)>();
  } else if (S >= 3 && ahead >= 1) {
    vm_wait<(S >= 3 ? PW : 0)>();
  } else {
    vm_wait<0>();
  }
}

template <int WM, int WN, int MT, int NT, int S, int EPI>
__global__ __launch_bounds__(WM * WN * 64, 1) void packed_gemm_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ wpk, int N,
    int K, int k_slice, uint16_t* __restrict__ out, int out_stride, float* __restrict__ ws) {
  constexpr int NW = WM * WN;
  static_assert(NW == 8 || NW == 4, "4 or 8 waves");
  constexpr int BM = WM * MT * 16, BN = WN * NT * 16;
  constexpr int A_PW = BM / (8 * NW);   // x DMA instructions per wave per stage (8 rows each)
  constexpr int B_PW = BN * 2 / (16 * NW);  // W DMA instructions per wave per stage (1 KiB each)
  constexpr int PW = A_PW + B_PW;
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  static_assert(S * STAGE <= 160 * 1024, "LDS");
  static_assert(EPI != kPgSilu || NT % 2 == 0, "SiLU pairs need an even NT");
  __shared__ __attribute__((aligned(16))) uint8_t smem[S * STAGE];

  const int lane = lane_id(), w = wave_id();
  const int wm = w / WN, wn = w % WN;
  const int l15 = lane & 15, g = lane >> 4;

  // tile id: XCD-aware bijective remap (guide §5), m fastest inside an n-block
  const int mt_tiles = (M + BM - 1) / BM;
  const int total = gridDim.x;
  const int orig = blockIdx.x;
  const int q = total / 8, r = total % 8, xcd = orig % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tn = wgid / mt_tiles, tm = wgid % mt_tiles;
  const int m0 = tm * BM, n0 = tn * BN;
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int nk = k_slice >> 6;
  const int ksteps = K >> 6;
  const int ntiles_all = N >> 4;

  const uint32_t lds0 = lds_off(smem);

  // per-lane DMA sources (k-step 0 of this split); advanced by 64 elements (x) or
  // one 2 KiB fragment block (W) per stage
  const uint16_t* a_src[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    const int inst = i * NW + w;
    const int rl = inst * 8 + (lane >> 3);
    const int slot = lane & 7;
    const int c = slot ^ ((rl >> 1) & 5);
    const int row = min(m0 + rl, M - 1);
    a_src[i] = x + (size_t)row * x_stride + kbeg + c * 8;
  }
  const uint16_t* b_src[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    const int inst = i * NW + w;
    const int ntl = inst >> 1, h = inst & 1;
    const int nt = min((n0 >> 4) + ntl, ntiles_all - 1);
    b_src[i] = wpk + ((size_t)nt * ksteps + (kbeg >> 6)) * 1024 + h * 512 + lane * 8;
  }

  auto issue = [&](int t) {
    const uint32_t base = lds0 + (t % S) * STAGE;
#pragma unroll
    for (int i = 0; i < A_PW; ++i) glds16(a_src[i] + t * 64, base + (i * NW + w) * 1024);
#pragma unroll
    for (int i = 0; i < B_PW; ++i)
      glds16(b_src[i] + (size_t)t * 1024, base + A_BYTES + (i * NW + w) * 1024);
  };

  pg_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = pg_floatx4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets inside a stage
  uint32_t a_off[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int rl = wm * MT * 16 + i * 16 + l15;
#pragma unroll
    for (int h = 0; h < 2; ++h) a_off[i][h] = rl * 128 + (((2 * g + h) ^ ((rl >> 1) & 5)) * 16);
  }
  const uint32_t b_off = A_BYTES + (wn * NT) * 2048 + lane * 16;

#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < nk) issue(t);

  for (int t = 0; t < nk; ++t) {
    // stage t landed (own DMAs), and every wave is done reading stage t-1's slot
    pg_wait_ahead<PW, S>(min(S - 2, nk - 1 - t));
    lgkm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (t + S - 1 < nk) issue(t + S - 1);
    const uint32_t base = lds0 + (t % S) * STAGE;
    uint4 bf[NT][2];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      bf[j][0] = ds_read16(base + b_off + j * 2048);
      bf[j][1] = ds_read16(base + b_off + j * 2048 + 1024);
    }
    uint4 af[2][2];
    af[0][0] = ds_read16(base + a_off[0][0]);
    af[0][1] = ds_read16(base + a_off[0][1]);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int cur = i & 1;
      if (i + 1 < MT) {
        af[cur ^ 1][0] = ds_read16(base + a_off[i + 1][0]);
        af[cur ^ 1][1] = ds_read16(base + a_off[i + 1][1]);
        lgkm_wait<2>();
      } else {
        lgkm_wait<0>();
      }
      dep(af[cur][0]);
      dep(af[cur][1]);
      if (i == 0) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          dep(bf[j][0]);
          dep(bf[j][1]);
        }
      }
      // raise this wave's issue priority over the MFMA cluster (guide §5 T2): the
      // other wave on the SIMD issues its LDS reads / DMAs in the gaps
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pg_frag(af[cur][0]), pg_frag(bf[j][0]),
                                                            acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pg_frag(af[cur][1]), pg_frag(bf[j][1]),
                                                            acc[i][j], 0, 0, 0);
      }
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // epilogue: C layout, lane (g, l15) holds rows 4g..4g+3 of column l15
  const int mw = m0 + wm * MT * 16;
  const int nw = n0 + wn * NT * 16;
  if (EPI == kPgSilu) {
    const int half_n = N >> 1;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; j += 2) {
        const int col = ((nw + 16 * j) >> 1) + l15;  // pair (gate tile, up tile) -> 16 outputs
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int m = mw + 16 * i + 4 * g + rr;
          if (m < M && col < half_n) {
            const float gv = acc[i][j][rr], uv = acc[i][j + 1][rr];
            out[(size_t)m * out_stride + col] = f32_to_bf16(gv / (1.f + __expf(-gv)) * uv);
          }
        }
      }
  } else {
    float* slab = ws + (size_t)s * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = nw + 16 * j + l15;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int m = mw + 16 * i + 4 * g + rr;
          if (m < M && n < N) {
            if (EPI == kPgSlab)
              slab[(size_t)m * N + n] = acc[i][j][rr];
            else
              out[(size_t)m * out_stride + n] = f32_to_bf16(acc[i][j][rr]);
          }
        }
      }
  }
}

// ---------------------------------------------------------------------------
// 256 x 256 "phased" variant (guide §5 "The 256² 8-phase template", adapted to
// the packed W image): each k-tile (64) is computed in 4 phases, one C quadrant
// (64 x 32 per wave) per phase, and the operand halves (A rows 0-127 / 128-255,
// W columns 0-127 / 128-255, 16 KiB each) are re-filled as soon as the last
// phase that reads them is over, so with only two LDS slots the next-but-one
// tile's halves are in flight while this tile computes.  Waves sit 2 (M) x 4 (N)
// and own rows {mq * 128 + wm * 64 + [0, 64)} x cols {nq * 128 + wn * 32 + [0, 32)}
// for quadrants (mq, nq), so every wave reads the same half in the same phase:
//   phase:        P0          P1          P2          P3
//   quadrant:   Alo.Blo     Alo.Bhi     Ahi.Blo     Ahi.Bhi
//   LDS reads:  Alo, Blo    Bhi         Ahi         -      (kept in registers)
//   DMA issue:  -           Alo,Blo     Bhi         Ahi    of tile t+2
// A half is refilled with tile t+2 one phase after its only read, so two whole
// tiles stay in flight with two LDS slots (6 phases between a half's DMA and its
// first read).  Each phase: counted vmcnt for the data the NEXT phase reads,
// this phase's ds_reads and DMA, s_barrier, MFMA cluster (setprio 1), s_barrier.
template <int EPI>
__global__ __launch_bounds__(512, 1) void packed_gemm8_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ wpk, int N,
    int K, int k_slice, uint16_t* __restrict__ out, int out_stride, float* __restrict__ ws) {
  constexpr int HALF = 16384;              // bytes per operand half-tile
  constexpr int SLOT = 4 * HALF;           // Alo | Ahi | Blo | Bhi
  constexpr int ALO = 0, AHI = HALF, BLO = 2 * HALF, BHI = 3 * HALF;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * SLOT];

  const int lane = lane_id(), w = wave_id();
  const int wm = w >> 2, wn = w & 3;
  const int l15 = lane & 15, g = lane >> 4;

  const int mt_tiles = (M + 255) / 256;
  const int total = gridDim.x;
  const int orig = blockIdx.x;
  const int q = total / 8, r = total % 8, xcd = orig % 8;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  const int tn = wgid / mt_tiles, tm = wgid % mt_tiles;
  const int m0 = tm * 256, n0 = tn * 256;
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int nk = k_slice >> 6;
  const int ksteps = K >> 6;
  const int ntiles_all = N >> 4;
  const uint32_t lds0 = lds_off(smem);

  // DMA sources: half-tile hf (0 = lo, 1 = hi) piece p = w + 8 i (i = 0, 1)
  const uint16_t* a_src[2][2];
  const uint16_t* b_src[2][2];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int piece = w + 8 * i;
      const int rl = piece * 8 + (lane >> 3);           // row within the half
      const int c = (lane & 7) ^ ((rl >> 1) & 5);
      const int row = min(m0 + hf * 128 + rl, M - 1);
      a_src[hf][i] = x + (size_t)row * x_stride + kbeg + c * 8;
      const int nt = min((n0 >> 4) + hf * 8 + (piece >> 1), ntiles_all - 1);
      b_src[hf][i] = wpk + ((size_t)nt * ksteps + (kbeg >> 6)) * 1024 + (piece & 1) * 512 + lane * 8;
    }
  auto issue_a = [&](int hf, int t) {
    const uint32_t base = lds0 + (t & 1) * SLOT + (hf ? AHI : ALO);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(a_src[hf][i] + t * 64, base + (w + 8 * i) * 1024);
  };
  auto issue_b = [&](int hf, int t) {
    const uint32_t base = lds0 + (t & 1) * SLOT + (hf ? BHI : BLO);
#pragma unroll
    for (int i = 0; i < 2; ++i) glds16(b_src[hf][i] + (size_t)t * 1024, base + (w + 8 * i) * 1024);
  };

  // fragment offsets inside a half: A rows wm*64 + i*16 + l15, W n-tiles wn*2 + j
  uint32_t a_off[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = wm * 64 + i * 16 + l15;
#pragma unroll
    for (int h = 0; h < 2; ++h) a_off[i][h] = rl * 128 + (((2 * g + h) ^ ((rl >> 1) & 5)) * 16);
  }
  const uint32_t b_off = (wn * 2) * 2048 + lane * 16;

  pg_floatx4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = pg_floatx4{0.f, 0.f, 0.f, 0.f};

  uint4 alo[4][2], ahi[4][2], blo[2][2], bhi[2][2];
  auto read_a = [&](uint4 (&a)[4][2], uint32_t base) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i][0] = ds_read16(base + a_off[i][0]);
      a[i][1] = ds_read16(base + a_off[i][1]);
    }
  };
  auto read_b = [&](uint4 (&b)[2][2], uint32_t base) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b[j][0] = ds_read16(base + b_off + j * 2048);
      b[j][1] = ds_read16(base + b_off + j * 2048 + 1024);
    }
  };
  auto quad = [&](uint4 (&a)[4][2], uint4 (&b)[2][2], int mq, int nq) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        pg_floatx4& c = acc[mq * 4 + i][nq * 2 + j];
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pg_frag(a[i][0]), pg_frag(b[j][0]), c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pg_frag(a[i][1]), pg_frag(b[j][1]), c, 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  auto dep_a = [&](uint4 (&a)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dep(a[i][0]);
      dep(a[i][1]);
    }
  };
  auto dep_b = [&](uint4 (&b)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      dep(b[j][0]);
      dep(b[j][1]);
    }
  };

  // prologue: tiles 0 and 1 whole (issue order = the steady-state order)
  issue_a(0, 0);
  issue_b(0, 0);
  issue_b(1, 0);
  issue_a(1, 0);
  if (nk > 1) {
    issue_a(0, 1);
    issue_b(0, 1);
    issue_b(1, 1);
    issue_a(1, 1);
    vm_wait<12>();  // tile 0's Alo, Blo
  } else {
    vm_wait<0>();
  }
  __builtin_amdgcn_s_barrier();

  for (int t = 0; t < nk; ++t) {
    const uint32_t base = lds0 + (t & 1) * SLOT;
    const bool steady = t + 2 < nk;   // every issue of the schedule happens
    // ---- P0: reads Alo, Blo (quadrant 0,0); retire Bhi(t) for P1
    if (steady) vm_wait<10>(); else vm_wait<0>();
    read_a(alo, base + ALO);
    read_b(blo, base + BLO);
    __builtin_amdgcn_s_barrier();
    lgkm_wait<0>();
    dep_a(alo);
    dep_b(blo);
    quad(alo, blo, 0, 0);
    __builtin_amdgcn_s_barrier();
    // ---- P1: reads Bhi (0,1); Alo/Blo(t) are in registers -> refill with tile t+2;
    // retire Ahi(t) for P2
    if (steady) vm_wait<8>(); else vm_wait<0>();
    read_b(bhi, base + BHI);
    if (t + 2 < nk) {
      issue_a(0, t + 2);
      issue_b(0, t + 2);
    }
    __builtin_amdgcn_s_barrier();
    lgkm_wait<0>();
    dep_b(bhi);
    quad(alo, bhi, 0, 1);
    __builtin_amdgcn_s_barrier();
    // ---- P2: reads Ahi (1,0); Bhi(t) free -> Bhi(t+2)
    read_a(ahi, base + AHI);
    if (t + 2 < nk) issue_b(1, t + 2);
    __builtin_amdgcn_s_barrier();
    lgkm_wait<0>();
    dep_a(ahi);
    quad(ahi, blo, 1, 0);
    __builtin_amdgcn_s_barrier();
    // ---- P3: (1,1) from registers; Ahi(t) free -> Ahi(t+2); retire Alo/Blo(t+1)
    if (steady) vm_wait<10>(); else vm_wait<0>();
    if (t + 2 < nk) issue_a(1, t + 2);
    __builtin_amdgcn_s_barrier();
    quad(ahi, bhi, 1, 1);
    __builtin_amdgcn_s_barrier();
  }

  // epilogue: acc[mq * 4 + i][nq * 2 + j] -> rows m0 + mq*128 + wm*64 + i*16 + 4g + rr,
  // cols n0 + nq*128 + wn*32 + j*16 + l15
  if (EPI == kPgSilu) {
    const int half_n = N >> 1;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int nq = 0; nq < 2; ++nq) {
        const int col = ((n0 + nq * 128 + wn * 32) >> 1) + l15;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int m = m0 + (mi >> 2) * 128 + wm * 64 + (mi & 3) * 16 + 4 * g + rr;
          if (m < M && col < half_n) {
            const float gv = acc[mi][nq * 2][rr], uv = acc[mi][nq * 2 + 1][rr];
            out[(size_t)m * out_stride + col] = f32_to_bf16(gv / (1.f + __expf(-gv)) * uv);
          }
        }
      }
  } else {
    float* slab = ws + (size_t)s * M * N;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) {
        const int n = n0 + (nj >> 1) * 128 + wn * 32 + (nj & 1) * 16 + l15;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int m = m0 + (mi >> 2) * 128 + wm * 64 + (mi & 3) * 16 + 4 * g + rr;
          if (m < M && n < N) {
            if (EPI == kPgSlab)
              slab[(size_t)m * N + n] = acc[mi][nj][rr];
            else
              out[(size_t)m * out_stride + n] = f32_to_bf16(acc[mi][nj][rr]);
          }
        }
      }
  }
}


// ---------------------------------------------------------------------------
// "pg32": the tile of packed_gemm_kernel with 32-deep stages in an S-slot LDS ring
// (BM x BN x 32 per slot, S = 5 for 256 x 256: the whole 160 KiB), so S - 1 stages
// (4 x 32 KiB for 256 x 256) are in flight while one computes -- packed_gemm_kernel's
// 64-deep stages fit two slots and keep ONE stage in flight, which at one workgroup
// per CU leaves the DMA latency exposed at every k-step (0.44-1.1 PF/s at 129-512
// rows, profiles/pg_probe_192_r04.log).  One raw s_barrier per stage; the slot a
// stage is loaded into was last read one stage earlier, and every wave consumed
// those reads in its MFMAs before it reached the barrier.
//   * stage t is half h = t & 1 of 64-deep k-step t >> 1, and in the packed image
//     half h of lane (g, r) holds k = 16 g + 8 h + [0, 8) of that k-step
//     (ops.pack_weight), so the A chunk c of a stage row is x[row][64 (t >> 1) +
//     16 c + 8 h + [0, 8)]: four 16-B pieces at a 32-B stride (the other half's
//     pieces fill the gaps one stage later, from the same L2 lines).
//   * A (x rows): 16 rows x 64 B per DMA instruction, the 16-B chunk c of local row
//     r at slot c ^ f[(r >> 2) & 3], f = {0, 2, 3, 1}: the four ds_read_b128 lane
//     groups of an A fragment (lane (g, r) reads row r, chunk g) then hit 16
//     distinct 16-B bank slots (conflict-free); the swizzle is applied on the
//     per-lane SOURCE address (the DMA destination is lane-linear).
//   * B (packed W): the two 32-deep halves of a 64-deep fragment block are
//     contiguous, so stage t of a column tile is 1 KiB at element offset 512 t;
//     the LDS image is in fragment order (lane l reads 16 B at 16 l).
//   * 8 waves as 2 (M) x 4 (N), each MT x NT 16 x 16 tiles, v_mfma_f32_16x16x32_bf16.
//   * bf16 / SiLU epilogues go through LDS (rows padded to 144 / 80 B, conflict
//     free) and leave as 16-B row stores; fp32 slabs are stored directly.
__device__ __forceinline__ int pg32_swz(int rq) { return (0x1320 >> (4 * (rq & 3))) & 3; }

template <int PW, int D>
__device__ __forceinline__ void pg32_wait(int ahead) {
  // retire everything but `ahead` stages (PW DMA instructions each) of this wave
  if constexpr (D >= 4) {
    if (ahead >= 3) { vm_wait<3 * PW>(); return; }
  }
  if constexpr (D >= 3) {
    if (ahead >= 2) { vm_wait<2 * PW>(); return; }
  }
  if constexpr (D >= 2) {
    if (ahead >= 1) { vm_wait<PW>(); return; }
  }
  vm_wait<0>();
}

template <int MT, int NT, int S, int EPI>
__global__ __launch_bounds__(512, 1) void pg32_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ wpk, int N,
    int K, int k_slice, uint16_t* __restrict__ out, int out_stride, float* __restrict__ ws) {
  constexpr int BM = 32 * MT, BN = 64 * NT;
  constexpr int A_BYTES = BM * 64, B_BYTES = BN * 64, SLOT = A_BYTES + B_BYTES;
  constexpr int A_INST = BM / 16, B_INST = BN / 16;   // 1 KiB DMA instructions per stage
  constexpr int A_PW = (A_INST + 7) / 8, B_PW = (B_INST + 7) / 8;
  constexpr int PW = A_PW + B_PW;
  constexpr int D = S - 1;   // stages in flight ahead of the computing one
  static_assert(S * SLOT <= 160 * 1024, "LDS");
  static_assert(D >= 1 && D <= 5, "ring depth");
  static_assert(EPI != kPgSilu || NT % 2 == 0, "SiLU pairs need an even NT");
  __shared__ __attribute__((aligned(16))) uint8_t smem[S * SLOT];

  const int lane = lane_id(), w = wave_id();
  const int wm = w >> 2, wn = w & 3;
  const int l15 = lane & 15, g = lane >> 4;

  // tile id: XCD-aware bijective remap, m fastest inside an n-block (the m-tiles that
  // read one weight slice run together on one XCD and share it through its L2)
  const int mt_tiles = (M + BM - 1) / BM;
  const int total = gridDim.x;
  const int orig = blockIdx.x;
  const int q = total / 8, r8 = total % 8, xcd = orig % 8;
  const int wgid = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
  const int tn = wgid / mt_tiles, tm = wgid % mt_tiles;
  const int m0 = tm * BM, n0 = tn * BN;
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int ns = k_slice >> 5;
  const int ksteps = K >> 6;
  const int ntiles_all = N >> 4;
  const uint32_t lds0 = lds_off(smem);

  // per-wave DMA instructions (every wave issues A_PW + B_PW per stage, so the
  // counted vmcnt waits are uniform; a wave without an instruction of its own
  // re-issues one of another wave: the same bytes to the same place)
  const uint16_t* a_src[A_PW];
  uint32_t a_dst[A_PW];
#pragma unroll
  for (int i = 0; i < A_PW; ++i) {
    int inst = w + 8 * i;
    if (inst >= A_INST) inst %= A_INST;
    const int rl = inst * 16 + (lane >> 2);
    const int c = (lane & 3) ^ pg32_swz(g);   // (rl & 15) >> 2 == lane >> 4
    const int row = min(m0 + rl, M - 1);
    a_src[i] = x + (size_t)row * x_stride + kbeg + c * 16;
    a_dst[i] = inst * 1024;
  }
  const uint16_t* b_src[B_PW];
  uint32_t b_dst[B_PW];
#pragma unroll
  for (int i = 0; i < B_PW; ++i) {
    int inst = w + 8 * i;
    if (inst >= B_INST) inst %= B_INST;
    const int nt = min((n0 >> 4) + inst, ntiles_all - 1);
    b_src[i] = wpk + ((size_t)nt * ksteps + (kbeg >> 6)) * 1024 + lane * 8;
    b_dst[i] = A_BYTES + inst * 1024;
  }
  auto issue = [&](int t, uint32_t base) {
#pragma unroll
    for (int i = 0; i < A_PW; ++i) glds16(a_src[i] + (t >> 1) * 64 + (t & 1) * 8, base + a_dst[i]);
#pragma unroll
    for (int i = 0; i < B_PW; ++i) glds16(b_src[i] + (size_t)t * 512, base + b_dst[i]);
  };

  pg_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = pg_floatx4{0.f, 0.f, 0.f, 0.f};

  const uint32_t a_off = (wm * MT) * 1024 + l15 * 64 + ((g ^ pg32_swz(l15 >> 2)) * 16);
  const uint32_t b_off = A_BYTES + (wn * NT) * 1024 + lane * 16;

#pragma unroll
  for (int t = 0; t < D; ++t)
    if (t < ns) issue(t, lds0 + t * SLOT);

  int slot = 0;        // slot of stage t
  int islot = D % S;   // slot of stage t + D
  for (int t = 0; t < ns; ++t) {
    pg32_wait<PW, D>(min(D - 1, ns - 1 - t));
    __builtin_amdgcn_s_barrier();
    if (t + D < ns) issue(t + D, lds0 + islot * SLOT);
    const uint32_t base = lds0 + slot * SLOT;
    uint4 bf[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bf[j] = ds_read16(base + b_off + j * 1024);
    uint4 af[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) af[i] = ds_read16(base + a_off + i * 1024);
    static_for<0, MT>([&](auto I) {
      constexpr int i = decltype(I)::value;
      lgkm_wait<MT - 1 - i>();
      dep(af[i]);
      if constexpr (i == 0) {
#pragma unroll
        for (int j = 0; j < NT; ++j) dep(bf[j]);
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pg_frag(af[i]), pg_frag(bf[j]),
                                                            acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    });
    slot = slot + 1 == S ? 0 : slot + 1;
    islot = islot + 1 == S ? 0 : islot + 1;
  }

  // epilogue: C layout, lane (g, l15) holds rows 4g..4g+3 of column l15 of each tile
  const int mw = m0 + wm * MT * 16;
  const int nw = n0 + wn * NT * 16;
  if constexpr (EPI == kPgSlab) {
    float* slab = ws + (size_t)s * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = nw + 16 * j + l15;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int m = mw + 16 * i + 4 * g + rr;
          if (m < M && n < N) slab[(size_t)m * N + n] = acc[i][j][rr];
        }
      }
    return;
  }
  // bf16 rows through LDS: this wave's (16 MT) x OC tile, rows padded to RS bytes
  constexpr int OC = EPI == kPgSilu ? 8 * NT : 16 * NT;   // output columns per wave
  constexpr int RS = OC * 2 + 16;
  static_assert(8 * 16 * MT * RS <= S * SLOT, "epilogue staging");
  __syncthreads();   // every wave is past its last fragment read; no DMA in flight
  uint8_t* sw = smem + w * (16 * MT * RS);
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 16 * i + 4 * g + rr;
      if constexpr (EPI == kPgSilu) {
#pragma unroll
        for (int j = 0; j < NT; j += 2) {
          const float gv = acc[i][j][rr], uv = acc[i][j + 1][rr];
          *reinterpret_cast<uint16_t*>(sw + row * RS + ((j >> 1) * 16 + l15) * 2) =
              f32_to_bf16(gv / (1.f + __expf(-gv)) * uv);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NT; ++j)
          *reinterpret_cast<uint16_t*>(sw + row * RS + (16 * j + l15) * 2) =
              f32_to_bf16(acc[i][j][rr]);
      }
    }
  // the wave reads back only its own staging rows (no other wave touches them)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  constexpr int CPR = OC / 8;             // 16-B chunks per output row
  constexpr int RPI = 64 / CPR;           // rows per wave instruction
  const int out_cols = EPI == kPgSilu ? (N >> 1) : N;
  const int oc0 = EPI == kPgSilu ? (nw >> 1) : nw;
#pragma unroll
  for (int r0 = 0; r0 < 16 * MT; r0 += RPI) {
    const int row = r0 + lane / CPR, ch = lane % CPR;
    const uint4 v = *reinterpret_cast<const uint4*>(sw + row * RS + ch * 16);
    const int m = mw + row, c = oc0 + ch * 8;
    if (m < M && c < out_cols)
      *reinterpret_cast<uint4*>(out + (size_t)m * out_stride + c) = v;
  }
}

}  // namespace ft

// cfg: 0 = 256x256 tile (2x4 waves of 128x64, 2 LDS slots), 1 = 128x256 (2x4 waves
// of 64x64, 3 slots), 2 = 256x128 (4x2 waves of 64x64, 3 slots), 3 = 256x256 phased,
// 5 = 192x256 (2x4 waves of 96x64, 2 slots), 6 = 192x128 (4x2 waves of 48x64, 3 slots).
// epi: 0 bf16 out, 1 fp32 slabs (splits > 1), 2 SiLU-mul of interleaved gate/up.
// Requirements (checked): N % 16 == 0 (N % 32 for SiLU), K % (64 * splits) == 0.
extern "C" int ft_packed_gemm(const void* x, int x_stride, int M, const void* wpk, int N, int K,
                              int splits, int epi, int cfg, void* out, int out_stride, float* ws,
                              hipStream_t stream) {
  if (M <= 0) return 0;
  if (N % 16 != 0 || (epi == 2 && N % 32 != 0)) return -2;
  if (splits < 1 || K % (64 * splits) != 0) return -3;
  if ((epi == 1) != (splits > 1)) return -4;
  if (epi == 1 && ws == nullptr) return -4;
  const int k_slice = K / splits;
  int bm, bn;
  switch (cfg) {
    case 0: bm = 256; bn = 256; break;
    case 1: bm = 128; bn = 256; break;
    case 2: bm = 256; bn = 128; break;
    case 3: bm = 256; bn = 256; break;
    case 4: bm = 256; bn = 256; break;
    case 5: bm = 192; bn = 256; break;
    case 6: bm = 192; bn = 128; break;
    case 10: bm = 256; bn = 256; break;
    case 11: bm = 192; bn = 256; break;
    case 12: bm = 128; bn = 256; break;
    case 13: bm = 256; bn = 128; break;
    case 14: bm = 64; bn = 256; break;
    default: return -5;
  }
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  dim3 grid(tiles, splits), block(cfg == 4 ? 256 : 512);
  if (cfg >= 10) {
    // pg32 (BK 32 ring): bf16 / SiLU epilogues store 16-B row chunks
    if (epi != 1 && (out_stride % 8 != 0 || (reinterpret_cast<uintptr_t>(out) & 15) != 0)) return -6;
  }
#define FT_PG(CFG, WM, WN, MT, NT, S)                                                          \
  if (cfg == CFG) {                                                                            \
    if (epi == 0)                                                                              \
      hipLaunchKernelGGL((ft::packed_gemm_kernel<WM, WN, MT, NT, S, ft::kPgStore>), grid,      \
                         block, 0, stream, (const uint16_t*)x, x_stride, M,                    \
                         (const uint16_t*)wpk, N, K, k_slice, (uint16_t*)out, out_stride, ws); \
    else if (epi == 1)                                                                         \
      hipLaunchKernelGGL((ft::packed_gemm_kernel<WM, WN, MT, NT, S, ft::kPgSlab>), grid,       \
                         block, 0, stream, (const uint16_t*)x, x_stride, M,                    \
                         (const uint16_t*)wpk, N, K, k_slice, (uint16_t*)out, out_stride, ws); \
    else                                                                                       \
      hipLaunchKernelGGL((ft::packed_gemm_kernel<WM, WN, MT, NT, S, ft::kPgSilu>), grid,       \
                         block, 0, stream, (const uint16_t*)x, x_stride, M,                    \
                         (const uint16_t*)wpk, N, K, k_slice, (uint16_t*)out, out_stride, ws); \
    return static_cast<int>(hipGetLastError());                                                \
  }
  if (cfg == 3) {
    if (epi == 0)
      hipLaunchKernelGGL((ft::packed_gemm8_kernel<ft::kPgStore>), grid, block, 0, stream,
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, N, K, k_slice,
                         (uint16_t*)out, out_stride, ws);
    else if (epi == 1)
      hipLaunchKernelGGL((ft::packed_gemm8_kernel<ft::kPgSlab>), grid, block, 0, stream,
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, N, K, k_slice,
                         (uint16_t*)out, out_stride, ws);
    else
      hipLaunchKernelGGL((ft::packed_gemm8_kernel<ft::kPgSilu>), grid, block, 0, stream,
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, N, K, k_slice,
                         (uint16_t*)out, out_stride, ws);
    return static_cast<int>(hipGetLastError());
  }
  FT_PG(0, 2, 4, 8, 4, 2)
  FT_PG(4, 2, 2, 8, 8, 2)
  FT_PG(1, 2, 4, 4, 4, 3)
  FT_PG(2, 4, 2, 4, 4, 3)
  // 192-row tiles: mixed steps of 129-192 / 257-384 rows pad to 192 / 384 instead of
  // 256 / 512 (a third fewer MFMA rows computed for nothing)
  FT_PG(5, 2, 4, 6, 4, 2)
  FT_PG(6, 4, 2, 3, 4, 3)
#undef FT_PG
#define FT_PG32(CFG, MT, NT, S)                                                              \
  if (cfg == CFG) {                                                                          \
    if (epi == 0)                                                                            \
      hipLaunchKernelGGL((ft::pg32_kernel<MT, NT, S, ft::kPgStore>), grid, block, 0, stream, \
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, N, K,        \
                         k_slice, (uint16_t*)out, out_stride, ws);                           \
    else if (epi == 1)                                                                       \
      hipLaunchKernelGGL((ft::pg32_kernel<MT, NT, S, ft::kPgSlab>), grid, block, 0, stream,  \
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, N, K,        \
                         k_slice, (uint16_t*)out, out_stride, ws);                           \
    else                                                                                     \
      hipLaunchKernelGGL((ft::pg32_kernel<MT, NT, S, ft::kPgSilu>), grid, block, 0, stream,  \
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, N, K,        \
                         k_slice, (uint16_t*)out, out_stride, ws);                           \
    return static_cast<int>(hipGetLastError());                                              \
  }
  FT_PG32(10, 8, 4, 5)
  FT_PG32(11, 6, 4, 5)
  FT_PG32(12, 4, 4, 6)
  FT_PG32(13, 8, 2, 6)
  FT_PG32(14, 2, 4, 6)
#undef FT_PG32
  return -5;
}

