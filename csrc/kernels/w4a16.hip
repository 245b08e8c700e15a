// E9 / K14: W4A16 (AWQ-style, group 128, asymmetric) weight-only GEMMs.
//   y[M, N] = x[M, K] . dequant(W)[N, K]^T,  dequant(W)[n, k] = (q[n,k] - z[n,g]) * s[n,g],
//   g = k / 128, q and z 4-bit.  Reference: --quantization awq
//   (docker-compose.vllm.yml:45-46, Llama-3.1-8B AWQ in app/utils/config.py:93-96).
//
// Decode (M <= 64) is a weight stream, and int4 cuts it 3.6x vs bf16, so the
// kernel is the packed-fragment skinny GEMM (skinny_gemm.hip, "pk") with the
// dequantization moved out of the inner loop:
//   * packed image [N/16][K/128][lane][4 x u32]: one 16-B load per lane = 1 KiB
//     of consecutive bytes per wave instruction = one 128-wide k-group for a
//     16-column tile.  Lane (n = l&15, g = l>>4) word w holds the 8 nibbles of
//     k = 128*grp + 64*(w>>1) + 16*g + 8*(w&1) + {0,2,4,6,1,3,5,7} (bit order),
//     so ((word >> 4i) & 0x000F000F) | 0x43004300 is the bf16 pair
//     (128 + q[2i], 128 + q[2i+1]) -- exact in bf16 -- and the four pairs are
//     the lane's MFMA B fragment: one shift + one and-or per two weights.
//   * acc_grp = x . (128 + q) over the group (exact bf16 products, fp32 sums),
//     xsum = x . 1 from two extra MFMAs per row tile (B = ones), then
//       y += s * (acc_grp - (128 + z) * xsum)       (2 FMAs per acc register)
//     with (s, 128 + z) as one float2 per (column, group) in a side array
//     [N/16][K/128][16].
//   * 4 waves split the groups of a column tile; with a workspace, split-K over
//     gridDim.y (1 split included) writes fp32 slabs reduced by the row
//     epilogues (fused_epilogue.hip), exactly as the bf16 packed path; without
//     one (1 split) it stores bf16.
// Above 64 rows the model runs packed_gemm.hip on a resident dequantized prefill
// image (models/llama.py _prepare_w4_prefill), or on one projection dequantized by
// w4_dequant_kernel into a packed scratch when that image is off.
#include "ft_common.h"
#include "ft_lds.h"

#include <type_traits>

namespace ft {

typedef __bf16 w4_bf16x8 __attribute__((ext_vector_type(8)));
typedef float w4_floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int w4_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 w4_nt_load16(const uint32_t* p) {
  const w4_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const w4_u32x4*>(p));
  return __builtin_bit_cast(uint4, v);
}

// one packed u32 (8 nibbles) -> the 8 bf16 values 128 + q of an MFMA B fragment
__device__ __forceinline__ w4_bf16x8 w4_frag(uint32_t w) {
  uint4 r;
  r.x = (w & 0x000F000Fu) | 0x43004300u;
  r.y = ((w >> 4) & 0x000F000Fu) | 0x43004300u;
  r.z = ((w >> 8) & 0x000F000Fu) | 0x43004300u;
  r.w = ((w >> 12) & 0x000F000Fu) | 0x43004300u;
  return __builtin_bit_cast(w4_bf16x8, r);
}

// the same with the two constants in VGPRs (opaque to the compiler): gfx950's VOP3
// encoding takes no literal, so with literal masks hipcc emitted v_and + v_or per
// output word (11 VALU per packed word); with register operands it is one
// v_and_or_b32 (7 per word)
__device__ __forceinline__ w4_bf16x8 w4_frag_r(uint32_t w, uint32_t vm, uint32_t vc) {
  uint4 r;
  r.x = (w & vm) | vc;
  r.y = ((w >> 4) & vm) | vc;
  r.z = ((w >> 8) & vm) | vc;
  r.w = ((w >> 12) & vm) | vc;
  return __builtin_bit_cast(w4_bf16x8, r);
}

__device__ __forceinline__ w4_bf16x8 w4_xfrag(const uint4& v) {
  return __builtin_bit_cast(w4_bf16x8, v);
}

template <int MT, int NT>
struct W4Stage {
  uint4 w[NT];      // one k-group of NT column tiles
  float2 sz[NT];    // (scale, 128 + zero) of this lane's column
  uint4 x[MT][4];   // 2 k-steps x 2 halves
};

template <int MT, int NT>
__global__ __launch_bounds__(256) void w4_skinny_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint32_t* __restrict__ wq,
    const float2* __restrict__ sz, int K, float* __restrict__ ws, uint16_t* __restrict__ out,
    int out_stride, int N, int k_slice) {
  __shared__ float s_red[4][MT * NT * 4][64];
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int groups_total = K >> 7;
  const int grp0 = kbeg >> 7;

  const uint32_t* wp[NT];
  const float2* sp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const size_t tile = (size_t)(n0 / 16 + j) * groups_total;
    wp[j] = wq + tile * 256 + lane * 4;
    sp[j] = sz + tile * 16 + l15;
  }
  const uint16_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = min(16 * i + l15, M - 1);
    xp[i] = x + (size_t)r * x_stride + kbeg + 16 * g;
  }

  w4_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = w4_floatx4{0.f, 0.f, 0.f, 0.f};

  const int ngroups = k_slice >> 7;
  const int my = ngroups > wave ? (ngroups - wave + 3) >> 2 : 0;
  const int last = my - 1;
  auto grp = [&](int t) { return wave + 4 * min(t, last); };
  auto load = [&](W4Stage<MT, NT>& st, int t) {
    const int gi = grp(t);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      st.w[j] = w4_nt_load16(wp[j] + (size_t)(grp0 + gi) * 256);
      st.sz[j] = sp[j][(size_t)(grp0 + gi) * 16];
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint4* p = reinterpret_cast<const uint4*>(xp[i] + gi * 128);
      st.x[i][0] = p[0];
      st.x[i][1] = p[1];
      st.x[i][2] = p[8];   // +64 elements: second k-step
      st.x[i][3] = p[9];
    }
  };
  const uint4 ones4 = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  const w4_bf16x8 ones = __builtin_bit_cast(w4_bf16x8, ones4);
  auto compute = [&](const W4Stage<MT, NT>& st) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      w4_floatx4 xs = w4_floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int h = 0; h < 4; ++h)
        xs = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w4_xfrag(st.x[i][h]), ones, xs, 0, 0, 0);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint32_t wd[4] = {st.w[j].x, st.w[j].y, st.w[j].z, st.w[j].w};
        w4_floatx4 a = w4_floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int h = 0; h < 4; ++h)
          a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w4_xfrag(st.x[i][h]), w4_frag(wd[h]), a, 0,
                                                      0, 0);
        const float sc = st.sz[j].x, zz = st.sz[j].y;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaf(sc, fmaf(-zz, xs[r], a[r]), acc[i][j][r]);
      }
    }
  };
  if (my > 0) {
    W4Stage<MT, NT> a, b;
    load(a, 0);
    int t = 0;
    for (; t + 2 <= my; t += 2) {
      load(b, t + 1);
      __builtin_amdgcn_sched_barrier(0);
      compute(a);
      __builtin_amdgcn_sched_barrier(0);
      load(a, t + 2);
      __builtin_amdgcn_sched_barrier(0);
      compute(b);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t < my) compute(a);
  }

  // The C fragment of a 16x16 MFMA: column = lane & 15, rows 4*(lane>>4) + r.
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_red[wave][(i * NT + j) * 4 + r][lane] = acc[i][j][r];
  __syncthreads();
  constexpr int NREG = MT * NT * 4;
  const int ln = threadIdx.x & 63;
  float* slab = ws + (size_t)s * M * N;
  for (int reg = threadIdx.x >> 6; reg < NREG; reg += 4) {
    const float v = s_red[0][reg][ln] + s_red[1][reg][ln] + s_red[2][reg][ln] + s_red[3][reg][ln];
    const int i = reg / (NT * 4), j = (reg / 4) % NT, r = reg & 3;
    const int m = 16 * i + (ln >> 4) * 4 + r;
    const int n = n0 + 16 * j + (ln & 15);
    if (m < M) {
      if (ws == nullptr)
        out[(size_t)m * out_stride + n] = f32_to_bf16(v);
      else
        slab[(size_t)m * N + n] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// "xr" W4 variant for 17..64 rows (the batched decode steps): at 64 rows the
// kernel above re-reads every x fragment per wave and column tile -- 16 B of x
// per lane and k-group against 16 B of int4 weights for 16 columns, so its x
// traffic is 16x the weight stream and the 64-row bucket ran no faster than the
// bf16 image (gate_up 47.5 vs 44.7 us).  Here, as in skinny_gemm.hip's "xr":
//   * the workgroup stages x for a 512-wide K chunk (4 groups) in LDS once
//     (double-buffered, one barrier per chunk); each staging thread loads one
//     (row, group) run of 128 k (256 B contiguous) and also writes that run's sum
//     xs = x . 1 to LDS, so the zero-point correction needs no MFMAs with ones;
//   * each wave streams NT column tiles; every group's weight registers are
//     refilled with the next chunk's fragment right after use (a register ring
//     across chunks: KS x NT x 16 B per lane in flight, no drain between chunks);
//   * per (group, tile) the 4 MFMAs give a = x . (128 + q) and
//     y += s * (a - (128 + z) * xs): 2 FMAs per accumulator register.
// EPI 1: SiLU epilogue on a gate/up image interleaved in 16-row groups
// (ops.quant.pack_w4 of interleave_gate_up(w, 1)): with NT = 2 a wave holds a gate
// tile and its up tile and writes h = silu(g) * u (N/2 columns, bf16).
template <int MT, int NT, int EPI>
__global__ __launch_bounds__(256, 1) void w4_xr_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint32_t* __restrict__ wq,
    const float2* __restrict__ sz, int K, float* __restrict__ ws, uint16_t* __restrict__ out,
    int out_stride, int N, int k_slice) {
  constexpr bool SILU = EPI == 1;
  static_assert(!SILU || NT % 2 == 0, "SiLU pairs a gate tile with its up tile");
  constexpr int KC = 512, NG = KC / 128;     // k per chunk, groups per chunk
  constexpr int ROWS = 16 * MT;
  constexpr int XR = 16;                      // 16-B loads per staging thread (one group)
  __shared__ __attribute__((aligned(16))) uint16_t s_x[2][ROWS * KC];
  __shared__ __attribute__((aligned(16))) float s_xs[2][NG][ROWS];
  const int tid = threadIdx.x;
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = (blockIdx.x * 4 + wave) * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int nch = k_slice / KC;
  const int groups_total = K >> 7;
  const int grp0 = kbeg >> 7;

  // staging thread -> (row, group) run of this chunk; threads past ROWS * NG idle
  const bool stager = tid < ROWS * NG;
  const int srow = tid / NG, sgrp = tid % NG;
  const uint16_t* xsrc = x + (size_t)min(srow, M - 1) * x_stride + kbeg + sgrp * 128;

  const uint32_t* wp[NT];
  const float2* sp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const size_t tile = (size_t)(min(n0 + 16 * j, N - 16) / 16) * groups_total + grp0;
    wp[j] = wq + tile * 256 + lane * 4;
    sp[j] = sz + tile * 16 + l15;
  }

  w4_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = w4_floatx4{0.f, 0.f, 0.f, 0.f};

  w4_u32x4 xr[XR];
  w4_u32x4 wr[NG][NT];
  float2 szr[NG][NT];
  auto load_x = [&](int c) {
    if (stager) {
#pragma unroll
      for (int p = 0; p < XR; ++p) xr[p] = *reinterpret_cast<const w4_u32x4*>(xsrc + (size_t)c * KC + p * 8);
    }
  };
  auto load_w = [&](int c, int gq) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      wr[gq][j] = __builtin_nontemporal_load(reinterpret_cast<const w4_u32x4*>(wp[j] + (size_t)(c * NG + gq) * 256));
      szr[gq][j] = sp[j][(size_t)(c * NG + gq) * 16];
    }
  };
  load_x(0);
#pragma unroll
  for (int gq = 0; gq < NG; ++gq) load_w(0, gq);

  auto chunk = [&](int c, auto more_tag) {
    constexpr bool MORE = decltype(more_tag)::value;
    uint16_t* sx = s_x[c & 1];
    if (stager) {
      // the run's 16 chunks -> LDS (16-B chunk swizzle as in skinny_gemm.hip), and its sum
      float sum = 0.f;
#pragma unroll
      for (int p = 0; p < XR; ++p) {
        const int ch = sgrp * 16 + p;
        const int slot = (ch & ~7) | ((ch & 7) ^ (srow & 7));
        *reinterpret_cast<w4_u32x4*>(&sx[srow * KC + slot * 8]) = xr[p];
        float f[8];
        load8(__builtin_bit_cast(uint4, xr[p]), f);
        sum += ((f[0] + f[1]) + (f[2] + f[3])) + ((f[4] + f[5]) + (f[6] + f[7]));
      }
      s_xs[c & 1][sgrp][srow] = sum;
    }
    if constexpr (MORE) load_x(c + 1);
    __syncthreads();   // chunk c visible; every wave is past chunk c-1's reads of the other buffer
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int row = 16 * i + l15;
        w4_u32x4 xf[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int ch = gq * 16 + 8 * (h >> 1) + 2 * g + (h & 1);
          const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
          xf[h] = *reinterpret_cast<const w4_u32x4*>(&sx[row * KC + slot * 8]);
        }
        float xs[4];
        {
          const float4 xs4 = *reinterpret_cast<const float4*>(&s_xs[c & 1][gq][16 * i + 4 * g]);
          xs[0] = xs4.x; xs[1] = xs4.y; xs[2] = xs4.z; xs[3] = xs4.w;
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          w4_floatx4 a = w4_floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int h = 0; h < 4; ++h)
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(w4_bf16x8, xf[h]),
                                                        w4_frag(wr[gq][j][h]), a, 0, 0, 0);
          const float sc = szr[gq][j].x, zz = szr[gq][j].y;
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaf(sc, fmaf(-zz, xs[r], a[r]), acc[i][j][r]);
        }
      }
      if constexpr (MORE) load_w(c + 1, gq);   // refill this group's registers
    }
  };
  for (int c = 0; c + 1 < nch; ++c) chunk(c, std::true_type{});
  chunk(nch - 1, std::false_type{});
  if (n0 >= N) return;
  if constexpr (SILU) {
#pragma unroll
    for (int j = 0; j < NT; j += 2) {
      const int col = ((n0 + 16 * j) >> 1) + l15;   // (gate tile, up tile) -> 16 h columns
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = 16 * i + g * 4 + r;
          if (m < M) {
            const float gt = acc[i][j][r], up = acc[i][j + 1][r];
            out[(size_t)m * out_stride + col] = f32_to_bf16(gt / (1.f + __expf(-gt)) * up);
          }
        }
    }
    return;
  }
  float* slab = ws + (size_t)s * M * N;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * i + g * 4 + r;
      if (m < M) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int n = n0 + 16 * j + l15;
          if (ws == nullptr)
            out[(size_t)m * out_stride + n] = f32_to_bf16(acc[i][j][r]);
          else
            slab[(size_t)m * N + n] = acc[i][j][r];
        }
      }
    }
}


// ---------------------------------------------------------------------------
// "mh" W4 variant for 33..64 rows (round 6).  Measured on MI355X at 50 rows
// (bench/w4mx_sweep.py, profiles/w4_mh_r06.log): qkv 12.2 vs 13.9 us, o 8.8 vs
// 9.2, gate_up + SiLU 38.5 vs 40.0 against xr / the register kernel; down stays on
// the register kernel.  Relative to xr:
//   * the zero-point term leaves the inner loop: y = sum_g s_g a_g - sum_g (s_g z'_g)
//     xs_g, a_g = x . (128 + q) over group g and xs_g = x . 1; the loop keeps one FMA
//     per accumulator register and group, the sums xs_g are parked in LDS, and
//     after the loop one v_mfma_f32_16x16x4_f32 per four groups subtracts
//     xs . (s z')^T (exact fp32 operands) into the same accumulators;
//   * the x . 1 sums come from the fragments the main loop already holds: for group
//     gi the column wave cw == gi % 4 of each row half adds 4 ones-MFMAs per row
//     tile (no VALU sums, no extra LDS reads, +12.5% MFMA);
//   * conflict-free x layout: 16-B piece ch of row r at slot ch ^ (r & 15) (each
//     16-lane group of a ds_read_b128 covers all 64 banks once; PMC: LDS bank
//     conflict cycles 4.6M -> 57k per 64 gate_up calls);
//   * two column tiles per wave (each x fragment read feeds two MFMAs), the rows
//     split over MH halves of two row tiles: waves (cw, mh), cw = column wave 0..3;
//     the two row halves of a column wave load the same weight bytes (served
//     on-chip the second time) and dequantize them each, so 8 waves (two per SIMD)
//     fit in 256 registers without spills;
//   * dequant with its constants in registers: one v_and_or_b32 per output word;
//   * weight ring RING chunks deep (KC 256 = 2 groups per chunk); XD = 2 keeps two
//     x chunks in flight (ring 2).
// What still bounds it (ablations, profiles/w4_mh_r06.log): the weight stream of
// this register-ring form alone -- no math, no x loads, no barriers, no scale loads
// -- takes 22 us for gate_up against 12.2 us for a plain 66 MB read
// (profiles/bw_blocks_r06.log): 8 KB of loads in flight per wave is what 256
// registers allow; going past it needs an LDS-DMA weight ring.
// Epilogues: bf16 out (ws == nullptr) or fp32 slabs ws[s][m][n]; EPI 1 SiLU of the
// in-wave gate / up tile pair of the 16-row interleaved image.  x rows >= M are
// never loaded (an MFMA row feeds only its own output row).
template <int MH, int RING, int EPI, int XD>
__global__ __launch_bounds__(256 * MH, 2) void w4_mh_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint32_t* __restrict__ wq,
    const float2* __restrict__ sz, int K, float* __restrict__ ws, uint16_t* __restrict__ out,
    int out_stride, int N, int k_slice) {
  constexpr bool SILU = EPI == 1;
  static_assert(XD == 1 || RING % 2 == 0, "two x register sets ride the ring-slot parity");
  constexpr int MTW = 2, NT = 2, KC = 256, NG = KC / 128;
  constexpr int NW = 4 * MH;
  constexpr int ROWS = 16 * MTW * MH;
  constexpr int NTH = 64 * NW;
  constexpr int CPR = KC / 8;                // 16-B x pieces per row per chunk
  constexpr int XL = (ROWS * CPR + NTH - 1) / NTH;
  constexpr int XSG = 32;                    // groups per K slice (host-checked)
  __shared__ __attribute__((aligned(16))) uint16_t s_x[2][ROWS * KC];
  __shared__ float s_xs[ROWS][XSG + 1];
  const int tid = threadIdx.x;
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int cw = wave & 3, mh = wave >> 2;
  const int t0 = (blockIdx.x * 4 + cw) * NT;          // first 16-column tile of this wave
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int nch = k_slice / KC;
  const int groups_total = K >> 7;
  const int grp0 = kbeg >> 7;
  const int ntiles = N >> 4;

  int xoff[XL];
  bool xok[XL];
#pragma unroll
  for (int p = 0; p < XL; ++p) {
    const int e = tid + NTH * p;
    const int row = e / CPR;
    xok[p] = e < ROWS * CPR && row < M;
    xoff[p] = min(row, M - 1) * x_stride + kbeg + (e % CPR) * 8;
  }
  const uint32_t* wp[NT];
  const float* sp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const size_t tile = (size_t)min(t0 + j, ntiles - 1) * groups_total + grp0;
    wp[j] = wq + tile * 256 + lane * 4;
    sp[j] = reinterpret_cast<const float*>(sz + tile * 16 + l15);
  }
  // this wave's LDS row base (row tile 2 mh + i, row l15 of it), swizzle key l15
  const int rbase = (16 * MTW * mh + l15) * KC;

  w4_floatx4 acc[MTW][NT];
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = w4_floatx4{0.f, 0.f, 0.f, 0.f};

  w4_u32x4 xr[XD][XL];
  w4_u32x4 wr[RING][NG][NT];
  float scr[RING][NG][NT];
  auto load_w = [&](int c, int sl) {
#pragma unroll
    for (int gq = 0; gq < NG; ++gq)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int gi = c * NG + gq;
        wr[sl][gq][j] = *reinterpret_cast<const w4_u32x4*>(wp[j] + (size_t)gi * 256);
        scr[sl][gq][j] = sp[j][(size_t)gi * 32];   // float2 stride: (tile, group) records of 16 columns
      }
  };
  const uint4 ones4 = make_uint4(0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u);
  const w4_bf16x8 ones = __builtin_bit_cast(w4_bf16x8, ones4);
  uint32_t vmask = 0x000F000Fu, vbias = 0x43004300u;
  asm volatile("" : "+v"(vmask), "+v"(vbias));

#pragma unroll
  for (int p = 0; p < XL; ++p)
    if (xok[p]) xr[0][p] = *reinterpret_cast<const w4_u32x4*>(x + xoff[p]);
  if (XD == 2 && nch > 1) {
#pragma unroll
    for (int p = 0; p < XL; ++p)
      if (xok[p]) xr[XD - 1][p] = *reinterpret_cast<const w4_u32x4*>(x + xoff[p] + KC);
  }
#pragma unroll
  for (int r = 0; r < RING; ++r)
    if (r < nch) load_w(r, r);

  auto chunk = [&](int c, auto sl_tag, auto more_tag) {
    constexpr int SL = decltype(sl_tag)::value;
    constexpr bool MORE = decltype(more_tag)::value;
    uint16_t* sx = s_x[c & 1];
#pragma unroll
    for (int p = 0; p < XL; ++p) {
      const int e = tid + NTH * p;
      const int row = e / CPR, ch = e % CPR;
      if (xok[p]) *reinterpret_cast<w4_u32x4*>(&sx[row * KC + (ch ^ (row & 15)) * 8]) = xr[XD == 2 ? (SL & 1) : 0][p];
    }
    if (c + XD < nch) {   // x of chunk c + XD into the register set just written out
#pragma unroll
      for (int p = 0; p < XL; ++p)
        if (xok[p]) xr[XD == 2 ? (SL & 1) : 0][p] = *reinterpret_cast<const w4_u32x4*>(x + xoff[p] + (c + XD) * KC);
    }
    __syncthreads();   // chunk c visible; every wave is past chunk c-1's reads of the other buffer
#pragma unroll
    for (int gq = 0; gq < NG; ++gq) {
      const int gi = c * NG + gq;
      w4_bf16x8 wf[NT][4];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int h = 0; h < 4; ++h) wf[j][h] = w4_frag_r(wr[SL][gq][j][h], vmask, vbias);
      float sc[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) sc[j] = scr[SL][gq][j];
      if constexpr (MORE) {   // refill this slot with chunk c + RING right away
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int gn = (c + RING) * NG + gq;
          wr[SL][gq][j] = *reinterpret_cast<const w4_u32x4*>(wp[j] + (size_t)gn * 256);
          scr[SL][gq][j] = sp[j][(size_t)gn * 32];
        }
      }
      const bool xs_duty = cw == (gi & 3);
#pragma unroll
      for (int i = 0; i < MTW; ++i) {
        w4_u32x4 xf[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int ch = gq * 16 + 8 * (h >> 1) + 2 * g + (h & 1);
          xf[h] = *reinterpret_cast<const w4_u32x4*>(&sx[rbase + 16 * i * KC + (ch ^ l15) * 8]);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          w4_floatx4 a = w4_floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int h = 0; h < 4; ++h)
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(w4_bf16x8, xf[h]), wf[j][h], a, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[i][j][r] = fmaf(sc[j], a[r], acc[i][j][r]);
        }
        if (xs_duty) {   // x . 1 of (row tile 2 mh + i, group gi) from the fragments in hand
          w4_floatx4 xm = w4_floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int h = 0; h < 4; ++h)
            xm = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(w4_bf16x8, xf[h]), ones, xm, 0, 0, 0);
          if (l15 == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) s_xs[16 * (MTW * mh + i) + 4 * g + r][gi] = xm[r];
          }
        }
      }
    }
  };
  for (int c = 0; c < nch; ++c) {   // ring slot c % RING; refill while chunk c + RING exists
    const bool more = c + RING < nch;
    static_for<0, RING>([&](auto sl) {
      if (c % RING == decltype(sl)::value) {
        if (more) chunk(c, sl, std::true_type{});
        else chunk(c, sl, std::false_type{});
      }
    });
  }
  __syncthreads();   // every wave's x sums are in s_xs
  // zero-point term: acc -= xs . (s z')^T, four groups per f32 MFMA
  const int ng = k_slice >> 7;
  for (int q = 0; q < ng; q += 4) {
    const bool gv = q + g < ng;
    float bz[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float2 v = reinterpret_cast<const float2*>(sp[j])[(size_t)min(q + g, ng - 1) * 16];
      bz[j] = gv ? -v.x * v.y : 0.f;
    }
#pragma unroll
    for (int i = 0; i < MTW; ++i) {
      const float xa = gv ? s_xs[16 * (MTW * mh + i) + l15][q + g] : 0.f;
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(xa, bz[j], acc[i][j], 0, 0, 0);
    }
  }
  if (t0 >= ntiles) return;
  if constexpr (SILU) {
    const int col = ((t0 * 16) >> 1) + l15;   // (gate tile, up tile) -> 16 h columns
#pragma unroll
    for (int i = 0; i < MTW; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * (MTW * mh + i) + g * 4 + r;
        if (m < M) {
          const float gt = acc[i][0][r], up = acc[i][1][r];
          out[(size_t)m * out_stride + col] = f32_to_bf16(gt / (1.f + __expf(-gt)) * up);
        }
      }
    return;
  }
  float* slab = ws + (size_t)s * M * N;
#pragma unroll
  for (int i = 0; i < MTW; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * (MTW * mh + i) + g * 4 + r;
      if (m < M) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int n = (t0 + j) * 16 + l15;
          if (t0 + j < ntiles) {
            if (ws == nullptr)
              out[(size_t)m * out_stride + n] = f32_to_bf16(acc[i][j][r]);
            else
              slab[(size_t)m * N + n] = acc[i][j][r];
          }
        }
      }
    }
}

// packed image -> bf16 [N, K] row-major (prefill path and tests).  One thread
// per (tile, group, lane): 32 weights = 4 runs of 8 consecutive k.
__global__ __launch_bounds__(256) void w4_dequant_kernel(const uint32_t* __restrict__ wq,
                                                         const float2* __restrict__ sz,
                                                         uint16_t* __restrict__ out, int N, int K) {
  const int groups = K >> 7;
  const long total = (long)(N / 16) * groups * 64;
  for (long t = blockIdx.x * 256L + threadIdx.x; t < total; t += (long)gridDim.x * 256L) {
    const int lane = (int)(t & 63);
    const long tg = t >> 6;  // tile * groups + group
    const int grp = (int)(tg % groups);
    const int tile = (int)(tg / groups);
    const int n = tile * 16 + (lane & 15), g = lane >> 4;
    const float2 p = sz[tg * 16 + (lane & 15)];
    const uint4 w4 = *reinterpret_cast<const uint4*>(wq + t * 4);
    const uint32_t wd[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int k = grp * 128 + 64 * (h >> 1) + 16 * g + 8 * (h & 1);
      float v[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[2 * i] = ((float)((wd[h] >> (4 * i)) & 15u) + 128.f - p.y) * p.x;
        v[2 * i + 1] = ((float)((wd[h] >> (4 * i + 16)) & 15u) + 128.f - p.y) * p.x;
      }
      *reinterpret_cast<uint4*>(out + (size_t)n * K + k) = store8(v);
    }
  }
}

}  // namespace ft

// Requirements (checked): M <= 64, N % (16*nt) == 0, K % (128*splits) == 0; ws
// (fp32 [splits][M][N] slabs) is required for splits > 1 and selects slab output.
extern "C" int ft_w4_gemm(const void* x, int x_stride, int M, const uint32_t* wq, const void* sz,
                          int N, int K, float* ws, void* out, int out_stride, int splits, int nt,
                          hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (128 * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  if (ws == nullptr && out == nullptr) return -6;
  const int mt = (M + 15) / 16;
  dim3 grid(N / (16 * nt), splits), block(256);
  const int k_slice = K / splits;
#define FT_W4(MT_, NT_)                                                                      \
  if (mt == MT_ && nt == NT_) {                                                              \
    hipLaunchKernelGGL((ft::w4_skinny_kernel<MT_, NT_>), grid, block, 0, stream,             \
                       (const uint16_t*)x, x_stride, M, wq, (const float2*)sz, K, ws,        \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_W4_NT(NT_) FT_W4(1, NT_) FT_W4(2, NT_) FT_W4(3, NT_) FT_W4(4, NT_)
  FT_W4_NT(1)
  FT_W4_NT(2)
  FT_W4_NT(4)
#undef FT_W4_NT
#undef FT_W4
  return -5;
}

// "xr" variant (17..64 rows): N % (64 * nt) == 0, K % (512 * splits) == 0; silu: nt even,
// out [M, N/2]; splits > 1 needs ws (slab output), silu needs splits == 1.
extern "C" int ft_w4_gemm_xr(const void* x, int x_stride, int M, const uint32_t* wq, const void* sz,
                             int N, int K, float* ws, void* out, int out_stride, int splits, int nt,
                             int silu, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (64 * nt) != 0) return -2;
  if (K % (512 * splits) != 0) return -3;
  if (splits > 1 && (ws == nullptr || silu)) return -4;
  if (ws == nullptr && out == nullptr) return -6;
  if (silu && nt % 2) return -7;
  const int mt = (M + 15) / 16;
  dim3 grid(N / (64 * nt), splits), block(256);
  const int k_slice = K / splits;
#define FT_W4X(MT_, NT_, E_)                                                                 \
  if (mt == MT_ && nt == NT_ && silu == E_) {                                                \
    hipLaunchKernelGGL((ft::w4_xr_kernel<MT_, NT_, E_>), grid, block, 0, stream,             \
                       (const uint16_t*)x, x_stride, M, wq, (const float2*)sz, K, ws,        \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_W4X_M(NT_, E_) FT_W4X(2, NT_, E_) FT_W4X(3, NT_, E_) FT_W4X(4, NT_, E_)
  FT_W4X_M(1, 0)
  FT_W4X_M(2, 0)
  FT_W4X_M(4, 0)
  FT_W4X_M(2, 1)
#undef FT_W4X_M
#undef FT_W4X
  return -5;
}

// "mh" variant (33..64 rows; 17..32 run one row half): N % 32 == 0, K % (256 * splits)
// == 0, K / splits <= 4096 (the x-sum table); ring 2 (two x chunks in flight too) or 3;
// silu: one split, out [M, N/2].
extern "C" int ft_w4_gemm_mh(const void* x, int x_stride, int M, const uint32_t* wq, const void* sz,
                             int N, int K, float* ws, void* out, int out_stride, int splits, int ring,
                             int silu, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % 32 != 0) return -2;
  if (K % (256 * splits) != 0 || K / splits > 4096) return -3;
  if (splits > 1 && (ws == nullptr || silu)) return -4;
  if (ws == nullptr && out == nullptr) return -6;
  if (ring != 2 && ring != 3) return -7;
  const int mh = M > 32 ? 2 : 1;
  dim3 grid((N / 16 + 7) / 8, splits), block(256 * mh);
  const int k_slice = K / splits;
#define FT_W4MH(MH_, R_, E_)                                                                     \
  if (mh == MH_ && ring == R_ && silu == E_) {                                                  \
    hipLaunchKernelGGL((ft::w4_mh_kernel<MH_, R_, E_, R_ == 2 ? 2 : 1>), grid, block, 0, stream,\
                       (const uint16_t*)x, x_stride, M, wq, (const float2*)sz, K, ws,           \
                       (uint16_t*)out, out_stride, N, k_slice);                                 \
    return static_cast<int>(hipGetLastError());                                                 \
  }
  FT_W4MH(1, 2, 0) FT_W4MH(1, 3, 0) FT_W4MH(2, 2, 0) FT_W4MH(2, 3, 0)
  FT_W4MH(1, 2, 1) FT_W4MH(1, 3, 1) FT_W4MH(2, 2, 1) FT_W4MH(2, 3, 1)
#undef FT_W4MH
  return -5;
}

extern "C" int ft_w4_dequant(const uint32_t* wq, const void* sz, void* out, int N, int K,
                             hipStream_t stream) {
  if (N % 16 != 0 || K % 128 != 0) return -1;
  const long total = (long)(N / 16) * (K / 128) * 64;
  const int blocks = (int)std::min<long>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(ft::w4_dequant_kernel, dim3(blocks), dim3(256), 0, stream, wq,
                     (const float2*)sz, (uint16_t*)out, N, K);
  return static_cast<int>(hipGetLastError());
}
