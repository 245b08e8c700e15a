// K3/K7/K8/K10/K11 at decode shapes: y[M, N] = x[M, K] . W[N, K]^T with M <= 64
// (one token per running sequence; "xc" also 65..128 rows: small mixed
// decode + prefill steps, still a weight stream), bf16 in, fp32 accumulate.
//
// At M <= 64 every projection is a weight stream (Llama-3-8B: 16 GB of weights
// per step vs < 1 MB of activations), so the kernels are built around the HBM
// read of W.  W is re-laid out once at load time into its MFMA-fragment image
// (ops.pack_weight: [N/16][K/64][half][lane][8]), so every wave instruction reads
// 1 KiB of consecutive bytes; A = x rows, B = W^T, v_mfma_f32_16x16x32_bf16.
//   * "pk": 16*NT columns per workgroup, the 4 waves split K by k-step, x
//     fragments straight from L2, the 4 partial tiles summed through LDS.
//   * "xc": x staged per 512-wide K chunk in LDS, every wave issues the whole
//     chunk's weight loads at once (deep streaming; gate_up and the LM head).
//   * split-K over gridDim.y: partial fp32 slabs ws[s][m][n] (plain stores) are
//     combined by the row-wise epilogue kernels in fused_epilogue.hip, which
//     also apply the op that follows the GEMM (residual add + RMSNorm, SiLU-mul,
//     bf16 store).  With gridDim.y == 1 the kernels store bf16 directly.
// Measured alternatives that lost and were removed (bench/gemm_sweep.py logs in
// profiles/): row-major-W streaming with U-deep k-blocks, K-split waves on
// row-major W, x-in-LDS double buffering, and a deep (4-6 stage) register ring
// over the packed image (profiles/pkd_sweep_r02.log: 5-20 % slower than pk/xc).
#include "ft_common.h"

#include <type_traits>

namespace ft {

typedef __bf16 sk_bf16x8 __attribute__((ext_vector_type(8)));
typedef float sk_floatx4 __attribute__((ext_vector_type(4)));

typedef unsigned int sk_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ sk_bf16x8 sk_frag(const uint4& v) {
  return __builtin_bit_cast(sk_bf16x8, v);
}

// streamed-once weight load: non-temporal (guide row "nt-weights": decode weights
// that one CU reads once)
__device__ __forceinline__ uint4 nt_load16(const uint16_t* p) {
  const sk_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const sk_u32x4*>(p));
  return __builtin_bit_cast(uint4, v);
}

__device__ __forceinline__ sk_u32x4 nt_load16v(const uint16_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const sk_u32x4*>(p));
}

// ---------------------------------------------------------------------------
// Stage of one 64-wide k-step: NT weight fragments + MT x fragments per lane.
template <int MT, int NT>
struct SkStage {
  uint4 w[NT][2];
  uint4 x[MT][2];
};

template <int MT, int NT>
__device__ __forceinline__ void sk_mma_stage(const SkStage<MT, NT>& st, sk_floatx4 (&acc)[MT][NT]) {
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(st.x[i][0]), sk_frag(st.w[j][0]),
                                                          acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(st.x[i][1]), sk_frag(st.w[j][1]),
                                                          acc[i][j], 0, 0, 0);
    }
}

// ---------------------------------------------------------------------------
// Variant "xc" (x chunks in LDS, deep weight streaming): per 512-wide K chunk
// the workgroup stages x[rows, 512] in LDS once (full-line loads, XOR
// swizzle) while every wave issues ALL of the chunk's weight loads for its
// 16*NT columns at once (8 k-steps x NT x 2 x 16 B per lane = 16-32 KiB per
// wave in flight), then runs the chunk's MFMAs as the weights land.  Two
// barriers per chunk; x loads are issued before the weight loads so the wait
// for x is an exact vmcnt that leaves the weight stream in flight.
template <int MT, int NT>
__global__ __launch_bounds__(256) void skinny_xc_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ w, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  constexpr int KC = MT <= 4 ? 512 : 256;          // k per chunk (8 / 4 MFMA k-steps of 64)
  constexpr int KS = KC / 64;
  constexpr int ROWS = 16 * MT;
  constexpr int CPR = KC / 8;                      // 16-B chunks per x row per chunk (64)
  constexpr int XL = ROWS * CPR / 256;             // x loads per thread per chunk
  __shared__ __attribute__((aligned(16))) uint16_t s_x[ROWS * KC];
  const int tid = threadIdx.x;
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = (blockIdx.x * 4 + wave) * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const bool active = n0 < N;

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    // packed fragment image: [N/16][K/64][half][lane][8]
    wp[j] = w + ((size_t)(min(n0 + 16 * j, N - 16) / 16) * (K >> 6) + (kbeg >> 6)) * 1024 + lane * 8;
  }

  sk_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = sk_floatx4{0.f, 0.f, 0.f, 0.f};

  for (int kc = 0; kc < k_slice; kc += KC) {
    // x chunk: element e = tid + 256*p -> row e / CPR, 16-B chunk e % CPR;
    // swizzle: chunk c of row r lives at slot c ^ (r & 7) (within its 128-B line group)
    uint4 xr[XL];
#pragma unroll
    for (int p = 0; p < XL; ++p) {
      const int e = tid + 256 * p;
      const int row = e / CPR, ch = e % CPR;
      xr[p] = *reinterpret_cast<const uint4*>(x + (size_t)min(row, M - 1) * x_stride + kbeg + kc +
                                              ch * 8);
    }
    uint4 wr[KS][NT][2];
#pragma unroll
    for (int st = 0; st < KS; ++st)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint16_t* p = wp[j] + (size_t)((kc >> 6) + st) * 1024;
        wr[st][j][0] = nt_load16(p);
        wr[st][j][1] = nt_load16(p + 512);
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int p = 0; p < XL; ++p) {
      const int e = tid + 256 * p;
      const int row = e / CPR, ch = e % CPR;
      const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
      *reinterpret_cast<uint4*>(&s_x[row * KC + slot * 8]) = xr[p];
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int st = 0; st < KS; ++st) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const int row = 16 * i + l15;
          uint4 xf[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int ch = st * 8 + 2 * g + h;
            const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
            xf[h] = *reinterpret_cast<const uint4*>(&s_x[row * KC + slot * 8]);
          }
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(xf[0]), sk_frag(wr[st][j][0]),
                                                                acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(xf[1]), sk_frag(wr[st][j][1]),
                                                                acc[i][j], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();
  }
  if (!active) return;
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
          if (gridDim.y == 1)
            out[(size_t)m * out_stride + n] = f32_to_bf16(acc[i][j][r]);
          else
            slab[(size_t)m * N + n] = acc[i][j][r];
        }
      }
    }
}


// ---------------------------------------------------------------------------
// Variant "xr" (x chunks in LDS, weight RING across chunks): "xc" with the
// chunk loop software-pipelined.  Measured (bench/xc_diag.py, 50 rows, cold):
// xc drains its weight stream at every 512-wide chunk -- the next chunk's
// loads are issued only after this chunk's MFMAs -- so a multi-chunk K slice
// (gate_up without split-K: 8 chunks) ran at 3.5 TB/s against 6 TB/s for its
// bare loads, which is why gate_up needed split-K slabs (+14.7 MB of fp32
// written and re-read by slab_silu).  Here each k-step's weight registers are
// refilled with the NEXT chunk's fragment right after their MFMAs, so every
// wave keeps KS k-steps (NT * 16 KiB) in flight without extra registers, and x
// is double-buffered in LDS (one barrier per chunk).  SILU: the gate_up image
// is interleaved in 16-column groups (interleave_gate_up(w, 1)), so with NT = 2
// a wave holds a gate tile and its up tile and writes h = silu(g) * u (bf16,
// N/2 columns) itself -- no slabs, no slab_silu launch.
// Epilogues: EPI 0 bf16 out (one split) / fp32 slabs ws[s][m][n]; EPI 1 SiLU
// (above).  (An in-launch split-K residual epilogue and an RMS-scaled SiLU variant
// were measured slower than the separate add+RMSNorm launches they replaced --
// profiles/ab_resid_layer_r02.log -- and removed.)
// NW: waves per workgroup.  8 waves share one staged x chunk between twice the
// weight columns: the per-CU load path carries x once per 8 waves' weights
// instead of once per 4 (at 50-64 rows x is as many bytes per workgroup as its
// weight slice), and a 128 KiB (KC 512) workgroup gets two waves per SIMD.
template <int MT, int NT, int KC, int EPI, int NW = 4>
__global__ __launch_bounds__(64 * NW, 1) void skinny_xr_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ w, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  constexpr bool SILU = EPI == 1;
  constexpr int KS = KC / 64;
  constexpr int ROWS = 16 * MT;
  constexpr int CPR = KC / 8;
  constexpr int NTH = 64 * NW;
  constexpr int XL = ROWS * CPR / NTH;
  static_assert(XL >= 1 && (ROWS * CPR) % NTH == 0, "x chunk must tile the workgroup");
  static_assert(!SILU || NT == 2, "the SiLU epilogue pairs a gate tile with its up tile");
  __shared__ __attribute__((aligned(16))) uint16_t s_x[2][ROWS * KC];
  const int tid = threadIdx.x;
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = (blockIdx.x * NW + wave) * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int nch = k_slice / KC;
  const bool active = n0 < N;

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    wp[j] = w + ((size_t)(min(n0 + 16 * j, N - 16) / 16) * (K >> 6) + (kbeg >> 6)) * 1024 + lane * 8;
  // this thread's x elements: row e / CPR, 16-B chunk e % CPR of each chunk, e = tid + NTH p
  const uint16_t* xsrc[XL];
#pragma unroll
  for (int p = 0; p < XL; ++p) {
    const int e = tid + NTH * p;
    xsrc[p] = x + (size_t)min(e / CPR, M - 1) * x_stride + kbeg + (e % CPR) * 8;
  }

  sk_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = sk_floatx4{0.f, 0.f, 0.f, 0.f};

  // native vector registers (the HIP uint4 struct defeats register promotion of
  // arrays that stay live across the chunk loop: they went to scratch)
  sk_u32x4 xr[XL];
  sk_u32x4 wr[KS][NT][2];
#pragma unroll
  for (int p = 0; p < XL; ++p) xr[p] = *reinterpret_cast<const sk_u32x4*>(xsrc[p]);
#pragma unroll
  for (int st = 0; st < KS; ++st)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      wr[st][j][0] = nt_load16v(wp[j] + (size_t)st * 1024);
      wr[st][j][1] = nt_load16v(wp[j] + (size_t)st * 1024 + 512);
    }
  // one chunk: x regs -> LDS buffer c&1, next chunk's x loads, barrier, MFMAs with
  // each k-step's weight registers refilled from chunk c+1 right after use.
  // MORE is a template constant (the last chunk is peeled) so the loop body is
  // branch-free: with conditional loads the waitcnt pass drained vmcnt(0) at
  // every chunk, which is the bubble this variant exists to remove.  Waves past
  // N (clamped weight pointers) compute and discard.
  auto chunk = [&](int c, auto more_tag) {
    constexpr bool MORE = decltype(more_tag)::value;
    uint16_t* sx = s_x[c & 1];
#pragma unroll
    for (int p = 0; p < XL; ++p) {
      const int e = tid + NTH * p;
      const int row = e / CPR, ch = e % CPR;
      const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
      *reinterpret_cast<sk_u32x4*>(&sx[row * KC + slot * 8]) = xr[p];
    }
    if constexpr (MORE) {
#pragma unroll
      for (int p = 0; p < XL; ++p) xr[p] = *reinterpret_cast<const sk_u32x4*>(xsrc[p] + (c + 1) * KC);
    }
    __syncthreads();   // chunk c visible; every wave is past chunk c-1's reads of the other buffer
    const size_t nxt = (size_t)(c + 1) * KS * 1024;
#pragma unroll
    for (int st = 0; st < KS; ++st) {
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int row = 16 * i + l15;
        sk_u32x4 xf[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ch = st * 8 + 2 * g + h;
          const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
          xf[h] = *reinterpret_cast<const sk_u32x4*>(&sx[row * KC + slot * 8]);
        }
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(sk_bf16x8, xf[0]), __builtin_bit_cast(sk_bf16x8, wr[st][j][0]),
              acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
              __builtin_bit_cast(sk_bf16x8, xf[1]), __builtin_bit_cast(sk_bf16x8, wr[st][j][1]),
              acc[i][j], 0, 0, 0);
        }
      }
      if constexpr (MORE) {   // refill this k-step's registers with the next chunk's fragments
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          wr[st][j][0] = nt_load16v(wp[j] + nxt + (size_t)st * 1024);
          wr[st][j][1] = nt_load16v(wp[j] + nxt + (size_t)st * 1024 + 512);
        }
      }
    }
  };
  for (int c = 0; c + 1 < nch; ++c) chunk(c, std::true_type{});
  chunk(nch - 1, std::false_type{});
  if (!active) return;
  if constexpr (SILU) {
    const int col = (n0 >> 1) + l15;   // 16-column gate group n0/32 -> h columns
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + g * 4 + r;
        if (m < M) {
          const float gt = acc[i][0][r], up = acc[i][1][r];
          out[(size_t)m * out_stride + col] = f32_to_bf16(gt / (1.f + __expf(-gt)) * up);
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
          if (gridDim.y == 1)
            out[(size_t)m * out_stride + n] = f32_to_bf16(acc[i][j][r]);
          else
            slab[(size_t)m * N + n] = acc[i][j][r];
        }
      }
    }
}


// ---------------------------------------------------------------------------
// Variant "pk" (pre-packed weights): W is re-laid out once at load time so that
// every (16-column tile, 64-wide k-step) MFMA B-fragment is 2 KiB contiguous
// in exactly the order the 64 lanes load it ([N/16][K/64][half][lane][8]).  A
// wave instruction then reads 1 KiB of consecutive bytes (whole lines, one
// DRAM page stream per wave) instead of 16 rows x 64 B, and a wave streaming
// its column tile along K walks one contiguous region.  Waves split K as in
// "ks"; x fragments come straight from L2.
template <int MT, int NT>
__global__ __launch_bounds__(256) void skinny_pk_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ wpk, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  __shared__ float s_red[4][MT * NT * 4][64];
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int ksteps_total = K >> 6;
  const int step0 = kbeg >> 6;

  // packed fragment base of column tile (n0/16 + j), k-step 0, this lane
  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    wp[j] = wpk + ((size_t)(n0 / 16 + j) * ksteps_total) * 1024 + lane * 8;
  const uint16_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = min(16 * i + l15, M - 1);
    xp[i] = x + (size_t)r * x_stride + kbeg + 16 * g;
  }

  sk_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = sk_floatx4{0.f, 0.f, 0.f, 0.f};

  const int nsteps = k_slice >> 6;
  const int my_steps = nsteps > wave ? (nsteps - wave + 3) >> 2 : 0;
  const int last = my_steps - 1;
  auto kst = [&](int t) { return wave + 4 * min(t, last); };  // k-step index within the split
  auto load = [&](SkStage<MT, NT>& st, int t) {
    const int ks = kst(t);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const uint16_t* p = wp[j] + (size_t)(step0 + ks) * 1024;
      st.w[j][0] = nt_load16(p);
      st.w[j][1] = nt_load16(p + 512);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint4* p = reinterpret_cast<const uint4*>(xp[i] + ks * 64);
      st.x[i][0] = p[0];
      st.x[i][1] = p[1];
    }
  };
  if (my_steps > 0) {
    SkStage<MT, NT> a, b;
    load(a, 0);
    int t = 0;
    for (; t + 2 <= my_steps; t += 2) {
      load(b, t + 1);
      __builtin_amdgcn_sched_barrier(0);
      sk_mma_stage<MT, NT>(a, acc);
      __builtin_amdgcn_sched_barrier(0);
      load(a, t + 2);
      __builtin_amdgcn_sched_barrier(0);
      sk_mma_stage<MT, NT>(b, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t < my_steps) sk_mma_stage<MT, NT>(a, acc);
  }

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
      if (gridDim.y == 1)
        out[(size_t)m * out_stride + n] = f32_to_bf16(v);
      else
        slab[(size_t)m * N + n] = v;
    }
  }
}


}  // namespace ft




// x-chunk variant.  Requirements (checked): M <= 128, N % (16*nt) == 0,
// K % (512*splits) == 0 (M <= 64) or K % (256*splits) == 0 (65..128 rows: the x
// chunk halves so 128 rows still fit 64 KiB of LDS).
extern "C" int ft_skinny_gemm_xc(const void* x, int x_stride, int M, const void* w, int N, int K,
                                 float* ws, void* out, int out_stride, int splits, int nt,
                                 hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 128 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % ((M > 64 ? 256 : 512) * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  const int cols = 4 * 16 * nt;
  dim3 grid((N + cols - 1) / cols, splits), block(256);
  const int k_slice = K / splits;
#define FT_XC(MT_, NT_)                                                                      \
  if (mt == MT_ && nt == NT_) {                                                              \
    hipLaunchKernelGGL((ft::skinny_xc_kernel<MT_, NT_>), grid, block, 0, stream,             \
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,           \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_XC_NT(NT_) FT_XC(1, NT_) FT_XC(2, NT_) FT_XC(3, NT_) FT_XC(4, NT_) \
  FT_XC(5, NT_) FT_XC(6, NT_) FT_XC(7, NT_) FT_XC(8, NT_)
  FT_XC_NT(1)
  FT_XC_NT(2)
#undef FT_XC_NT
#undef FT_XC
  return -5;
}

// Ring-pipelined x-chunk variant.  Requirements (checked): M <= 64,
// N % (16*nt) == 0, K % (kc*splits) == 0 with kc = 512 (nt 2) / 256 (nt 1; two
// 4-wave workgroups per CU).  epi 0: out (one split) or ws [splits, M, N];
// epi 1 (SiLU): nt 2, one split, out = [M, N/2].  nw: 4 or 8 waves per workgroup.
extern "C" int ft_skinny_gemm_xr(const void* x, int x_stride, int M, const void* w, int N, int K,
                                 float* ws, void* out, int out_stride, int splits, int nt, int epi,
                                 int nw, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (nt != 1 && nt != 2) return -5;
  if (nw != 4 && nw != 8) return -7;
  if (N % (16 * nt) != 0) return -2;
  const int kc = nt == 2 ? 512 : 256;
  if (K % (kc * splits) != 0) return -3;
  if (epi < 0 || epi > 1) return -6;
  if (epi == 1 && (nt != 2 || splits != 1)) return -6;
  if (epi == 0 && splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  const int cols = nw * 16 * nt;
  dim3 grid((N + cols - 1) / cols, splits), block(64 * nw);
  const int k_slice = K / splits;
#define FT_XR(MT_, NT_, KC_, E_, NW_)                                                         \
  if (mt == MT_ && nt == NT_ && epi == E_ && nw == NW_) {                                     \
    hipLaunchKernelGGL((ft::skinny_xr_kernel<MT_, NT_, KC_, E_, NW_>), grid, block, 0, stream,\
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,            \
                       (uint16_t*)out, out_stride, N, k_slice);                               \
    return static_cast<int>(hipGetLastError());                                               \
  }
#define FT_XR_MT(MT_, NW_) FT_XR(MT_, 1, 256, 0, NW_) FT_XR(MT_, 2, 512, 0, NW_) FT_XR(MT_, 2, 512, 1, NW_)
  FT_XR_MT(1, 4)
  FT_XR_MT(2, 4)
  FT_XR_MT(3, 4)
  FT_XR_MT(4, 4)
  FT_XR_MT(1, 8)
  FT_XR_MT(2, 8)
  FT_XR_MT(3, 8)
  FT_XR_MT(4, 8)
#undef FT_XR_MT
#undef FT_XR
  return -5;
}

// Pre-packed-weight variant (wpk from ft_pack_weights layout).  Requirements
// (checked): M <= 64, N % (16*nt) == 0, K % (64*splits) == 0.
extern "C" int ft_skinny_gemm_pk(const void* x, int x_stride, int M, const void* wpk, int N, int K,
                                 float* ws, void* out, int out_stride, int splits, int nt,
                                 hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (64 * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  dim3 grid(N / (16 * nt), splits), block(256);
  const int k_slice = K / splits;
#define FT_PK(MT_, NT_)                                                                      \
  if (mt == MT_ && nt == NT_) {                                                              \
    hipLaunchKernelGGL((ft::skinny_pk_kernel<MT_, NT_>), grid, block, 0, stream,             \
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, K, ws,         \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_PK_NT(NT_) FT_PK(1, NT_) FT_PK(2, NT_) FT_PK(3, NT_) FT_PK(4, NT_)
  FT_PK_NT(1)
  FT_PK_NT(2)
  FT_PK_NT(4)
#undef FT_PK_NT
#undef FT_PK
  return -5;
}

