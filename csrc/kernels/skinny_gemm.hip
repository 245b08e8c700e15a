// K3/K7/K8/K10/K11 at decode shapes: y[M, N] = x[M, K] . W[N, K]^T with M <= 64
// (one token per running sequence), bf16 in, fp32 accumulate.
//
// At M <= 64 every projection is a weight stream (Llama-3-8B: 16 GB of weights
// per step vs < 1 MB of activations), so the kernel is built around the HBM read
// of W, following the "GEMV / M <= 16 decode weights" guidance: no LDS round trip,
// both operands go straight to VGPRs in MFMA fragment order.
//   * v_mfma_f32_16x16x32_bf16; A = x (16 rows per m-tile), B = W^T.
//   * a k-block is 64 wide: lane (r = lane&15, g = lane>>4) loads 32 contiguous
//     bytes of row r at k = 16g..16g+15, i.e. every wave instruction pair reads
//     16 rows x 128 B = whole cache lines; the two 8-element halves feed two
//     MFMAs (the k permutation is applied identically to A and B).
//   * each wave owns NT 16-column tiles; 4 waves per workgroup share the x rows
//     through L1; U k-blocks are loaded before any MFMA so each lane keeps
//     2*NT*U 16-B weight loads in flight.
//   * split-K over gridDim.y: partial fp32 slabs ws[s][m][n] (plain stores) are
//     combined by the row-wise epilogue kernels in fused_epilogue.hip, which
//     also apply the op that follows the GEMM (residual add + RMSNorm, SiLU-mul,
//     bf16 store).  With gridDim.y == 1 the kernel stores bf16 directly.
#include "ft_common.h"

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

template <int MT, int NT, int U>
__global__ __launch_bounds__(256) void skinny_gemm_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ w, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = (blockIdx.x * 4 + wave) * (16 * NT);
  if (n0 >= N) return;
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;

  sk_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = sk_floatx4{0.f, 0.f, 0.f, 0.f};

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wp[j] = w + (size_t)(n0 + 16 * j + l15) * K + kbeg + 16 * g;
  const uint16_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = min(16 * i + l15, M - 1);
    xp[i] = x + (size_t)r * x_stride + kbeg + 16 * g;
  }

  for (int kb = 0; kb < k_slice; kb += 64 * U) {
    uint4 wf[U][NT][2];
    uint4 xf[U][MT][2];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint16_t* p = wp[j] + kb + 64 * u;
        wf[u][j][0] = nt_load16(p);
        wf[u][j][1] = nt_load16(p + 8);
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const uint4* p = reinterpret_cast<const uint4*>(xp[i] + kb + 64 * u);
        xf[u][i][0] = p[0];
        xf[u][i][1] = p[1];
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(xf[u][i][0]),
                                                              sk_frag(wf[u][j][0]), acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(xf[u][i][1]),
                                                              sk_frag(wf[u][j][1]), acc[i][j], 0, 0, 0);
        }
  }

  // C layout: col = lane & 15 (n), row = (lane >> 4) * 4 + r (m)
  if (gridDim.y == 1) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + g * 4 + r;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < NT; ++j)
            out[(size_t)m * out_stride + n0 + 16 * j + l15] = f32_to_bf16(acc[i][j][r]);
        }
      }
  } else {
    float* slab = ws + (size_t)s * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + g * 4 + r;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < NT; ++j) slab[(size_t)m * N + n0 + 16 * j + l15] = acc[i][j][r];
        }
      }
  }
}


// ---------------------------------------------------------------------------
// Variant "ks" (K-split waves): the 4 waves of a workgroup share the SAME
// 16*NT output columns and split the workgroup's K range between them (wave w
// takes the 64-wide k-steps w, w+4, ...), so every byte of x a workgroup needs
// is fetched once by one wave (x traffic = M/(16*NT) of the weight traffic,
// 4x less than column-split waves).  Each wave double-buffers its loads: the
// next k-step's weight and x fragments are in flight while the current one
// feeds the MFMAs.  The four partial tiles are summed through LDS at the end
// and written as bf16 (gridDim.y == 1) or as an fp32 split-K slab.
template <int MT, int NT>
struct SkStage {
  uint4 w[NT][2];
  uint4 x[MT][2];
};

template <int MT, int NT>
__device__ __forceinline__ void sk_load_stage(SkStage<MT, NT>& st, const uint16_t* const (&wp)[NT],
                                              const uint16_t* const (&xp)[MT], int k) {
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    st.w[j][0] = nt_load16(wp[j] + k);
    st.w[j][1] = nt_load16(wp[j] + k + 8);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const uint4* p = reinterpret_cast<const uint4*>(xp[i] + k);
    st.x[i][0] = p[0];
    st.x[i][1] = p[1];
  }
}

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

template <int MT, int NT>
__global__ __launch_bounds__(256) void skinny_ks_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ w, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  __shared__ float s_red[4][MT * NT * 4][64];  // [wave][acc register][lane]
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wp[j] = w + (size_t)(n0 + 16 * j + l15) * K + kbeg + 16 * g;
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

  // this wave's k-steps are wave, wave + 4, ...; the prefetch of step t+1 is issued
  // before the MFMAs of step t.  Every load is unconditional (an index past the
  // end re-reads the last step, an L2 hit) so the compiler can count vmcnt
  // exactly instead of draining the whole queue at a control-flow merge.
  const int nsteps = k_slice >> 6;
  const int my_steps = nsteps > wave ? (nsteps - wave + 3) >> 2 : 0;
  const int last = my_steps - 1;
  auto koff = [&](int t) { return (wave + 4 * min(t, last)) * 64; };
  if (my_steps > 0) {
    SkStage<MT, NT> a, b;
    sk_load_stage<MT, NT>(a, wp, xp, koff(0));
    int t = 0;
    // sched_barrier(0) pins the order: the compiler's scheduler would otherwise
    // sink the prefetch below the MFMAs and wait vmcnt(0) on it
    for (; t + 2 <= my_steps; t += 2) {
      sk_load_stage<MT, NT>(b, wp, xp, koff(t + 1));
      __builtin_amdgcn_sched_barrier(0);
      sk_mma_stage<MT, NT>(a, acc);
      __builtin_amdgcn_sched_barrier(0);
      sk_load_stage<MT, NT>(a, wp, xp, koff(t + 2));
      __builtin_amdgcn_sched_barrier(0);
      sk_mma_stage<MT, NT>(b, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (t < my_steps) sk_mma_stage<MT, NT>(a, acc);
  }

  // ---- sum the 4 waves' partial tiles through LDS ----------------------------------
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_red[wave][(i * NT + j) * 4 + r][lane] = acc[i][j][r];
  __syncthreads();
  // thread t of the workgroup finalises register slots t/64 + 4q of lane t%64
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


// ---------------------------------------------------------------------------
// Variant "xs" (x staged in LDS): the 4 waves split the columns (16*NT each)
// and share one copy of the x k-step in LDS.  x is fetched in whole 128-B
// lines (thread t: row t/8, 16-B chunk t%8) -- fragment-shaped x loads touch
// 16 lines per wave instruction and were measured to cost ~3 us per 16 rows
// of M on the Llama-3-8B down projection -- and written XOR-swizzled (chunk c
// of row r at slot c ^ (r & 7)) so the fragment reads are near conflict-free.
// W streams straight to registers (nontemporal), double buffered; x is double
// buffered in LDS with one barrier per 64-wide k-step.  Within an iteration
// the x loads are issued BEFORE the weight prefetch so waiting for them never
// drains the weight pipeline (vmcnt counts in issue order).
template <int MT, int NT>
__device__ __forceinline__ void xs_load_w(uint4 (&wr)[NT][2], const uint16_t* const (&wp)[NT], int k) {
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    wr[j][0] = nt_load16(wp[j] + k);
    wr[j][1] = nt_load16(wp[j] + k + 8);
  }
}

template <int MT, int NT>
__device__ __forceinline__ void xs_mma(const uint4 (&wr)[NT][2], const uint16_t* xs, int l15, int g,
                                       sk_floatx4 (&acc)[MT][NT]) {
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int row = 16 * i + l15;
    uint4 xf[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = 2 * g + h;
      xf[h] = *reinterpret_cast<const uint4*>(xs + row * 64 + ((c ^ (row & 7)) * 8));
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(xf[0]), sk_frag(wr[j][0]),
                                                          acc[i][j], 0, 0, 0);
      acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sk_frag(xf[1]), sk_frag(wr[j][1]),
                                                          acc[i][j], 0, 0, 0);
    }
  }
}

template <int MT, int NT>
__global__ __launch_bounds__(256) void skinny_xs_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ w, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  constexpr int ROWS = 16 * MT;                 // x rows staged (M rounded up to 16)
  constexpr int XPASS = (ROWS * 8 + 255) / 256;  // 16-B chunks per thread per k-step
  __shared__ __attribute__((aligned(16))) uint16_t s_x[2][ROWS * 64];
  const int tid = threadIdx.x;
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = (blockIdx.x * 4 + wave) * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int nsteps = k_slice >> 6;
  const bool active = n0 < N;  // a trailing wave past N only helps stage x

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    wp[j] = w + (size_t)min(n0 + 16 * j + l15, N - 1) * K + kbeg + 16 * g;
  // x staging: thread -> (row, chunk) of each pass; rows past M re-read row M-1
  const uint16_t* xsrc[XPASS];
  int xdst[XPASS];
#pragma unroll
  for (int p = 0; p < XPASS; ++p) {
    const int e = tid + 256 * p;
    const int row = min(e >> 3, ROWS - 1), ch = e & 7;
    xsrc[p] = x + (size_t)min(row, M - 1) * x_stride + kbeg + ch * 8;
    xdst[p] = row * 64 + ((ch ^ (row & 7)) * 8);
  }
  auto x_load = [&](uint4 (&xr)[XPASS], int t) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p) xr[p] = *reinterpret_cast<const uint4*>(xsrc[p] + t * 64);
  };
  auto x_store = [&](const uint4 (&xr)[XPASS], int buf) {
#pragma unroll
    for (int p = 0; p < XPASS; ++p)
      if (tid + 256 * p < ROWS * 8) *reinterpret_cast<uint4*>(&s_x[buf][xdst[p]]) = xr[p];
  };

  sk_floatx4 acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = sk_floatx4{0.f, 0.f, 0.f, 0.f};

  uint4 xr[XPASS];
  uint4 wa[NT][2], wb[NT][2];
  const int last = nsteps - 1;
  x_load(xr, 0);
  xs_load_w<MT, NT>(wa, wp, 0);
  x_store(xr, 0);
  __syncthreads();
  // step t: x(t) is in s_x[t&1], W(t) in registers; prefetch x(t+1) then W(t+1)
  int t = 0;
  for (; t + 2 <= nsteps; t += 2) {
    x_load(xr, min(t + 1, last));
    xs_load_w<MT, NT>(wb, wp, min(t + 1, last) * 64);
    __builtin_amdgcn_sched_barrier(0);
    if (active) xs_mma<MT, NT>(wa, s_x[0], l15, g, acc);
    __builtin_amdgcn_sched_barrier(0);
    x_store(xr, 1);
    __syncthreads();
    x_load(xr, min(t + 2, last));
    xs_load_w<MT, NT>(wa, wp, min(t + 2, last) * 64);
    __builtin_amdgcn_sched_barrier(0);
    if (active) xs_mma<MT, NT>(wb, s_x[1], l15, g, acc);
    __builtin_amdgcn_sched_barrier(0);
    x_store(xr, 0);
    __syncthreads();
  }
  if (t < nsteps && active) xs_mma<MT, NT>(wa, s_x[0], l15, g, acc);
  if (!active) return;

  // C layout: col = lane & 15 (n), row = (lane >> 4) * 4 + r (m)
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
// Variant "xc" (x chunks in LDS, deep weight streaming): per 512-wide K chunk
// the workgroup stages x[rows, 512] in LDS once (full-line loads, XOR
// swizzle) while every wave issues ALL of the chunk's weight loads for its
// 16*NT columns at once (8 k-steps x NT x 2 x 16 B per lane = 16-32 KiB per
// wave in flight), then runs the chunk's MFMAs as the weights land.  Two
// barriers per chunk; x loads are issued before the weight loads so the wait
// for x is an exact vmcnt that leaves the weight stream in flight.
template <int MT, int NT, bool PACKED>
__global__ __launch_bounds__(256) void skinny_xc_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ w, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  constexpr int KC = 512;                          // k per chunk (8 MFMA k-steps of 64)
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
    if constexpr (PACKED)  // fragment image: [N/16][K/64][half][lane][8]
      wp[j] = w + ((size_t)(min(n0 + 16 * j, N - 16) / 16) * (K >> 6) + (kbeg >> 6)) * 1024 + lane * 8;
    else
      wp[j] = w + (size_t)min(n0 + 16 * j + l15, N - 1) * K + kbeg + 16 * g;
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
    uint4 wr[8][NT][2];
#pragma unroll
    for (int st = 0; st < 8; ++st)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        if constexpr (PACKED) {
          const uint16_t* p = wp[j] + (size_t)((kc >> 6) + st) * 1024;
          wr[st][j][0] = nt_load16(p);
          wr[st][j][1] = nt_load16(p + 512);
        } else {
          wr[st][j][0] = nt_load16(wp[j] + kc + st * 64);
          wr[st][j][1] = nt_load16(wp[j] + kc + st * 64 + 8);
        }
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
      for (int st = 0; st < 8; ++st) {
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


// ---------------------------------------------------------------------------
// Variant "pkd" (packed, deep weight ring): pk's decomposition (16*NT columns
// per workgroup, the 4 waves split the K range by k-step) with the weight stream
// in an R-deep register ring -- R-1 k-steps (R-1 x NT x 2 KiB per wave) stay in
// flight while one feeds the MFMAs -- and x (L2-resident, shorter latency)
// double-buffered on its own.  At decode shapes every CU holds 1-3 of these
// workgroups, so bytes in flight per CU, not MFMA or VALU, set the rate (pk keeps
// one k-step in flight per wave: ~32 KiB per CU at 1 workgroup/CU).
template <int MT, int NT, int R>
__global__ __launch_bounds__(256) void skinny_pkd_kernel(
    const uint16_t* __restrict__ x, int x_stride, int M, const uint16_t* __restrict__ wpk, int K,
    float* __restrict__ ws, uint16_t* __restrict__ out, int out_stride, int N, int k_slice) {
  static_assert(R % 2 == 0, "the x ring is indexed by step parity");
  __shared__ float s_red[4][MT * NT * 4][64];
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * k_slice;
  const int ksteps_total = K >> 6;
  const int step0 = kbeg >> 6;

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    wp[j] = wpk + ((size_t)(n0 / 16 + j) * ksteps_total + step0) * 1024 + lane * 8;
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
  auto kst = [&](int t) { return wave + 4 * min(t, last); };  // past the end: re-load the last
  uint4 wr[R][NT][2];
  uint4 xr[2][MT][2];
  auto load_w = [&](uint4 (&st)[NT][2], int t) {
    const size_t off = (size_t)kst(t) * 1024;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      st[j][0] = nt_load16(wp[j] + off);
      st[j][1] = nt_load16(wp[j] + off + 512);
    }
  };
  auto load_x = [&](uint4 (&st)[MT][2], int t) {
    const int k = kst(t) * 64;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint4* p = reinterpret_cast<const uint4*>(xp[i] + k);
      st[i][0] = p[0];
      st[i][1] = p[1];
    }
  };
  if (my_steps > 0) {
#pragma unroll
    for (int r = 0; r + 1 < R; ++r) load_w(wr[r], r);
    load_x(xr[0], 0);
    for (int t = 0; t < my_steps; t += R) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        load_w(wr[(r + R - 1) % R], t + r + R - 1);
        load_x(xr[(r + 1) & 1], t + r + 1);
        __builtin_amdgcn_sched_barrier(0);
        if (t + r < my_steps) {
#pragma unroll
          for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) {
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  sk_frag(xr[r & 1][i][0]), sk_frag(wr[r][j][0]), acc[i][j], 0, 0, 0);
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                  sk_frag(xr[r & 1][i][1]), sk_frag(wr[r][j][1]), acc[i][j], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
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

// Returns 0 on success.  Requirements (checked): M <= 64, N % (16*nt) == 0,
// K % (64*u*splits) == 0, 16-B aligned rows.
extern "C" int ft_skinny_gemm(const void* x, int x_stride, int M, const void* w, int N, int K,
                              float* ws, void* out, int out_stride, int splits, int nt, int u,
                              hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (64 * u * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  const int cols_per_block = 4 * 16 * nt;
  dim3 grid((N + cols_per_block - 1) / cols_per_block, splits), block(256);
  const int k_slice = K / splits;
#define FT_SK(MT_, NT_, U_)                                                                   \
  if (mt == MT_ && nt == NT_ && u == U_) {                                                    \
    hipLaunchKernelGGL((ft::skinny_gemm_kernel<MT_, NT_, U_>), grid, block, 0, stream,        \
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,            \
                       (uint16_t*)out, out_stride, N, k_slice);                               \
    return static_cast<int>(hipGetLastError());                                               \
  }
#define FT_SK_NT(NT_, U_) FT_SK(1, NT_, U_) FT_SK(2, NT_, U_) FT_SK(3, NT_, U_) FT_SK(4, NT_, U_)
  FT_SK_NT(1, 2)
  FT_SK_NT(1, 4)
  FT_SK_NT(2, 2)
  FT_SK_NT(2, 4)
  FT_SK_NT(4, 1)
  FT_SK_NT(4, 2)
#undef FT_SK_NT
#undef FT_SK
  return -5;
}

// K-split-wave variant.  Requirements (checked): M <= 64, N % (16*nt) == 0,
// K % (64*splits) == 0.
extern "C" int ft_skinny_gemm_ks(const void* x, int x_stride, int M, const void* w, int N, int K,
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
#define FT_KS(MT_, NT_)                                                                      \
  if (mt == MT_ && nt == NT_) {                                                              \
    hipLaunchKernelGGL((ft::skinny_ks_kernel<MT_, NT_>), grid, block, 0, stream,             \
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,           \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_KS_NT(NT_) FT_KS(1, NT_) FT_KS(2, NT_) FT_KS(3, NT_) FT_KS(4, NT_)
  FT_KS_NT(1)
  FT_KS_NT(2)
  FT_KS_NT(4)
#undef FT_KS_NT
#undef FT_KS
  return -5;
}

// x-in-LDS variant.  Requirements (checked): M <= 64, N % (16*nt) == 0,
// K % (64*splits) == 0.
extern "C" int ft_skinny_gemm_xs(const void* x, int x_stride, int M, const void* w, int N, int K,
                                 float* ws, void* out, int out_stride, int splits, int nt,
                                 hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (64 * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  const int cols = 4 * 16 * nt;
  dim3 grid((N + cols - 1) / cols, splits), block(256);
  const int k_slice = K / splits;
#define FT_XS(MT_, NT_)                                                                      \
  if (mt == MT_ && nt == NT_) {                                                              \
    hipLaunchKernelGGL((ft::skinny_xs_kernel<MT_, NT_>), grid, block, 0, stream,             \
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,           \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_XS_NT(NT_) FT_XS(1, NT_) FT_XS(2, NT_) FT_XS(3, NT_) FT_XS(4, NT_)
  FT_XS_NT(1)
  FT_XS_NT(2)
  FT_XS_NT(4)
#undef FT_XS_NT
#undef FT_XS
  return -5;
}

// x-chunk variant.  Requirements (checked): M <= 64, N % (16*nt) == 0,
// K % (512*splits) == 0.
extern "C" int ft_skinny_gemm_xc(const void* x, int x_stride, int M, const void* w, int N, int K,
                                 float* ws, void* out, int out_stride, int splits, int nt,
                                 int packed, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (512 * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  const int cols = 4 * 16 * nt;
  dim3 grid((N + cols - 1) / cols, splits), block(256);
  const int k_slice = K / splits;
#define FT_XC(MT_, NT_)                                                                      \
  if (mt == MT_ && nt == NT_) {                                                              \
    if (packed)                                                                              \
      hipLaunchKernelGGL((ft::skinny_xc_kernel<MT_, NT_, true>), grid, block, 0, stream,     \
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,         \
                         (uint16_t*)out, out_stride, N, k_slice);                            \
    else                                                                                     \
      hipLaunchKernelGGL((ft::skinny_xc_kernel<MT_, NT_, false>), grid, block, 0, stream,    \
                         (const uint16_t*)x, x_stride, M, (const uint16_t*)w, K, ws,         \
                         (uint16_t*)out, out_stride, N, k_slice);                            \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_XC_NT(NT_) FT_XC(1, NT_) FT_XC(2, NT_) FT_XC(3, NT_) FT_XC(4, NT_)
  FT_XC_NT(1)
  FT_XC_NT(2)
#undef FT_XC_NT
#undef FT_XC
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

// Pre-packed-weight variant with an R-deep weight ring (depth 2, 4 or 6).
// Requirements (checked): M <= 64, N % (16*nt) == 0, K % (64*splits) == 0.
extern "C" int ft_skinny_gemm_pkd(const void* x, int x_stride, int M, const void* wpk, int N,
                                  int K, float* ws, void* out, int out_stride, int splits, int nt,
                                  int depth, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (64 * splits) != 0) return -3;
  if (splits > 1 && ws == nullptr) return -4;
  const int mt = (M + 15) / 16;
  dim3 grid(N / (16 * nt), splits), block(256);
  const int k_slice = K / splits;
#define FT_PKD(MT_, NT_, R_)                                                                 \
  if (mt == MT_ && nt == NT_ && depth == R_) {                                               \
    hipLaunchKernelGGL((ft::skinny_pkd_kernel<MT_, NT_, R_>), grid, block, 0, stream,        \
                       (const uint16_t*)x, x_stride, M, (const uint16_t*)wpk, K, ws,         \
                       (uint16_t*)out, out_stride, N, k_slice);                              \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_PKD_MT(NT_, R_) FT_PKD(1, NT_, R_) FT_PKD(2, NT_, R_) FT_PKD(3, NT_, R_) FT_PKD(4, NT_, R_)
  FT_PKD_MT(1, 2) FT_PKD_MT(1, 4) FT_PKD_MT(1, 6)
  FT_PKD_MT(2, 2) FT_PKD_MT(2, 4) FT_PKD_MT(2, 6)
  FT_PKD_MT(4, 2) FT_PKD_MT(4, 4)
#undef FT_PKD_MT
#undef FT_PKD
  return -5;
}
