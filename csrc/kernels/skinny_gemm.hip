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
