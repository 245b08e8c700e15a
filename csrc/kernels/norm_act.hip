// K2 (RMSNorm / fused residual-add + RMSNorm) and K9 (SiLU-and-mul) for gfx950.
//
// Both are HBM-bound streaming ops.  Layout decisions:
//   * one wave64 per row, 4 rows per 256-thread workgroup; every lane moves
//     16 B (8 x bf16) per access so one wave instruction covers 1 KiB of a row;
//     the row stays in registers between the reduction and the scaled store
//     (single HBM read + single write per tensor, no LDS round trip).
//   * the fused variant writes the updated residual (bf16) and the normalised
//     row in one pass, which is the "fuse elementwise into the producer" rule:
//     the residual add never exists as a separate kernel.
//   * SiLU-and-mul reads gate and up halves of the gate_up GEMM output with
//     16-B loads and does the math in fp32 with a single rounding.
#include "ft_common.h"

namespace ft {

// ----------------------------------------------------------------------------
// RMSNorm: out[r] = bf16(bf16(x[r] * rsqrt(mean(x^2)+eps)) * w)   (HF Llama order)
// If RESIDUAL: r = bf16(x + res); res <- r; out <- norm(r).
// ----------------------------------------------------------------------------
template <int NCHUNK, bool RESIDUAL>
__global__ __launch_bounds__(256) void rmsnorm_kernel(uint16_t* __restrict__ out,
                                                      const uint16_t* __restrict__ x,
                                                      uint16_t* __restrict__ residual,
                                                      const uint16_t* __restrict__ weight,
                                                      int rows, int hidden, int x_stride,
                                                      int out_stride, float eps) {
  const int row = blockIdx.x * 4 + wave_id();
  if (row >= rows) return;
  const int lane = lane_id();
  const uint4* xr = reinterpret_cast<const uint4*>(x + (size_t)row * x_stride);
  uint4 v[NCHUNK];
#pragma unroll
  for (int c = 0; c < NCHUNK; ++c) v[c] = xr[c * 64 + lane];

  if constexpr (RESIDUAL) {
    uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * hidden);
#pragma unroll
    for (int c = 0; c < NCHUNK; ++c) {
      float a[8], b[8];
      load8(v[c], a);
      load8(rr[c * 64 + lane], b);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] += b[j];
      v[c] = store8(a);          // round the sum to bf16 (it is stored as bf16)
      rr[c * 64 + lane] = v[c];
    }
  }

  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCHUNK; ++c) {
    float a[8];
    load8(v[c], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)hidden + eps);

  const uint4* wr = reinterpret_cast<const uint4*>(weight);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * out_stride);
#pragma unroll
  for (int c = 0; c < NCHUNK; ++c) {
    float a[8], w[8];
    load8(v[c], a);
    load8(wr[c * 64 + lane], w);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float n = bf16_to_f32(f32_to_bf16(a[j] * inv));
      a[j] = n * w[j];
    }
    orow[c * 64 + lane] = store8(a);
  }
}

template <bool RESIDUAL>
static int launch_rmsnorm(uint16_t* out, const uint16_t* x, uint16_t* residual, const uint16_t* w,
                          int rows, int hidden, int x_stride, int out_stride, float eps,
                          hipStream_t stream) {
  if (rows <= 0) return 0;
  if (hidden % 512 != 0) return -1;
  dim3 grid(ceil_div(rows, 4)), block(256);
  const int nchunk = hidden / 512;
#define FT_RMS_CASE(N)                                                                    \
  case N:                                                                                 \
    hipLaunchKernelGGL((rmsnorm_kernel<N, RESIDUAL>), grid, block, 0, stream, out, x,     \
                       residual, w, rows, hidden, x_stride, out_stride, eps);             \
    break;
  switch (nchunk) {
    FT_RMS_CASE(1)
    FT_RMS_CASE(2)
    FT_RMS_CASE(3)
    FT_RMS_CASE(4)
    FT_RMS_CASE(5)
    FT_RMS_CASE(6)
    FT_RMS_CASE(8)
    FT_RMS_CASE(10)
    FT_RMS_CASE(12)
    FT_RMS_CASE(16)
    default:
      return -2;
  }
#undef FT_RMS_CASE
  return static_cast<int>(hipGetLastError());
}

// ----------------------------------------------------------------------------
// K1 + first K2: embedding gather fused with the first layer's RMSNorm.
//   residual[t] = table[ids[t]]   (the residual stream starts as the embedding)
//   out[t]      = rmsnorm(table[ids[t]]) * w
// One wave per token row, the gathered row stays in registers between the
// reduction and both stores (the embedding row is read from HBM once).
// ----------------------------------------------------------------------------
template <int NCHUNK>
__global__ __launch_bounds__(256) void embed_rmsnorm_kernel(uint16_t* __restrict__ out,
                                                            uint16_t* __restrict__ residual,
                                                            const int* __restrict__ ids,
                                                            const uint16_t* __restrict__ table,
                                                            const uint16_t* __restrict__ weight,
                                                            int rows, int hidden, int vocab,
                                                            float eps) {
  const int row = blockIdx.x * 4 + wave_id();
  if (row >= rows) return;
  const int lane = lane_id();
  const int tok = min(max(FT_CHECK_IDX(ids[row], vocab, kCkTokenId, row), 0), vocab - 1);
  const uint4* xr = reinterpret_cast<const uint4*>(table + (size_t)tok * hidden);
  uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * hidden);
  uint4 v[NCHUNK];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCHUNK; ++c) {
    v[c] = xr[c * 64 + lane];
    rr[c * 64 + lane] = v[c];
    float a[8];
    load8(v[c], a);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += a[j] * a[j];
  }
  ss = wave_sum(ss);
  const float inv = rsqrtf(ss / (float)hidden + eps);
  const uint4* wr = reinterpret_cast<const uint4*>(weight);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * hidden);
#pragma unroll
  for (int c = 0; c < NCHUNK; ++c) {
    float a[8], w[8];
    load8(v[c], a);
    load8(wr[c * 64 + lane], w);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = bf16_to_f32(f32_to_bf16(a[j] * inv)) * w[j];
    orow[c * 64 + lane] = store8(a);
  }
}

// ----------------------------------------------------------------------------
// SiLU-and-mul: out[t, i] = silu(gu[t, i]) * gu[t, I + i]
// ----------------------------------------------------------------------------
// il: gate/up rows interleaved in groups of 16 (ops.interleave_gate_up(w, 1), the
// single gate_up image of the packed model): gate column c sits at
// (c / 16) * 32 + c % 16, its up column 16 further.
__global__ __launch_bounds__(256) void silu_mul_kernel(uint16_t* __restrict__ out,
                                                       const uint16_t* __restrict__ gu, int rows,
                                                       int inter, int il) {
  const int vec_per_row = inter / 8;
  const long total = (long)rows * vec_per_row;
  for (long idx = (long)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (long)gridDim.x * blockDim.x) {
    const long r = idx / vec_per_row;
    const int c = (int)(idx - r * vec_per_row);
    const uint4* g4 = reinterpret_cast<const uint4*>(gu + r * 2 * (long)inter);
    float g[8], u[8];
    const int gi = il ? ((c >> 1) << 2) + (c & 1) : c;       // uint4 index of the gate chunk
    load8(g4[gi], g);
    load8(g4[il ? gi + 2 : vec_per_row + c], u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    reinterpret_cast<uint4*>(out + r * (long)inter)[c] = store8(g);
  }
}

}  // namespace ft

extern "C" int ft_rmsnorm(void* out, const void* x, const void* w, int rows, int hidden,
                          int x_stride, int out_stride, float eps, hipStream_t stream) {
  return ft::launch_rmsnorm<false>((uint16_t*)out, (const uint16_t*)x, nullptr,
                                   (const uint16_t*)w, rows, hidden, x_stride, out_stride, eps,
                                   stream);
}

extern "C" int ft_fused_add_rmsnorm(void* out, const void* x, void* residual, const void* w,
                                    int rows, int hidden, int x_stride, int out_stride,
                                    float eps, hipStream_t stream) {
  return ft::launch_rmsnorm<true>((uint16_t*)out, (const uint16_t*)x, (uint16_t*)residual,
                                  (const uint16_t*)w, rows, hidden, x_stride, out_stride, eps,
                                  stream);
}

extern "C" int ft_silu_mul(void* out, const void* gu, int rows, int inter, int il,
                           hipStream_t stream) {
  if (rows <= 0) return 0;
  if (inter % 8 != 0) return -1;
  const long total = (long)rows * (inter / 8);
  int grid = (int)((total + 255) / 256);
  if (grid > 256 * 16) grid = 256 * 16;
  hipLaunchKernelGGL(ft::silu_mul_kernel, dim3(grid), dim3(256), 0, stream, (uint16_t*)out,
                     (const uint16_t*)gu, rows, inter, il);
  return static_cast<int>(hipGetLastError());
}

extern "C" int ft_embed_rmsnorm(void* out, void* residual, const int* ids, const void* table,
                                const void* w, int rows, int hidden, int vocab, float eps,
                                hipStream_t stream) {
  if (rows <= 0) return 0;
  if (hidden % 512 != 0) return -1;
  dim3 grid(ft::ceil_div(rows, 4)), block(256);
#define FT_EMB_CASE(N)                                                                      \
  case N:                                                                                   \
    hipLaunchKernelGGL((ft::embed_rmsnorm_kernel<N>), grid, block, 0, stream, (uint16_t*)out, \
                       (uint16_t*)residual, ids, (const uint16_t*)table, (const uint16_t*)w,  \
                       rows, hidden, vocab, eps);                                          \
    break;
  switch (hidden / 512) {
    FT_EMB_CASE(1)
    FT_EMB_CASE(2)
    FT_EMB_CASE(3)
    FT_EMB_CASE(4)
    FT_EMB_CASE(6)
    FT_EMB_CASE(8)
    FT_EMB_CASE(16)
    default:
      return -2;
  }
#undef FT_EMB_CASE
  return static_cast<int>(hipGetLastError());
}

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(norm_act)
