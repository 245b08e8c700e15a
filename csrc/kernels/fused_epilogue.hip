// Row-wise epilogues that consume GEMM output -- either a bf16 matrix or the
// fp32 split-K slabs of skinny_gemm.hip -- and apply the op that follows the
// GEMM in a Llama layer, so the split-K reduction, the residual add, RMSNorm,
// SiLU-and-mul and RoPE + paged-KV write never make a separate HBM pass:
//
//   add_rmsnorm  : x = sum_s slab (or bf16 x); residual += x; out = rmsnorm(residual)*w   (K2)
//   silu_mul     : h = silu(sum gate) * sum up                                              (K9)
//   rope_kv      : rotate q/k of sum_s slab, write q (bf16) and k/v into the paged cache      (K4)
//   store        : out = bf16(sum_s slab)
//
// add_rmsnorm uses one 256-thread workgroup per row (16 elements per lane at
// H = 4096, all loads issued before the reduction): at decode batch sizes the
// old one-wave-per-row kernel ran on only B/4 CUs and took ~10 us for 50 rows.
#include "ft_common.h"

namespace ft {

struct SrcBf16 {
  const uint16_t* p;
  int stride;
  __device__ __forceinline__ void load8(int row, int col, float (&f)[8]) const {
    load8v(*reinterpret_cast<const uint4*>(p + (size_t)row * stride + col), f);
  }
  __device__ __forceinline__ static void load8v(const uint4& v, float (&f)[8]) { ft::load8(v, f); }
};

struct SrcSlab {
  const float* ws;
  int splits, rows, cols;
  // Slabs are read 4 at a time with clamped (always valid) addresses, so up to 4
  // loads per half are in flight instead of one dependent round trip per split.
  __device__ __forceinline__ void load8(int row, int col, float (&f)[8]) const {
    const float* p = ws + (size_t)row * cols + col;
    const size_t slab = (size_t)rows * cols;
    float4 a = reinterpret_cast<const float4*>(p)[0];
    float4 b = reinterpret_cast<const float4*>(p)[1];
    for (int s0 = 1; s0 < splits; s0 += 4) {
      float4 c[4], d[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* q = p + (size_t)min(s0 + u, splits - 1) * slab;
        c[u] = reinterpret_cast<const float4*>(q)[0];
        d[u] = reinterpret_cast<const float4*>(q)[1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float k = s0 + u < splits ? 1.f : 0.f;
        a.x += k * c[u].x; a.y += k * c[u].y; a.z += k * c[u].z; a.w += k * c[u].w;
        b.x += k * d[u].x; b.y += k * d[u].y; b.z += k * d[u].z; b.w += k * d[u].w;
      }
    }
    f[0] = a.x; f[1] = a.y; f[2] = a.z; f[3] = a.w;
    f[4] = b.x; f[5] = b.y; f[6] = b.z; f[7] = b.w;
  }
};

// ---------------------------------------------------------------------------------
// add + RMSNorm, one 256-thread workgroup per row; VPT = 8-element vectors per lane
// ---------------------------------------------------------------------------------
template <int VPT, bool RESIDUAL, typename Src>
__global__ __launch_bounds__(256) void row_add_rmsnorm_kernel(Src src, uint16_t* __restrict__ out,
                                                              int out_stride,
                                                              uint16_t* __restrict__ residual,
                                                              const uint16_t* __restrict__ weight,
                                                              int hidden, float eps) {
  __shared__ float red[4];
  const int row = blockIdx.x;
  float v[VPT][8];
  uint4 wv[VPT];
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    const int col = (c * 256 + threadIdx.x) * 8;
    src.load8(row, col, v[c]);
    wv[c] = *reinterpret_cast<const uint4*>(weight + col);
  }
  if constexpr (RESIDUAL) {
    uint4* rr = reinterpret_cast<uint4*>(residual + (size_t)row * hidden);
#pragma unroll
    for (int c = 0; c < VPT; ++c) {
      float r[8];
      load8(rr[c * 256 + threadIdx.x], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] += r[j];
      const uint4 rb = store8(v[c]);
      rr[c * 256 + threadIdx.x] = rb;
      load8(rb, v[c]);  // continue from the bf16-rounded residual
    }
  }
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < VPT; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += v[c][j] * v[c][j];
  ss = wave_sum(ss);
  if (lane_id() == 0) red[wave_id()] = ss;
  __syncthreads();
  ss = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(ss / (float)hidden + eps);
  uint4* orow = reinterpret_cast<uint4*>(out + (size_t)row * out_stride);
#pragma unroll
  for (int c = 0; c < VPT; ++c) {
    float wf[8];
    load8(wv[c], wf);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[c][j] = bf16_to_f32(f32_to_bf16(v[c][j] * inv)) * wf[j];
    orow[c * 256 + threadIdx.x] = store8(v[c]);
  }
}

// ---------------------------------------------------------------------------------
// SiLU-and-mul / store over split-K slabs (grid-stride, 8 outputs per thread)
// ---------------------------------------------------------------------------------
// il: interleaved gate/up columns (groups of 16, see silu_mul_kernel)
__global__ __launch_bounds__(256) void slab_silu_kernel(SrcSlab src, uint16_t* __restrict__ out,
                                                        int out_stride, int rows, int inter, int il) {
  const int vec = inter / 8;
  const long total = (long)rows * vec;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int r = (int)(idx / vec), c = (int)(idx - (long)r * vec) * 8;
    float g[8], u[8];
    const int gc = il ? ((c >> 4) << 5) + (c & 15) : c;
    src.load8(r, gc, g);
    src.load8(r, il ? gc + 16 : inter + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) g[j] = g[j] / (1.f + __expf(-g[j])) * u[j];
    *reinterpret_cast<uint4*>(out + (size_t)r * out_stride + c) = store8(g);
  }
}

__global__ __launch_bounds__(256) void slab_store_kernel(SrcSlab src, uint16_t* __restrict__ out,
                                                         int out_stride, int rows, int cols) {
  const int vec = cols / 8;
  const long total = (long)rows * vec;
  for (long idx = (long)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    const int r = (int)(idx / vec), c = (int)(idx - (long)r * vec) * 8;
    float f[8];
    src.load8(r, c, f);
    *reinterpret_cast<uint4*>(out + (size_t)r * out_stride + c) = store8(f);
  }
}

// ---------------------------------------------------------------------------------
// RoPE + paged KV write from split-K slabs of the QKV projection
// ---------------------------------------------------------------------------------
// KV8: fp8 (e4m3) caches (ft_common.h fp8x*), same layouts with 1-byte elements
template <int D, bool KV8>
__global__ __launch_bounds__(256) void slab_rope_kv_kernel(
    SrcSlab src, uint16_t* __restrict__ q_out, int q_stride, const int* __restrict__ positions,
    const float* __restrict__ cos_sin, const int* __restrict__ slot_mapping,
    void* __restrict__ k_cache, void* __restrict__ v_cache, int nq, int nkv,
    int block_size, const uint16_t* __restrict__ residual, int hidden, float eps, int cos_rows,
    int num_slots) {
  constexpr int HALF = D / 2;
  constexpr int CPH = HALF / 8;
  const int t = blockIdx.x;
  const int pos = FT_CHECK_IDX(positions[t], cos_rows, kCkPosition, t);
  int slot = slot_mapping[t];
  if (slot >= 0) slot = FT_CHECK_IDX(slot, num_slots, kCkSlot, t);
  const float* cs = cos_sin + (size_t)pos * D;
  const int blk = slot >= 0 ? slot / block_size : 0;
  const int off = slot >= 0 ? slot - blk * block_size : 0;
  // fused decode layer: the QKV GEMM ran on the raw residual stream with the
  // input-norm weight folded into W, so the RMS scale of the row applies here
  // (RoPE is linear): qkv = rsqrt(mean(res^2) + eps) * sum(slabs)
  float rs = 1.f;
  if (residual != nullptr) {
    __shared__ float red[4];
    const uint4* rr = reinterpret_cast<const uint4*>(residual + (size_t)t * hidden);
    float ss = 0.f;
    for (int c = threadIdx.x; c < hidden / 8; c += blockDim.x) {
      float f[8];
      load8(rr[c], f);
#pragma unroll
      for (int j = 0; j < 8; ++j) ss += f[j] * f[j];
    }
    ss = wave_sum(ss);
    if (lane_id() == 0) red[wave_id()] = ss;
    __syncthreads();
    rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)hidden + eps);
  }
  const int n_rot = (nq + nkv) * CPH;
  const int tid = blockIdx.y * blockDim.x + threadIdx.x, nthr = gridDim.y * blockDim.x;
  for (int item = tid; item < n_rot; item += nthr) {
    const int head = item / CPH, c = item - (item / CPH) * CPH;
    float x1[8], x2[8];
    src.load8(t, head * D + c * 8, x1);
    src.load8(t, head * D + HALF + c * 8, x2);
    float y1[8], y2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float co = cs[c * 8 + j], si = cs[HALF + c * 8 + j];
      x1[j] *= rs;
      x2[j] *= rs;
      y1[j] = x1[j] * co - x2[j] * si;
      y2[j] = x2[j] * co + x1[j] * si;
    }
    if (head < nq) {
      uint16_t* qp = q_out + (size_t)t * q_stride + head * D;
      *reinterpret_cast<uint4*>(qp + c * 8) = store8(y1);
      *reinterpret_cast<uint4*>(qp + HALF + c * 8) = store8(y2);
    } else if (slot >= 0) {
      const size_t e = (((size_t)blk * nkv + (head - nq)) * block_size + off) * D;
      if constexpr (KV8) {
        uint8_t* kp = reinterpret_cast<uint8_t*>(k_cache) + e;
        *reinterpret_cast<uint2*>(kp + c * 8) = fp8x8_pack(y1);
        *reinterpret_cast<uint2*>(kp + HALF + c * 8) = fp8x8_pack(y2);
      } else {
        uint16_t* kp = reinterpret_cast<uint16_t*>(k_cache) + e;
        *reinterpret_cast<uint4*>(kp + c * 8) = store8(y1);
        *reinterpret_cast<uint4*>(kp + HALF + c * 8) = store8(y2);
      }
    }
  }
  if (slot >= 0) {
    const int nv = nkv * (D / 8);
    for (int item = tid; item < nv; item += nthr) {
      const int kh = item / (D / 8), c = item - kh * (D / 8);
      float f[8];
      src.load8(t, (nq + nkv) * D + kh * D + c * 8, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] *= rs;
      // V blocks are transposed ([D][block_size], rope_kv.hip)
      const size_t e = (((size_t)blk * nkv + kh) * D + c * 8) * block_size + off;
      if constexpr (KV8) {
        const uint2 q8 = fp8x8_pack(f);
        uint8_t* vp = reinterpret_cast<uint8_t*>(v_cache) + e;
#pragma unroll
        for (int j = 0; j < 8; ++j) vp[j * block_size] = (uint8_t)(((j < 4 ? q8.x : q8.y) >> (8 * (j & 3))) & 0xffu);
      } else {
        uint16_t* vp = reinterpret_cast<uint16_t*>(v_cache) + e;
#pragma unroll
        for (int j = 0; j < 8; ++j) vp[j * block_size] = f32_to_bf16(f[j]);
      }
    }
  }
}

template <bool RES, typename Src>
static int launch_row_norm(Src src, uint16_t* out, int out_stride, uint16_t* residual,
                           const uint16_t* w, int rows, int hidden, float eps, hipStream_t st) {
  if (hidden % 2048 != 0) return -1;
  const int vpt = hidden / 2048;
  dim3 grid(rows), block(256);
#define FT_RN(V)                                                                              \
  case V:                                                                                     \
    hipLaunchKernelGGL((row_add_rmsnorm_kernel<V, RES, Src>), grid, block, 0, st, src, out,   \
                       out_stride, residual, w, hidden, eps);                                 \
    break;
  switch (vpt) {
    FT_RN(1)
    FT_RN(2)
    FT_RN(3)
    FT_RN(4)
    default:
      return -2;
  }
#undef FT_RN
  return static_cast<int>(hipGetLastError());
}

}  // namespace ft

// x (bf16 rows) or slabs (ws != null) -> [residual +=] -> rmsnorm -> out
extern "C" int ft_row_rmsnorm(const void* x, int x_stride, const float* ws, int splits, void* out,
                              int out_stride, void* residual, const void* w, int rows, int hidden,
                              float eps, hipStream_t stream) {
  if (rows <= 0) return 0;
  uint16_t* res = (uint16_t*)residual;
  if (ws) {
    ft::SrcSlab src{ws, splits, rows, hidden};
    return res ? ft::launch_row_norm<true>(src, (uint16_t*)out, out_stride, res, (const uint16_t*)w,
                                           rows, hidden, eps, stream)
               : ft::launch_row_norm<false>(src, (uint16_t*)out, out_stride, res,
                                            (const uint16_t*)w, rows, hidden, eps, stream);
  }
  ft::SrcBf16 src{(const uint16_t*)x, x_stride};
  return res ? ft::launch_row_norm<true>(src, (uint16_t*)out, out_stride, res, (const uint16_t*)w,
                                         rows, hidden, eps, stream)
             : ft::launch_row_norm<false>(src, (uint16_t*)out, out_stride, res, (const uint16_t*)w,
                                          rows, hidden, eps, stream);
}

extern "C" int ft_slab_silu(const float* ws, int splits, int rows, int inter, void* out,
                            int out_stride, int il, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (inter % 8) return -1;
  ft::SrcSlab src{ws, splits, rows, 2 * inter};
  const long total = (long)rows * (inter / 8);
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(ft::slab_silu_kernel, dim3(grid), dim3(256), 0, stream, src, (uint16_t*)out,
                     out_stride, rows, inter, il);
  return static_cast<int>(hipGetLastError());
}

extern "C" int ft_slab_store(const float* ws, int splits, int rows, int cols, void* out,
                             int out_stride, hipStream_t stream) {
  if (rows <= 0) return 0;
  if (cols % 8) return -1;
  ft::SrcSlab src{ws, splits, rows, cols};
  const long total = (long)rows * (cols / 8);
  int grid = (int)((total + 255) / 256);
  if (grid > 4096) grid = 4096;
  hipLaunchKernelGGL(ft::slab_store_kernel, dim3(grid), dim3(256), 0, stream, src, (uint16_t*)out,
                     out_stride, rows, cols);
  return static_cast<int>(hipGetLastError());
}

extern "C" int ft_slab_rope_kv(const float* ws, int splits, int rows, int cols, void* q_out,
                               int q_stride, const int* positions, const float* cos_sin,
                               const int* slot_mapping, void* k_cache, void* v_cache, int nq,
                               int nkv, int head_dim, int block_size, const void* residual,
                               int hidden, float eps, int cos_rows, int num_slots, int kv8,
                               hipStream_t stream) {
  if (rows <= 0) return 0;
  if (residual != nullptr && hidden % 8 != 0) return -2;
  ft::SrcSlab src{ws, splits, rows, cols};
#define FT_SRK(DD, K8)                                                                          \
  hipLaunchKernelGGL((ft::slab_rope_kv_kernel<DD, K8>), dim3(rows, 2), dim3(256), 0, stream, src, \
                     (uint16_t*)q_out, q_stride, positions, cos_sin, slot_mapping, k_cache,       \
                     v_cache, nq, nkv, block_size, (const uint16_t*)residual, hidden, eps,        \
                     cos_rows, num_slots)
  if (head_dim == 128) {
    if (kv8) FT_SRK(128, true); else FT_SRK(128, false);
  } else if (head_dim == 64) {
    if (kv8) FT_SRK(64, true); else FT_SRK(64, false);
  } else {
    return -1;
  }
#undef FT_SRK
  return static_cast<int>(hipGetLastError());
}

// checked build: this unit's error-word / limits hook (ft_common.h)
FT_CHECK_HOOK(fused_epilogue)
