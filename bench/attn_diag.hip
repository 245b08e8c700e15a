// Diagnostic (not part of the package): the paged decode attention's memory
// stream alone -- same flattened partition, block-table walk, per-lane K / V^T
// addressing and R-deep register ring as csrc/kernels/attn_decode.hip, with the
// MFMAs and softmax replaced by an XOR fold.  MODE 0: K and V, 1: K only,
// 2: V only.  Splits the kernel's time into "stream" and "everything else".
// hipcc -I csrc/include -O3 --offload-arch=gfx950 -shared -fPIC bench/attn_diag.hip -o bench/libattndiag.so
#include "../csrc/kernels/attn_decode.hip"

namespace ftd {
using namespace ft;

template <int D, int R, int MODE>
__global__ __launch_bounds__(256, 2) void attn_loads(const uint16_t* __restrict__ k_cache,
                                                     const uint16_t* __restrict__ v_cache,
                                                     const int* __restrict__ block_tables, int bt_stride,
                                                     const int* __restrict__ seq_lens, int batch, int nkv,
                                                     int bs_shift, unsigned* __restrict__ sink) {
  __shared__ int s_pre[kDecMaxBatch + 1];
  if (wave_id() == 0) dec_prefix(s_pre, seq_lens, batch, 1);
  __syncthreads();
  const int total = nkv * s_pre[batch];
  const int nw = dec_num_waves(total, gridDim.x * 4, kDecMinTiles);
  const int w = wave_id() * gridDim.x + blockIdx.x;
  if (total == 0 || w >= nw) return;
  int f = (int)(((long long)w * total) / nw);
  const int f1 = (int)(((long long)(w + 1) * total) / nw);
  const int lane = lane_id();
  const int n = lane & 15, g = lane >> 4;
  const int bsz = 1 << bs_shift, bmask = bsz - 1;
  const size_t blk_stride = (size_t)nkv * bsz * D;
  const int koff = n * D + 8 * g;
  const int voff = n * bsz + 4 * g;
  unsigned fold = 0;
  while (f < f1) {
    int lo = 0, hi = batch - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (nkv * s_pre[mid] <= f) lo = mid; else hi = mid - 1;
    }
    const int b = lo;
    const int nb = s_pre[b + 1] - s_pre[b];
    const int rel = f - nkv * s_pre[b];
    const int h = rel / nb;
    const int t0 = rel - h * nb;
    const int cnt = min(f1 - f, nb - t0);
    const int* bt = block_tables + (size_t)b * bt_stride;
    for (int c0 = 0; c0 < cnt; c0 += 64) {
      const int cc = min(64, cnt - c0);
      int my_blk = 0, my_off = 0;
      if (lane < cc) {
        const int tok = (t0 + c0 + lane) << 4;
        my_blk = bt[tok >> bs_shift];
        my_off = tok & bmask;
      }
      auto ld = [&](MTile<D>& t, int i) {
        const int j = min(i, cc - 1);
        const size_t blk = (size_t)(uint32_t)__builtin_amdgcn_readlane(my_blk, j);
        const int off = __builtin_amdgcn_readlane(my_off, j);
        const size_t hb = blk * blk_stride + (size_t)h * bsz * D;
        const uint16_t* kb = k_cache + hb + (size_t)off * D;
        const uint16_t* vb = v_cache + hb + off;
        if (MODE == 3) {   // both tiles as whole 1-KiB wave instructions (fragment-ordered layout)
#pragma unroll
          for (int kc = 0; kc < D / 32; ++kc) t.k[kc] = *reinterpret_cast<const uint4*>(kb + lane * 8 + kc * 512);
          const uint16_t* vt = v_cache + hb + (size_t)off * D;
#pragma unroll
          for (int nd = 0; nd < D / 32; ++nd) {
            const uint4 v4 = *reinterpret_cast<const uint4*>(vt + lane * 8 + nd * 512);
            t.v[2 * nd] = make_uint2(v4.x, v4.y);
            t.v[2 * nd + 1] = make_uint2(v4.z, v4.w);
          }
          return;
        }
        if (MODE == 4) {   // the kernel's addressing with non-temporal loads
          typedef unsigned int u4v __attribute__((ext_vector_type(4)));
          typedef unsigned int u2v __attribute__((ext_vector_type(2)));
#pragma unroll
          for (int kc = 0; kc < D / 32; ++kc)
            t.k[kc] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(
                                                    reinterpret_cast<const u4v*>(kb + koff + kc * 32)));
#pragma unroll
          for (int nd = 0; nd < D / 16; ++nd)
            t.v[nd] = __builtin_bit_cast(uint2, __builtin_nontemporal_load(
                                                    reinterpret_cast<const u2v*>(vb + voff + nd * 16 * bsz)));
          return;
        }
        if (MODE != 2) {
#pragma unroll
          for (int kc = 0; kc < D / 32; ++kc) t.k[kc] = *reinterpret_cast<const uint4*>(kb + koff + kc * 32);
        }
        if (MODE != 1) {
#pragma unroll
          for (int nd = 0; nd < D / 16; ++nd)
            t.v[nd] = *reinterpret_cast<const uint2*>(vb + voff + nd * 16 * bsz);
        }
      };
      auto consume = [&](const MTile<D>& t) {
        if (MODE != 2) {
#pragma unroll
          for (int kc = 0; kc < D / 32; ++kc) fold ^= t.k[kc].x ^ t.k[kc].y ^ t.k[kc].z ^ t.k[kc].w;
        }
        if (MODE != 1) {
#pragma unroll
          for (int nd = 0; nd < D / 16; ++nd) fold ^= t.v[nd].x ^ t.v[nd].y;
        }
      };
      MTile<D> ring[R];
#pragma unroll
      for (int r = 0; r + 1 < R; ++r) ld(ring[r], r);
      for (int i = 0; i < cc; i += R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          ld(ring[(r + R - 1) % R], i + r + R - 1);
          __builtin_amdgcn_sched_barrier(0);
          if (i + r < cc) consume(ring[r]);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    f += cnt;
  }
  if (fold == 0x9e3779b9u) sink[threadIdx.x] = fold;
}
}  // namespace ftd

extern "C" int attn_loads_launch(const void* k, const void* v, const int* bt, int bt_stride, const int* sl,
                                 int batch, int nkv, int mode, int ring, int wpc, int bs_shift,
                                 unsigned* sink, hipStream_t stream) {
  const int nwg = ft_num_cus() * wpc;
#define L(MM, RR)                                                                                      \
  if (mode == MM && ring == RR) {                                                                      \
    hipLaunchKernelGGL((ftd::attn_loads<128, RR, MM>), dim3(nwg), dim3(256), 0, stream,                \
                       (const uint16_t*)k, (const uint16_t*)v, bt, bt_stride, sl, batch, nkv, bs_shift, sink); \
    return (int)hipGetLastError();                                                                     \
  }
  L(0, 3) L(1, 3) L(2, 3) L(0, 4) L(0, 6) L(3, 3) L(3, 4) L(4, 2) L(4, 3) L(4, 4)
#undef L
  return -1;
}
