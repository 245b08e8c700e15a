// Diagnostic (not part of the package): the fp8 decode attention's memory stream
// alone -- the flattened partition, block-table walk and register ring of
// csrc/kernels/attn_decode.hip's KV8 path at 4 waves per workgroup, with the MFMAs,
// conversions and softmax replaced by an XOR fold.  V MODE 0: the kernel's V^T
// addressing (8 x 4-B loads per lane per tile); MODE 1: the same bytes in a
// fragment-ordered V layout (2 x 16-B loads per lane per tile); MODE 2: K only.
// hipcc -I csrc/include -O3 --offload-arch=gfx950 -shared -fPIC bench/attn_fp8_diag.hip -o bench/libattnfp8diag.so
#include "../csrc/kernels/attn_decode.hip"

namespace ftd8 {
using namespace ft;

template <int R, int MODE>
__global__ __launch_bounds__(256, 1) void attn8_loads(const uint8_t* __restrict__ k_cache,
                                                      const uint8_t* __restrict__ v_cache,
                                                      const int* __restrict__ block_tables, int bt_stride,
                                                      const int* __restrict__ seq_lens, int batch, int nkv,
                                                      int bs_shift, unsigned* __restrict__ sink) {
  constexpr int D = 128;
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
  const int koff = n * D + 16 * g;
  const int voff = n * bsz + 4 * g;
  unsigned fold = 0;
  struct T8 { uint4 k[2]; uint4 v[2]; };
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
      auto ld = [&](T8& t, int i) {
        const int j = min(i, cc - 1);
        const size_t blk = (size_t)(uint32_t)__builtin_amdgcn_readlane(my_blk, j);
        const int off = __builtin_amdgcn_readlane(my_off, j);
        const size_t hb = blk * blk_stride + (size_t)h * bsz * D;
        const __amdgpu_buffer_rsrc_t kr = __builtin_amdgcn_make_buffer_rsrc(
            uniform_ptr(k_cache + hb + (size_t)off * D), 0, 16 * D, 0x00020000);
        t.k[0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(kr, koff, 0, 2));
        t.k[1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(kr, koff + 64, 0, 2));
        if (MODE == 0) {
          const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
              uniform_ptr(v_cache + hb + off), 0, 0x7fffffff, 0x00020000);
          uint32_t vv[8];
#pragma unroll
          for (int nd = 0; nd < 8; ++nd) vv[nd] = __builtin_amdgcn_raw_buffer_load_b32(vr, voff, nd * 16 * bsz, 2);
          t.v[0] = make_uint4(vv[0], vv[1], vv[2], vv[3]);
          t.v[1] = make_uint4(vv[4], vv[5], vv[6], vv[7]);
        } else if (MODE == 1) {   // fragment-ordered 16-token V tile: lane l's 32 B at 32 l
          const __amdgpu_buffer_rsrc_t vr = __builtin_amdgcn_make_buffer_rsrc(
              uniform_ptr(v_cache + hb + (size_t)off * D), 0, 16 * D, 0x00020000);
          t.v[0] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(vr, lane * 32, 0, 2));
          t.v[1] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(vr, lane * 32 + 16, 0, 2));
        }
      };
      auto consume = [&](const T8& t) {
        fold ^= t.k[0].x ^ t.k[0].y ^ t.k[0].z ^ t.k[0].w ^ t.k[1].x ^ t.k[1].y ^ t.k[1].z ^ t.k[1].w;
        if (MODE != 2) fold ^= t.v[0].x ^ t.v[0].y ^ t.v[0].z ^ t.v[0].w ^ t.v[1].x ^ t.v[1].y ^ t.v[1].z ^ t.v[1].w;
      };
      T8 ring[R];
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
}  // namespace ftd8

extern "C" int attn8_loads_launch(const void* k, const void* v, const int* bt, int bt_stride, const int* sl,
                                  int batch, int nkv, int mode, int ring, int bs_shift, unsigned* sink,
                                  hipStream_t stream) {
  const int nwg = ft_num_cus();
#define L(MM, RR)                                                                                      \
  if (mode == MM && ring == RR) {                                                                      \
    hipLaunchKernelGGL((ftd8::attn8_loads<RR, MM>), dim3(nwg), dim3(256), 0, stream,                   \
                       (const uint8_t*)k, (const uint8_t*)v, bt, bt_stride, sl, batch, nkv, bs_shift, sink); \
    return (int)hipGetLastError();                                                                     \
  }
  L(0, 2) L(1, 2) L(2, 2) L(0, 3) L(1, 3)
#undef L
  return -1;
}
