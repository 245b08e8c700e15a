// Decode GEMMs of the fused decode layer (M <= 64 rows: one token per running
// sequence): y[M, N] = x[M, K] . W[N, K]^T, bf16 in, fp32 accumulate, streaming
// pre-packed weights through an S-deep register ring, with fused epilogues.
//
// Why a ring (profiles/bench_kernels_packed.txt, 50 sessions -> batch bucket 64):
// the 2-stage "pk" kernel (skinny_gemm.hip) streamed the down projection at
// 3.9 TB/s and hipBLASLt the gate_up at 4.9 TB/s, against 6.3 TB/s for an HBM
// copy.  At ~10 B/clk/CU and 1.5-2 us of loaded HBM latency a CU needs 35-70 KiB
// of weight loads in flight; a 2-stage NT=4 wave keeps 8 KiB, an S-stage one
// S * NT * 2 KiB.
//
// Layout ("pk" contract): W is the MFMA-fragment image [N/16][K/64][half][lane][8]
// (ops.pack_weight), so a weight load is 1 KiB contiguous per wave instruction.
// The 4 waves of a workgroup split K (wave w: k-steps w, w+4, ...) over the same
// 16*NT output columns; x fragments come straight from L2; the four partial
// tiles are summed through LDS into wave 0, which runs the epilogue:
//   EPI_STORE  bf16 y (out given and one split) or fp32 split-K slabs ws[s][m][n]
//   EPI_SILU   one split; the packing interleaves gate and up so tiles j and
//              j + NT/2 of a workgroup are the gate / up columns of the same
//              outputs (ops.interleave_gate_up): h = silu(g) * u.  With NORM the
//              rows of x are RMS-normalised on the fly -- the sum of squares comes
//              from the streamed x fragments (v_dot2) and the norm weight is
//              folded into W -- so the post-attention RMSNorm, gate_up and
//              SiLU-mul are one launch.
//   EPI_RESID  residual[m][n] += y in place (fp32 add, bf16 store).  Split-K
//              partials are reduced inside the launch: each split stores its slab,
//              publishes it (agent-scope release), takes a ticket, and the last
//              split of a column tile sums every slab in split order (the result
//              does not depend on arrival order), updates the residual and
//              re-arms the ticket (cdna_hip_programming.md, "In-launch split-K
//              reduction").  O and down projections need no separate add launch.
//
// WN (wave-split-N, for 33-64 rows): the K-split layout above makes every wave read
// its own x fragments, so x leaves L2 (N / 16NT) * M * K * 2 bytes per launch --
// at M = 64 four times the weight bytes of the O projection, and the kernel fell to
// half of hipBLASLt.  With WN the 4 waves own 4 * NT adjacent column tiles and walk
// the same k-steps, so one x fragment load serves the workgroup through L1 and no
// LDS reduction is needed; every wave runs the epilogue of its own tile.
#include "ft_common.h"

namespace ft {

typedef __bf16 pr_bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 pr_bf16x2 __attribute__((ext_vector_type(2)));
typedef float pr_floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned int pr_u32x4 __attribute__((ext_vector_type(4)));

constexpr int kEpiStore = 0, kEpiSilu = 1, kEpiResid = 2;

struct PrArgs {
  const uint16_t* x;
  const uint16_t* wpk;
  float* ws;
  uint16_t* out;
  uint16_t* residual;
  int* tickets;
  int x_stride, M, K, N, k_slice, out_stride, res_stride;
  float eps;
};

__device__ __forceinline__ pr_bf16x8 pr_frag(const uint4& v) {
  return __builtin_bit_cast(pr_bf16x8, v);
}

// streamed-once weights: non-temporal loads
__device__ __forceinline__ uint4 pr_nt_load16(const uint16_t* p) {
  const pr_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const pr_u32x4*>(p));
  return __builtin_bit_cast(uint4, v);
}

// c + a.lo^2 + a.hi^2 for a word holding two bf16
__device__ __forceinline__ float pr_sq2(uint32_t w, float c) {
  const pr_bf16x2 a = __builtin_bit_cast(pr_bf16x2, w);
  return __builtin_amdgcn_fdot2_f32_bf16(a, a, c, false);
}

template <int MT, int NT>
struct PrStage {
  uint4 w[NT][2];
  uint4 x[MT][2];
};

template <int MT, int NT, int S, int EPI, bool NORM, bool WN>
__global__ __launch_bounds__(256) void skinny_pkr_kernel(PrArgs a) {
  // waves 1..3 hand their partial tiles to wave 0 through LDS
  __shared__ float s_red[3][MT * NT * 4][64];
  __shared__ float s_ss[4][MT * 16];
  const int lane = lane_id(), wave = wave_id();
  const int l15 = lane & 15, g = lane >> 4;
  const int M = a.M, N = a.N;
  const int tile = WN ? blockIdx.x * 4 + wave : blockIdx.x;  // 16*NT-column tile
  const int n0 = tile * (16 * NT);
  const int s = blockIdx.y;
  const int kbeg = s * a.k_slice;
  const int ksteps_total = a.K >> 6;
  const int step0 = kbeg >> 6;

  const uint16_t* wp[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j)
    wp[j] = a.wpk + ((size_t)(n0 / 16 + j) * ksteps_total + step0) * 1024 + lane * 8;
  const uint16_t* xp[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int r = min(16 * i + l15, M - 1);
    xp[i] = a.x + (size_t)r * a.x_stride + kbeg + 16 * g;
  }

  pr_floatx4 acc[MT][NT];
  float ss[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    ss[i] = 0.f;
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = pr_floatx4{0.f, 0.f, 0.f, 0.f};
  }

  const int nsteps = a.k_slice >> 6;
  const int my_steps = WN ? nsteps : nsteps > wave ? (nsteps - wave + 3) >> 2 : 0;

  auto load = [&](PrStage<MT, NT>& st, int t) {
    const int ks = WN ? t : wave + 4 * t;  // k-step within this split
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const uint16_t* p = wp[j] + (size_t)ks * 1024;
      st.w[j][0] = pr_nt_load16(p);
      st.w[j][1] = pr_nt_load16(p + 512);
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const uint4* p = reinterpret_cast<const uint4*>(xp[i] + ks * 64);
      st.x[i][0] = p[0];
      st.x[i][1] = p[1];
    }
  };
  auto mma = [&](const PrStage<MT, NT>& st) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pr_frag(st.x[i][0]), pr_frag(st.w[j][0]),
                                                            acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pr_frag(st.x[i][1]), pr_frag(st.w[j][1]),
                                                            acc[i][j], 0, 0, 0);
      }
    if constexpr (NORM) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          ss[i] = pr_sq2(st.x[i][h].x, ss[i]);
          ss[i] = pr_sq2(st.x[i][h].y, ss[i]);
          ss[i] = pr_sq2(st.x[i][h].z, ss[i]);
          ss[i] = pr_sq2(st.x[i][h].w, ss[i]);
        }
    }
  };

  // The loop body is branch-free (loads past the last step re-read it, clamped) so
  // the compiler keeps counted vmcnt waits across the back edge; a conditional
  // load there makes it drain to vmcnt(0) at the top of every iteration.
  if (my_steps > 0) {
    const int last = my_steps - 1;
    PrStage<MT, NT> ring[S];
#pragma unroll
    for (int q = 0; q < S; ++q) load(ring[q], min(q, last));
    int t = 0;
    for (; t + S < my_steps; t += S) {
#pragma unroll
      for (int q = 0; q < S; ++q) {
        __builtin_amdgcn_sched_barrier(0);
        mma(ring[q]);
        __builtin_amdgcn_sched_barrier(0);
        load(ring[q], min(t + q + S, last));
      }
    }
    // the last 1..S steps are already in the ring
#pragma unroll
    for (int q = 0; q < S; ++q)
      if (t + q < my_steps) mma(ring[q]);
  }

  if constexpr (NORM) {
    // lane (l15, g) holds row 16 i + l15's squares of its k offsets: sum over g
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v = ss[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g == 0) s_ss[wave][i * 16 + l15] = v;
    }
  }
  // WN: the wave's own sums of squares cover all of K; s_ss[wave] is written and
  // read by this wave only (LDS ops of a wave complete in order)
  if constexpr (WN) {
  } else {
  if (wave > 0) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) s_red[wave - 1][(i * NT + j) * 4 + r][lane] = acc[i][j][r];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int reg = (i * NT + j) * 4 + r;
        acc[i][j][r] += s_red[0][reg][lane] + s_red[1][reg][lane] + s_red[2][reg][lane];
      }
  }

  // C layout: col = lane & 15 (n), row = (lane >> 4) * 4 + r (m)
  if constexpr (EPI == kEpiSilu) {
    constexpr int NH = NT / 2;
    const int c0 = tile * (16 * NH);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * g + r;
        float rs = 1.f;
        if constexpr (NORM) {
          const int q = i * 16 + 4 * g + r;
          const float sq = WN ? s_ss[wave][q] : s_ss[0][q] + s_ss[1][q] + s_ss[2][q] + s_ss[3][q];
          rs = rsqrtf(sq / (float)a.K + a.eps);
        }
        if (m < M) {
#pragma unroll
          for (int j = 0; j < NH; ++j) {
            const float gt = acc[i][j][r] * rs, up = acc[i][j + NH][r] * rs;
            a.out[(size_t)m * a.out_stride + c0 + 16 * j + l15] =
                f32_to_bf16(gt / (1.f + __expf(-gt)) * up);
          }
        }
      }
    return;
  }

  if constexpr (EPI == kEpiStore) {
    const bool bf16_out = a.out != nullptr && gridDim.y == 1;
    float* slab = a.ws + (size_t)s * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * g + r;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int n = n0 + 16 * j + l15;
            if (bf16_out)
              a.out[(size_t)m * a.out_stride + n] = f32_to_bf16(acc[i][j][r]);
            else
              slab[(size_t)m * N + n] = acc[i][j][r];
          }
        }
      }
    return;
  }

  // ---- EPI_RESID ----------------------------------------------------------------
  // the residual tile is read before the slab handshake so its latency overlaps it
  float res_pre[MT][NT][4];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = min(16 * i + 4 * g + r, M - 1);
#pragma unroll
      for (int j = 0; j < NT; ++j)
        res_pre[i][j][r] = bf16_to_f32(a.residual[(size_t)m * a.res_stride + n0 + 16 * j + l15]);
    }
  if (gridDim.y > 1) {
    float* slab = a.ws + (size_t)s * M * N;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = 16 * i + 4 * g + r;
        if (m < M) {
#pragma unroll
          for (int j = 0; j < NT; ++j) slab[(size_t)m * N + n0 + 16 * j + l15] = acc[i][j][r];
        }
      }
    // publish the slab, then take a ticket; the last split of this tile reduces
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int prev = 0;
    if (lane == 0)
      prev = __hip_atomic_fetch_add(a.tickets + tile, 1, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT);
    prev = __shfl(prev, 0, 64);
    if (prev != (int)gridDim.y - 1) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // every slab in split order (deterministic whoever arrives last)
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[i][j] = pr_floatx4{0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < (int)gridDim.y; ++sp) {
      const float* sl = a.ws + (size_t)sp * M * N;
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int m = min(16 * i + 4 * g + r, M - 1);
#pragma unroll
          for (int j = 0; j < NT; ++j) acc[i][j][r] += sl[(size_t)m * N + n0 + 16 * j + l15];
        }
    }
    if (lane == 0) a.tickets[tile] = 0;  // re-arm for the next launch
  }
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 16 * i + 4 * g + r;
      if (m < M) {
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          a.residual[(size_t)m * a.res_stride + n0 + 16 * j + l15] =
              f32_to_bf16(res_pre[i][j][r] + acc[i][j][r]);
        }
      }
    }
}

}  // namespace ft

// Requirements (checked): M <= 64, N % (16*nt) == 0, K % (64*splits) == 0.
//   epi 0 (store): out (one split) or ws [splits, M, N]
//   epi 1 (silu):  one split, nt even, out [M, N/2]; norm: x rows RMS-normalised
//   epi 2 (resid): residual [M, N] (row stride res_stride); splits > 1 needs ws and
//                  N/(16*nt) zeroed tickets (left zeroed on return)
extern "C" int ft_pkr_gemm(const void* x, int x_stride, int M, const void* wpk, int N, int K,
                           float* ws, void* out, int out_stride, void* residual, int res_stride,
                           int* tickets, int splits, int nt, int depth, int epi, int norm,
                           int wn, float eps, hipStream_t stream) {
  if (M <= 0) return 0;
  if (M > 64 || splits < 1 || splits > 64) return -1;
  if (N % (16 * nt) != 0) return -2;
  if (K % (64 * splits) != 0) return -3;
  if (epi == ft::kEpiStore && !(out != nullptr && splits == 1) && ws == nullptr) return -4;
  if (epi == ft::kEpiSilu && (splits != 1 || nt % 2 != 0 || out == nullptr)) return -6;
  if (epi == ft::kEpiResid &&
      (residual == nullptr || (splits > 1 && (ws == nullptr || tickets == nullptr))))
    return -7;
  if (norm && epi != ft::kEpiSilu) return -8;
  const int mt = (M + 15) / 16;
  if (wn && (N % (64 * nt) != 0 || mt < 3)) return -9;
  ft::PrArgs a{(const uint16_t*)x, (const uint16_t*)wpk, ws, (uint16_t*)out, (uint16_t*)residual,
               tickets, x_stride, M, K, N, K / splits, out_stride, res_stride, eps};
  dim3 grid(N / (16 * nt) / (wn ? 4 : 1), splits), block(256);
#define FT_PRW(MT_, NT_, S_, E_, N_, W_)                                                     \
  if (mt == MT_ && nt == NT_ && depth == S_ && epi == E_ && (norm != 0) == N_ &&             \
      (wn != 0) == W_) {                                                                     \
    hipLaunchKernelGGL((ft::skinny_pkr_kernel<MT_, NT_, S_, E_, N_, W_>), grid, block, 0,     \
                       stream, a);                                                           \
    return static_cast<int>(hipGetLastError());                                              \
  }
#define FT_PR(MT_, NT_, S_, E_, N_) FT_PRW(MT_, NT_, S_, E_, N_, false)
#define FT_PR_MT(NT_, S_, E_, N_)                                                   \
  FT_PR(1, NT_, S_, E_, N_) FT_PR(2, NT_, S_, E_, N_) FT_PR(3, NT_, S_, E_, N_)     \
  FT_PR(4, NT_, S_, E_, N_) FT_PRW(3, NT_, S_, E_, N_, true) FT_PRW(4, NT_, S_, E_, N_, true)
  // ring stages stay within ~192 VGPRs: S * (MT + NT) * 8 <= 192 at MT = 4
#define FT_PR_PLAIN(NT_, S_) FT_PR_MT(NT_, S_, 0, false) FT_PR_MT(NT_, S_, 2, false)
#define FT_PR_SILU(NT_, S_) FT_PR_MT(NT_, S_, 1, true)
  FT_PR_PLAIN(1, 2)
  FT_PR_PLAIN(1, 4)
  FT_PR_PLAIN(2, 2)
  FT_PR_PLAIN(2, 3)
  FT_PR_PLAIN(2, 4)
  FT_PR_PLAIN(4, 2)
  FT_PR_PLAIN(4, 3)
  FT_PR_SILU(2, 2)
  FT_PR_SILU(2, 3)
  FT_PR_SILU(2, 4)
  FT_PR_SILU(4, 2)
  FT_PR_SILU(4, 3)
#undef FT_PR_SILU
#undef FT_PR_PLAIN
#undef FT_PR_MT
#undef FT_PR
#undef FT_PRW
  return -5;
}
