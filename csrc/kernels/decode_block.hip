// Persistent post-attention decode block (33..64 rows, also 1..32): ONE launch per
// layer runs
//     residual += attn . Wo^T                  (phase O, split-K, in-launch combine)
//     h = silu(g) * u,  [g|u] = rms(residual) . Wgu'^T      (phase GU, ln2 folded in W)
//     residual += h . Wd^T                     (phase D, split-K, in-launch combine)
// with the workgroups resident (one 8-wave workgroup per CU, grid = #CUs) and the
// phases joined by grid-wide arrival counters.  It replaces five launches of the
// unfused decode layer (o GEMM, add+RMSNorm, gate_up+SiLU GEMM, down GEMM,
// add+RMSNorm: 96 us per layer at 50 rows on MI355X, profiles/prof_driver_config_r05.txt)
// whose costs beyond the 61 us weight stream were per-launch ramps and tails, the two
// row kernels, and 224-of-256-CU gate_up grids.  What the single launch buys:
//   * each phase's first weight chunks are loaded BEFORE the grid barrier that
//     precedes it (weights never depend on activations), so the barrier latency and
//     the seam work overlap the next phase's HBM stream (guide: MI355X_MICROARCH.md,
//     "prefetch-credit");
//   * the post-attention RMSNorm is an epilogue scale: gate_up runs on the raw
//     residual (ln2 folded into the packed image) and every workgroup computes the
//     rows' sums of squares while it stages them anyway (it reads all of K), so no
//     norm kernel and no extra pass; the next layer's input norm is applied by
//     slab_rope_kv from the residual (the fused ring layer's convention);
//   * gate_up tiles are dealt 7 per workgroup on all 256 CUs (1,792 16-column tiles):
//     a gate/up pair split between two workgroups meets through a 2-way ticket.
// Weights: the packed MFMA-fragment images (ops.pack_weight: [N/16][K/64][half][lane][8]),
// streamed non-temporal into a per-wave register ring two 256-deep K chunks ahead;
// x (attn / residual / h rows) is staged per chunk in LDS once per workgroup (the xr
// kernel's swizzle, skinny_gemm.hip) and read as MFMA A fragments
// (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
// Phase geometry (Llama-3-8B, G = 256): O and D deal 64 columns x K/4 per workgroup
// (the 4 K-slices of a column group on one XCD, speed only); the 8 waves split the
// workgroup's 4 column tiles x 2 k-step parities and meet in LDS.  GU deals 7 tiles
// x all of K, one tile per wave (wave 7 stages x only).
// Hand-offs (cdna_hip_programming.md Guideline 16, R1): everything another
// workgroup reads in this launch (split-K slabs, residual rows, h rows, split-pair
// tiles) is stored write-through (sc1), every storing wave drains vmcnt(0), one lane
// signals with an agent-scope atomic; slab / pair consumers read with sc1 loads,
// phase consumers poll the grid counter relaxed and run ONE agent acquire.  Every
// counter is left zeroed for the next launch (last arriver / last finisher resets);
// every spin is bounded and a give-up sets the sticky error word ctl[2] (checked by
// the runner: engine/runner.py).
#include "ft_common.h"

#include <stdlib.h>

namespace ft {
namespace dblk {

// 4 waves per workgroup, one per SIMD: each wave may hold ~400 VGPRs, most of them a
// weight ring several 256-deep K chunks deep (192-224 KiB in flight per CU; the first
// 8-wave version kept 64 KiB and its phases ran at ~28 GB/s per CU)
constexpr int NW = 4, NTH = 64 * NW;
constexpr int KC = 256, KS = KC / 64, CPR = KC / 8;
#ifndef FT_DB_RC_G
#define FT_DB_RC_G 4
#endif
#ifndef FT_DB_RC_D
#define FT_DB_RC_D 7
#endif
#ifndef FT_DB_DEPTH_O
#define FT_DB_DEPTH_O 4
#endif
constexpr int RC_G = FT_DB_RC_G, RC_D = FT_DB_RC_D, DEPTH_O = FT_DB_DEPTH_O;
constexpr int kCtlBar = 0, kCtlDone = 1, kCtlErr = 2, kCtlTkD = 320;
constexpr int kCtlWords = 1024;
constexpr unsigned kSpinLimit = 1u << 20;   // ~1-2 s per barrier
constexpr int kPollWave = NW - 1;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int V>
struct IC { static constexpr int value = V; };
template <bool V>
struct BC { static constexpr bool value = V; };

template <int J, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (J < N) {
    f(IC<J>{});
    static_for<J + 1, N>(f);
  }
}

struct Args {
  const uint16_t* attn;   // [M, Ko]
  uint16_t* residual;     // [M, H] in / out
  uint16_t* h;            // [M, I] scratch (row stride I)
  const uint16_t* wo;     // packed [H/16][Ko/64][...]
  const uint16_t* wgu;    // packed, gate/up interleaved in 16-row groups, ln2 folded
  const uint16_t* wd;     // packed [H/16][I/64][...]
  float* ws;              // split-K slabs of D (C-fragment layout)
  int* ctl;               // counters, zeroed (kCtlWords)
  long long* stamps;      // optional per-workgroup phase timestamps [G][16] (probe)
  int M, H, Ko, I;
  int sd;                 // D K-splits
  float eps;
};

__device__ __forceinline__ void* uniform_ptr(const void* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(uniform_ptr(base), 0, 0x7fffffff, 0x00020000);
}

// write-through 16-B store / L2-served 16-B load (aux 16 = sc1)
__device__ __forceinline__ void st_wt(void* base, int byte_off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, rsrc(base), byte_off, 0, 16);
}
__device__ __forceinline__ u32x4 ld_wt(const void* base, int byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b128(rsrc(base), byte_off, 0, 16);
}

__device__ __forceinline__ float sq2(uint32_t w, float c) {
  const bf16x2 v = __builtin_bit_cast(bf16x2, w);
  return __builtin_amdgcn_fdot2_f32_bf16(v, v, c, false);
}

__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// probe: wall-clock (100 MHz) stamp k of this workgroup
__device__ __forceinline__ void stamp(long long* st, int k) {
  if (st != nullptr && threadIdx.x == 0) st[blockIdx.x * 16 + k] = wall_clock64();
}

__device__ __forceinline__ void set_err(int* ctl, int code) {
  __hip_atomic_fetch_or(ctl + kCtlErr, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Grid-wide barrier, arrive half: every storing wave has drained (vmcnt(0)) and the
// workgroup passed a barrier; one lane adds (relaxed agent atomic).
__device__ __forceinline__ void grid_arrive(int* ctl) {
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(ctl + kCtlBar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wait half: lane 0 of the poll wave polls relaxed with s_sleep between polls (its
// first poll returns behind the wave's own prefetch: vmcnt is in order).  No acquire fence: every
// byte handed off inside the launch is stored sc1 and loaded sc1 (x staging, slabs,
// residual re-reads), the guide's R1 form without the acquire (cdna_hip_programming.md
// Guideline 16, Rule); the wavefront-scope fence keeps the compiler from hoisting
// those loads above the poll.
__device__ __forceinline__ void grid_wait(int* ctl, int target) {
  if (threadIdx.x == kPollWave * 64) {
    unsigned spins = 0;
    while (__hip_atomic_load(ctl + kCtlBar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        set_err(ctl, 1);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  __syncthreads();
}

// ---------------------------------------------------------------------------
// A wave's weight stream: buffer loads off an SGPR descriptor at its first tile, one
// VGPR offset (lane * 16 B) for every load, tile / k-step in soffset: the ring costs
// no address registers.  aux 2 = nt: decode weights are read once per step.
struct WStream {
  __amdgpu_buffer_rsrc_t r;
  int voff;
  int tile_bytes;   // bytes between adjacent 16-column tiles (K / 64 * 2 KiB)
};

__device__ __forceinline__ WStream wstream(const uint16_t* tile_base, int K, int lane) {
  return WStream{rsrc(tile_base), lane * 16, (K >> 6) * 2048};
}

template <int NT>
__device__ __forceinline__ void ring_load(u32x4 (&r)[KS][NT][2], const WStream& w, int chunk) {
#pragma unroll
  for (int s = 0; s < KS; ++s)
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int so = j * w.tile_bytes + (chunk * KS + s) * 2048;
      r[s][j][0] = __builtin_amdgcn_raw_buffer_load_b128(w.r, w.voff, so, 2);
      r[s][j][1] = __builtin_amdgcn_raw_buffer_load_b128(w.r, w.voff, so + 1024, 2);
    }
}

// x staging: thread tid moves 16-B chunk (tid % 32) of rows tid / 32 + 8 p; the
// per-lane byte offsets are loop-invariant, the chunk's k offset rides in soffset.
// sc1 loads (aux 16): the residual / h rows were written by other workgroups in
// this launch (write-through); these loads stand in for the acquire.
constexpr int RPP = NTH / CPR;   // rows per staging pass (8)

template <int MT>
struct XStream {
  __amdgpu_buffer_rsrc_t r;
  int voff[2 * MT];
};

template <int MT>
__device__ __forceinline__ XStream<MT> xstream(const uint16_t* x, int stride, int M, int tid) {
  XStream<MT> s;
  s.r = rsrc(x);
#pragma unroll
  for (int p = 0; p < 2 * MT; ++p)
    s.voff[p] = (min(tid / CPR + RPP * p, M - 1) * stride + (tid % CPR) * 8) * 2;
  return s;
}

template <int MT>
__device__ __forceinline__ void x_load(u32x4 (&xr)[2 * MT], const XStream<MT>& xs, int k0) {
#pragma unroll
  for (int p = 0; p < 2 * MT; ++p) xr[p] = __builtin_amdgcn_raw_buffer_load_b128(xs.r, xs.voff[p], k0 * 2, 16);
}

template <int MT, bool NORM>
__device__ __forceinline__ void x_store(uint16_t* sx, const u32x4 (&xr)[2 * MT], int tid,
                                        float (&ss)[2 * MT]) {
#pragma unroll
  for (int p = 0; p < 2 * MT; ++p) {
    const int row = tid / CPR + RPP * p, ch = tid % CPR;
    const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
    *reinterpret_cast<u32x4*>(&sx[row * KC + slot * 8]) = xr[p];
    if constexpr (NORM) {
      ss[p] = sq2(xr[p].x, ss[p]);
      ss[p] = sq2(xr[p].y, ss[p]);
      ss[p] = sq2(xr[p].z, ss[p]);
      ss[p] = sq2(xr[p].w, ss[p]);
    }
  }
}

// One phase GEMM over nch 256-deep chunks of x[:, k0 : k0 + 256 nch] for the wave's
// NT column tiles: the ring holds chunks c .. c+RC-1 (its first RC chunks issued by
// the caller, possibly before a grid barrier); each k-step's registers are refilled
// with chunk c+RC right after their MFMAs.  Loop bodies are branch-free (refill /
// next-x flags compile-time, the last RC chunks peeled) so the compiler keeps counted
// vmcnt waits; nch must be a multiple of RC.  Inactive waves (ACTIVE false) stage x
// and meet the barriers only.
template <int MT, int NT, int RC, bool NORM, bool ACTIVE>
__device__ __forceinline__ void run_phase(u32x4 (&ring)[RC][KS][NT][2], f32x4 (&acc)[MT][NT],
                                          float (&ss)[2 * MT], const uint16_t* x, int xstride, int M,
                                          int k0, int nch, const WStream& wp, uint16_t* sxb, int tid,
                                          int l15, int g) {
  const XStream<MT> xs = xstream<MT>(x, xstride, M, tid);
  u32x4 xr[2 * MT];
  x_load<MT>(xr, xs, k0);
  auto chunk = [&](int c, auto slot_tag, auto refill_tag, auto xnext_tag) {
    constexpr int SL = decltype(slot_tag)::value;
    constexpr bool REFILL = decltype(refill_tag)::value;
    constexpr bool XNEXT = decltype(xnext_tag)::value;
    uint16_t* sx = sxb + (c & 1) * (64 * KC);
    // keep the next chunk's x-staging math (the NORM squares) out of this chunk's MFMA
    // section: hoisted there it waits for the x loads just issued, and the in-order
    // vmcnt turns that into a wait for every weight load before them
    __builtin_amdgcn_sched_barrier(0);
    x_store<MT, NORM>(sx, xr, tid, ss);
    if constexpr (XNEXT) x_load<MT>(xr, xs, k0 + (c + 1) * KC);
    __syncthreads();   // chunk c visible; every wave is past chunk c-1's reads of the other buffer
    if constexpr (ACTIVE) {
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          const int row = 16 * i + l15;
          u32x4 xf[2];
#pragma unroll
          for (int hh = 0; hh < 2; ++hh) {
            const int ch = s * 8 + 2 * g + hh;
            const int slot = (ch & ~7) | ((ch & 7) ^ (row & 7));
            xf[hh] = *reinterpret_cast<const u32x4*>(&sx[row * KC + slot * 8]);
          }
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xf[0]),
                                                                __builtin_bit_cast(bf16x8, ring[SL][s][j][0]),
                                                                acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, xf[1]),
                                                                __builtin_bit_cast(bf16x8, ring[SL][s][j][1]),
                                                                acc[i][j], 0, 0, 0);
          }
        }
        if constexpr (REFILL) {
#pragma unroll
          for (int j = 0; j < NT; ++j) {
            const int so = j * wp.tile_bytes + ((c + RC) * KS + s) * 2048;
            ring[SL][s][j][0] = __builtin_amdgcn_raw_buffer_load_b128(wp.r, wp.voff, so, 2);
            ring[SL][s][j][1] = __builtin_amdgcn_raw_buffer_load_b128(wp.r, wp.voff, so + 1024, 2);
          }
        }
        // one k-step at a time: hoisting later k-steps' fragment reads above these
        // MFMAs only adds registers (the chunk is LDS-resident, the MFMAs are not the
        // bottleneck) and spilled the deep-ring kernels
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  auto group = [&](int c0, auto refill_tag, auto last_tag) {
    constexpr bool REFILL = decltype(refill_tag)::value;
    constexpr bool LAST = decltype(last_tag)::value;
    static_for<0, RC>([&](auto jt) {
      constexpr int J = decltype(jt)::value;
      chunk(c0 + J, IC<J>{}, BC<REFILL>{}, BC<!(LAST && J == RC - 1)>{});
    });
  };
  // do-while (nch >= 2 RC, checked by the plan): with a zero-trip path around the loop
  // hipcc kept the prefetched ring in other registers than the loop's and copied it at
  // the loop entry, doubling the ring's registers (spills at RC 4)
  int c = 0;
  do {
    group(c, BC<true>{}, BC<false>{});
    c += RC;
  } while (c + 2 * RC <= nch);
  group(c, BC<false>{}, BC<true>{});
}

// NT x 16 columns x MT*16 rows of bf16 from the C layout (lane (l15, g): rows
// 16 i + 4 g + r, column l15 of tile j) -> row segments through the wave's LDS tile ->
// 16-B write-through stores (rows < M)
template <int MT>
__device__ __forceinline__ void store_tile(const float (&v)[MT][4], uint16_t* tr, uint16_t* dst,
                                           int stride, int col0, int M, int lane) {
  const int l15 = lane & 15, g = lane >> 4;
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) tr[(16 * i + 4 * g + r) * 16 + l15] = f32_to_bf16(v[i][r]);
  lds_drain();
  for (int piece = lane; piece < 32 * MT; piece += 64) {
    const int row = piece >> 1, half = piece & 1;
    if (row < M) {
      const u32x4 d = *reinterpret_cast<const u32x4*>(&tr[row * 16 + half * 8]);
      st_wt(dst, (row * stride + col0 + half * 8) * 2, d);
    }
  }
  lds_drain();   // the tile buffer is reused by the next call
}

// column group / K-slice of workgroup b in phase D: the S slices of a column group go
// to blocks with equal b % 8 (one XCD under round-robin placement; speed only)
__device__ __forceinline__ void item_of(int b, int G, int S, int& cg, int& split) {
  if ((G & 7) == 0 && ((G >> 3) % S) == 0) {
    const int xcd = b & 7, idx = b >> 3;
    cg = xcd + 8 * (idx / S);
    split = idx % S;
  } else {
    cg = b / S;
    split = b % S;
  }
}

// Phase O, whole K per workgroup: its 16-column tile of Wo (128 KiB) against all of
// attn; the waves take contiguous K ranges and stream their x fragments straight from
// L2 (no x byte is shared between waves, so LDS staging would buy nothing), then meet
// in LDS.  No split-K seam: the first version split K four ways and its ticket ->
// slab -> residual chain cost ~10 us per layer (profiles/decode_block_r06.log).
template <int MT>
__device__ __forceinline__ void o_phase(f32x4 (&acc)[MT], const Args& a, int tile, int wave, int lane) {
  const int l15 = lane & 15, g = lane >> 4;
  const int KW = (a.Ko >> 6) / NW;    // k-steps per wave (a multiple of DEPTH_O)
  const int ks0 = wave * KW;
  const __amdgpu_buffer_rsrc_t wr = rsrc(a.wo + (size_t)tile * (a.Ko >> 6) * 1024);
  const __amdgpu_buffer_rsrc_t xr = rsrc(a.attn);
  int xoff[MT];
#pragma unroll
  for (int i = 0; i < MT; ++i) xoff[i] = (min(16 * i + l15, a.M - 1) * a.Ko + 16 * g) * 2;
  struct St {
    u32x4 w[2];
    u32x4 x[MT][2];
  };
  auto load = [&](St& st, int ks) {
    st.w[0] = __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 16, ks * 2048, 2);
    st.w[1] = __builtin_amdgcn_raw_buffer_load_b128(wr, lane * 16, ks * 2048 + 1024, 2);
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      st.x[i][0] = __builtin_amdgcn_raw_buffer_load_b128(xr, xoff[i], ks * 128, 0);
      st.x[i][1] = __builtin_amdgcn_raw_buffer_load_b128(xr, xoff[i], ks * 128 + 16, 0);
    }
  };
  auto mma = [&](const St& st) {
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, st.x[i][0]),
                                                       __builtin_bit_cast(bf16x8, st.w[0]), acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, st.x[i][1]),
                                                       __builtin_bit_cast(bf16x8, st.w[1]), acc[i], 0, 0, 0);
    }
  };
  St ring[DEPTH_O];
#pragma unroll
  for (int d = 0; d < DEPTH_O; ++d) load(ring[d], ks0 + d);
  int s = 0;
  for (; s + DEPTH_O < KW; s += DEPTH_O) {
#pragma unroll
    for (int d = 0; d < DEPTH_O; ++d) {
      mma(ring[d]);
      load(ring[d], ks0 + s + DEPTH_O + d);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH_O; ++d) mma(ring[d]);
}

// gate/up pairs of workgroup b: `base` each, one more for half the workgroups when the
// pairs do not divide evenly (every other group of 8 consecutive blocks: each XCD gets
// as many of the longer workgroups under round-robin placement; speed only)
__device__ __forceinline__ void gu_pairs(int b, int P, int G, int& np, int& p0) {
  const int base = P / G;
  if (P % G == 0) {
    np = base;
    p0 = b * base;
  } else {   // P % G == G / 2 (checked by the plan)
    np = base + (((b >> 3) & 1) == 0 ? 1 : 0);
    p0 = b * base + 8 * (b >> 4) + min(b & 15, 8);
  }
}

template <int MT, bool PF>
__global__ __launch_bounds__(NTH, 1) void decode_block_kernel(Args a) {
  // ONE shared array (a second __shared__ object can make hipcc drain vmcnt before
  // every ds_read: cdna_hip_programming.md §5 trap (a))
  //   [0, 64K)    x double buffer [2][64 rows][KC] bf16; also the O-phase wave partials
  //               [NW][MT][64][f32x4]
  //   [64K, 72K)  per-wave bf16 store tiles [NW][64][16]
  //   [72K, +256) row sums of squares; then flags
  __shared__ __attribute__((aligned(16))) uint8_t smem[73728 + 256 + 64];
  uint16_t* sxb = reinterpret_cast<uint16_t*>(smem);
  f32x4* sx4 = reinterpret_cast<f32x4*>(smem);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform
  const int l15 = lane & 15, g = lane >> 4;
  uint16_t* tr = reinterpret_cast<uint16_t*>(smem + 65536) + wave * 1024;
  float* s_ss = reinterpret_cast<float*>(smem + 73728);
  int* sflag = reinterpret_cast<int*>(smem + 73728 + 256);
  const int b = blockIdx.x, G = gridDim.x;
  const int M = a.M;

  // old residual of this workgroup's 16 columns (phase O's epilogue), loaded now so
  // its latency hides under the O stream: wave i holds m-tile i
  float res_old[4];
  if (wave < MT) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = min(16 * wave + 4 * g + r, M - 1);
      res_old[r] = bf16_to_f32(a.residual[(size_t)m * a.H + b * 16 + l15]);
    }
  }

  // gate_up: whole pairs per workgroup, a wave holds one pair (gate tile + up tile)
  int np, p0;
  gu_pairs(b, a.I / 16, G, np, p0);
  const bool gact = wave < np;
  const int pw = min(p0 + wave, a.I / 16 - 1);   // this wave's pair
  const WStream wpg = wstream(a.wgu + (size_t)(2 * pw) * (a.H >> 6) * 1024, a.H, lane);
  u32x4 ring_g[RC_G][KS][2][2];
  auto prefetch_g = [&]() {
    if (gact) {
#pragma unroll
      for (int c = 0; c < RC_G; ++c) ring_load<2>(ring_g[c], wpg, c);
    }
  };

  stamp(a.stamps, 0);
  // ------------------------------------------------------------ phase O
  {
    f32x4 acc[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    o_phase<MT>(acc, a, b, wave, lane);
    stamp(a.stamps, 1);
#pragma unroll
    for (int i = 0; i < MT; ++i) sx4[(wave * MT + i) * 64 + lane] = acc[i];
    __syncthreads();
    if (wave < MT) {   // wave i: m-tile i of the workgroup's 16 residual columns
      const int i = wave;
      f32x4 sum = sx4[i * 64 + lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) sum += sx4[(w * MT + i) * 64 + lane];
#pragma unroll
      for (int r = 0; r < 4; ++r) tr[(4 * g + r) * 16 + l15] = f32_to_bf16(res_old[r] + sum[r]);
      lds_drain();
      if (lane < 32) {
        const int row = 16 * i + (lane >> 1), half = lane & 1;
        if (row < M)
          st_wt(a.residual, (row * a.H + b * 16 + half * 8) * 2,
                *reinterpret_cast<const u32x4*>(&tr[(lane >> 1) * 16 + half * 8]));
      }
      drain();
    }
  }
  __syncthreads();
  grid_arrive(a.ctl);
  // ONE definition of the ring (two made hipcc copy it through phis).  PF: in flight
  // while the barrier resolves; else issued after it, so hand-offs do not queue
  // behind a saturated weight stream
  if constexpr (PF) prefetch_g();
  stamp(a.stamps, 2);
  grid_wait(a.ctl, G);
  if constexpr (!PF) prefetch_g();
  stamp(a.stamps, 3);

  // ------------------------------------------------------------ phase GU
  float ss[2 * MT];
#pragma unroll
  for (int p = 0; p < 2 * MT; ++p) ss[p] = 0.f;
  {
    f32x4 acc[MT][2];
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (gact)
      run_phase<MT, 2, RC_G, true, true>(ring_g, acc, ss, a.residual, a.H, M, 0, a.H / KC, wpg, sxb, tid,
                                         l15, g);
    else
      run_phase<MT, 2, RC_G, true, false>(ring_g, acc, ss, a.residual, a.H, M, 0, a.H / KC, wpg, sxb,
                                          tid, l15, g);
    stamp(a.stamps, 4);
    // rows' sums of squares: thread tid holds rows tid/32 + 8 p over its 16-B column
    // chunks of every K chunk -> half-wave sums
#pragma unroll
    for (int p = 0; p < 2 * MT; ++p) {
      const float v = group_sum<32>(ss[p]);
      if ((lane & 31) == 0) s_ss[tid / CPR + RPP * p] = v;
    }
    __syncthreads();
    if (gact) {   // h = silu(g) * u of the RMS-scaled pair, written through
      const float inv_h = 1.f / (float)a.H;
      float hv[MT][4];
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float rs = rsqrtf(s_ss[16 * i + 4 * g + r] * inv_h + a.eps);
          const float gt = acc[i][0][r] * rs, up = acc[i][1][r] * rs;
          hv[i][r] = gt / (1.f + __expf(-gt)) * up;
        }
      store_tile<MT>(hv, tr, a.h, a.I, pw * 16, M, lane);
      drain();
    }
  }
  __syncthreads();
  grid_arrive(a.ctl);
  stamp(a.stamps, 5);

  // ------------------------------------------------------------ phase D
  int cg, split;
  item_of(b, G, a.sd, cg, split);
  const int kslice = a.I / a.sd;
  const WStream wpd = wstream(a.wd + ((size_t)(cg * 4 + wave) * (a.I >> 6) + (kslice >> 6) * split) * 1024,
                              a.I, lane);
  u32x4 ring_d[RC_D][KS][1][2];
  if constexpr (PF) {
#pragma unroll
    for (int c = 0; c < RC_D; ++c) ring_load<1>(ring_d[c], wpd, c);
  }
  grid_wait(a.ctl, 2 * G);
  if constexpr (!PF) {
#pragma unroll
    for (int c = 0; c < RC_D; ++c) ring_load<1>(ring_d[c], wpd, c);
  }
  stamp(a.stamps, 6);
  f32x4 acc[MT][1];
#pragma unroll
  for (int i = 0; i < MT; ++i) acc[i][0] = f32x4{0.f, 0.f, 0.f, 0.f};
  run_phase<MT, 1, RC_D, false, true>(ring_d, acc, ss, a.h, a.I, M, split * kslice, kslice / KC, wpd, sxb,
                                      tid, l15, g);
  stamp(a.stamps, 7);

  // split-K seam: every K slice publishes its 64-column slab (write-through), takes a
  // ticket; the last one sums the slabs in slice order (deterministic) onto the residual
  const int S = a.sd;
  float* slab0 = a.ws + (size_t)cg * S * NW * MT * 256;   // [S][4 tiles][MT][64 lanes][4]
  bool last = true;
  if (S > 1) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
      st_wt(slab0, (((split * NW + wave) * MT + i) * 64 + lane) * 16, __builtin_bit_cast(u32x4, acc[i][0]));
    drain();
    __syncthreads();
    if (tid == 0)
      *sflag = __hip_atomic_fetch_add(a.ctl + kCtlTkD + cg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    last = *sflag == S - 1;
  }
  if (last) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // keep the loads below the ticket
    const int col0 = cg * 64 + wave * 16;
    float old[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = min(16 * i + 4 * g + r, M - 1);
        // sc1: phase O of another workgroup wrote these columns in this launch
        old[i][r] = bf16_to_f32((uint16_t)__hip_atomic_load(
            reinterpret_cast<const unsigned short*>(a.residual) + (size_t)m * a.H + col0 + l15,
            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      }
    f32x4 tot[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) tot[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < S; ++sp) {
      f32x4 part[MT];
#pragma unroll
      for (int i = 0; i < MT; ++i)
        part[i] = __builtin_bit_cast(f32x4, ld_wt(slab0, (((sp * NW + wave) * MT + i) * 64 + lane) * 16));
#pragma unroll
      for (int i = 0; i < MT; ++i) tot[i] += sp == split ? acc[i][0] : part[i];
    }
    float v[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[i][r] = old[i][r] + tot[i][r];
    store_tile<MT>(v, tr, a.residual, a.H, col0, M, lane);
    if (tid == 0 && S > 1)
      __hip_atomic_store(a.ctl + kCtlTkD + cg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    drain();
  }
  stamp(a.stamps, 8);
  __syncthreads();
  // last finisher re-arms the grid counter (every workgroup is past its last poll)
  if (tid == 0) {
    const int d = __hip_atomic_fetch_add(a.ctl + kCtlDone, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (d == G - 1) {
      __hip_atomic_store(a.ctl + kCtlBar, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.ctl + kCtlDone, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace dblk
}  // namespace ft

static int ft_cu_count() {
  static int n = -1;
  if (n < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 0;
  }
  return n;
}

// Geometry for (H, Ko, I) on this device: 0 and (so, sd, pairs, grid) when the block
// kernel covers the shape, else a negative code (the caller runs the unfused layer).
//   O: one 16-column tile of Wo per workgroup (H / 16 == grid), each wave a multiple
//      of DEPTH_O K steps;  GU: whole gate/up pairs, <= NW per workgroup, the remainder
//      0 or half the grid;  D: 64-column groups x sd K slices == grid, RC_D | chunks.
extern "C" int ft_decode_block_plan(int H, int Ko, int I, int* so, int* sd, int* tpw, int* grid) {
  using namespace ft::dblk;
  const int G = ft_cu_count();
  if (G <= 0 || G % 16) return -1;
  if (H % (KC * RC_G) || Ko % (64 * NW * DEPTH_O) || I % 64) return -2;
  if (H / 16 != G) return -3;
  const int cgs = H / 64;
  if (G % cgs) return -3;
  const int s_d = G / cgs;
  if (I % (s_d * KC * RC_D) || I / s_d < 2 * KC * RC_D || H < 2 * KC * RC_G) return -4;
  const int P = I / 16;
  if (P % G != 0 && P % G != G / 2) return -5;
  const int np = P / G + (P % G ? 1 : 0);
  if (np < 1 || np > NW) return -6;
  *so = 1;
  *sd = s_d;
  *tpw = np;
  *grid = G;
  return 0;
}

extern "C" size_t ft_decode_block_ws_floats(int H, int M) {
  const int mt = (M + 15) / 16;
  const int G = ft_cu_count();
  const int cgs = H / 64;
  const int s = G > 0 && cgs > 0 ? G / cgs : 1;
  return (size_t)cgs * s * ft::dblk::NW * mt * 256;
}

extern "C" int ft_decode_block(const void* attn, int attn_stride, void* residual, int res_stride,
                               void* h, int h_stride, const void* wo, const void* wgu, const void* wd,
                               float* ws, long ws_floats, float* xg, long xg_floats, int* ctl,
                               long long* stamps, int M, int H, int Ko, int I, float eps,
                               hipStream_t stream) {
  (void)xg;
  (void)xg_floats;
  if (M <= 0) return 0;
  if (M > 64) return -1;
  int so = 0, sd = 0, tpw = 0, G = 0;
  const int rc = ft_decode_block_plan(H, Ko, I, &so, &sd, &tpw, &G);
  if (rc) return rc - 10;
  if (attn_stride != Ko || res_stride != H || h_stride != I) return -20;
  if ((size_t)ws_floats < ft_decode_block_ws_floats(H, M)) return -21;
  ft::dblk::Args a{(const uint16_t*)attn, (uint16_t*)residual, (uint16_t*)h, (const uint16_t*)wo,
                   (const uint16_t*)wgu, (const uint16_t*)wd, ws, ctl, stamps, M, H, Ko, I, sd, eps};
  dim3 grid(G), block(ft::dblk::NTH);
  static const bool pf = getenv("FT_DB_PREFETCH") == nullptr || getenv("FT_DB_PREFETCH")[0] != '0';
#define FT_DB(MT_)                                                                             \
  if (pf) hipLaunchKernelGGL((ft::dblk::decode_block_kernel<MT_, true>), grid, block, 0, stream, a); \
  else hipLaunchKernelGGL((ft::dblk::decode_block_kernel<MT_, false>), grid, block, 0, stream, a);
  switch ((M + 15) / 16) {
    case 1: FT_DB(1) break;
    case 2: FT_DB(2) break;
    case 3: FT_DB(3) break;
    default: FT_DB(4) break;
  }
#undef FT_DB
  return static_cast<int>(hipGetLastError());
}

extern "C" int ft_decode_block_ctl_words() { return ft::dblk::kCtlWords; }
