// PyTorch bindings for the gfx950 kernels in csrc/kernels (extension `_C`).
//
// Every op: validates dtype/device/shape on the host (a mis-shaped launch of a
// hand-written kernel can fault the GPU, so we refuse it here), then calls the
// extern "C" launcher on the caller's current HIP stream, so ops are
// hipGraph-capturable (no allocation, no synchronisation).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int ft_rmsnorm(void* out, const void* x, const void* w, int rows, int hidden, int x_stride,
               int out_stride, float eps, hipStream_t stream);
int ft_fused_add_rmsnorm(void* out, const void* x, void* residual, const void* w, int rows,
                         int hidden, int x_stride, int out_stride, float eps, hipStream_t stream);
int ft_silu_mul(void* out, const void* gu, int rows, int inter, int il, hipStream_t stream);
int ft_rope_kv_write(void* qkv, int qkv_stride, const int* positions, const float* cos_sin,
                     const int* slot_mapping, void* k_cache, void* v_cache, int tokens, int nq,
                     int nkv, int head_dim, int block_size, int cos_rows, int num_slots, int kv8,
                     hipStream_t stream);
int ft_decode_waves();
int ft_decode_max_batch();
int ft_paged_decode_attention(void* out, int out_stride, float* tmp_out, float* tmp_ml,
                              const void* q, int q_stride, const void* k_cache,
                              const void* v_cache, const int* block_tables, int bt_stride,
                              const int* seq_lens, int batch, int nq, int nkv, int head_dim,
                              int block_size, float scale, int* counters, int piece,
                              int slot_cap, int num_blocks, int kv8, hipStream_t stream);
int ft_prefill_tile_tokens(int nq, int nkv);
int ft_prefill_attention(void* out, int out_stride, const void* q, int q_stride,
                         const void* k_cache, const void* v_cache, const int* block_tables,
                         int bt_stride, const int* seq_lens, const int* q_start_loc,
                         const int* tile_info, int num_tiles, int nq, int nkv, int head_dim,
                         int block_size, float scale, float* part_o, float* part_ml,
                         const int* combine, int num_combine, int invariant, int num_blocks,
                         int kv8, hipStream_t stream);
int ft_sample(int* out_tokens, const void* logits, int logits_is_bf16, long logit_stride,
              int batch, int vocab, const float* temperature, const float* top_p,
              const int* top_k, const long long* seeds, const int* steps,
              const uint32_t* allow_mask, int mask_words, float* ws, hipStream_t stream);
int ft_sample_ws_floats();
int ft_kv_block_copy(void* k_cache, void* v_cache, const int* src_dst, int num_pairs,
                     long block_elems, int num_blocks, hipStream_t stream);
int ft_w4_gemm(const void* x, int x_stride, int M, const uint32_t* wq, const void* sz, int N, int K,
               float* ws, void* out, int out_stride, int splits, int nt, hipStream_t stream);
int ft_w4_dequant(const uint32_t* wq, const void* sz, void* out, int N, int K, hipStream_t stream);
int ft_w4_gemm_xr(const void* x, int x_stride, int M, const uint32_t* wq, const void* sz, int N, int K,
                  float* ws, void* out, int out_stride, int splits, int nt, int silu,
                  hipStream_t stream);
int ft_w4_gemm_mh(const void* x, int x_stride, int M, const uint32_t* wq, const void* sz, int N, int K,
                  float* ws, void* out, int out_stride, int splits, int ring, int silu,
                  hipStream_t stream);
int ft_kv_swap(const uint64_t* ptrs_dev, int ncache, const int* ids_dev, int n, void* staging,
               long block_elems, int to_staging, int num_blocks, hipStream_t stream);
int ft_skinny_gemm_xc(const void* x, int x_stride, int M, const void* w, int N, int K, float* ws,
                      void* out, int out_stride, int splits, int nt, hipStream_t stream);
int ft_embed_rmsnorm(void* out, void* residual, const int* ids, const void* table, const void* w,
                     int rows, int hidden, int vocab, float eps, hipStream_t stream);
size_t ft_ar_header_bytes();
void ft_ar_set_max_blocks(int n);
int ft_ar_alloc(size_t bytes, void** ptr);
int ft_ar_free(void* ptr);
int ft_ar_ipc_handle(void* ptr, char* out64);
int ft_ar_ipc_open(const char* in64, void** ptr);
int ft_ar_ipc_close(void* ptr);
int ft_ar_read_error(void* mine, int* err);
int ft_ar_add_rmsnorm(void* out, int out_stride, void* residual, const void* weight, float eps,
                      const float* ws, int splits, const void* x, int x_stride, long rows, long hidden,
                      const uint64_t* peers_dev, int rank, int world, size_t max_bytes,
                      unsigned spin_budget, hipStream_t stream);
int ft_ar_allreduce(void* out, const void* x, long n, const uint64_t* peers_dev, int rank, int world,
                    size_t max_bytes, unsigned spin_budget, int two_shot, hipStream_t stream);
int ft_ar_allgather(void* out, const void* x, long rows, long row_elems, const uint64_t* peers_dev,
                    int rank, int world, size_t max_bytes, unsigned spin_budget, hipStream_t stream);
int ft_ar_export_error(int* dst, const uint64_t* peers_dev, int world, hipStream_t stream);
int ft_skinny_gemm_pk(const void* x, int x_stride, int M, const void* wpk, int N, int K, float* ws,
                      void* out, int out_stride, int splits, int nt, hipStream_t stream);
int ft_skinny_gemm_xr(const void* x, int x_stride, int M, const void* w, int N, int K, float* ws,
                      void* out, int out_stride, int splits, int nt, int epi, int nw,
                      hipStream_t stream);
int ft_packed_gemm(const void* x, int x_stride, int M, const void* wpk, int N, int K, int splits,
                   int epi, int cfg, void* out, int out_stride, float* ws, hipStream_t stream);
int ft_pkr_gemm(const void* x, int x_stride, int M, const void* wpk, int N, int K, float* ws,
                void* out, int out_stride, void* residual, int res_stride, int* tickets,
                int splits, int nt, int depth, int epi, int norm, int wn, float eps,
                hipStream_t stream);
int ft_decode_block_plan(int H, int Ko, int I, int* so, int* sd, int* tpw, int* grid);
size_t ft_decode_block_ws_floats(int H, int M);
int ft_decode_block_ctl_words();
int ft_decode_block(const void* attn, int attn_stride, void* residual, int res_stride, void* h,
                    int h_stride, const void* wo, const void* wgu, const void* wd, float* ws,
                    long ws_floats, float* xg, long xg_floats, int* ctl, long long* stamps, int M,
                    int H, int Ko, int I, float eps, hipStream_t stream);
int ft_row_rmsnorm(const void* x, int x_stride, const float* ws, int splits, void* out,
                   int out_stride, void* residual, const void* w, int rows, int hidden, float eps,
                   hipStream_t stream);
int ft_slab_silu(const float* ws, int splits, int rows, int inter, void* out, int out_stride, int il,
                 hipStream_t stream);
int ft_slab_store(const float* ws, int splits, int rows, int cols, void* out, int out_stride,
                  hipStream_t stream);
int ft_slab_rope_kv(const float* ws, int splits, int rows, int cols, void* q_out, int q_stride,
                    const int* positions, const float* cos_sin, const int* slot_mapping,
                    void* k_cache, void* v_cache, int nq, int nkv, int head_dim, int block_size,
                    const void* residual, int hidden, float eps, int cos_rows, int num_slots,
                    int kv8, hipStream_t stream);
}

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_dev(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}
void check_bf16(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, name, " must be bfloat16");
}
void check_i32(const at::Tensor& t, const char* name) {
  check_dev(t, name);
  TORCH_CHECK(t.scalar_type() == at::kInt, name, " must be int32");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_rc(int rc, const char* op) { TORCH_CHECK(rc == 0, op, " launch failed, code ", rc); }
void check_rows(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2, name, " must be 2-D");
  TORCH_CHECK(t.stride(1) == 1, name, " rows must be contiguous");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-B aligned");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
}

// KV caches: K [blocks, nkv, block_size, D] (token rows), V [blocks, nkv, D,
// block_size] (transposed, rope_kv.hip); a mismatched V layout would be read as
// garbage by the attention kernels, so every op touching the caches checks both
// returns true for fp8 (e4m3) caches, false for bf16
bool check_kv_caches(const at::Tensor& k_cache, const at::Tensor& v_cache, int64_t nkv,
                     int64_t head_dim) {
  check_dev(k_cache, "k_cache");
  check_dev(v_cache, "v_cache");
  const bool kv8 = k_cache.scalar_type() == at::kFloat8_e4m3fn;
  TORCH_CHECK(kv8 || k_cache.scalar_type() == at::kBFloat16, "KV caches must be bfloat16 or float8_e4m3fn");
  TORCH_CHECK(v_cache.scalar_type() == k_cache.scalar_type(), "K and V caches must share a dtype");
  TORCH_CHECK(!kv8 || k_cache.size(2) >= 16, "fp8 KV caches need block_size >= 16");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous(), "KV caches must be contiguous");
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == nkv && k_cache.size(3) == head_dim,
              "k_cache must be [blocks, nkv, block_size, head_dim]");
  TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(0) == k_cache.size(0) && v_cache.size(1) == nkv &&
                  v_cache.size(2) == head_dim && v_cache.size(3) == k_cache.size(2),
              "v_cache must be [blocks, nkv, head_dim, block_size] (transposed V blocks)");
  return kv8;
}

void rmsnorm(at::Tensor out, at::Tensor x, at::Tensor w, double eps) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  check_bf16(w, "weight");
  check_rows(out, "out");
  check_rows(x, "x");
  TORCH_CHECK(w.is_contiguous() && w.numel() == x.size(1), "weight shape");
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == x.size(1), "out shape");
  check_rc(ft_rmsnorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), (int)x.size(0), (int)x.size(1),
                      (int)x.stride(0), (int)out.stride(0), (float)eps, cur_stream()),
           "rmsnorm");
}

void fused_add_rmsnorm(at::Tensor out, at::Tensor x, at::Tensor residual, at::Tensor w,
                       double eps) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  check_bf16(residual, "residual");
  check_bf16(w, "weight");
  check_rows(out, "out");
  check_rows(x, "x");
  TORCH_CHECK(residual.is_contiguous() && residual.sizes() == x.sizes(), "residual shape");
  TORCH_CHECK(w.is_contiguous() && w.numel() == x.size(1), "weight shape");
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == x.size(1), "out shape");
  check_rc(ft_fused_add_rmsnorm(out.data_ptr(), x.data_ptr(), residual.data_ptr(), w.data_ptr(),
                                (int)x.size(0), (int)x.size(1), (int)x.stride(0),
                                (int)out.stride(0), (float)eps, cur_stream()),
           "fused_add_rmsnorm");
}

void silu_mul(at::Tensor out, at::Tensor gu, bool il) {
  check_bf16(out, "out");
  check_bf16(gu, "gate_up");
  TORCH_CHECK(gu.is_contiguous() && out.is_contiguous(), "contiguous tensors required");
  TORCH_CHECK(gu.dim() == 2 && out.dim() == 2 && gu.size(0) == out.size(0) &&
                  gu.size(1) == 2 * out.size(1),
              "silu_mul shapes");
  TORCH_CHECK(!il || out.size(1) % 16 == 0, "interleaved silu_mul: inter % 16");
  check_rc(ft_silu_mul(out.data_ptr(), gu.data_ptr(), (int)out.size(0), (int)out.size(1), il ? 1 : 0,
                       cur_stream()),
           "silu_mul");
}

void rope_kv_write(at::Tensor qkv, at::Tensor positions, at::Tensor cos_sin,
                   at::Tensor slot_mapping, at::Tensor k_cache, at::Tensor v_cache, int64_t nq,
                   int64_t nkv, int64_t head_dim) {
  check_bf16(qkv, "qkv");
  check_rows(qkv, "qkv");
  check_i32(positions, "positions");
  check_i32(slot_mapping, "slot_mapping");
  check_dev(cos_sin, "cos_sin");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.is_contiguous() &&
                  cos_sin.size(1) == head_dim,
              "cos_sin must be fp32 [max_pos, head_dim]");
  const bool kv8 = check_kv_caches(k_cache, v_cache, nkv, head_dim);
  TORCH_CHECK(qkv.size(1) >= (nq + 2 * nkv) * head_dim, "qkv width");
  const int tokens = (int)qkv.size(0);
  TORCH_CHECK(positions.numel() >= tokens && slot_mapping.numel() >= tokens, "metadata length");
  check_rc(ft_rope_kv_write(qkv.data_ptr(), (int)qkv.stride(0), positions.data_ptr<int>(),
                            cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int>(),
                            k_cache.data_ptr(), v_cache.data_ptr(), tokens, (int)nq, (int)nkv,
                            (int)head_dim, (int)k_cache.size(2), (int)cos_sin.size(0),
                            (int)(k_cache.size(0) * k_cache.size(2)), kv8 ? 1 : 0, cur_stream()),
           "rope_kv_write");
}

void paged_decode_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                            at::Tensor block_tables, at::Tensor seq_lens, at::Tensor tmp_out,
                            at::Tensor tmp_ml, int64_t nq, int64_t nkv, int64_t head_dim,
                            double scale, c10::optional<at::Tensor> counters, int64_t piece) {
  check_bf16(out, "out");
  check_bf16(q, "q");
  check_rows(out, "out");
  check_rows(q, "q");
  const bool kv8 = check_kv_caches(k_cache, v_cache, nkv, head_dim);
  check_i32(block_tables, "block_tables");
  check_i32(seq_lens, "seq_lens");
  const int batch = (int)q.size(0);
  TORCH_CHECK(out.size(0) >= batch && seq_lens.numel() >= batch && block_tables.size(0) >= batch,
              "batch sizes");
  TORCH_CHECK(batch <= ft_decode_max_batch(), "decode batch above ", ft_decode_max_batch());
  TORCH_CHECK(nq % nkv == 0 && nq / nkv <= 16, "GQA group must be <= 16");
  // partial slots: one per (sequence, kv head) + one per wave of the grid
  const int64_t slots = (int64_t)batch * nkv + ft_decode_waves();
  TORCH_CHECK(tmp_out.scalar_type() == at::kFloat && tmp_ml.scalar_type() == at::kFloat,
              "tmp buffers fp32");
  TORCH_CHECK(tmp_out.numel() >= slots * (nq / nkv) * head_dim &&
                  tmp_ml.numel() >= slots * (nq / nkv) * 2,
              "decode workspace too small (ops.decode_workspace)");
  int* cnt = nullptr;
  if (counters.has_value()) {  // fused combine: zeroed int32 [>= batch * nkv], left zeroed
    check_i32(*counters, "counters");
    TORCH_CHECK(counters->numel() >= (int64_t)batch * nkv, "decode counters too small");
    cnt = counters->data_ptr<int>();
  }
  const int64_t slot_cap = std::min(tmp_out.numel() / ((nq / nkv) * head_dim), tmp_ml.numel() / ((nq / nkv) * 2));
  if (piece > 0) {  // batch-invariant pieces: one slot per piece of the longest possible segment
    TORCH_CHECK(cnt != nullptr, "piece mode merges in-launch: counters required");
    const int64_t max_tiles = (block_tables.size(1) * k_cache.size(2) + 15) / 16;
    TORCH_CHECK(slot_cap >= (int64_t)batch * nkv * ((max_tiles + piece - 1) / piece),
                "decode workspace too small for piece mode (ops.decode_workspace pieces=)");
  }
  check_rc(ft_paged_decode_attention(out.data_ptr(), (int)out.stride(0), tmp_out.data_ptr<float>(),
                                     tmp_ml.data_ptr<float>(), q.data_ptr(), (int)q.stride(0),
                                     k_cache.data_ptr(), v_cache.data_ptr(),
                                     block_tables.data_ptr<int>(), (int)block_tables.stride(0),
                                     seq_lens.data_ptr<int>(), batch, (int)nq, (int)nkv,
                                     (int)head_dim, (int)k_cache.size(2), (float)scale, cnt,
                                     (int)piece, (int)std::min<int64_t>(slot_cap, INT32_MAX),
                                     (int)k_cache.size(0), kv8 ? 1 : 0,
                                     cur_stream()),
           "paged_decode_attention");
}

void prefill_attention(at::Tensor out, at::Tensor q, at::Tensor k_cache, at::Tensor v_cache,
                       at::Tensor block_tables, at::Tensor seq_lens, at::Tensor q_start_loc,
                       at::Tensor tile_info, int64_t num_tiles, int64_t nq, int64_t nkv,
                       int64_t head_dim, double scale, c10::optional<at::Tensor> part_o,
                       c10::optional<at::Tensor> part_ml, c10::optional<at::Tensor> combine,
                       int64_t num_combine, int64_t num_partials, bool invariant) {
  check_bf16(out, "out");
  check_bf16(q, "q");
  check_rows(out, "out");
  check_rows(q, "q");
  const bool kv8 = check_kv_caches(k_cache, v_cache, nkv, head_dim);
  check_i32(block_tables, "block_tables");
  check_i32(seq_lens, "seq_lens");
  check_i32(q_start_loc, "q_start_loc");
  check_i32(tile_info, "tile_info");
  // the prefill kernel stages a sequence's block-table row in LDS (4096 entries)
  TORCH_CHECK(block_tables.size(1) <= 4096, "prefill: at most 4096 KV blocks per sequence");
  // work items: (sequence, first query token, KV tile range, partial slot)
  TORCH_CHECK(tile_info.numel() >= 4 * num_tiles, "tile_info too small");
  float* po = nullptr;
  float* pml = nullptr;
  const int* cb = nullptr;
  if (num_partials > 0 || num_combine > 0) {
    TORCH_CHECK(part_o.has_value() && part_ml.has_value() && combine.has_value(),
                "split-KV prefill needs part_o, part_ml and combine");
    TORCH_CHECK(part_o->scalar_type() == at::kFloat && part_ml->scalar_type() == at::kFloat,
                "partials fp32");
    check_dev(*part_o, "part_o");
    check_dev(*part_ml, "part_ml");
    check_i32(*combine, "combine");
    // partial slots hold 256 rows (token x GQA head) of D floats per kv head
    TORCH_CHECK(part_o->numel() >= num_partials * nkv * 256 * head_dim, "part_o too small");
    TORCH_CHECK(part_ml->numel() >= num_partials * nkv * 256 * 2, "part_ml too small");
    TORCH_CHECK(combine->numel() >= 4 * num_combine, "combine too small");
    po = part_o->data_ptr<float>();
    pml = part_ml->data_ptr<float>();
    cb = combine->data_ptr<int>();
  }
  check_rc(ft_prefill_attention(out.data_ptr(), (int)out.stride(0), q.data_ptr(),
                                (int)q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                                block_tables.data_ptr<int>(), (int)block_tables.stride(0),
                                seq_lens.data_ptr<int>(), q_start_loc.data_ptr<int>(),
                                tile_info.data_ptr<int>(), (int)num_tiles, (int)nq, (int)nkv,
                                (int)head_dim, (int)k_cache.size(2), (float)scale, po, pml, cb,
                                (int)num_combine, (int)invariant, (int)k_cache.size(0), kv8 ? 1 : 0,
                                cur_stream()),
           "prefill_attention");
}

void sample(at::Tensor out_tokens, at::Tensor logits, at::Tensor temperature, at::Tensor top_p,
            at::Tensor top_k, at::Tensor seeds, at::Tensor steps, c10::optional<at::Tensor> mask) {
  check_i32(out_tokens, "out_tokens");
  check_dev(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V] with contiguous rows");
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(is_bf16 || logits.scalar_type() == at::kFloat, "logits fp32 or bf16");
  const int batch = (int)logits.size(0), vocab = (int)logits.size(1);
  TORCH_CHECK(out_tokens.numel() >= batch, "out_tokens too small");
  TORCH_CHECK(temperature.scalar_type() == at::kFloat && top_p.scalar_type() == at::kFloat,
              "temperature/top_p fp32");
  check_i32(top_k, "top_k");
  check_i32(steps, "steps");
  TORCH_CHECK(seeds.scalar_type() == at::kLong && seeds.is_cuda(), "seeds int64");
  TORCH_CHECK(temperature.numel() >= batch && top_p.numel() >= batch && top_k.numel() >= batch &&
                  seeds.numel() >= batch && steps.numel() >= batch,
              "sampling param length");
  const uint32_t* mp = nullptr;
  int words = 0;
  if (mask.has_value() && mask->defined()) {
    check_i32(*mask, "mask");
    words = (int)mask->size(1);
    TORCH_CHECK(mask->size(0) >= batch && words * 32 >= vocab, "mask shape");
    mp = reinterpret_cast<const uint32_t*>(mask->data_ptr<int>());
  }
  // per-row scratch of the multi-workgroup sampler (stream-ordered: safe to reuse
  // from the caching allocator, graph-capturable); FT_SAMPLER_ONE_WG=1 keeps the
  // single-workgroup kernel for every row
  static const bool one_wg = [] {
    const char* e = getenv("FT_SAMPLER_ONE_WG");
    return e && e[0] == '1';
  }();
  at::Tensor ws;
  if (!one_wg) ws = at::empty({(int64_t)batch * ft_sample_ws_floats()}, logits.options().dtype(at::kFloat));
  check_rc(ft_sample(out_tokens.data_ptr<int>(), logits.data_ptr(), is_bf16 ? 1 : 0,
                     (long)logits.stride(0), batch, vocab, temperature.data_ptr<float>(),
                     top_p.data_ptr<float>(), top_k.data_ptr<int>(),
                     reinterpret_cast<const long long*>(seeds.data_ptr<int64_t>()),
                     steps.data_ptr<int>(), mp, words, one_wg ? nullptr : ws.data_ptr<float>(),
                     cur_stream()),
           "sample");
}

void kv_block_copy(at::Tensor k_cache, at::Tensor v_cache, at::Tensor src_dst) {
  check_dev(k_cache, "k_cache");
  check_dev(v_cache, "v_cache");
  TORCH_CHECK(k_cache.scalar_type() == v_cache.scalar_type() &&
                  (k_cache.scalar_type() == at::kBFloat16 || k_cache.scalar_type() == at::kFloat8_e4m3fn),
              "KV caches bfloat16 or float8_e4m3fn");
  check_i32(src_dst, "src_dst");
  TORCH_CHECK(k_cache.is_contiguous() && v_cache.is_contiguous(), "caches contiguous");
  // the kernel copies 16-B words; it counts a block in 2-byte units
  const long block_bytes = (long)(k_cache.numel() / k_cache.size(0)) * (long)k_cache.element_size();
  TORCH_CHECK(block_bytes % 16 == 0, "block size");
  const long block_elems = block_bytes / 2;
  check_rc(ft_kv_block_copy(k_cache.data_ptr(), v_cache.data_ptr(), src_dst.data_ptr<int>(),
                            (int)(src_dst.numel() / 2), block_elems, (int)k_cache.size(0),
                            cur_stream()),
           "kv_block_copy");
}

// ptrs: int64 device [2L] cache base pointers (every cache [nblk, ...] bf16 with
// block_elems elements per block); ids: int32 device [n]; staging: bf16 device
// [n, 2L, block_elems].  The caller bounds-checks ids against the pool size.
void kv_swap(at::Tensor ptrs, at::Tensor ids, at::Tensor staging, int64_t block_elems,
             bool to_staging, int64_t num_blocks) {
  check_dev(ptrs, "ptrs");
  TORCH_CHECK(ptrs.scalar_type() == at::kLong && ptrs.is_contiguous(), "ptrs int64");
  check_i32(ids, "ids");
  check_dev(staging, "staging");
  TORCH_CHECK(staging.scalar_type() == at::kBFloat16 || staging.scalar_type() == at::kFloat8_e4m3fn,
              "staging in the caches' dtype (bfloat16 or float8_e4m3fn)");
  TORCH_CHECK(staging.is_contiguous(), "staging contiguous");
  const int n = (int)ids.numel();
  TORCH_CHECK(staging.numel() >= (int64_t)n * ptrs.numel() * block_elems, "staging too small");
  // the kernel moves 16-B words and counts a block in 2-byte units
  const int64_t block_bytes = block_elems * (int64_t)staging.element_size();
  TORCH_CHECK(block_bytes % 16 == 0, "block bytes must be a multiple of 16");
  check_rc(ft_kv_swap(reinterpret_cast<const uint64_t*>(ptrs.data_ptr<int64_t>()),
                      (int)ptrs.numel(), ids.data_ptr<int>(), n, staging.data_ptr(), block_bytes / 2,
                      to_staging ? 1 : 0, (int)num_blocks, cur_stream()),
           "kv_swap");
}

void check_ws(const at::Tensor& ws, int64_t need) {
  check_dev(ws, "workspace");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && ws.is_contiguous(), "workspace fp32 contiguous");
  TORCH_CHECK(ws.numel() >= need, "workspace too small: need ", need, " have ", ws.numel());
}

// y = x W^T for M <= 64 rows; splits > 1 writes fp32 slabs [splits, M, N] into ws
// W4A16: wq int32 packed image [N/16][K/128][64][4], sz fp32 [N/16][K/128][16][2]
// (scale, 128 + zero); see w4a16.hip.
void check_w4(const at::Tensor& wq, const at::Tensor& sz, int64_t N, int64_t K) {
  check_dev(wq, "wq");
  check_dev(sz, "sz");
  TORCH_CHECK(wq.scalar_type() == at::kInt && wq.is_contiguous(), "wq int32 contiguous");
  TORCH_CHECK(sz.scalar_type() == at::kFloat && sz.is_contiguous(), "sz fp32 contiguous");
  TORCH_CHECK(N % 16 == 0 && K % 128 == 0, "W4 needs N % 16 == 0 and K % 128 == 0");
  TORCH_CHECK(wq.numel() == N * K / 8, "wq size");
  TORCH_CHECK(sz.numel() == N * (K / 128) * 2, "sz size");
}

void w4_gemm(at::Tensor x, at::Tensor wq, at::Tensor sz, int64_t N, c10::optional<at::Tensor> out,
             c10::optional<at::Tensor> ws, int64_t splits, int64_t nt, int64_t xr, bool silu) {
  check_bf16(x, "x");
  check_rows(x, "x");
  const int M = (int)x.size(0), K = (int)x.size(1);
  check_w4(wq, sz, N, K);
  TORCH_CHECK(M <= 64, "w4_gemm supports M <= 64");
  float* wsp = nullptr;
  void* op = nullptr;
  int ostride = 0;
  if (ws.has_value()) {  // fp32 slabs (any split count)
    check_ws(*ws, (int64_t)splits * M * N);
    wsp = ws->data_ptr<float>();
  } else {
    TORCH_CHECK(splits == 1, "splits > 1 needs a workspace");
    TORCH_CHECK(out.has_value(), "no workspace: needs out");
    check_bf16(*out, "out");
    TORCH_CHECK(out->dim() == 2 && out->stride(1) == 1 && out->size(0) >= M &&
                    out->size(1) >= (silu ? N / 2 : N),
                "out shape");
    op = out->data_ptr();
    ostride = (int)out->stride(0);
  }
  TORCH_CHECK(!silu || (xr && !ws.has_value()), "the SiLU epilogue is an xr bf16-output variant");
  if (xr == 4 || xr == 5) {   // "mh": two tiles per wave, rows over wave pairs; ring 2 (+2 x chunks) / 3
    check_rc(ft_w4_gemm_mh(x.data_ptr(), (int)x.stride(0), M,
                           reinterpret_cast<const uint32_t*>(wq.data_ptr<int>()), sz.data_ptr(),
                           (int)N, K, wsp, op, ostride, (int)splits, xr == 4 ? 2 : 3, silu ? 1 : 0,
                           cur_stream()),
             "w4_gemm_mh");
    return;
  }
  if (xr) {   // "xr": x chunks in LDS, x sums while staging
    check_rc(ft_w4_gemm_xr(x.data_ptr(), (int)x.stride(0), M,
                           reinterpret_cast<const uint32_t*>(wq.data_ptr<int>()), sz.data_ptr(),
                           (int)N, K, wsp, op, ostride, (int)splits, (int)nt, silu ? 1 : 0,
                           cur_stream()),
             "w4_gemm_xr");
    return;
  }
  check_rc(ft_w4_gemm(x.data_ptr(), (int)x.stride(0), M,
                      reinterpret_cast<const uint32_t*>(wq.data_ptr<int>()), sz.data_ptr(), (int)N,
                      K, wsp, op, ostride, (int)splits, (int)nt, cur_stream()),
           "w4_gemm");
}

void w4_dequant(at::Tensor wq, at::Tensor sz, at::Tensor out) {
  check_bf16(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.is_contiguous(), "out [N, K] contiguous");
  const int64_t N = out.size(0), K = out.size(1);
  check_w4(wq, sz, N, K);
  check_rc(ft_w4_dequant(reinterpret_cast<const uint32_t*>(wq.data_ptr<int>()), sz.data_ptr(),
                         out.data_ptr(), (int)N, (int)K, cur_stream()),
           "w4_dequant");
}

void skinny_gemm(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> out,
                 c10::optional<at::Tensor> ws, int64_t splits, int64_t nt, int64_t u) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_rows(x, "x");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "w must be the packed [N, K] image");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "K mismatch");
  TORCH_CHECK(M <= (u == -4 ? 128 : 64), "skinny_gemm supports M <= 64 (pk, xr) / 128 (xc)");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "w alignment");
  TORCH_CHECK(u >= -8 && u <= -3,
              "skinny_gemm variant: -3 (pk), -4 (xc), -5 (xr), -6 (xr + SiLU), -7 / -8 (the same "
              "xr on 8-wave workgroups), packed weights");
  const bool silu = u == -6 || u == -8;
  TORCH_CHECK(!silu || (splits == 1 && nt == 2 && N % 32 == 0),
              "xr SiLU epilogue: one split, nt 2, interleaved gate_up image");
  float* wsp = nullptr;
  void* op = nullptr;
  int ostride = 0;
  if (splits > 1) {
    TORCH_CHECK(ws.has_value(), "splits > 1 needs a workspace");
    check_ws(*ws, (int64_t)splits * M * N);
    wsp = ws->data_ptr<float>();
  } else {
    TORCH_CHECK(out.has_value(), "splits == 1 needs out");
    check_bf16(*out, "out");
    TORCH_CHECK(out->dim() == 2 && out->stride(1) == 1 && out->size(0) >= M &&
                    out->size(1) >= (silu ? N / 2 : N),
                "out shape");
    op = out->data_ptr();
    ostride = (int)out->stride(0);
  }
  if (u <= -5)
    check_rc(ft_skinny_gemm_xr(x.data_ptr(), (int)x.stride(0), M, w.data_ptr(), N, K, wsp, op,
                               ostride, (int)splits, (int)nt, silu ? 1 : 0, u <= -7 ? 8 : 4,
                               cur_stream()),
             "skinny_gemm_xr");
  else if (u == -3)  // w is the packed [N/16][K/64][2][64][8] image (ops.pack_weight)
    check_rc(ft_skinny_gemm_pk(x.data_ptr(), (int)x.stride(0), M, w.data_ptr(), N, K, wsp, op,
                               ostride, (int)splits, (int)nt, cur_stream()),
             "skinny_gemm_pk");
  else
    check_rc(ft_skinny_gemm_xc(x.data_ptr(), (int)x.stride(0), M, w.data_ptr(), N, K, wsp, op,
                               ostride, (int)splits, (int)nt, cur_stream()),
             "skinny_gemm_xc");
}

// "xr" decode GEMM (csrc/kernels/skinny_gemm.hip): epi 0 bf16 out / fp32 slabs,
// epi 1 SiLU of the interleaved gate/up image.
void skinny_gemm_xr(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> out,
                    c10::optional<at::Tensor> ws, int64_t splits, int64_t nt, int64_t epi,
                    int64_t nw) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_rows(x, "x");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "w must be the packed [N, K] image");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K && M <= 64, "xr: K mismatch or M > 64");
  void* op = nullptr;
  int ostride = 0;
  if (epi == 1 || (epi == 0 && splits == 1)) {
    TORCH_CHECK(out.has_value(), "xr: out required");
    check_bf16(*out, "out");
    TORCH_CHECK(out->dim() == 2 && out->stride(1) == 1 && out->size(0) >= M &&
                    out->size(1) >= (epi == 1 ? N / 2 : N), "xr: out shape");
    op = out->data_ptr();
    ostride = (int)out->stride(0);
  }
  float* wsp = nullptr;
  if (splits > 1) {
    TORCH_CHECK(ws.has_value(), "xr: splits > 1 needs a workspace");
    check_ws(*ws, (int64_t)splits * M * N);
    wsp = ws->data_ptr<float>();
  }
  check_rc(ft_skinny_gemm_xr(x.data_ptr(), (int)x.stride(0), M, w.data_ptr(), N, K, wsp, op, ostride,
                             (int)splits, (int)nt, (int)epi, (int)nw, cur_stream()),
           "skinny_gemm_xr");
}

// Packed-image GEMM for M > 64 rows (csrc/kernels/packed_gemm.hip).
// epi: 0 bf16 out [M, N], 1 fp32 slabs ws [splits, M, N], 2 SiLU-mul out [M, N/2]
// (interleaved gate/up image).
void packed_gemm(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> out,
                 c10::optional<at::Tensor> ws, int64_t splits, int64_t epi, int64_t cfg) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_rows(x, "x");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "w must be the packed [N, K] image");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "K mismatch");
  TORCH_CHECK(N % 16 == 0 && K % 64 == 0, "packed_gemm: N % 16, K % 64");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && x.stride(0) % 8 == 0,
              "x rows must be 16-B aligned");
  TORCH_CHECK(epi >= 0 && epi <= 2 && (epi == 1) == (splits > 1), "packed_gemm: epi/splits");
  float* wsp = nullptr;
  void* op = nullptr;
  int ostride = 0;
  if (epi == 1) {
    TORCH_CHECK(ws.has_value(), "splits > 1 needs a workspace");
    check_ws(*ws, (int64_t)splits * M * N);
    wsp = ws->data_ptr<float>();
  } else {
    TORCH_CHECK(out.has_value(), "needs out");
    check_bf16(*out, "out");
    const int64_t cols = epi == 2 ? N / 2 : N;
    TORCH_CHECK(out->dim() == 2 && out->stride(1) == 1 && out->size(0) >= M && out->size(1) >= cols,
                "out shape");
    op = out->data_ptr();
    ostride = (int)out->stride(0);
  }
  check_rc(ft_packed_gemm(x.data_ptr(), (int)x.stride(0), M, w.data_ptr(), N, K, (int)splits,
                          (int)epi, (int)cfg, op, ostride, wsp, cur_stream()),
           "packed_gemm");
}


// Ring-pipelined packed decode GEMM with fused epilogues (csrc/kernels/skinny_pkr.hip).
// epi: 0 store (out or slabs), 1 silu (gate/up interleaved, out [M, N/2]), 2 resid.
void pkr_gemm(at::Tensor x, at::Tensor w, c10::optional<at::Tensor> out,
              c10::optional<at::Tensor> ws, c10::optional<at::Tensor> residual,
              c10::optional<at::Tensor> tickets, int64_t splits, int64_t nt, int64_t depth,
              int64_t epi, bool norm, double eps, bool wn) {
  check_bf16(x, "x");
  check_bf16(w, "w");
  check_rows(x, "x");
  TORCH_CHECK(w.dim() == 2 && w.is_contiguous(), "w must be contiguous [N, K]");
  const int M = (int)x.size(0), K = (int)x.size(1), N = (int)w.size(0);
  TORCH_CHECK(w.size(1) == K, "K mismatch");
  TORCH_CHECK(M <= 64, "pkr_gemm supports M <= 64");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0, "w alignment");
  float* wsp = nullptr;
  void* op = nullptr;
  void* rp = nullptr;
  int* tp = nullptr;
  int ostride = 0, rstride = 0;
  if (ws.has_value()) {
    check_ws(*ws, splits * M * N);
    wsp = ws->data_ptr<float>();
  }
  if (out.has_value()) {
    check_bf16(*out, "out");
    TORCH_CHECK(out->dim() == 2 && out->stride(1) == 1 && out->size(0) >= M &&
                    out->size(1) >= (epi == 1 ? N / 2 : N),
                "out shape");
    op = out->data_ptr();
    ostride = (int)out->stride(0);
  }
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    check_rows(*residual, "residual");
    TORCH_CHECK(residual->size(0) >= M && residual->size(1) == N, "residual shape");
    rp = residual->data_ptr();
    rstride = (int)residual->stride(0);
  }
  if (tickets.has_value()) {
    check_i32(*tickets, "tickets");
    TORCH_CHECK(tickets->numel() >= N / (16 * nt), "tickets too small");
    tp = tickets->data_ptr<int>();
  }
  check_rc(ft_pkr_gemm(x.data_ptr(), (int)x.stride(0), M, w.data_ptr(), N, K, wsp, op, ostride, rp,
                       rstride, tp, (int)splits, (int)nt, (int)depth, (int)epi, norm ? 1 : 0,
                       wn ? 1 : 0, (float)eps, cur_stream()),
           "pkr_gemm");
}

// Persistent post-attention decode block (csrc/kernels/decode_block.hip):
// residual += attn Wo^T; h = silu . rms-scaled (residual Wgu^T); residual += h Wd^T.
void decode_block(at::Tensor attn, at::Tensor residual, at::Tensor h, at::Tensor wo, at::Tensor wgu,
                  at::Tensor wd, at::Tensor ws, at::Tensor xg, at::Tensor ctl, double eps,
                  c10::optional<at::Tensor> stamps) {
  long long* sp = nullptr;
  if (stamps.has_value()) {
    check_dev(*stamps, "stamps");
    TORCH_CHECK(stamps->scalar_type() == at::kLong && stamps->numel() >= 16 * 1024, "stamps int64 [>= 16K]");
    sp = reinterpret_cast<long long*>(stamps->data_ptr<int64_t>());
  }
  for (auto* t : {&attn, &residual, &h, &wo, &wgu, &wd}) {
    check_bf16(*t, "decode_block operand");
    TORCH_CHECK(t->dim() == 2 && t->is_contiguous(), "decode_block operands must be contiguous 2-D");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "decode_block alignment");
  }
  check_dev(ws, "ws");
  check_dev(xg, "xg");
  TORCH_CHECK(ws.scalar_type() == at::kFloat && xg.scalar_type() == at::kFloat, "ws / xg float32");
  TORCH_CHECK(ws.is_contiguous() && xg.is_contiguous(), "ws / xg contiguous");
  check_i32(ctl, "ctl");
  TORCH_CHECK(ctl.numel() >= ft_decode_block_ctl_words(), "ctl too small");
  const int M = (int)attn.size(0), Ko = (int)attn.size(1), H = (int)residual.size(1);
  const int I = (int)h.size(1);
  TORCH_CHECK(M >= 1 && M <= 64, "decode_block: 1..64 rows");
  TORCH_CHECK(residual.size(0) == M && h.size(0) >= M, "decode_block rows");
  TORCH_CHECK(wo.size(0) == H && wo.size(1) == Ko, "wo shape");
  TORCH_CHECK(wgu.size(0) == 2 * I && wgu.size(1) == H, "wgu shape");
  TORCH_CHECK(wd.size(0) == H && wd.size(1) == I, "wd shape");
  check_rc(ft_decode_block(attn.data_ptr(), Ko, residual.data_ptr(), H, h.data_ptr(), I,
                           wo.data_ptr(), wgu.data_ptr(), wd.data_ptr(), ws.data_ptr<float>(),
                           (long)ws.numel(), xg.data_ptr<float>(), (long)xg.numel(),
                           ctl.data_ptr<int>(), sp, M, H, Ko, I, (float)eps, cur_stream()),
           "decode_block");
}

py::object decode_block_plan(int64_t H, int64_t Ko, int64_t I) {
  int so = 0, sd = 0, tpw = 0, grid = 0;
  if (ft_decode_block_plan((int)H, (int)Ko, (int)I, &so, &sd, &tpw, &grid) != 0) return py::none();
  return py::make_tuple(so, sd, tpw, grid);
}

// ---- custom one-shot all-reduce (csrc/kernels/custom_ar.hip) ----------------------
int64_t custom_ar_alloc(int64_t bytes) {
  void* p = nullptr;
  check_rc(ft_ar_alloc((size_t)bytes, &p), "custom_ar_alloc");
  return (int64_t)(uintptr_t)p;
}
void custom_ar_free(int64_t p) { check_rc(ft_ar_free((void*)(uintptr_t)p), "custom_ar_free"); }
py::bytes custom_ar_handle(int64_t p) {
  char h[64] = {0};
  check_rc(ft_ar_ipc_handle((void*)(uintptr_t)p, h), "custom_ar_handle");
  return py::bytes(h, 64);
}
int64_t custom_ar_open(py::bytes h) {
  std::string s = h;
  TORCH_CHECK(s.size() == 64, "ipc handle must be 64 bytes");
  void* p = nullptr;
  check_rc(ft_ar_ipc_open(s.data(), &p), "custom_ar_open");
  return (int64_t)(uintptr_t)p;
}
void custom_ar_close(int64_t p) { check_rc(ft_ar_ipc_close((void*)(uintptr_t)p), "custom_ar_close"); }
int64_t custom_ar_error(int64_t p) {
  int e = 0;
  check_rc(ft_ar_read_error((void*)(uintptr_t)p, &e), "custom_ar_error");
  return e;
}
void custom_ar_allreduce(at::Tensor out, at::Tensor x, at::Tensor peers, int64_t rank, int64_t world,
                         int64_t max_bytes, int64_t spin_budget, bool two_shot) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && out.numel() == x.numel(), "contiguous");
  TORCH_CHECK(peers.scalar_type() == at::kLong && peers.is_cuda() && peers.numel() == world, "peers");
  TORCH_CHECK(x.numel() % 8 == 0 && x.numel() * 2 <= max_bytes, "custom_ar_allreduce: size");
  check_rc(ft_ar_allreduce(out.data_ptr(), x.data_ptr(), (long)x.numel(),
                           reinterpret_cast<const uint64_t*>(peers.data_ptr<int64_t>()), (int)rank,
                           (int)world, (size_t)max_bytes, (unsigned)spin_budget, two_shot ? 1 : 0,
                           cur_stream()),
           "custom_ar_allreduce");
}
// residual += all-reduce(partial); out = rmsnorm(residual) * weight.  partial: fp32
// split-K slabs ws[splits][rows][hidden] (ws given) or bf16 x [rows, hidden].
void custom_ar_add_rmsnorm(at::Tensor out, at::Tensor residual, at::Tensor weight, double eps,
                           c10::optional<at::Tensor> ws, int64_t splits, c10::optional<at::Tensor> x,
                           int64_t rows, at::Tensor peers, int64_t rank, int64_t world,
                           int64_t max_bytes, int64_t spin_budget) {
  check_bf16(out, "out");
  check_bf16(residual, "residual");
  check_bf16(weight, "weight");
  const int64_t hidden = residual.size(1);
  TORCH_CHECK(residual.is_contiguous() && residual.size(0) >= rows, "residual");
  TORCH_CHECK(out.size(0) >= rows && out.size(1) == hidden && out.stride(1) == 1, "out");
  TORCH_CHECK(weight.numel() == hidden, "weight");
  TORCH_CHECK(peers.scalar_type() == at::kLong && peers.is_cuda() && peers.numel() == world, "peers");
  const float* wsp = nullptr;
  const void* xp = nullptr;
  int x_stride = 0;
  if (ws.has_value()) {
    TORCH_CHECK(ws->scalar_type() == at::kFloat && ws->numel() >= splits * rows * hidden, "ws");
    wsp = ws->data_ptr<float>();
  } else {
    TORCH_CHECK(x.has_value(), "ws or x");
    check_bf16(*x, "x");
    TORCH_CHECK(x->size(1) == hidden && x->stride(1) == 1 && x->size(0) >= rows, "x");
    xp = x->data_ptr();
    x_stride = (int)x->stride(0);
  }
  check_rc(ft_ar_add_rmsnorm(out.data_ptr(), (int)out.stride(0), residual.data_ptr(), weight.data_ptr(),
                             (float)eps, wsp, (int)splits, xp, x_stride, (long)rows, (long)hidden,
                             reinterpret_cast<const uint64_t*>(peers.data_ptr<int64_t>()), (int)rank,
                             (int)world, (size_t)max_bytes, (unsigned)spin_budget, cur_stream()),
           "custom_ar_add_rmsnorm");
}
// x: [rows, shard] bf16 -> out: [rows, world * shard]
void custom_ar_allgather(at::Tensor out, at::Tensor x, at::Tensor peers, int64_t rank, int64_t world,
                         int64_t max_bytes, int64_t spin_budget) {
  check_bf16(out, "out");
  check_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && out.dim() == 2 && x.is_contiguous() && out.is_contiguous(), "2-D contiguous");
  TORCH_CHECK(out.size(0) == x.size(0) && out.size(1) == x.size(1) * world, "allgather shapes");
  TORCH_CHECK(x.size(1) % 8 == 0 && x.numel() * 2 <= max_bytes, "custom_ar_allgather: size");
  TORCH_CHECK(peers.scalar_type() == at::kLong && peers.is_cuda() && peers.numel() == world, "peers");
  check_rc(ft_ar_allgather(out.data_ptr(), x.data_ptr(), (long)x.size(0), (long)x.size(1),
                           reinterpret_cast<const uint64_t*>(peers.data_ptr<int64_t>()), (int)rank,
                           (int)world, (size_t)max_bytes, (unsigned)spin_budget, cur_stream()),
           "custom_ar_allgather");
}
void custom_ar_export_error(at::Tensor dst, at::Tensor peers, int64_t world) {
  TORCH_CHECK(dst.is_cuda() && dst.scalar_type() == at::kInt && dst.numel() >= 1, "dst: int32 device");
  TORCH_CHECK(peers.scalar_type() == at::kLong && peers.is_cuda() && peers.numel() == world, "peers");
  check_rc(ft_ar_export_error(dst.data_ptr<int>(), reinterpret_cast<const uint64_t*>(peers.data_ptr<int64_t>()),
                              (int)world, cur_stream()),
           "custom_ar_export_error");
}

// residual = table[ids]; out = rmsnorm(residual) * w  (embedding + first RMSNorm)
void embed_rmsnorm(at::Tensor out, at::Tensor residual, at::Tensor ids, at::Tensor table,
                   at::Tensor w, double eps) {
  check_bf16(out, "out");
  check_bf16(residual, "residual");
  check_bf16(table, "table");
  check_bf16(w, "w");
  check_i32(ids, "ids");
  TORCH_CHECK(table.dim() == 2 && table.is_contiguous(), "table must be contiguous [V, H]");
  const int rows = (int)ids.numel(), hidden = (int)table.size(1);
  TORCH_CHECK(out.is_contiguous() && residual.is_contiguous() && out.numel() >= (int64_t)rows * hidden &&
                  residual.numel() >= (int64_t)rows * hidden && w.numel() == hidden,
              "embed_rmsnorm shapes");
  check_rc(ft_embed_rmsnorm(out.data_ptr(), residual.data_ptr(), ids.data_ptr<int>(),
                            table.data_ptr(), w.data_ptr(), rows, hidden, (int)table.size(0),
                            (float)eps, cur_stream()),
           "embed_rmsnorm");
}

// out = rmsnorm([residual +=] src) * w where src = bf16 x or the fp32 slabs in ws
void row_rmsnorm(at::Tensor out, c10::optional<at::Tensor> x, c10::optional<at::Tensor> ws,
                 int64_t splits, c10::optional<at::Tensor> residual, at::Tensor w, int64_t rows,
                 double eps) {
  check_bf16(out, "out");
  check_rows(out, "out");
  check_bf16(w, "weight");
  const int hidden = (int)w.numel();
  TORCH_CHECK(out.size(0) >= rows && out.size(1) == hidden, "out shape");
  void* rp = nullptr;
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) >= rows &&
                    residual->size(1) == hidden, "residual shape");
    rp = residual->data_ptr();
  }
  if (ws.has_value()) {
    check_ws(*ws, (int64_t)splits * rows * hidden);
    check_rc(ft_row_rmsnorm(nullptr, 0, ws->data_ptr<float>(), (int)splits, out.data_ptr(),
                            (int)out.stride(0), rp, w.data_ptr(), (int)rows, hidden, (float)eps,
                            cur_stream()), "row_rmsnorm");
  } else {
    TORCH_CHECK(x.has_value(), "need x or ws");
    check_bf16(*x, "x");
    check_rows(*x, "x");
    TORCH_CHECK(x->size(0) >= rows && x->size(1) == hidden, "x shape");
    check_rc(ft_row_rmsnorm(x->data_ptr(), (int)x->stride(0), nullptr, 1, out.data_ptr(),
                            (int)out.stride(0), rp, w.data_ptr(), (int)rows, hidden, (float)eps,
                            cur_stream()), "row_rmsnorm");
  }
}

void slab_silu(at::Tensor ws, int64_t splits, int64_t rows, int64_t inter, at::Tensor out, bool il) {
  check_ws(ws, splits * rows * 2 * inter);
  check_bf16(out, "out");
  check_rows(out, "out");
  TORCH_CHECK(out.size(0) >= rows && out.size(1) >= inter, "out shape");
  TORCH_CHECK(!il || inter % 16 == 0, "interleaved slab_silu: inter % 16");
  check_rc(ft_slab_silu(ws.data_ptr<float>(), (int)splits, (int)rows, (int)inter, out.data_ptr(),
                        (int)out.stride(0), il ? 1 : 0, cur_stream()), "slab_silu");
}

void slab_store(at::Tensor ws, int64_t splits, int64_t rows, int64_t cols, at::Tensor out) {
  check_ws(ws, splits * rows * cols);
  check_bf16(out, "out");
  check_rows(out, "out");
  TORCH_CHECK(out.size(0) >= rows && out.size(1) >= cols, "out shape");
  check_rc(ft_slab_store(ws.data_ptr<float>(), (int)splits, (int)rows, (int)cols, out.data_ptr(),
                         (int)out.stride(0), cur_stream()), "slab_store");
}

void slab_rope_kv(at::Tensor ws, int64_t splits, int64_t rows, int64_t cols, at::Tensor q_out,
                  at::Tensor positions, at::Tensor cos_sin, at::Tensor slot_mapping,
                  at::Tensor k_cache, at::Tensor v_cache, int64_t nq, int64_t nkv,
                  int64_t head_dim, c10::optional<at::Tensor> residual, double eps) {
  check_ws(ws, splits * rows * cols);
  const void* rp = nullptr;
  int hidden = 0;
  if (residual.has_value()) {
    check_bf16(*residual, "residual");
    TORCH_CHECK(residual->is_contiguous() && residual->size(0) >= rows, "residual shape");
    rp = residual->data_ptr();
    hidden = (int)residual->size(1);
  }
  check_bf16(q_out, "q_out");
  check_rows(q_out, "q_out");
  check_i32(positions, "positions");
  check_i32(slot_mapping, "slot_mapping");
  TORCH_CHECK(cols == (nq + 2 * nkv) * head_dim, "cols");
  TORCH_CHECK(q_out.size(0) >= rows && q_out.size(1) >= nq * head_dim, "q_out shape");
  TORCH_CHECK(cos_sin.scalar_type() == at::kFloat && cos_sin.size(1) == head_dim, "cos_sin");
  const bool kv8 = check_kv_caches(k_cache, v_cache, nkv, head_dim);
  TORCH_CHECK(positions.numel() >= rows && slot_mapping.numel() >= rows, "metadata length");
  check_rc(ft_slab_rope_kv(ws.data_ptr<float>(), (int)splits, (int)rows, (int)cols,
                           q_out.data_ptr(), (int)q_out.stride(0), positions.data_ptr<int>(),
                           cos_sin.data_ptr<float>(), slot_mapping.data_ptr<int>(),
                           k_cache.data_ptr(), v_cache.data_ptr(), (int)nq, (int)nkv,
                           (int)head_dim, (int)k_cache.size(2), rp, hidden, (float)eps,
                           (int)cos_sin.size(0), (int)(k_cache.size(0) * k_cache.size(2)),
                           kv8 ? 1 : 0, cur_stream()), "slab_rope_kv");
}

#if defined(FT_KERNEL_CHECKS) && FT_KERNEL_CHECKS
// checked build: every instrumented kernel unit's hook (ft_common.h FT_CHECK_HOOK)
extern "C" {
#define FT_HOOK_DECL(NAME) int ft_check_hook_##NAME(uint32_t*);
FT_HOOK_DECL(attn_decode)
FT_HOOK_DECL(attn_prefill)
FT_HOOK_DECL(rope_kv)
FT_HOOK_DECL(fused_epilogue)
FT_HOOK_DECL(norm_act)
FT_HOOK_DECL(sampling)
FT_HOOK_DECL(kv_copy)
#undef FT_HOOK_DECL
}

// word: int32 [4] device tensor (violations, first code, context, value); the process's
// checked kernels report into it until it is replaced
void set_kernel_checks(torch::Tensor word) {
  TORCH_CHECK(word.is_cuda() && word.scalar_type() == at::kInt && word.numel() >= 4, "check word");
  uint32_t* w = reinterpret_cast<uint32_t*>(word.data_ptr<int>());
  using Hook = int (*)(uint32_t*);
  const Hook hooks[] = {ft_check_hook_attn_decode, ft_check_hook_attn_prefill,
                        ft_check_hook_rope_kv,     ft_check_hook_fused_epilogue,
                        ft_check_hook_norm_act,    ft_check_hook_sampling,
                        ft_check_hook_kv_copy};
  for (Hook h : hooks) check_rc(h(w), "set_kernel_checks");
}
#endif

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "FastTalk MI355X (gfx950) HIP kernels";
#if defined(FT_KERNEL_CHECKS) && FT_KERNEL_CHECKS
  m.attr("kernel_checks") = true;
  m.def("set_kernel_checks", &set_kernel_checks);
#else
  m.attr("kernel_checks") = false;
#endif
  m.def("rmsnorm", &rmsnorm);
  m.def("fused_add_rmsnorm", &fused_add_rmsnorm);
  m.def("silu_mul", &silu_mul);
  m.def("rope_kv_write", &rope_kv_write);
  m.def("paged_decode_attention", &paged_decode_attention, py::arg("out"), py::arg("q"),
        py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"), py::arg("seq_lens"),
        py::arg("tmp_out"), py::arg("tmp_ml"), py::arg("nq"), py::arg("nkv"), py::arg("head_dim"),
        py::arg("scale"), py::arg("counters") = py::none(), py::arg("piece") = 0);
  m.def("decode_waves", []() { return ft_decode_waves(); });
  m.def("decode_max_batch", []() { return ft_decode_max_batch(); });
  m.def("prefill_attention", &prefill_attention, py::arg("out"), py::arg("q"), py::arg("k_cache"),
        py::arg("v_cache"), py::arg("block_tables"), py::arg("seq_lens"), py::arg("q_start_loc"),
        py::arg("tile_info"), py::arg("num_tiles"), py::arg("nq"), py::arg("nkv"),
        py::arg("head_dim"), py::arg("scale"), py::arg("part_o") = py::none(),
        py::arg("part_ml") = py::none(), py::arg("combine") = py::none(),
        py::arg("num_combine") = 0, py::arg("num_partials") = 0, py::arg("invariant") = false);
  m.def("prefill_tile_tokens", [](int64_t nq, int64_t nkv) { return ft_prefill_tile_tokens((int)nq, (int)nkv); });
  m.def("sample", &sample, py::arg("out_tokens"), py::arg("logits"), py::arg("temperature"),
        py::arg("top_p"), py::arg("top_k"), py::arg("seeds"), py::arg("steps"),
        py::arg("mask") = py::none());
  m.def("kv_block_copy", &kv_block_copy);
  m.def("kv_swap", &kv_swap, py::arg("ptrs"), py::arg("ids"), py::arg("staging"),
        py::arg("block_elems"), py::arg("to_staging"), py::arg("num_blocks") = 0);
  m.def("w4_gemm", &w4_gemm, py::arg("x"), py::arg("wq"), py::arg("sz"), py::arg("N"),
        py::arg("out") = py::none(), py::arg("ws") = py::none(), py::arg("splits") = 1,
        py::arg("nt") = 1, py::arg("xr") = false, py::arg("silu") = false);
  m.def("w4_dequant", &w4_dequant);
  m.def("skinny_gemm_xr", &skinny_gemm_xr, py::arg("x"), py::arg("w"), py::arg("out") = py::none(),
        py::arg("ws") = py::none(), py::arg("splits") = 1, py::arg("nt") = 2, py::arg("epi") = 0,
        py::arg("nw") = 4);
  m.def("skinny_gemm", &skinny_gemm, py::arg("x"), py::arg("w"), py::arg("out") = py::none(),
        py::arg("ws") = py::none(), py::arg("splits") = 1, py::arg("nt") = 1, py::arg("u") = -3);
  m.def("pkr_gemm", &pkr_gemm, py::arg("x"), py::arg("w"), py::arg("out") = py::none(),
        py::arg("ws") = py::none(), py::arg("residual") = py::none(),
        py::arg("tickets") = py::none(), py::arg("splits") = 1, py::arg("nt") = 2,
        py::arg("depth") = 3, py::arg("epi") = 0, py::arg("norm") = false, py::arg("eps") = 0.0,
        py::arg("wn") = false);
  m.def("decode_block", &decode_block, py::arg("attn"), py::arg("residual"), py::arg("h"),
        py::arg("wo"), py::arg("wgu"), py::arg("wd"), py::arg("ws"), py::arg("xg"), py::arg("ctl"),
        py::arg("eps"), py::arg("stamps") = py::none());
  m.def("decode_block_plan", &decode_block_plan);
  m.def("decode_block_ws_floats",
        [](int64_t H, int64_t M) { return (int64_t)ft_decode_block_ws_floats((int)H, (int)M); });
  m.def("decode_block_ctl_words", []() { return (int64_t)ft_decode_block_ctl_words(); });
  m.def("row_rmsnorm", &row_rmsnorm, py::arg("out"), py::arg("x") = py::none(),
        py::arg("ws") = py::none(), py::arg("splits") = 1, py::arg("residual") = py::none(),
        py::arg("w"), py::arg("rows"), py::arg("eps"));
  m.def("embed_rmsnorm", &embed_rmsnorm);
  m.def("custom_ar_header_bytes", []() { return (int64_t)ft_ar_header_bytes(); });
  m.def("custom_ar_set_max_blocks", [](int64_t n) { ft_ar_set_max_blocks((int)n); });
  m.def("custom_ar_alloc", &custom_ar_alloc);
  m.def("custom_ar_free", &custom_ar_free);
  m.def("custom_ar_handle", &custom_ar_handle);
  m.def("custom_ar_open", &custom_ar_open);
  m.def("custom_ar_close", &custom_ar_close);
  m.def("custom_ar_error", &custom_ar_error);
  m.def("custom_ar_allreduce", &custom_ar_allreduce);
  m.def("custom_ar_add_rmsnorm", &custom_ar_add_rmsnorm);
  m.def("packed_gemm", &packed_gemm);
  m.def("custom_ar_allgather", &custom_ar_allgather);
  m.def("custom_ar_export_error", &custom_ar_export_error);
  m.def("slab_silu", &slab_silu);
  m.def("slab_store", &slab_store);
  m.def("slab_rope_kv", &slab_rope_kv, py::arg("ws"), py::arg("splits"), py::arg("rows"),
        py::arg("cols"), py::arg("q_out"), py::arg("positions"), py::arg("cos_sin"),
        py::arg("slot_mapping"), py::arg("k_cache"), py::arg("v_cache"), py::arg("nq"),
        py::arg("nkv"), py::arg("head_dim"), py::arg("residual") = py::none(),
        py::arg("eps") = 0.0);
}
