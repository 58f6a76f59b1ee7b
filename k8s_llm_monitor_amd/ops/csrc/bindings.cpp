// PyTorch bindings for the gfx950 kernels.  The kernels themselves are plain HIP compiled by
// hipcc (no torch headers); this translation unit validates tensors, picks the current HIP
// stream (so every op is hipGraph-capturable) and calls the C launchers.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

extern "C" {
int k8sllm_rmsnorm(void* out, const void* x, void* residual, const void* w, long rows, int d, float eps,
                   long x_stride, long out_stride, hipStream_t s);
int k8sllm_layernorm(void* out, const void* x, const void* w, const void* b, long rows, int d, float eps,
                     hipStream_t s);
int k8sllm_silu_mul(void* out, const void* x, long rows, int F, int interleaved, hipStream_t s);
int k8sllm_gelu_tanh(void* out, const void* x, long n, hipStream_t s);
int k8sllm_embedding(void* out, const int* ids, const void* weight, long T, int d, int vocab_start, int rows,
                     hipStream_t s);
int k8sllm_resolve_ids(int* out, const int* ids, const int* src, const int* prev, int n, hipStream_t s);
int k8sllm_rope_cache(void* qkv, long qkv_stride, const int* positions, const float* cos_sin, void* k_cache,
                      void* v_cache, const int* slot_mapping, long T, int Hq, int Hkv, int D, int block_size,
                      int apply_rope, const float* partial, int S, hipStream_t s);
int k8sllm_paged_decode(void* out, long out_stride, float* part_out, float* part_ml, const void* q, long q_stride,
                        const void* k_cache, const void* v_cache, const int* block_tables, int bt_stride,
                        const int* seq_lens, int B, int Hq, int Hkv, int D, int S, float scale, hipStream_t s);
void k8sllm_decode_tw_force(int tw);
int k8sllm_paged_decode_fused(void* out, long out_stride, float* part_out, float* part_ml, const float* slabs,
                              int nslabs, const int* positions, const float* cos_sin, const int* slot_mapping,
                              void* k_cache, void* v_cache, const int* block_tables, int bt_stride,
                              const int* seq_lens, int B, int Hq, int Hkv, int D, int S, float scale, int* merge_ctr,
                              hipStream_t s);
int k8sllm_flash_prefill(void* out, long out_stride, const void* qkv, long qkv_stride, const int* cu_seqlens,
                         const int* qb_seq, const int* qb_start, int n_qblocks, int Hq, int Hkv, int D, float scale,
                         const int* ctx_start, const void* k_cache, const void* v_cache, const int* block_tables,
                         int bt_stride, hipStream_t s);
int k8sllm_sample(int* out, const void* logits, int is_fp32, long B, long stride, int V, const float* temps,
                  const int* top_k, const float* top_p, const int64_t* rng, float* pv, int* pi, int advance, hipStream_t s);
int k8sllm_sample_parts(long B, int V);
int k8sllm_moe_route(const void* logits, long T, int E, int K, int renorm, int* topk_ids, float* topk_w,
                     hipStream_t s);
int k8sllm_moe_router(const void* x, const void* wr, long T, int d, int E, int K, int renorm, int* ids, float* w,
                      float* wd, hipStream_t s);
int k8sllm_moe_align(const int* topk_ids, long n, int E, int* expert_offsets, int* sorted_idx, int* inv_idx,
                     hipStream_t s);
int k8sllm_moe_combine(void* out, const void* expert_out, const int* inv_idx, const float* topk_w, long T, int K,
                       int d, hipStream_t s);
int k8sllm_gather_rows(void* out, const void* x, const int* idx, long n, int d, int div, hipStream_t s);
int k8sllm_gemm_tile(const void* X, const void* W, void* Y, int M, int N, int K, const int* offsets, int E, long w_es,
                     int epi, int algo, const int* rope_pos, const float* rope_cs, int rope_heads,
                     const float* rs_part, int rs_np, float rs_eps, void* resid, void* hw, const void* norm_w,
                     float* ss_out, int wpk, hipStream_t s);
int k8sllm_moe_grouped_gemm(const void* X, const void* W, void* Y, const int* offsets, int E, long rows, int N, int K,
                            long w_es, int epi, hipStream_t s);
int k8sllm_gemm_skinny(const void* A, long lda, const void* Wp, float* partial, void* Y, long ldy, int M, int N, int K,
                       int S, int epi, int nt_tiles, int a_packed, const float* rn_ss, int rn_nc, int rn_d,
                       float rn_eps, int waves, int experts, long w_es, long a_es, long y_es,
                       const float* row_w, int row_w_ld, int w_rm, hipStream_t s);
int k8sllm_gemm_skinny_auto_splits(int M, int N, int K);
int k8sllm_gemm_dec(const void* A, const void* Wp, float* partial, void* Y, long ldy, int M, int N, int K, int splits,
                    int epi, int ntw, int waves, int depth, const float* rn_ss, int rn_nc, int rn_d, float rn_eps,
                    int experts, long a_es, long w_es, long y_es, const float* rw, int rw_ld, hipStream_t s);
int k8sllm_gemm_dec_rc(const void* A, const void* Wp, void* resid, const void* nw, void* xw, float* ss, int M, int N,
                       int K, hipStream_t s);
int k8sllm_add_norm_partial(void* out, long out_stride, void* residual, const float* partial, int S, int M,
                            const void* w, int d, float* ss_part, hipStream_t s);
int k8sllm_embed_norm_partial(void* out, long out_stride, void* residual, const int* ids, const int* src,
                              const int* prev, const void* emb, int vocab, const void* w, int M, int d,
                              float* ss_part, hipStream_t s);
int k8sllm_gemm_skinny_slabs(int K, int S);
int k8sllm_reduce_slabs(void* out, const float* partial, int S, long n, hipStream_t s);
int k8sllm_reduce_add_rmsnorm(void* out, void* residual, const float* partial, int S, int M, const void* w, int d,
                              float eps, long out_stride, void* out2, hipStream_t s);
void* k8sllm_car_create(int rank, int world, long max_elems, void* handles, int* err);
int k8sllm_car_handle_size();
int k8sllm_car_open(void* state, const void* all_handles);
int k8sllm_car_all_reduce(void* state, const void* in, void* out, long n, long spin_limit, int algo, hipStream_t s);
int k8sllm_car_fused_tail(void* state, const float* slabs, int ns, long slab_stride, void* residual, const void* w,
                          void* out, long ldo, int M, int d, float eps, int packed, long spin_limit, int algo,
                          hipStream_t s);
int k8sllm_car_error(void* state);
int k8sllm_car_all_gather(void* state, const void* in, void* out, long n, long spin_limit, hipStream_t s);
int k8sllm_car_all_to_all(void* state, const void* in, void* out, long n, long spin_limit, hipStream_t s);
int k8sllm_car_error_async(void* state, void* host_dst, hipStream_t s);
void k8sllm_car_destroy(void* state);
}

namespace {

hipStream_t cur() { return c10::hip::getCurrentHIPStream().stream(); }

void check(int rc, const char* what) { TORCH_CHECK(rc == 0, "k8sllm kernel launch failed: ", what, " rc=", rc); }

void dev_bf16(const torch::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, n, " must be bfloat16");
}

void dev_i32(const torch::Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == torch::kInt32, n, " must be int32");
  TORCH_CHECK(t.is_contiguous(), n, " must be contiguous");
}

void rms_norm(torch::Tensor out, torch::Tensor x, torch::Tensor w, double eps) {
  dev_bf16(out, "out"); dev_bf16(x, "x"); dev_bf16(w, "w");
  const int d = (int)x.size(-1);
  TORCH_CHECK(x.stride(-1) == 1 && out.stride(-1) == 1 && w.is_contiguous(), "rms_norm: inner dim must be contiguous");
  const long rows = x.numel() / d;
  const long xs = x.dim() > 1 ? x.stride(-2) : d, os = out.dim() > 1 ? out.stride(-2) : d;
  check(k8sllm_rmsnorm(out.data_ptr(), x.data_ptr(), nullptr, w.data_ptr(), rows, d, (float)eps, xs, os, cur()),
        "rms_norm");
}

void fused_add_rms_norm(torch::Tensor out, torch::Tensor x, torch::Tensor residual, torch::Tensor w, double eps) {
  dev_bf16(out, "out"); dev_bf16(x, "x"); dev_bf16(residual, "residual"); dev_bf16(w, "w");
  TORCH_CHECK(residual.is_contiguous() && w.is_contiguous() && x.stride(-1) == 1, "fused_add_rms_norm layout");
  const int d = (int)x.size(-1);
  const long rows = x.numel() / d;
  TORCH_CHECK(residual.numel() == rows * d, "residual shape");
  const long xs = x.dim() > 1 ? x.stride(-2) : d, os = out.dim() > 1 ? out.stride(-2) : d;
  check(k8sllm_rmsnorm(out.data_ptr(), x.data_ptr(), residual.data_ptr(), w.data_ptr(), rows, d, (float)eps, xs, os,
                       cur()),
        "fused_add_rms_norm");
}

void layer_norm(torch::Tensor out, torch::Tensor x, torch::Tensor w, torch::Tensor b, double eps) {
  dev_bf16(out, "out"); dev_bf16(x, "x"); dev_bf16(w, "w"); dev_bf16(b, "b");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "layer_norm: contiguous");
  const int d = (int)x.size(-1);
  check(k8sllm_layernorm(out.data_ptr(), x.data_ptr(), w.data_ptr(), b.data_ptr(), x.numel() / d, d, (float)eps, cur()),
        "layer_norm");
}

// interleaved: x columns are [64 gate | 64 up] per 128 (ops.interleave_gate_up) instead of [F | F]
void silu_mul(torch::Tensor out, torch::Tensor x, bool interleaved) {
  dev_bf16(out, "out"); dev_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous(), "silu_mul: contiguous");
  const int F = (int)out.size(-1);
  TORCH_CHECK(x.size(-1) == 2 * F, "silu_mul: x last dim must be 2*F");
  TORCH_CHECK(!interleaved || F % 64 == 0, "silu_mul: interleaved gate/up needs F % 64 == 0");
  check(k8sllm_silu_mul(out.data_ptr(), x.data_ptr(), out.numel() / F, F, interleaved ? 1 : 0, cur()), "silu_mul");
}

void gelu_tanh(torch::Tensor out, torch::Tensor x) {
  dev_bf16(out, "out"); dev_bf16(x, "x");
  TORCH_CHECK(x.is_contiguous() && out.is_contiguous() && x.numel() == out.numel(), "gelu: shape");
  check(k8sllm_gelu_tanh(out.data_ptr(), x.data_ptr(), x.numel(), cur()), "gelu_tanh");
}

void embedding(torch::Tensor out, torch::Tensor ids, torch::Tensor weight, int64_t vocab_start) {
  dev_bf16(out, "out"); dev_bf16(weight, "weight"); dev_i32(ids, "ids");
  TORCH_CHECK(weight.is_contiguous() && out.is_contiguous(), "embedding: contiguous");
  const int d = (int)weight.size(1);
  check(k8sllm_embedding(out.data_ptr(), ids.data_ptr<int>(), weight.data_ptr(), ids.numel(), d, (int)vocab_start,
                         (int)weight.size(0), cur()),
        "embedding");
}

void resolve_ids(torch::Tensor out, torch::Tensor ids, torch::Tensor src, torch::Tensor prev) {
  dev_i32(out, "out"); dev_i32(ids, "ids"); dev_i32(src, "src"); dev_i32(prev, "prev");
  TORCH_CHECK(out.is_contiguous() && ids.is_contiguous() && src.is_contiguous() && prev.is_contiguous(),
              "resolve_ids: contiguous");
  TORCH_CHECK(ids.numel() == out.numel() && src.numel() == out.numel(), "resolve_ids: sizes");
  check(k8sllm_resolve_ids(out.data_ptr<int>(), ids.data_ptr<int>(), src.data_ptr<int>(), prev.data_ptr<int>(),
                           (int)out.numel(), cur()),
        "resolve_ids");
}

void rope_and_cache(torch::Tensor qkv, torch::Tensor positions, torch::Tensor cos_sin, torch::Tensor k_cache,
                    torch::Tensor v_cache, torch::Tensor slot_mapping, int64_t Hq, int64_t Hkv, int64_t D,
                    bool apply_rope, c10::optional<torch::Tensor> partial, int64_t S) {
  dev_bf16(qkv, "qkv"); dev_i32(positions, "positions");
  TORCH_CHECK(qkv.stride(-1) == 1 && qkv.dim() == 2, "qkv must be [T, (Hq+2Hkv)*D] with unit inner stride");
  TORCH_CHECK(qkv.size(1) >= (Hq + 2 * Hkv) * D, "qkv width");
  TORCH_CHECK(cos_sin.scalar_type() == torch::kFloat32 && cos_sin.is_contiguous() && cos_sin.size(1) == D, "cos_sin");
  const bool has_cache = slot_mapping.numel() > 0;
  int block_size = 16;
  if (has_cache) {
    dev_i32(slot_mapping, "slot_mapping");
    dev_bf16(k_cache, "k_cache"); dev_bf16(v_cache, "v_cache");
    // k_cache [NB, Hkv, D/8, BS, 8], v_cache [NB, Hkv, D, BS]
    TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(1) == Hkv && k_cache.size(4) == 8, "k_cache layout");
    TORCH_CHECK(v_cache.dim() == 4 && v_cache.size(1) == Hkv && v_cache.size(2) == D, "v_cache layout");
    block_size = (int)k_cache.size(3);
  }
  const float* pp = nullptr;
  if (partial.has_value()) {  // qkv = sum of S fp32 split-K slabs [S][T][(Hq+2Hkv)*D]
    TORCH_CHECK(partial->is_cuda() && partial->scalar_type() == torch::kFloat32 && partial->is_contiguous(), "partial");
    TORCH_CHECK(partial->numel() >= S * qkv.size(0) * (Hq + 2 * Hkv) * D, "partial too small");
    pp = partial->data_ptr<float>();
  }
  check(k8sllm_rope_cache(qkv.data_ptr(), qkv.stride(0), positions.data_ptr<int>(), cos_sin.data_ptr<float>(),
                          has_cache ? k_cache.data_ptr() : nullptr, has_cache ? v_cache.data_ptr() : nullptr,
                          has_cache ? slot_mapping.data_ptr<int>() : nullptr, qkv.size(0), (int)Hq, (int)Hkv, (int)D,
                          block_size, apply_rope ? 1 : 0, pp, (int)S, cur()),
        "rope_and_cache");
}

void paged_decode(torch::Tensor out, torch::Tensor q, torch::Tensor k_cache, torch::Tensor v_cache,
                  torch::Tensor block_tables, torch::Tensor seq_lens, torch::Tensor part_out, torch::Tensor part_ml,
                  int64_t Hq, int64_t Hkv, int64_t D, double scale, int64_t splits) {
  dev_bf16(out, "out"); dev_bf16(q, "q"); dev_bf16(k_cache, "k_cache"); dev_bf16(v_cache, "v_cache");
  dev_i32(block_tables, "block_tables"); dev_i32(seq_lens, "seq_lens");
  TORCH_CHECK(q.dim() == 2 && q.stride(1) == 1, "q must be [B, >=Hq*D] rows");
  const bool packed = out.dim() == 4;  // fragment-packed [ceil(B/16), Hq*D/32, 64, 8] for gemm_skinny
  if (packed) {
    TORCH_CHECK(out.is_contiguous() && out.size(1) * 32 == Hq * D && out.size(2) == 64 && out.size(3) == 8 &&
                    out.size(0) * 16 >= seq_lens.size(0),
                "packed out must be [ceil(B/16), Hq*D/32, 64, 8]");
  } else {
    TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) == Hq * D, "out must be [B, Hq*D]");
  }
  TORCH_CHECK(k_cache.size(3) == 16 && v_cache.size(3) == 16, "paged_decode expects block_size 16");
  TORCH_CHECK(part_out.scalar_type() == torch::kFloat32 && part_ml.scalar_type() == torch::kFloat32, "partials fp32");
  const int B = (int)seq_lens.size(0);
  TORCH_CHECK(splits >= 1 && splits <= 64, "splits must be in [1, 64]");
  TORCH_CHECK(part_out.numel() >= (int64_t)B * Hq * splits * D && part_ml.numel() >= (int64_t)B * Hq * splits * 2,
              "decode workspace too small for batch x splits");
  check(k8sllm_paged_decode(out.data_ptr(), packed ? -(long)(Hq * D / 32) : (long)out.stride(0),
                            part_out.data_ptr<float>(), part_ml.data_ptr<float>(),
                            q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                            block_tables.data_ptr<int>(), (int)block_tables.stride(0), seq_lens.data_ptr<int>(), B,
                            (int)Hq, (int)Hkv, (int)D, (int)splits, (float)scale, cur()),
        "paged_decode");
}

// paged_decode with the new token's q / k / v taken from the qkv projection's fp32 split-K slabs
// [nslabs, B, (Hq + 2 Hkv) * D] (summed, rounded, RoPE at positions, k / v written to the cache at
// slot_mapping inside the attention kernel: rope_and_cache folded in).  D = 128.
void paged_decode_fused(torch::Tensor out, torch::Tensor slabs, int64_t nslabs, torch::Tensor positions,
                        torch::Tensor cos_sin, torch::Tensor slot_mapping, torch::Tensor k_cache,
                        torch::Tensor v_cache, torch::Tensor block_tables, torch::Tensor seq_lens,
                        torch::Tensor part_out, torch::Tensor part_ml, int64_t Hq, int64_t Hkv, int64_t D,
                        double scale, int64_t splits, torch::Tensor merge_ctr) {
  dev_bf16(out, "out"); dev_bf16(k_cache, "k_cache"); dev_bf16(v_cache, "v_cache");
  dev_i32(block_tables, "block_tables"); dev_i32(seq_lens, "seq_lens"); dev_i32(positions, "positions");
  TORCH_CHECK(D == 128, "paged_decode_fused: head_dim 128");
  const int B = (int)seq_lens.size(0);
  TORCH_CHECK(slabs.is_cuda() && slabs.scalar_type() == torch::kFloat32 && slabs.is_contiguous() &&
                  slabs.numel() >= nslabs * B * (Hq + 2 * Hkv) * D && nslabs >= 1,
              "paged_decode_fused: slabs must hold nslabs x [B, (Hq + 2 Hkv) * D] fp32");
  TORCH_CHECK(positions.numel() >= B, "paged_decode_fused: positions [B]");
  TORCH_CHECK(cos_sin.is_cuda() && cos_sin.scalar_type() == torch::kFloat32 && cos_sin.is_contiguous() &&
                  cos_sin.size(1) == D, "paged_decode_fused: cos_sin [max_pos, D] fp32");
  const bool has_slots = slot_mapping.numel() > 0;
  if (has_slots) {
    dev_i32(slot_mapping, "slot_mapping");
    TORCH_CHECK(slot_mapping.numel() >= B, "paged_decode_fused: slot_mapping [B]");
  }
  const bool packed = out.dim() == 4;
  if (packed) {
    TORCH_CHECK(out.is_contiguous() && out.size(1) * 32 == Hq * D && out.size(2) == 64 && out.size(3) == 8 &&
                    out.size(0) * 16 >= B, "packed out must be [ceil(B/16), Hq*D/32, 64, 8]");
  } else {
    TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) == Hq * D, "out must be [B, Hq*D]");
  }
  TORCH_CHECK(k_cache.dim() == 5 && k_cache.size(1) == Hkv && k_cache.size(3) == 16 && v_cache.size(3) == 16,
              "paged_decode_fused: caches [NB, Hkv, D/8, 16, 8] / [NB, Hkv, D, 16]");
  TORCH_CHECK(splits >= 1 && splits <= 64, "splits must be in [1, 64]");
  TORCH_CHECK(part_out.numel() >= (int64_t)B * Hq * splits * D && part_ml.numel() >= (int64_t)B * Hq * splits * 2,
              "decode workspace too small for batch x splits");
  // merge_ctr (numel > 0): B x Hkv int32 counters, zero between launches (the kernel resets them)
  const bool merge = merge_ctr.numel() > 0;
  if (merge) {
    dev_i32(merge_ctr, "merge_ctr");
    TORCH_CHECK(merge_ctr.numel() >= (int64_t)B * Hkv, "paged_decode_fused: merge_ctr must hold B x Hkv counters");
  }
  check(k8sllm_paged_decode_fused(out.data_ptr(), packed ? -(long)(Hq * D / 32) : (long)out.stride(0),
                                  part_out.data_ptr<float>(), part_ml.data_ptr<float>(), slabs.data_ptr<float>(),
                                  (int)nslabs, positions.data_ptr<int>(), cos_sin.data_ptr<float>(),
                                  has_slots ? slot_mapping.data_ptr<int>() : nullptr, k_cache.data_ptr(),
                                  v_cache.data_ptr(), block_tables.data_ptr<int>(), (int)block_tables.stride(0),
                                  seq_lens.data_ptr<int>(), B, (int)Hq, (int)Hkv, (int)D, (int)splits, (float)scale,
                                  merge ? merge_ctr.data_ptr<int>() : nullptr, cur()),
        "paged_decode_fused");
}

// paged (optional, all or none): ctx_start [S] (cached tokens before each sequence's new rows),
// k_cache / v_cache (already holding the new tokens), block_tables [S, W] -> attention over the
// whole context from the paged cache (prefix caching / chunked prefill).
void flash_prefill(torch::Tensor out, torch::Tensor qkv, torch::Tensor cu_seqlens, torch::Tensor qb_seq,
                   torch::Tensor qb_start, int64_t Hq, int64_t Hkv, int64_t D, double scale,
                   c10::optional<torch::Tensor> ctx_start, c10::optional<torch::Tensor> k_cache,
                   c10::optional<torch::Tensor> v_cache, c10::optional<torch::Tensor> block_tables) {
  dev_bf16(out, "out"); dev_bf16(qkv, "qkv");
  dev_i32(cu_seqlens, "cu_seqlens"); dev_i32(qb_seq, "qb_seq"); dev_i32(qb_start, "qb_start");
  TORCH_CHECK(qkv.dim() == 2 && qkv.stride(1) == 1, "qkv rows");
  TORCH_CHECK(out.dim() == 2 && out.stride(1) == 1 && out.size(1) == Hq * D, "out must be [T, Hq*D]");
  const int* cs = nullptr;
  const void *kc = nullptr, *vc = nullptr;
  const int* bt = nullptr;
  int bts = 0;
  if (ctx_start.has_value()) {
    TORCH_CHECK(k_cache.has_value() && v_cache.has_value() && block_tables.has_value(), "paged prefill needs caches");
    dev_i32(*ctx_start, "ctx_start"); dev_i32(*block_tables, "block_tables");
    dev_bf16(*k_cache, "k_cache"); dev_bf16(*v_cache, "v_cache");
    TORCH_CHECK(k_cache->dim() == 5 && k_cache->size(1) == Hkv && k_cache->size(3) == 16 && k_cache->size(4) == 8,
                "k_cache layout [NB, Hkv, D/8, 16, 8]");
    TORCH_CHECK(v_cache->dim() == 4 && v_cache->size(1) == Hkv && v_cache->size(2) == D && v_cache->size(3) == 16,
                "v_cache layout [NB, Hkv, D, 16]");
    TORCH_CHECK(block_tables->dim() == 2 && block_tables->size(0) == cu_seqlens.numel() - 1, "block_tables [S, W]");
    cs = ctx_start->data_ptr<int>();
    kc = k_cache->data_ptr();
    vc = v_cache->data_ptr();
    bt = block_tables->data_ptr<int>();
    bts = (int)block_tables->stride(0);
  }
  check(k8sllm_flash_prefill(out.data_ptr(), out.stride(0), qkv.data_ptr(), qkv.stride(0), cu_seqlens.data_ptr<int>(),
                             qb_seq.data_ptr<int>(), qb_start.data_ptr<int>(), (int)qb_seq.numel(), (int)Hq, (int)Hkv,
                             (int)D, (float)scale, cs, kc, vc, bt, bts, cur()),
        "flash_prefill");
}

void sample(torch::Tensor out, torch::Tensor logits, c10::optional<torch::Tensor> temps,
            c10::optional<torch::Tensor> top_k, c10::optional<torch::Tensor> top_p, c10::optional<torch::Tensor> rng,
            bool advance) {
  dev_i32(out, "out");
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1, "logits [B, V]");
  const bool f32 = logits.scalar_type() == torch::kFloat32;
  TORCH_CHECK(f32 || logits.scalar_type() == torch::kBFloat16, "logits must be fp32 or bf16");
  const float* t = temps && temps->numel() ? temps->data_ptr<float>() : nullptr;
  const int* k = top_k && top_k->numel() ? top_k->data_ptr<int>() : nullptr;
  const float* p = top_p && top_p->numel() ? top_p->data_ptr<float>() : nullptr;
  const int64_t* r = rng && rng->numel() ? rng->data_ptr<int64_t>() : nullptr;
  const long B = logits.size(0);
  const int V = (int)logits.size(1);
  const int64_t np = B * k8sllm_sample_parts(B, V);
  // partial (value, index) workspace: stream-ordered caching allocator (graph-pool safe)
  auto pv = torch::empty({np}, logits.options().dtype(torch::kFloat32));
  auto pi = torch::empty({np}, logits.options().dtype(torch::kInt32));
  check(k8sllm_sample(out.data_ptr<int>(), logits.data_ptr(), f32 ? 1 : 0, B, logits.stride(0), V, t, k, p, r,
                      pv.data_ptr<float>(), pi.data_ptr<int>(), advance ? 1 : 0, cur()),
        "sample");
}

void moe_router(torch::Tensor x, torch::Tensor wr, torch::Tensor ids, torch::Tensor w, torch::Tensor wd, bool renorm) {
  dev_bf16(x, "x"); dev_bf16(wr, "router"); dev_i32(ids, "ids");
  TORCH_CHECK(x.is_contiguous() && x.dim() == 2 && wr.is_contiguous() && wr.dim() == 2 && wr.size(1) == x.size(1),
              "moe_router: x [T, d], router [E, d]");
  const long T = x.size(0);
  const int E = (int)wr.size(0), K = (int)ids.size(1);
  TORCH_CHECK(ids.dim() == 2 && ids.size(0) == T && w.is_cuda() && w.scalar_type() == torch::kFloat32 &&
                  w.sizes() == ids.sizes() && wd.is_cuda() && wd.scalar_type() == torch::kFloat32 &&
                  wd.is_contiguous() && wd.numel() == T * E, "moe_router: ids / w [T, K], wd [T, E] fp32");
  check(k8sllm_moe_router(x.data_ptr(), wr.data_ptr(), T, (int)x.size(1), E, K, renorm ? 1 : 0, ids.data_ptr<int>(),
                          w.data_ptr<float>(), wd.data_ptr<float>(), cur()),
        "moe_router");
}

void moe_route(torch::Tensor logits, torch::Tensor topk_ids, torch::Tensor topk_w, bool renorm) {
  TORCH_CHECK(logits.is_cuda() && logits.is_contiguous(), "router logits");
  TORCH_CHECK(logits.scalar_type() == torch::kFloat32, "router logits must be fp32");
  dev_i32(topk_ids, "topk_ids");
  const int E = (int)logits.size(1);
  const int K = (int)topk_ids.size(1);
  TORCH_CHECK(E <= 64 && K <= E, "moe_route supports up to 64 experts");
  check(k8sllm_moe_route(logits.data_ptr(), logits.size(0), E, K, renorm ? 1 : 0, topk_ids.data_ptr<int>(),
                         topk_w.data_ptr<float>(), cur()),
        "moe_route");
}

void moe_align(torch::Tensor topk_ids, int64_t E, torch::Tensor expert_offsets, torch::Tensor sorted_idx,
               torch::Tensor inv_idx) {
  dev_i32(topk_ids, "topk_ids"); dev_i32(expert_offsets, "expert_offsets");
  dev_i32(sorted_idx, "sorted_idx"); dev_i32(inv_idx, "inv_idx");
  TORCH_CHECK(expert_offsets.numel() == E + 1, "expert_offsets size");
  check(k8sllm_moe_align(topk_ids.data_ptr<int>(), topk_ids.numel(), (int)E, expert_offsets.data_ptr<int>(),
                         sorted_idx.data_ptr<int>(), inv_idx.data_ptr<int>(), cur()),
        "moe_align");
}

void moe_combine(torch::Tensor out, torch::Tensor expert_out, torch::Tensor inv_idx, torch::Tensor topk_w) {
  dev_bf16(out, "out"); dev_bf16(expert_out, "expert_out"); dev_i32(inv_idx, "inv_idx");
  TORCH_CHECK(out.is_contiguous() && expert_out.is_contiguous(), "moe_combine contiguous");
  const int d = (int)out.size(1);
  check(k8sllm_moe_combine(out.data_ptr(), expert_out.data_ptr(), inv_idx.data_ptr<int>(), topk_w.data_ptr<float>(),
                           out.size(0), (int)topk_w.size(1), d, cur()),
        "moe_combine");
}

// Grouped expert GEMM over expert-sorted rows (moe_gemm.hip): x [rows, K], w [E, N, K], offsets
// [E + 1] int32 absolute row offsets of the experts in x (device, from moe_align; no host sync).
// swiglu: w gate/up-interleaved per 128 rows, y [rows, N / 2] = silu(gate) * up; else y [rows, N].
// Rows outside [offsets[0], offsets[E]) are not written.
void moe_grouped_gemm(torch::Tensor y, torch::Tensor x, torch::Tensor w, torch::Tensor offsets, bool swiglu) {
  dev_bf16(y, "y"); dev_bf16(x, "x"); dev_bf16(w, "w"); dev_i32(offsets, "offsets");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && w.dim() == 3 && w.is_contiguous() && y.is_contiguous(),
              "moe_grouped_gemm: x [rows, K], w [E, N, K] contiguous");
  const int E = (int)w.size(0), N = (int)w.size(1), K = (int)w.size(2);
  TORCH_CHECK(x.size(1) == K, "moe_grouped_gemm: K mismatch");
  TORCH_CHECK(offsets.numel() == E + 1, "moe_grouped_gemm: offsets must hold E + 1 entries");
  TORCH_CHECK(N % 128 == 0 && K % 64 == 0, "moe_grouped_gemm: N % 128 == 0 and K % 64 == 0");
  TORCH_CHECK(y.size(0) == x.size(0) && y.size(1) == (swiglu ? N / 2 : N), "moe_grouped_gemm: y shape");
  check(k8sllm_moe_grouped_gemm(x.data_ptr(), w.data_ptr(), y.data_ptr(), offsets.data_ptr<int>(), E, x.size(0), N, K,
                                (long)N * K, swiglu ? 1 : 0, cur()),
        "moe_grouped_gemm");
}

// 256 x 256 MFMA GEMM (gemm_tile.hip) for prefill-sized projections: y = x . w^T, x [M, K], w [N, K]
// (dense, offsets None) or w [E, N, K] with device offsets [E + 1] (grouped over expert-sorted rows,
// no host sync).  swiglu: w gate/up-interleaved per 128 rows, y [M, N / 2] = silu(gate) * up.
// rope_pos / rope_cs (dense, N % 128 == 0): the qkv projection with the rotary embedding of heads
// 0 .. rope_heads - 1 (q and k, head_dim 128) applied in the epilogue (TILE_EPI_ROPE)
// swiglu: 0 none, 1 = gate/up interleaved per 128 rows (interleave_gate_up), 8 = per 16 rows
// (interleave_gate_up8, the decode GEMMs' packed copy)
void gemm_tile(torch::Tensor y, torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> offsets, int64_t swiglu,
               int64_t algo, c10::optional<torch::Tensor> rope_pos, c10::optional<torch::Tensor> rope_cs,
               int64_t rope_heads, c10::optional<torch::Tensor> rs_part, double rs_eps,
               c10::optional<torch::Tensor> resid, c10::optional<torch::Tensor> hw,
               c10::optional<torch::Tensor> norm_w, c10::optional<torch::Tensor> ss_out) {
  dev_bf16(y, "y"); dev_bf16(x, "x"); dev_bf16(w, "w");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && w.is_contiguous() && y.is_contiguous(),
              "gemm_tile: x [M, K], w contiguous, y contiguous");
  const bool grouped = offsets.has_value();
  // w row-major [N, K] / [E, N, K], or fragment-packed [N/16, K/32, 64, 8] / [E, ...] (pack_skinny)
  const bool wpk = w.dim() == (grouped ? 5 : 4);
  TORCH_CHECK(w.dim() == (grouped ? 3 : 2) || (wpk && w.size(-2) == 64 && w.size(-1) == 8),
              "gemm_tile: w [N, K] (dense) or [E, N, K] (grouped), or their fragment-packed forms");
  const int E = grouped ? (int)w.size(0) : 1;
  const int N = wpk ? (int)w.size(w.dim() - 4) * 16 : (int)w.size(w.dim() - 2);
  const int K = wpk ? (int)w.size(w.dim() - 3) * 32 : (int)w.size(w.dim() - 1);
  const int M = (int)x.size(0);
  TORCH_CHECK(x.size(1) == K, "gemm_tile: K mismatch");
  TORCH_CHECK(algo >= 0 && algo <= 1, "gemm_tile: algo 0 (one barrier per k-tile) or 1 (two)");
  TORCH_CHECK(N % 16 == 0 && K % 64 == 0 && K >= 64 && (!swiglu || N % 256 == 0),
              "gemm_tile: N % 16 == 0 (SwiGLU: % 256), K % 64 == 0");
  TORCH_CHECK(y.dim() == 2 && y.size(0) == M && y.size(1) == (swiglu ? N / 2 : N), "gemm_tile: y shape");
  const int* op = nullptr;
  if (grouped) {
    dev_i32(*offsets, "offsets");
    TORCH_CHECK(offsets->numel() == E + 1, "gemm_tile: offsets must hold E + 1 entries");
    op = offsets->data_ptr<int>();
  }
  const int* rp = nullptr;
  const float* rc = nullptr;
  if (rope_pos.has_value()) {
    TORCH_CHECK(!grouped && !swiglu && rope_cs.has_value() && N % 128 == 0, "gemm_tile: rope epilogue is dense qkv");
    dev_i32(*rope_pos, "rope_pos");
    TORCH_CHECK(rope_pos->numel() >= M, "gemm_tile: rope_pos needs a position per row");
    TORCH_CHECK(rope_heads >= 0 && rope_heads * 128 <= N, "gemm_tile: rope_heads * 128 must fit in N");
    TORCH_CHECK(rope_cs->is_cuda() && rope_cs->scalar_type() == torch::kFloat32 && rope_cs->is_contiguous() &&
                    rope_cs->dim() == 2 && rope_cs->size(1) == 128,
                "gemm_tile: rope_cs must be [max_pos, 128] fp32 (head_dim 128)");
    rp = rope_pos->data_ptr<int>();
    rc = rope_cs->data_ptr<float>();
  }
  // row scale (deferred RMSNorm of the A rows): rs_part [M][K / 128] fp32 partial sums of squares
  const float* rsp = nullptr;
  int rs_np = 0;
  if (rs_part.has_value()) {
    TORCH_CHECK(!grouped && K % 128 == 0, "gemm_tile: row scale needs dense, K % 128 == 0");
    TORCH_CHECK(rs_part->is_cuda() && rs_part->scalar_type() == torch::kFloat32 && rs_part->is_contiguous() &&
                    rs_part->dim() == 2 && rs_part->size(0) >= M && rs_part->size(1) == K / 128,
                "gemm_tile: rs_part must be [M, K / 128] fp32");
    rsp = rs_part->data_ptr<float>();
    rs_np = K / 128;
  }
  // residual epilogue: resid [M][N] += y (in place), hw = resid * norm_w, ss_out [M][N / 128]
  const bool rsd = resid.has_value();
  if (rsd) {
    TORCH_CHECK(!grouped && !swiglu && !rp && !rsp && N % 128 == 0 && hw.has_value() && norm_w.has_value() &&
                    ss_out.has_value(), "gemm_tile: residual epilogue is dense, N % 128 == 0, with hw / norm_w / ss_out");
    dev_bf16(*resid, "resid"); dev_bf16(*hw, "hw"); dev_bf16(*norm_w, "norm_w");
    TORCH_CHECK(resid->is_contiguous() && resid->dim() == 2 && resid->size(0) == M && resid->size(1) == N,
                "gemm_tile: resid [M, N]");
    TORCH_CHECK(hw->is_contiguous() && hw->dim() == 2 && hw->size(0) == M && hw->size(1) == N, "gemm_tile: hw [M, N]");
    TORCH_CHECK(norm_w->is_contiguous() && norm_w->numel() == N, "gemm_tile: norm_w [N]");
    TORCH_CHECK(ss_out->is_cuda() && ss_out->scalar_type() == torch::kFloat32 && ss_out->is_contiguous() &&
                    ss_out->numel() >= (long)M * (N / 128), "gemm_tile: ss_out [M, N / 128] fp32");
  }
  TORCH_CHECK(swiglu == 0 || swiglu == 1 || swiglu == 8, "gemm_tile: swiglu 0, 1 or 8");
  const int epi = rsd ? 3 : rp ? 2 : (swiglu == 8 ? 4 : swiglu ? 1 : 0);
  check(k8sllm_gemm_tile(x.data_ptr(), w.data_ptr(), rsd ? resid->data_ptr() : y.data_ptr(), M, N, K, op, E,
                         (long)N * K, epi, (int)algo, rp, rc, (int)rope_heads, rsp, rs_np, (float)rs_eps,
                         rsd ? resid->data_ptr() : nullptr, rsd ? hw->data_ptr() : nullptr,
                         rsd ? norm_w->data_ptr() : nullptr, rsd ? ss_out->data_ptr<float>() : nullptr, wpk ? 1 : 0,
                         cur()),
        "gemm_tile");
}

void gather_rows(torch::Tensor out, torch::Tensor x, torch::Tensor idx, int64_t div) {
  dev_bf16(out, "out"); dev_bf16(x, "x"); dev_i32(idx, "idx");
  TORCH_CHECK(out.is_contiguous() && x.is_contiguous(), "gather_rows contiguous");
  check(k8sllm_gather_rows(out.data_ptr(), x.data_ptr(), idx.data_ptr<int>(), idx.numel(), (int)x.size(1), (int)div,
                           cur()),
        "gather_rows");
}

}  // namespace

// Deferred RMSNorm operand: per-row partial sums of squares [M, nc] over nc equal column chunks
// of the K columns (add_norm_partial: 512-column chunks; the RESNORM epilogue: one per workgroup).
static void rownorm_args(const c10::optional<torch::Tensor>& rn_ss, int M, int K, const float*& rp, int& rn_nc) {
  if (!rn_ss.has_value()) return;
  TORCH_CHECK(rn_ss->is_cuda() && rn_ss->scalar_type() == torch::kFloat32 && rn_ss->is_contiguous() &&
                  rn_ss->dim() == 2 && rn_ss->size(0) >= M && rn_ss->size(1) >= 1 && K % rn_ss->size(1) == 0,
              "gemm_skinny: rn_ss must be [M, nc] fp32 with nc | K");
  rp = rn_ss->data_ptr<float>();
  rn_nc = (int)rn_ss->size(1);
}

// Weight of a skinny GEMM: fragment-packed [N/16, K/32, 64, 8] (a decode-only copy), or the
// row-major [N, K] tensor itself (gemm_skinny_rm_kernel, the single resident copy prefill's GEMMs
// read as well).  `lead` = leading (expert) dimensions.  Returns w_rm.
static int skinny_weight_dims(const torch::Tensor& wp, int lead, int& N, int& K, const char* what) {
  TORCH_CHECK(wp.is_contiguous(), what, ": weight must be contiguous");
  if (wp.dim() == lead + 4 && wp.size(lead + 2) == 64 && wp.size(lead + 3) == 8) {
    N = (int)wp.size(lead) * 16;
    K = (int)wp.size(lead + 1) * 32;
    return 0;
  }
  TORCH_CHECK(wp.dim() == lead + 2, what, ": weight must be fragment-packed [N/16, K/32, 64, 8] or row-major [N, K]");
  N = (int)wp.size(lead);
  K = (int)wp.size(lead + 1);
  TORCH_CHECK(N % 64 == 0 && K % 64 == 0, what, ": row-major weight needs N % 64 == 0 and K % 64 == 0");
  return 1;
}

// Skinny decode GEMM over a fragment-packed weight wp [N/16][K/32][64][8] or the row-major [N][K]
// weight (gemm_skinny.hip).
// epi 0: fp32 split-K slabs partial[S'][M][N], returns S'; epi 1: y = bf16(a . W^T);
// epi 2: y[M, N/2] = silu(gate) * up over a [32 gate | 32 up]-interleaved weight; epi 3: the same
// written fragment-packed.  Returns the
// number of slabs written (1 for epi 1/2).
int64_t gemm_skinny(torch::Tensor a, torch::Tensor wp, c10::optional<torch::Tensor> partial,
                    c10::optional<torch::Tensor> y, int64_t splits, int64_t epi, int64_t nt_tiles, int64_t rows,
                    c10::optional<torch::Tensor> rn_ss, double rn_eps, int64_t waves) {
  dev_bf16(a, "a"); dev_bf16(wp, "wp");
  int N, K;
  const int w_rm = skinny_weight_dims(wp, 0, N, K, "gemm_skinny");
  const bool a_packed = a.dim() == 4;
  TORCH_CHECK(!w_rm || a_packed, "gemm_skinny: a row-major weight needs a fragment-packed a");
  int M;
  if (a_packed) {  // fragment-packed activations [ceil(M/16), K/32, 64, 8]; `rows` = valid rows
    TORCH_CHECK(a.is_contiguous() && a.size(1) * 32 == K && a.size(2) == 64 && a.size(3) == 8,
                "gemm_skinny: packed a must be [ceil(M/16), K/32, 64, 8]");
    M = (int)rows;
    TORCH_CHECK(M > 0 && (M + 15) / 16 <= a.size(0), "gemm_skinny: rows exceed the packed a");
  } else {
    TORCH_CHECK(a.dim() == 2 && a.stride(1) == 1 && a.stride(0) % 8 == 0, "gemm_skinny: a layout");
    TORCH_CHECK(a.size(1) == K, "gemm_skinny: a has ", a.size(1), " columns, weight K=", K);
    M = (int)a.size(0);
  }
  TORCH_CHECK(M <= 64, "gemm_skinny: at most 64 rows");
  TORCH_CHECK(N % (16 * nt_tiles) == 0, "gemm_skinny: N not divisible by the workgroup tile");
  if (epi == 0 && splits <= 0) splits = k8sllm_gemm_skinny_auto_splits(M, N, K);
  const int S = epi == 0 ? k8sllm_gemm_skinny_slabs(K, (int)splits) : 1;
  float* pp = nullptr;
  void* yp = nullptr;
  long ldy = 0;
  if (epi == 0) {
    TORCH_CHECK(partial.has_value(), "gemm_skinny: split-K needs a partial buffer");
    TORCH_CHECK(partial->is_cuda() && partial->scalar_type() == torch::kFloat32 && partial->is_contiguous(),
                "partial must be contiguous fp32 on the GPU");
    TORCH_CHECK(partial->numel() >= (int64_t)S * M * N, "partial buffer too small");
    pp = partial->data_ptr<float>();
  } else {
    TORCH_CHECK(y.has_value(), "gemm_skinny: output tensor required");
    dev_bf16(*y, "y");
    if (epi == 3) {  // SwiGLU written fragment-packed [ceil(M/16), F/32, 64, 8]
      TORCH_CHECK(y->dim() == 4 && y->is_contiguous() && y->size(0) * 16 >= M && y->size(1) * 64 == N &&
                      y->size(2) == 64 && y->size(3) == 8,
                  "gemm_skinny: packed SwiGLU output must be [ceil(M/16), F/32, 64, 8]");
      TORCH_CHECK(y->size(0) == (M + 15) / 16, "gemm_skinny: packed output m-tiles");
    } else {
      const int ncol = epi == 2 ? N / 2 : N;
      TORCH_CHECK(y->dim() == 2 && y->size(0) >= M && y->size(1) == ncol && y->stride(1) == 1,
                  "gemm_skinny: y shape");
      ldy = y->stride(0);
    }
    yp = y->data_ptr();
  }
  const float* rp = nullptr;
  int rn_nc = 0;
  rownorm_args(rn_ss, M, K, rp, rn_nc);
  check(k8sllm_gemm_skinny(a.data_ptr(), a_packed ? 0 : a.stride(0), wp.data_ptr(), pp, yp, ldy, M, N, K,
                           epi == 0 ? (int)splits : 1, (int)epi, (int)nt_tiles, a_packed ? 1 : 0, rp, rn_nc, K,
                           (float)rn_eps, (int)waves, 1, 0, 0, 0, nullptr, 0, w_rm, cur()),
        "gemm_skinny");
  return S;
}

// Decode GEMM over a fragment-packed weight copy with A shared through LDS (gemm_decode.hip):
// a packed [ceil(M/16), K/32, 64, 8] (`rows` valid), wp packed [N/16, K/32, 64, 8] (for epi 2 the
// rows interleaved per 16-row n-tile as [8 gate | 8 up]).  epi 0: fp32 slabs partial[S][M][N],
// returns S = splits; epi 1: y [M, N] bf16 (row stride y.stride(0)); epi 2: packed SwiGLU
// y [ceil(M/16), N/64, 64, 8].  Returns the slab count (1 for epi 1/2); -1 if the configuration
// is not available (the caller falls back to gemm_skinny).
int64_t gemm_dec(torch::Tensor a, torch::Tensor wp, c10::optional<torch::Tensor> partial, c10::optional<torch::Tensor> y,
                 int64_t splits, int64_t epi, int64_t ntw, int64_t waves, int64_t depth, int64_t rows,
                 c10::optional<torch::Tensor> rn_ss, double rn_eps) {
  dev_bf16(a, "a"); dev_bf16(wp, "wp");
  TORCH_CHECK(wp.dim() == 4 && wp.is_contiguous() && wp.size(2) == 64 && wp.size(3) == 8,
              "gemm_dec: wp must be fragment-packed [N/16, K/32, 64, 8]");
  const int N = (int)wp.size(0) * 16, K = (int)wp.size(1) * 32, M = (int)rows;
  TORCH_CHECK(a.dim() == 4 && a.is_contiguous() && a.size(1) * 32 == K && a.size(2) == 64 && a.size(3) == 8,
              "gemm_dec: a must be fragment-packed [ceil(M/16), K/32, 64, 8]");
  TORCH_CHECK(M > 0 && M <= 64 && (M + 15) / 16 <= a.size(0), "gemm_dec: 1..64 rows within the packed a");
  float* pp = nullptr;
  void* yp = nullptr;
  long ldy = 0;
  if (epi == 0) {
    TORCH_CHECK(partial.has_value() && partial->is_cuda() && partial->scalar_type() == torch::kFloat32 &&
                    partial->is_contiguous() && partial->numel() >= splits * M * N,
                "gemm_dec: partial must be contiguous fp32 with splits x M x N elements");
    pp = partial->data_ptr<float>();
  } else {
    TORCH_CHECK(splits == 1, "gemm_dec: bf16 / SwiGLU epilogues need splits == 1");
    TORCH_CHECK(y.has_value(), "gemm_dec: output tensor required");
    dev_bf16(*y, "y");
    if (epi == 2) {
      TORCH_CHECK(y->dim() == 4 && y->is_contiguous() && y->size(0) == (M + 15) / 16 && y->size(1) * 64 == N &&
                      y->size(2) == 64 && y->size(3) == 8,
                  "gemm_dec: packed SwiGLU output must be [ceil(M/16), N/64, 64, 8]");
    } else {
      TORCH_CHECK(y->dim() == 2 && y->size(0) >= M && y->size(1) == N && y->stride(1) == 1, "gemm_dec: y [M, N]");
      ldy = y->stride(0);
    }
    yp = y->data_ptr();
  }
  const float* rp = nullptr;
  int rn_nc = 0;
  rownorm_args(rn_ss, M, K, rp, rn_nc);
  const int rc = k8sllm_gemm_dec(a.data_ptr(), wp.data_ptr(), pp, yp, ldy, M, N, K, (int)splits, (int)epi, (int)ntw,
                                 (int)waves, (int)depth, rp, rn_nc, K, (float)rn_eps, 1, 0, 0, 0, nullptr, 0, cur());
  if (rc < 0) return -1;
  check(rc, "gemm_dec");
  return epi == 0 ? splits : 1;
}

// Grouped decode GEMM over the local experts of a MoE layer (grid.z = expert): wp [E, N/16, K/32,
// 64, 8]; a packed [ceil(M/16), K/32, 64, 8] shared by every expert (gate_up) or [E, ceil(M/16),
// K/32, 64, 8] per expert (down).  epi 2: y [E, ceil(M/16), N/64, 64, 8] packed SwiGLU per expert;
// epi 0: fp32 slabs [E * splits, M, N] scaled by row_w [M, E] (the routing weights of these
// experts).  Returns the slab count (epi 0) or 1; -1 for a shape / configuration it does not take.
int64_t gemm_dec_grouped(torch::Tensor a, torch::Tensor wp, c10::optional<torch::Tensor> partial,
                         c10::optional<torch::Tensor> y, int64_t splits, int64_t epi, int64_t ntw, int64_t waves,
                         int64_t depth, int64_t rows, c10::optional<torch::Tensor> row_w) {
  dev_bf16(a, "a"); dev_bf16(wp, "wp");
  TORCH_CHECK(wp.dim() == 5 && wp.is_contiguous() && wp.size(3) == 64 && wp.size(4) == 8,
              "gemm_dec_grouped: wp must be [E, N/16, K/32, 64, 8]");
  const int E = (int)wp.size(0), N = (int)wp.size(1) * 16, K = (int)wp.size(2) * 32, M = (int)rows;
  const int MT = (M + 15) / 16;
  TORCH_CHECK(M > 0 && M <= 64 && E >= 1, "gemm_dec_grouped: 1..64 rows, >= 1 expert");
  const bool per_e = a.dim() == 5;
  TORCH_CHECK(a.is_contiguous() && (per_e ? (a.size(0) == E && a.size(1) >= MT && a.size(2) * 32 == K &&
                                             a.size(3) == 64 && a.size(4) == 8)
                                          : (a.dim() == 4 && a.size(0) >= MT && a.size(1) * 32 == K &&
                                             a.size(2) == 64 && a.size(3) == 8)),
              "gemm_dec_grouped: a packed [ceil(M/16), K/32, 64, 8] or [E, ...]");
  const long a_es = per_e ? a.stride(0) : 0, w_es = wp.stride(0);
  float* pp = nullptr;
  void* yp = nullptr;
  long y_es = 0;
  const float* rw = nullptr;
  int rw_ld = 0;
  if (epi == 0) {
    TORCH_CHECK(partial.has_value() && partial->is_cuda() && partial->scalar_type() == torch::kFloat32 &&
                    partial->is_contiguous() && partial->numel() >= (long)E * splits * M * N,
                "gemm_dec_grouped: partial must hold E x splits x M x N fp32");
    pp = partial->data_ptr<float>();
    if (row_w.has_value()) {
      TORCH_CHECK(row_w->is_cuda() && row_w->scalar_type() == torch::kFloat32 && row_w->dim() == 2 &&
                      row_w->size(0) >= M && row_w->size(1) == E && row_w->stride(1) == 1,
                  "gemm_dec_grouped: row_w [M, E] fp32");
      rw = row_w->data_ptr<float>();
      rw_ld = (int)row_w->stride(0);
    }
  } else {
    TORCH_CHECK(epi == 2 && splits == 1 && y.has_value(), "gemm_dec_grouped: SwiGLU output needs splits 1 and y");
    dev_bf16(*y, "y");
    TORCH_CHECK(y->dim() == 5 && y->is_contiguous() && y->size(0) == E && y->size(1) == MT && y->size(2) * 64 == N &&
                    y->size(3) == 64 && y->size(4) == 8, "gemm_dec_grouped: y [E, ceil(M/16), N/64, 64, 8]");
    yp = y->data_ptr();
    y_es = y->stride(0);
  }
  const int rc = k8sllm_gemm_dec(a.data_ptr(), wp.data_ptr(), pp, yp, 0, M, N, K, (int)splits, (int)epi, (int)ntw,
                                 (int)waves, (int)depth, nullptr, 0, K, 0.f, E, a_es, w_es, y_es, rw, rw_ld, cur());
  if (rc < 0) return -1;
  check(rc, "gemm_dec_grouped");
  return epi == 0 ? (int64_t)E * splits : 1;
}

// Row-complete decode GEMM + residual add + deferred-norm operands (gemm_decode.hip
// gemm_dec_rc_kernel): a packed [ceil(M/16), K/32, 64, 8] (`rows` valid), wp packed [N/16, K/32,
// 64, 8]; resid [M, N] bf16 += a . wp^T (in place); xw packed [ceil(M/16), N/32, 64, 8] = resid *
// nw; ss [M, N/16] fp32 per-16-column sums of resid^2.  Returns false for a shape it does not tile.
bool gemm_dec_rc(torch::Tensor a, torch::Tensor wp, torch::Tensor resid, torch::Tensor nw, torch::Tensor xw,
                 torch::Tensor ss, int64_t rows) {
  dev_bf16(a, "a"); dev_bf16(wp, "wp"); dev_bf16(resid, "resid"); dev_bf16(nw, "nw"); dev_bf16(xw, "xw");
  TORCH_CHECK(wp.dim() == 4 && wp.is_contiguous() && wp.size(2) == 64 && wp.size(3) == 8, "gemm_dec_rc: wp packed");
  const int N = (int)wp.size(0) * 16, K = (int)wp.size(1) * 32, M = (int)rows;
  TORCH_CHECK(a.dim() == 4 && a.is_contiguous() && a.size(1) * 32 == K && a.size(2) == 64 && a.size(3) == 8 &&
                  M > 0 && M <= 64 && (M + 15) / 16 <= a.size(0), "gemm_dec_rc: a packed [ceil(M/16), K/32, 64, 8]");
  TORCH_CHECK(resid.dim() == 2 && resid.is_contiguous() && resid.size(0) >= M && resid.size(1) == N,
              "gemm_dec_rc: resid [M, N]");
  TORCH_CHECK(nw.numel() == N && nw.is_contiguous(), "gemm_dec_rc: nw [N]");
  TORCH_CHECK(xw.dim() == 4 && xw.is_contiguous() && xw.size(0) == (M + 15) / 16 && xw.size(1) * 32 == N,
              "gemm_dec_rc: xw packed [ceil(M/16), N/32, 64, 8]");
  TORCH_CHECK(ss.is_cuda() && ss.scalar_type() == torch::kFloat32 && ss.is_contiguous() && ss.dim() == 2 &&
                  ss.size(0) >= M && ss.size(1) == N / 16, "gemm_dec_rc: ss [M, N/16] fp32");
  const int rc = k8sllm_gemm_dec_rc(a.data_ptr(), wp.data_ptr(), resid.data_ptr(), nw.data_ptr(), xw.data_ptr(),
                                    ss.data_ptr<float>(), M, N, K, cur());
  if (rc == -1) return false;
  check(rc, "gemm_dec_rc");
  return true;
}

// Grouped (MoE) skinny GEMM: wp [E, N/16, K/32, 64, 8] (one packed weight per local expert).
// a: packed [MT, K/32, 64, 8] shared by every expert, or [E, MT, K/32, 64, 8] per expert.
// epi 3: y = packed SwiGLU [E, MT, F/32, 64, 8]; epi 0: fp32 slabs partial[E * S'][M][N] with
// row m of expert x's output scaled by row_w[m][x] (row_w [M, E] fp32, routing weights).
// Returns E * S' (the slab count for the residual-add kernels) or 1.
int64_t gemm_skinny_grouped(torch::Tensor a, torch::Tensor wp, c10::optional<torch::Tensor> partial,
                            c10::optional<torch::Tensor> y, int64_t splits, int64_t epi, int64_t rows,
                            c10::optional<torch::Tensor> row_w, int64_t waves) {
  dev_bf16(a, "a"); dev_bf16(wp, "wp");
  int N, K;
  const int w_rm = skinny_weight_dims(wp, 1, N, K, "gemm_skinny_grouped");
  TORCH_CHECK(epi == 0 || epi == 3, "gemm_skinny_grouped: epi must be 0 (slabs) or 3 (packed SwiGLU)");
  const int E = (int)wp.size(0), M = (int)rows;
  const long w_es = wp[0].numel();
  TORCH_CHECK(M > 0 && (M <= 64 || (M <= 128 && w_rm && E > 1)),
              "gemm_skinny_grouped: 1..64 rows (1..128 over row-major expert weights)");
  const int MT = (M + 15) / 16;
  long a_es = 0;
  TORCH_CHECK(a.is_contiguous() && a.size(-1) == 8 && a.size(-2) == 64 && a.size(-3) * 32 == K,
              "gemm_skinny_grouped: a must be fragment-packed with K = ", K);
  if (a.dim() == 5) {
    TORCH_CHECK(a.size(0) == E && a.size(1) == MT, "gemm_skinny_grouped: per-expert a must be [E, MT, K/32, 64, 8]");
    a_es = a[0].numel();
  } else {
    TORCH_CHECK(a.dim() == 4 && a.size(0) == MT, "gemm_skinny_grouped: shared a must be [MT, K/32, 64, 8]");
  }
  float* pp = nullptr;
  void* yp = nullptr;
  long y_es = 0;
  const float* rw = nullptr;
  int S = 1;
  if (epi == 0) {
    if (splits <= 0) splits = 1;
    S = k8sllm_gemm_skinny_slabs(K, (int)splits);
    TORCH_CHECK(partial.has_value() && partial->is_cuda() && partial->scalar_type() == torch::kFloat32 &&
                    partial->is_contiguous() && partial->numel() >= (int64_t)E * S * M * N,
                "gemm_skinny_grouped: partial must be fp32 with room for E * S * M * N");
    pp = partial->data_ptr<float>();
    if (row_w.has_value()) {
      TORCH_CHECK(row_w->is_cuda() && row_w->scalar_type() == torch::kFloat32 && row_w->is_contiguous() &&
                      row_w->dim() == 2 && row_w->size(0) >= M && row_w->size(1) == E,
                  "gemm_skinny_grouped: row_w must be [M, E] fp32");
      rw = row_w->data_ptr<float>();
    }
  } else {
    TORCH_CHECK(y.has_value(), "gemm_skinny_grouped: output required");
    dev_bf16(*y, "y");
    TORCH_CHECK(y->dim() == 5 && y->is_contiguous() && y->size(0) == E && y->size(1) == MT &&
                    y->size(2) * 64 == N && y->size(3) == 64 && y->size(4) == 8,
                "gemm_skinny_grouped: y must be [E, MT, N/64, 64, 8]");
    yp = y->data_ptr();
    y_es = (*y)[0].numel();
  }
  check(k8sllm_gemm_skinny(a.data_ptr(), 0, wp.data_ptr(), pp, yp, 0, M, N, K, epi == 0 ? (int)splits : 1,
                           (int)epi, 4, 1, nullptr, 0, K, 0.f, (int)waves, E, w_es, a_es, y_es, rw, E, w_rm,
                           cur()),
        "gemm_skinny_grouped");
  return epi == 0 ? (int64_t)E * S : 1;
}

// residual += sum of S slabs; out = residual * w (row-major or fragment-packed); ss_part[m][c] =
// sum of residual^2 over columns [512 c, 512 c + 512) - the deferred-RMSNorm producer.
// decode front end: resolved ids -> embedding rows (residual) + the first layer's deferred-norm operands
void embed_norm_partial(torch::Tensor out, torch::Tensor residual, torch::Tensor ids, c10::optional<torch::Tensor> src,
                        c10::optional<torch::Tensor> prev, torch::Tensor emb, torch::Tensor w, torch::Tensor ss_part) {
  dev_bf16(out, "out"); dev_bf16(residual, "residual"); dev_bf16(emb, "emb"); dev_bf16(w, "w"); dev_i32(ids, "ids");
  TORCH_CHECK(residual.is_contiguous() && residual.dim() == 2 && emb.is_contiguous() && emb.dim() == 2 &&
                  w.is_contiguous(), "embed_norm_partial layout");
  const int M = (int)residual.size(0), d = (int)residual.size(1);
  TORCH_CHECK(d % 512 == 0 && emb.size(1) == d && w.numel() == d && ids.numel() >= M, "embed_norm_partial shapes");
  TORCH_CHECK(src.has_value() == prev.has_value(), "embed_norm_partial: src and prev go together");
  const int* sp = nullptr;
  const int* pp = nullptr;
  if (src.has_value()) {
    dev_i32(*src, "src"); dev_i32(*prev, "prev");
    TORCH_CHECK(src->numel() >= M, "embed_norm_partial: src [M]");
    sp = src->data_ptr<int>();
    pp = prev->data_ptr<int>();
  }
  TORCH_CHECK(ss_part.is_cuda() && ss_part.scalar_type() == torch::kFloat32 && ss_part.is_contiguous() &&
                  ss_part.numel() >= (int64_t)M * (d / 512), "ss_part");
  long ostride = d;
  if (out.dim() == 4) {
    TORCH_CHECK(out.size(0) == (M + 15) / 16 && out.size(1) * 32 == d && out.size(2) == 64 && out.size(3) == 8,
                "packed out must be [ceil(M/16), d/32, 64, 8]");
    ostride = -(long)(d / 32);
  } else {
    TORCH_CHECK(out.numel() == (int64_t)M * d, "out shape");
  }
  check(k8sllm_embed_norm_partial(out.data_ptr(), ostride, residual.data_ptr(), ids.data_ptr<int>(), sp, pp,
                                  emb.data_ptr(), (int)emb.size(0), w.data_ptr(), M, d, ss_part.data_ptr<float>(), cur()),
        "embed_norm_partial");
}

void add_norm_partial(torch::Tensor out, torch::Tensor residual, c10::optional<torch::Tensor> partial, int64_t S,
                      torch::Tensor w, torch::Tensor ss_part) {
  dev_bf16(out, "out"); dev_bf16(residual, "residual"); dev_bf16(w, "w");
  TORCH_CHECK(residual.is_contiguous() && out.is_contiguous() && w.is_contiguous() && residual.dim() == 2,
              "add_norm_partial layout");
  const int M = (int)residual.size(0), d = (int)residual.size(1);
  TORCH_CHECK(d % 512 == 0, "add_norm_partial: d % 512 != 0");
  TORCH_CHECK(ss_part.is_cuda() && ss_part.scalar_type() == torch::kFloat32 && ss_part.is_contiguous() &&
                  ss_part.numel() >= (int64_t)M * (d / 512), "ss_part");
  const float* pp = nullptr;
  if (S > 0) {
    TORCH_CHECK(partial.has_value() && partial->scalar_type() == torch::kFloat32 && partial->is_contiguous() &&
                    partial->numel() >= S * M * d, "partial");
    pp = partial->data_ptr<float>();
  }
  long ostride = d;
  if (out.dim() == 4) {
    TORCH_CHECK(out.size(0) == (M + 15) / 16 && out.size(1) * 32 == d && out.size(2) == 64 && out.size(3) == 8,
                "packed out must be [ceil(M/16), d/32, 64, 8]");
    ostride = -(long)(d / 32);
  } else {
    TORCH_CHECK(out.numel() == (int64_t)M * d, "out shape");
  }
  check(k8sllm_add_norm_partial(out.data_ptr(), ostride, residual.data_ptr(), pp, (int)S, M, w.data_ptr(), d,
                                ss_part.data_ptr<float>(), cur()),
        "add_norm_partial");
}

void reduce_slabs(torch::Tensor out, torch::Tensor partial, int64_t S) {
  dev_bf16(out, "out");
  TORCH_CHECK(out.is_contiguous(), "reduce_slabs: out must be contiguous");
  TORCH_CHECK(partial.is_cuda() && partial.scalar_type() == torch::kFloat32 && partial.is_contiguous(), "partial");
  TORCH_CHECK(partial.numel() >= S * out.numel(), "reduce_slabs: partial too small");
  check(k8sllm_reduce_slabs(out.data_ptr(), partial.data_ptr<float>(), (int)S, out.numel(), cur()), "reduce_slabs");
}

void reduce_add_rms_norm(torch::Tensor out, torch::Tensor residual, c10::optional<torch::Tensor> partial, int64_t S,
                         torch::Tensor w, double eps, c10::optional<torch::Tensor> out_packed) {
  dev_bf16(out, "out"); dev_bf16(residual, "residual"); dev_bf16(w, "w");
  TORCH_CHECK(residual.is_contiguous() && out.is_contiguous() && w.is_contiguous(), "reduce_add_rms_norm layout");
  const int d = (int)residual.size(-1);
  const int M = (int)(residual.numel() / d);
  const float* pp = nullptr;
  if (S > 0) {
    TORCH_CHECK(partial.has_value() && partial->is_cuda() && partial->scalar_type() == torch::kFloat32 &&
                    partial->is_contiguous(), "partial");
    TORCH_CHECK(partial->numel() >= S * M * d, "reduce_add_rms_norm: partial too small");
    pp = partial->data_ptr<float>();
  }
  long ostride = d;
  if (out.dim() == 4) {  // fragment-packed [ceil(M/16), d/32, 64, 8] for the next gemm_skinny
    TORCH_CHECK(out.size(0) == (M + 15) / 16 && out.size(1) * 32 == d && out.size(2) == 64 && out.size(3) == 8,
                "packed out must be [ceil(M/16), d/32, 64, 8]");
    ostride = -(long)(d / 32);
  } else {
    TORCH_CHECK(out.numel() == (int64_t)M * d, "reduce_add_rms_norm shapes");
  }
  void* out2 = nullptr;
  if (out_packed.has_value()) {  // a second, fragment-packed copy of the normed rows
    const auto& o2 = *out_packed;
    dev_bf16(o2, "out_packed");
    TORCH_CHECK(o2.dim() == 4 && o2.is_contiguous() && o2.size(0) == (M + 15) / 16 && o2.size(1) * 32 == d &&
                    o2.size(2) == 64 && o2.size(3) == 8, "out_packed must be [ceil(M/16), d/32, 64, 8]");
    out2 = o2.data_ptr();
  }
  check(k8sllm_reduce_add_rmsnorm(out.data_ptr(), residual.data_ptr(), pp, (int)S, M, w.data_ptr(), d, (float)eps,
                                  ostride, out2, cur()),
        "reduce_add_rms_norm");
}

// One-shot IPC all-reduce (custom_ar.hip).  The state is an opaque pointer held by Python.
py::tuple car_create(int64_t rank, int64_t world, int64_t max_elems) {
  std::string h(2 * k8sllm_car_handle_size(), '\0');
  int err = 0;
  void* st = k8sllm_car_create((int)rank, (int)world, (long)max_elems, h.data(), &err);
  TORCH_CHECK(st != nullptr, "custom all-reduce: allocation / IPC handle failed, hip error ", err);
  return py::make_tuple((int64_t)(intptr_t)st, py::bytes(h));
}

void car_open(int64_t state, py::bytes all_handles) {
  std::string a = all_handles;
  check(k8sllm_car_open((void*)(intptr_t)state, a.data()), "car_open (hipIpcOpenMemHandle)");
}

void car_all_reduce(int64_t state, torch::Tensor in, torch::Tensor out, int64_t spin_limit, int64_t algo) {
  dev_bf16(in, "in"); dev_bf16(out, "out");
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel(), "car_all_reduce layout");
  check(k8sllm_car_all_reduce((void*)(intptr_t)state, in.data_ptr(), out.data_ptr(), (long)in.numel(),
                              (long)spin_limit, (int)algo, cur()),
        "car_all_reduce");
}

// TP row-parallel tail in one launch: slabs [ns, M, d] fp32 -> reduced over ranks -> residual +=,
// RMSNorm * w -> out (row-major [M, d] or fragment-packed when packed).
void car_fused_tail(int64_t state, torch::Tensor slabs, int64_t ns, torch::Tensor residual, torch::Tensor w,
                    torch::Tensor out, double eps, bool packed, int64_t spin_limit, int64_t algo) {
  dev_bf16(residual, "residual"); dev_bf16(w, "w"); dev_bf16(out, "out");
  TORCH_CHECK(slabs.is_cuda() && slabs.scalar_type() == torch::kFloat32 && slabs.is_contiguous(), "slabs fp32");
  TORCH_CHECK(residual.dim() == 2 && residual.is_contiguous() && w.is_contiguous() && out.is_contiguous(),
              "car_fused_tail layout");
  const int M = (int)residual.size(0), d = (int)residual.size(1);
  TORCH_CHECK(slabs.numel() >= ns * (long)M * d && w.numel() == d, "car_fused_tail sizes");
  TORCH_CHECK(packed ? out.numel() >= (long)((M + 15) / 16) * 16 * d : out.numel() >= (long)M * d,
              "car_fused_tail out size");
  check(k8sllm_car_fused_tail((void*)(intptr_t)state, slabs.data_ptr<float>(), (int)ns, (long)M * d,
                              residual.data_ptr(), w.data_ptr(), out.data_ptr(), d, M, d, (float)eps, packed ? 1 : 0,
                              (long)spin_limit, (int)algo, cur()),
        "car_fused_tail");
}

void car_all_gather(int64_t state, torch::Tensor in, torch::Tensor out, int64_t spin_limit) {
  dev_bf16(in, "in"); dev_bf16(out, "out");
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && out.numel() % in.numel() == 0 &&
                  out.data_ptr() != in.data_ptr(), "car_all_gather layout");
  check(k8sllm_car_all_gather((void*)(intptr_t)state, in.data_ptr(), out.data_ptr(), (long)in.numel(),
                              (long)spin_limit, cur()),
        "car_all_gather");
}

void car_all_to_all(int64_t state, torch::Tensor in, torch::Tensor out, int64_t spin_limit) {
  dev_bf16(in, "in"); dev_bf16(out, "out");
  TORCH_CHECK(in.is_contiguous() && out.is_contiguous() && out.numel() == in.numel() &&
                  out.data_ptr() != in.data_ptr(), "car_all_to_all layout");
  check(k8sllm_car_all_to_all((void*)(intptr_t)state, in.data_ptr(), out.data_ptr(), (long)in.numel(),
                              (long)spin_limit, cur()),
        "car_all_to_all");
}

int64_t car_error(int64_t state) { return k8sllm_car_error((void*)(intptr_t)state); }

void car_error_async(int64_t state, torch::Tensor host) {
  TORCH_CHECK(!host.is_cuda() && host.scalar_type() == torch::kInt32 && host.numel() >= 1, "host int32 flag");
  check(k8sllm_car_error_async((void*)(intptr_t)state, host.data_ptr(), cur()), "car_error_async");
}

void car_destroy(int64_t state) { k8sllm_car_destroy((void*)(intptr_t)state); }

PYBIND11_MODULE(_k8sllm_ops, m) {
  m.doc() = "gfx950 HIP kernels for k8s-llm-monitor-amd";
  m.def("rms_norm", &rms_norm);
  m.def("fused_add_rms_norm", &fused_add_rms_norm);
  m.def("layer_norm", &layer_norm);
  m.def("silu_mul", &silu_mul);
  m.def("moe_grouped_gemm", &moe_grouped_gemm);
  m.def("gemm_tile", &gemm_tile, py::arg("y"), py::arg("x"), py::arg("w"), py::arg("offsets"), py::arg("swiglu"),
        py::arg("algo") = 1, py::arg("rope_pos") = py::none(), py::arg("rope_cs") = py::none(),
        py::arg("rope_heads") = 0, py::arg("rs_part") = py::none(), py::arg("rs_eps") = 1e-5,
        py::arg("resid") = py::none(), py::arg("hw") = py::none(), py::arg("norm_w") = py::none(),
        py::arg("ss_out") = py::none());
  m.def("gelu_tanh", &gelu_tanh);
  m.def("embedding", &embedding);
  m.def("resolve_ids", &resolve_ids);
  m.def("rope_and_cache", &rope_and_cache);
  m.def("paged_decode", &paged_decode);
  m.def("paged_decode_fused", &paged_decode_fused);
  m.def("decode_tw_force", [](int64_t tw) { k8sllm_decode_tw_force((int)tw); });
  m.def("flash_prefill", &flash_prefill);
  m.def("embed_norm_partial", &embed_norm_partial);
  m.def("sample", &sample, py::arg("out"), py::arg("logits"), py::arg("temps"), py::arg("top_k"), py::arg("top_p"),
        py::arg("rng"), py::arg("advance") = false);
  m.def("moe_route", &moe_route);
  m.def("moe_router", &moe_router);
  m.def("moe_align", &moe_align);
  m.def("moe_combine", &moe_combine);
  m.def("gather_rows", &gather_rows);
  m.def("gemm_skinny", &gemm_skinny);
  m.def("gemm_skinny_grouped", &gemm_skinny_grouped);
  m.def("gemm_dec", &gemm_dec);
  m.def("gemm_dec_grouped", &gemm_dec_grouped);
  m.def("gemm_dec_rc", &gemm_dec_rc);
  m.def("reduce_add_rms_norm", &reduce_add_rms_norm);
  m.def("reduce_slabs", &reduce_slabs);
  m.def("add_norm_partial", &add_norm_partial);
  m.def("car_create", &car_create);
  m.def("car_open", &car_open);
  m.def("car_all_reduce", &car_all_reduce, py::arg("state"), py::arg("in"), py::arg("out"), py::arg("spin_limit"),
        py::arg("algo") = -1);
  m.def("car_fused_tail", &car_fused_tail);
  m.def("car_all_to_all", &car_all_to_all);
  m.def("car_error", &car_error);
  m.def("car_all_gather", &car_all_gather);
  m.def("car_error_async", &car_error_async);
  m.def("car_destroy", &car_destroy);
}
