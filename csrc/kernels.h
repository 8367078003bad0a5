// Host-callable launchers of the gfx950 kernel library.  Raw pointers + an explicit
// stream keep the .hip translation units free of torch headers (fast rebuilds) and
// make every launcher capturable in a hipGraph (no allocation, no sync inside).
// Return 0 on success, <0 for an unsupported shape (checked before launch).
#pragma once
#include <hip/hip_runtime.h>

typedef unsigned short bf16_t;

// Launch-failure return codes (common.h LK_CHECK_LAUNCH / LK_SET_MAX_LDS): the bindings raise
// with the HIP error string instead of handing back an uninitialised output.
constexpr int kLkLaunchError = -1000;  // rc = kLkLaunchError - hipError_t
constexpr int kLkAttrError = -2000;    // rc = kLkAttrError - hipError_t (dynamic-LDS opt-in refused)

// norm.hip
int lk_rmsnorm(bf16_t* out, bf16_t* residual, const bf16_t* x, const bf16_t* w, long rows, int H,
               float eps, long xs, long os, long rs, hipStream_t st);
int lk_splitk_rmsnorm(bf16_t* out, bf16_t* residual, const float* part, int S, const bf16_t* w, long rows, int H,
                      float eps, long os, long rs, hipStream_t st);
int lk_layernorm(bf16_t* out, const bf16_t* x, const bf16_t* res, bf16_t* res_out, const bf16_t* w,
                 const bf16_t* b, long rows, int H, float eps, long xs, long os, long rs,
                 hipStream_t st);
int lk_embed_layernorm(bf16_t* out, const int* ids, const int* pos_ids, const int* type_ids,
                       const bf16_t* tok, const bf16_t* pos, const bf16_t* typ, const bf16_t* w,
                       const bf16_t* b, long rows, int H, float eps, hipStream_t st);

// activation.hip
int lk_silu_mul(bf16_t* out, const bf16_t* x, long rows, int I, long xs, long os, hipStream_t st);
int lk_activation(bf16_t* x, const bf16_t* bias, long rows, int N, long xs, int kind,
                  hipStream_t st);

// skinny_gemm.hip (decode-regime linear, optional fused SwiGLU)
int lk_skinny_splits(int M, int N, int K, int swiglu);
int lk_skinny_gemm(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int S, int swiglu,
                   bf16_t* out, long ldo, float* part, hipStream_t st);

void lk_wsgemm_plan(int M, int N, int K, int swiglu, int* bn_out, int* s_out);
int lk_wsgemm_pro(int kind, bf16_t* x, const bf16_t* w, int M, int N, int K, int BN, int S, int swiglu,
                  bf16_t* out, long ldo, float* part, const float* pp, int pS, const bf16_t* res, bf16_t* res_out,
                  long rs, const bf16_t* gamma, float eps, const float* po, const float* pml, const int* ctx, int Hq,
                  int D, int max_splits, int split, hipStream_t st);
int lk_wsgemm(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int BN, int S, int swiglu,
              bf16_t* out, long ldo, float* part, hipStream_t st);

// gemv_decode.hip (decode GEMV for M <= 2 rows; mode 0 out, 1 res += out, 2 SwiGLU, 3 RoPE + paged KV;
// gamma != nullptr: RMSNorm prologue over x; po != nullptr (mode 1): x = the paged-decode split merge)
int lk_gemv_supported(int M, int N, int K, int mode);
void lk_gemv_set_wgs(int wgs);
void lk_gemv_set_ksplit(int on);
int lk_l3_prefetch(const void* p, long bytes, int wgs, unsigned* sink, hipStream_t st);
int lk_gemv_decode(int mode, const bf16_t* x, long ldx, const bf16_t* gamma, float eps, const bf16_t* w, int M, int N,
                   int K, bf16_t* out, long ldo, bf16_t* res, long ldr, const int* positions, const float* cos_sin,
                   int Hq, int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
                   const float* po, const float* pml, const int* ctx, int max_splits, int split, hipStream_t st);

// GEMM part only (S >= 2): f32 partial slabs part[S][M][N], for a consumer that fuses the
// split-K reduction (lk_splitk_rmsnorm, lk_splitk_rope_kv)
int lk_wsgemm_set_variant(int M, int N, int K, int swiglu, int variant);  // -1 = back to the default
int lk_wsgemm_part(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int BN, int S, float* part,
                   hipStream_t st);
// the same split-K GEMM with the reduction fused into its last workgroup(s): RoPE + paged-KV
// write per head (BN == D == 128), or residual + RMSNorm for M <= 4 (skinny_gemm.hip WsTail)
int lk_ws_rope_kv_fused(const bf16_t* x, long ldx, const bf16_t* w, int M, int K, int BN, int S, float* part,
                        int* tickets, bf16_t* qkv, long qs, const int* positions, const float* cos_sin, int Hq,
                        int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
                        int write_k_inplace, hipStream_t st);
int lk_ws_rmsnorm_fused(const bf16_t* x, long ldx, const bf16_t* w, int M, int N, int K, int BN, int S, float* part,
                        int* tickets, bf16_t* out, long os, bf16_t* residual, long rs, const bf16_t* norm_w, float eps,
                        hipStream_t st);

void lk_wsgemm_set_rot(int rot_mul);  // K-step rotation per column tile (0 = off, -1 = policy)

int lk_ws_scores_f32(const bf16_t* x, long ldx, const bf16_t* w, int M, long N, int K, float* out, long ldo,
                     hipStream_t st);

// xgmi_allreduce.hip (one-shot / two-shot all-reduce over IPC-mapped peer buffers, K14)
int lk_xgmi_ar_sig_words();
int lk_xgmi_gather(bf16_t* const* data, unsigned* const* sig, int rank, int world, int root, const void* in,
                   void* out, long nbytes, int* err, hipStream_t st);
int lk_xgmi_allreduce2(bf16_t* const* data, unsigned* const* sig, long red_off, int rank, int world,
                       const bf16_t* in, bf16_t* residual, const bf16_t* w, bf16_t* out, int T, int H, float eps,
                       int norm, int* err, hipStream_t st);
int lk_xgmi_ar_max_ranks();
int lk_xgmi_allreduce_rmsnorm(bf16_t* const* data, unsigned* const* sig, int rank, int world, const bf16_t* in,
                              bf16_t* residual, const bf16_t* w, bf16_t* out, int T, int H, float eps, int* err,
                              hipStream_t st);
int lk_xgmi_allreduce(bf16_t* const* data, unsigned* const* sig, int rank, int world, const bf16_t* in,
                      bf16_t* out, long n, int* err, hipStream_t st);

// gemm.hip (prefill / encoder-regime linear, 256 x {256,192} MFMA tiles, fused epilogues)
// epi: 0 none, 1 SwiGLU (W = [Wg; Wu]), 2 bias, 3 bias + GELU(erf), 4 bias + ReLU; bn: 256 | 192
// ks > 1: split-K over ks K-ranges, fp32 partials in ws [ks, M, N], then a reduce applies the
// epilogue (not SwiGLU) -- for shapes with fewer tiles than CUs
int lk_gemm_supported(int M, int N, int K, int epi, int bn, int ks = 1);
int lk_gemm_streamk(int mode);
// Fused prefill-chain epilogues of lk_gemm (the RMSNorm of the pre-norm decoder block folded
// into its neighbouring GEMMs, the norm weight g folded into the consumer's weight rows):
//   row scale (any of epi NONE / SWIGLU / QKV, when ss_in is set): acc *= rsqrt(sum_t
//     ss_in[t * ss_ld + row] / H + eps) before the epilogue -- the consumer side of the norm;
//   epi RESID (6): r = bf16(r + bf16(acc)) in place in resid [M, ldr], and the per-row partial
//     sums of squares of the new r over this column tile into ss_out[tn * ss_out_ld + row]
//     (tn = column tile of 256) -- the producer side; `out` is not written;
//   epi QKV (7): out = the qkv row, q / k heads rotated with interleaved-pair RoPE (weights
//     permuted at load: models/llama.py), K / V scattered into the paged cache at slots[row]
//     (slot < 0: not cached).
struct LkEpi {
  const float* ss_in = nullptr;  // [nt][ss_ld] fp32 partial sums of squares (row scale)
  int ss_nt = 0;                 // partials per row (<= 32)
  long ss_ld = 0;                // row stride of one partial plane (>= M)
  float inv_h = 0.f;             // 1 / hidden size
  float eps = 0.f;
  bf16_t* resid = nullptr;       // RESID: residual stream, updated in place
  long ldr = 0;
  float* ss_out = nullptr;       // RESID: [N / 256][ss_out_ld] partial sums of squares
  long ss_out_ld = 0;
  const int* pos = nullptr;      // QKV: positions [M]
  const float* cos_sin = nullptr;  // QKV: [max_pos, D] = [cos(D/2) | sin(D/2)]
  const int* slots = nullptr;    // QKV: cache slot per row (block * bs + offset), -1 = skip
  bf16_t* kc = nullptr;          // QKV: paged caches [num_blocks, hkv, bs, hd]
  bf16_t* vc = nullptr;
  int bs = 0, hq = 0, hkv = 0, hd = 0;
};
// variant: K-loop schedule of gemm.hip (0 / 1 / 2), or 3 = gemm1w.hip (bn 256)
int lk_gemm(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int N, int K, int epi, int bn,
            int variant, bf16_t* out, long ldo, hipStream_t st, int ks = 1, float* ws = nullptr,
            const LkEpi* ea = nullptr);

// gemm1w.hip: the one-wave-per-SIMD bm x 256 prefill GEMM (hipBLASLt's gfx950 K-loop schedule,
// every lk_gemm epilogue); lk_gemm routes variants 3 / 4 / 5 here (row tile bm = 256 / 192 / 128).
// Needs K % 64 == 0 and >= 3 K-tiles per split, N % 256 == 0 (SwiGLU: N/2 % 128).
// group_m <= 0: LK_GEMM_GROUP_M (4).
// Variants 6 / 7: a column split -- the column tiles that fill whole waves of the CUs on 256-row
// tiles, the remaining (less than a wave) on 128 / 192-row tiles, as two launches.
constexpr int LK_GEMM1W_SPLIT128 = 1, LK_GEMM1W_SPLIT192 = 2;
inline int lk_gemm1w_bm(int variant) {
  return variant == 3 ? 256 : variant == 4 ? 192 : variant == 5 ? 128 : variant == 6 ? LK_GEMM1W_SPLIT128
       : variant == 7 ? LK_GEMM1W_SPLIT192 : 0;
}
// 256-wide column tiles of a variant 6 / 7 split that run on 256-row tiles (0 or all: no split)
int lk_gemm1w_split_cols(int M, int TN, int cus);
int lk_gemm1w_supported(int M, int N, int K, int epi, int ks, int bm = 256);
int lk_gemm1w(const bf16_t* x, long ldx, const bf16_t* w, const bf16_t* bias, int M, int N, int K, int epi,
              bf16_t* out, long ldo, hipStream_t st, int ks, float* ws, const LkEpi* ea, int group_m, int bm = 256);

// rope_kv.hip
int lk_rope_kv(bf16_t* qkv, long qs, const int* positions, const float* cos_sin, long T, int Hq,
               int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
               int write_k_inplace, hipStream_t st);
// RoPE + paged-KV write fused with the split-K reduction of the QKV projection:
// part[S][T][N] f32 -> qkv [T, N] bf16 (q rotated, k as lk_rope_kv leaves it, v) + caches
int lk_splitk_rope_kv(const float* part, int S, bf16_t* qkv, long qs, const int* positions, const float* cos_sin,
                      long T, int Hq, int Hkv, int D, bf16_t* kc, bf16_t* vc, const int* slots, int BS, int neox,
                      int write_k_inplace, hipStream_t st);
int lk_kv_write(const bf16_t* k, long ks, const bf16_t* v, long vs, bf16_t* kc, bf16_t* vc,
                const int* slots, long T, int Hkv, int D, int BS, hipStream_t st);

// attn_decode.hip
int lk_decode_split_size(int B, int Hkv);
int lk_decode_splits(int max_context, int split);
int lk_paged_decode(const bf16_t* q, long qs, const bf16_t* kc, const bf16_t* vc,
                    const int* block_tables, int bt_stride, const int* ctx_lens, bf16_t* out,
                    long os, float* part_o, float* part_ml, int B, int Hq, int Hkv, int D, int BS,
                    int max_splits, int split, float scale, const int* k_start, const float* pp_o,
                    const float* pp_ml, hipStream_t st, int* tickets = nullptr, int reduce = 1);

// attn_prefill.hip
int lk_prefill_rows_per_tile(int G, int D);
int lk_flash_prefill(const bf16_t* q, long qs, const bf16_t* k, const bf16_t* v, long ks, long vs,
                     const int* block_tables, int bt_stride, const int* cu_q, const int* ctx_lens,
                     const int* tile_seq, const int* tile_q0, int ntiles, bf16_t* out, long os,
                     int Hq, int Hkv, int D, int BS, float scale, int causal, int paged,
                     float* part_o, float* part_ml, const int* q_past, hipStream_t st);

// knn.hip
int lk_knn_nblocks(long N);
int lk_knn_partial(const bf16_t* corpus, const float* cnorm, long N, int D, const bf16_t* queries,
                   const float* qnorm, int nq, int K, float* part_s, int* part_i, hipStream_t st);
int lk_knn_score_chunks(long N);
int lk_knn_score_topk(const float* scores, long ld, const float* cnorm, const float* qnorm, long N, int nq, int K,
                      float* part_s, int* part_i, hipStream_t st);
int lk_knn_merge(const float* cand_s, const int* cand_i, int nq, int ncand, int K, float* out_s,
                 int* out_i, hipStream_t st);

// pooling.hip
int lk_pool_normalize(const bf16_t* hidden, long hs, const int* cu, int B, int H, int mode,
                      int normalize, void* out, long os, int out_bf16, hipStream_t st);
int lk_row_norms(const bf16_t* x, long N, int D, float* out, hipStream_t st);

// sampling.hip
// plan: int32 [B flags | B+1 offsets | allowed ids] (ids in [0, V), checked by the caller)
int lk_select_allowed(const void* logits, int is_bf16, long ls, int B, int V, const float* temps,
                      unsigned long long seed, int step, const int* plan, int* out, hipStream_t st);
int lk_select_tokens(const void* logits, int is_bf16, long ls, int B, int V, const float* temps,
                     unsigned long long seed, int step, int* out, hipStream_t st);
// vocab-parallel greedy: per row an order-preserving int64 key of (max value, vocab_lo + argmax)
// (larger = larger value, then lower id); keys_to_ids: the max over W gathered key rows -> ids
int lk_argmax_key(const void* logits, int is_bf16, long ls, int B, int V, int vocab_lo, long long* keys, hipStream_t st);
int lk_keys_to_ids(const long long* keys, int W, int R, int* ids, hipStream_t st);
int lk_repeat_penalty(void* logits, int is_bf16, long ls, int B, const int* window, int W,
                      const float* penalty, hipStream_t st);
// Ollama-default sampling (repeat penalty from a device history ring, top-k, top-p,
// temperature; greedy rows = argmax).  prm: int32 [B, 8] = temperature, top_p, penalty (f32
// bits), top_k, last_n, slot, reset, seed.  hist: int32 [slots, W] ring, hist_len: [slots].
// logits (f32, modified in place by the penalty) -> out int32 [B]; the token is appended to the ring.
int lk_sample(float* logits, long ls, int B, int V, const int* prm, int* hist, int* hist_len, int W,
              unsigned long long seed, int* out, hipStream_t st);

// csrc/marker.hip: a one-wave marker kernel bounding a timed window in kernel traces
int lk_window_mark(int id, hipStream_t st);
// a launch the runtime rejects (2048 threads): returns the LK_CHECK_LAUNCH code, runs nothing
int lk_debug_invalid_launch(hipStream_t st);

// csrc/step_ops.hip: the forward's small per-step gathers (no framework kernels in a step)
int lk_embed_rows(bf16_t* out, const bf16_t* table, const int* ids, long T, int H, long lo, long n_local,
                  hipStream_t st, int strict = 0);
int lk_embed_errors();  // out-of-table ids seen by strict lk_embed_rows since the last call
int lk_scatter_ids(int* ids, const long* dst, const int* prev, const long* src, int n, hipStream_t st);
int lk_gather_rows(bf16_t* out, const bf16_t* x, long xs, const long* idx, long R, int H, hipStream_t st);
