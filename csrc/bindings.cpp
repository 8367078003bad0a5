// PyTorch bindings for the gfx950 kernel library (module `_C`).
// Every op validates device / dtype / shape on the host BEFORE launching: a bad
// launch shape on the GPU box can fault the device for every tenant, so nothing
// reaches a kernel unchecked.  Kernels run on PyTorch's current HIP stream, so the
// ops compose with torch.cuda.graphs (hipGraph capture) and stream semantics.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include "kernels.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bfloat16")
#define CHECK_I32(x) TORCH_CHECK((x).scalar_type() == at::kInt, #x " must be int32")
#define CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be float32")
#define CHECK_LASTDIM(x) TORCH_CHECK((x).stride(-1) == 1, #x " must be contiguous in its last dim")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
// Every launcher's return code AND the HIP launch state are checked after each op: a rejected
// launch raises here instead of returning an uninitialised output (common.h LK_CHECK_LAUNCH).
void check_rc(int rc, const char* name) {
  const hipError_t e = hipGetLastError();  // launchers that do not check their own launches
  if (rc <= kLkAttrError && rc > kLkAttrError - 1000)
    TORCH_CHECK(false, name, ": kernel dynamic-LDS attribute refused: ", hipGetErrorString((hipError_t)(kLkAttrError - rc)));
  if (rc <= kLkLaunchError && rc > kLkLaunchError - 1000)
    TORCH_CHECK(false, name, ": kernel launch failed: ", hipGetErrorString((hipError_t)(kLkLaunchError - rc)));
  TORCH_CHECK(rc == 0, name, ": unsupported shape/config (code ", rc, ")");
  TORCH_CHECK(e == hipSuccess, name, ": kernel launch failed: ", hipGetErrorString(e));
}
#define CHECK_RC(rc, name) check_rc((rc), (name))

inline bf16_t* bp(const at::Tensor& t) { return reinterpret_cast<bf16_t*>(t.data_ptr()); }
inline bf16_t* bpo(const c10::optional<at::Tensor>& t) { return t ? bp(*t) : nullptr; }
inline const int* ip(const at::Tensor& t) { return t.data_ptr<int>(); }
inline const int* ipo(const c10::optional<at::Tensor>& t) { return t ? ip(*t) : nullptr; }

// shape support of the prefill GEMM for a schedule variant (3 / 4 / 5: gemm1w.hip, 256-wide column
// tiles, 256 / 192 / 128-row tiles)
bool gemm_shape_ok(int M, int N, int K, int epi, int bn, int splits, int variant) {
  if (lk_gemm1w_bm(variant)) return bn == 256 && lk_gemm1w_supported(M, N, K, epi, splits, lk_gemm1w_bm(variant)) != 0;
  return lk_gemm_supported(M, N, K, epi, bn, splits) != 0;
}

// 16-byte alignment of every row start (vector loads)
void check_rows16(const at::Tensor& t, const char* name) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
  if (t.dim() >= 2) TORCH_CHECK((t.stride(0) * t.element_size()) % 16 == 0, name, " row stride must be a multiple of 16 bytes");
}

at::Tensor rmsnorm(const at::Tensor& x, const at::Tensor& w, double eps,
                   const c10::optional<at::Tensor>& residual, const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2, "x must be [T, H]");
  const long T = x.size(0);
  const int H = x.size(1);
  TORCH_CHECK(w.numel() == H && w.is_contiguous(), "weight shape");
  check_rows16(x, "x");
  at::Tensor out = out_ ? *out_ : at::empty({T, H}, x.options());
  CHECK_LASTDIM(out); check_rows16(out, "out");
  TORCH_CHECK(out.size(0) == T && out.size(1) == H, "out shape");
  long rs = 0;
  if (residual) {
    CHECK_BF16(*residual); CHECK_LASTDIM(*residual); check_rows16(*residual, "residual");
    TORCH_CHECK(residual->size(0) == T && residual->size(1) == H, "residual shape");
    rs = residual->stride(0);
  }
  int rc = lk_rmsnorm(bp(out), bpo(residual), bp(x), bp(w), T, H, (float)eps, x.stride(0),
                      out.stride(0), rs, cur_stream());
  CHECK_RC(rc, "rmsnorm");
  return out;
}

at::Tensor layernorm(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& b,
                     double eps, const c10::optional<at::Tensor>& residual, bool write_residual) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2, "x must be [T, H]");
  const long T = x.size(0);
  const int H = x.size(1);
  TORCH_CHECK(w.numel() == H, "weight shape");
  if (b) { CHECK_BF16(*b); TORCH_CHECK(b->numel() == H, "bias shape"); }
  check_rows16(x, "x");
  at::Tensor out = at::empty({T, H}, x.options());
  long rs = 0;
  if (residual) {
    CHECK_BF16(*residual); CHECK_LASTDIM(*residual); check_rows16(*residual, "residual");
    TORCH_CHECK(residual->size(0) == T && residual->size(1) == H, "residual shape");
    rs = residual->stride(0);
  }
  int rc = lk_layernorm(bp(out), bp(x), bpo(residual), (residual && write_residual) ? bp(*residual) : nullptr,
                        bp(w), bpo(b), T, H, (float)eps, x.stride(0), out.stride(0), rs, cur_stream());
  CHECK_RC(rc, "layernorm");
  return out;
}

at::Tensor embed_layernorm(const at::Tensor& ids, const c10::optional<at::Tensor>& pos_ids,
                           const c10::optional<at::Tensor>& type_ids, const at::Tensor& tok,
                           const c10::optional<at::Tensor>& pos, const c10::optional<at::Tensor>& typ,
                           const at::Tensor& w, const at::Tensor& b, double eps) {
  CHECK_CUDA(ids); CHECK_I32(ids); CHECK_BF16(tok); CHECK_CONTIG(tok); CHECK_CONTIG(ids);
  const long T = ids.numel();
  const int H = tok.size(1);
  if (pos) { CHECK_BF16(*pos); CHECK_CONTIG(*pos); TORCH_CHECK(pos_ids.has_value(), "pos_ids required"); CHECK_I32(*pos_ids); TORCH_CHECK(pos_ids->numel() == T, "pos_ids"); TORCH_CHECK(pos->size(1) == H, "pos table"); }
  if (typ) { CHECK_BF16(*typ); CHECK_CONTIG(*typ); TORCH_CHECK(typ->size(1) == H, "type table"); }
  if (type_ids) { CHECK_I32(*type_ids); TORCH_CHECK(type_ids->numel() == T, "type_ids"); }
  at::Tensor out = at::empty({T, H}, tok.options());
  int rc = lk_embed_layernorm(bp(out), ip(ids), ipo(pos_ids), ipo(type_ids), bp(tok), bpo(pos), bpo(typ),
                              bp(w), bp(b), T, H, (float)eps, cur_stream());
  CHECK_RC(rc, "embed_layernorm");
  return out;
}

at::Tensor silu_mul(const at::Tensor& x, const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 2 == 0, "x must be [T, 2I]");
  check_rows16(x, "x");
  const long T = x.size(0);
  const int I = x.size(1) / 2;
  at::Tensor out = out_ ? *out_ : at::empty({T, I}, x.options());
  TORCH_CHECK(out.size(0) == T && out.size(1) == I, "out shape"); CHECK_LASTDIM(out);
  check_rows16(out, "out");
  int rc = lk_silu_mul(bp(out), bp(x), T, I, x.stride(0), out.stride(0), cur_stream());
  CHECK_RC(rc, "silu_mul");
  return out;
}

// Decode-regime linear: x [M, K] (M <= 256, row-contiguous) . w[N, K]^T -> [M, N];
// swiglu=true: w = [Wg; Wu] (2I rows) -> silu(x Wg^T) * (x Wu^T) [M, I].  Rows beyond
// 128 are processed as a second launch (the weight stream is re-read; still far
// below the library GEMM at these shapes).
at::Tensor skinny_linear(const at::Tensor& x, const at::Tensor& w, bool swiglu, int64_t splits,
                         const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "x [M,K], w [N,K]");
  check_rows16(x, "x"); check_rows16(w, "w");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 256, "skinny_linear: M must be in [1, 256]");
  const int n_out = swiglu ? N / 2 : N;
  at::Tensor out = out_ ? *out_ : at::empty({M, n_out}, x.options());
  CHECK_BF16(out); CHECK_LASTDIM(out); check_rows16(out, "out");
  TORCH_CHECK(out.size(0) == M && out.size(1) == n_out, "out shape");
  const int S = splits > 0 ? (int)splits : lk_skinny_splits(std::min(M, 128), N, K, swiglu);
  at::Tensor part;
  if (S > 1) part = at::empty({(long)S * std::min(M, 128) * N}, x.options().dtype(at::kFloat));
  for (int m0 = 0; m0 < M; m0 += 128) {
    const int mc = std::min(128, M - m0);
    int rc = lk_skinny_gemm(bp(x) + (long)m0 * x.stride(0), x.stride(0), bp(w), mc, N, K, S, swiglu ? 1 : 0,
                            bp(out) + (long)m0 * out.stride(0), out.stride(0),
                            S > 1 ? part.data_ptr<float>() : nullptr, cur_stream());
    CHECK_RC(rc, "skinny_linear");
  }
  return out;
}

// Weight-streaming GEMM for 64 < M <= 256 (LDS-DMA staged, csrc/skinny_gemm.hip wsgemm)
at::Tensor ws_linear(const at::Tensor& x, const at::Tensor& w, bool swiglu, int64_t bn, int64_t splits,
                     const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "x [M,K], w [N,K]");
  check_rows16(x, "x"); check_rows16(w, "w");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(M >= 1 && M <= 256, "ws_linear: M must be in [1, 256]");
  const int n_out = swiglu ? N / 2 : N;
  at::Tensor out = out_ ? *out_ : at::empty({M, n_out}, x.options());
  CHECK_BF16(out); CHECK_LASTDIM(out);
  TORCH_CHECK(out.size(0) == M && out.size(1) == n_out, "out shape");
  int BN = (int)bn, S = (int)splits;
  if (BN <= 0 || S <= 0) {
    int pb = 64, ps = 1;
    lk_wsgemm_plan(M, N, K, swiglu ? 1 : 0, &pb, &ps);
    if (BN <= 0) BN = pb;
    if (S <= 0) S = ps;
  }
  at::Tensor part;
  if (S > 1) part = at::empty({(long)S * M * N}, x.options().dtype(at::kFloat));
  int rc = lk_wsgemm(bp(x), x.stride(0), bp(w), M, N, K, BN, S, swiglu ? 1 : 0, bp(out), out.stride(0),
                     S > 1 ? part.data_ptr<float>() : nullptr, cur_stream());
  CHECK_RC(rc, "ws_linear");
  return out;
}

// Decode-step fusions (split-K weight-streaming GEMM whose reduction is done by the
// consumer kernel): the partial slabs never become a bf16 tensor, one launch fewer each.
namespace {
struct WsSplit {
  int M, N, K, BN, S;
};
WsSplit ws_split(const at::Tensor& x, const at::Tensor& w, int64_t bn, int64_t splits, const char* name) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), name, ": x [M,K], w [N,K]");
  check_rows16(x, "x"); check_rows16(w, "w");
  WsSplit p{(int)x.size(0), (int)w.size(0), (int)x.size(1), (int)bn, (int)splits};
  TORCH_CHECK(p.M >= 1 && p.M <= 256, name, ": M must be in [1, 256]");
  if (p.BN <= 0 || p.S <= 0) {
    int pb = 64, ps = 1;
    lk_wsgemm_plan(p.M, p.N, p.K, 0, &pb, &ps);
    if (p.BN <= 0) p.BN = pb;
    if (p.S <= 0) p.S = ps;
  }
  TORCH_CHECK(p.S >= 2, name, ": needs a split-K plan (S >= 2)");
  return p;
}
}  // namespace

// out = RMSNorm(x W^T + residual) * norm_w, residual += x W^T (bf16, in place)
at::Tensor ws_linear_rmsnorm(const at::Tensor& x, const at::Tensor& w, at::Tensor& residual,
                             const at::Tensor& norm_w, double eps, int64_t bn, int64_t splits,
                             const c10::optional<at::Tensor>& tickets) {
  const WsSplit p = ws_split(x, w, bn, splits, "ws_linear_rmsnorm");
  CHECK_CUDA(residual); CHECK_BF16(residual); CHECK_LASTDIM(residual); check_rows16(residual, "residual");
  TORCH_CHECK(residual.dim() == 2 && residual.size(0) == p.M && residual.size(1) == p.N, "residual shape");
  CHECK_BF16(norm_w); TORCH_CHECK(norm_w.numel() == p.N && norm_w.is_contiguous(), "norm weight shape");
  at::Tensor part = at::empty({(long)p.S * p.M * p.N}, x.options().dtype(at::kFloat));
  at::Tensor out = at::empty({p.M, p.N}, x.options());
  if (tickets && p.M <= 4 && (p.S == 2 || p.S == 4 || p.S == 8)) {  // reduction fused into the GEMM
    CHECK_CUDA(*tickets); CHECK_I32(*tickets); CHECK_CONTIG(*tickets);
    TORCH_CHECK(tickets->numel() >= 1, "tickets");
    int rc = lk_ws_rmsnorm_fused(bp(x), x.stride(0), bp(w), p.M, p.N, p.K, p.BN, p.S, part.data_ptr<float>(),
                                 tickets->data_ptr<int>(), bp(out), out.stride(0), bp(residual), residual.stride(0),
                                 bp(norm_w), (float)eps, cur_stream());
    CHECK_RC(rc, "ws_linear_rmsnorm (fused)");
    return out;
  }
  int rc = lk_wsgemm_part(bp(x), x.stride(0), bp(w), p.M, p.N, p.K, p.BN, p.S, part.data_ptr<float>(), cur_stream());
  CHECK_RC(rc, "ws_linear_rmsnorm (gemm)");
  rc = lk_splitk_rmsnorm(bp(out), bp(residual), part.data_ptr<float>(), p.S, bp(norm_w), p.M, p.N, (float)eps,
                         out.stride(0), residual.stride(0), cur_stream());
  CHECK_RC(rc, "ws_linear_rmsnorm (norm)");
  return out;
}

// qkv = x W^T with RoPE applied and K/V scattered into the paged cache (as rope_kv_)
at::Tensor ws_linear_rope_kv(const at::Tensor& x, const at::Tensor& w, const at::Tensor& positions,
                             const at::Tensor& cos_sin, int64_t Hq, int64_t Hkv, int64_t D,
                             const c10::optional<at::Tensor>& k_cache, const c10::optional<at::Tensor>& v_cache,
                             const c10::optional<at::Tensor>& slots, bool neox, bool write_k_inplace, int64_t bn,
                             int64_t splits, const c10::optional<at::Tensor>& tickets) {
  const WsSplit p = ws_split(x, w, bn, splits, "ws_linear_rope_kv");
  TORCH_CHECK(p.N == (Hq + 2 * Hkv) * D, "w must be the fused [(Hq + 2 Hkv) * D, K] projection");
  CHECK_I32(positions); CHECK_F32(cos_sin); CHECK_CONTIG(cos_sin); CHECK_CONTIG(positions);
  TORCH_CHECK(positions.numel() == p.M, "positions");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  int BS = 1;
  if (k_cache || v_cache) {
    TORCH_CHECK(k_cache && v_cache && slots, "k_cache, v_cache and slots go together");
    CHECK_BF16(*k_cache); CHECK_BF16(*v_cache); CHECK_CONTIG(*k_cache); CHECK_CONTIG(*v_cache);
    CHECK_I32(*slots); TORCH_CHECK(slots->numel() == p.M, "slots");
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == Hkv && k_cache->size(3) == D, "k_cache must be [NB, Hkv, BS, D]");
    TORCH_CHECK(v_cache->sizes() == k_cache->sizes(), "v_cache shape");
    BS = k_cache->size(2);
  }
  at::Tensor part = at::empty({(long)p.S * p.M * p.N}, x.options().dtype(at::kFloat));
  at::Tensor qkv = at::empty({p.M, p.N}, x.options());
  if (tickets && p.BN == D && D == 128 && (p.S == 2 || p.S == 4 || p.S == 8)) {  // reduction fused into the GEMM
    CHECK_CUDA(*tickets); CHECK_I32(*tickets); CHECK_CONTIG(*tickets);
    TORCH_CHECK(tickets->numel() >= Hq + 2 * Hkv, "tickets: one per head");
    int rc = lk_ws_rope_kv_fused(bp(x), x.stride(0), bp(w), p.M, p.K, p.BN, p.S, part.data_ptr<float>(),
                                 tickets->data_ptr<int>(), bp(qkv), qkv.stride(0), ip(positions),
                                 cos_sin.data_ptr<float>(), (int)Hq, (int)Hkv, (int)D, bpo(k_cache), bpo(v_cache),
                                 ipo(slots), BS, neox ? 1 : 0, write_k_inplace ? 1 : 0, cur_stream());
    CHECK_RC(rc, "ws_linear_rope_kv (fused)");
    return qkv;
  }
  int rc = lk_wsgemm_part(bp(x), x.stride(0), bp(w), p.M, p.N, p.K, p.BN, p.S, part.data_ptr<float>(), cur_stream());
  CHECK_RC(rc, "ws_linear_rope_kv (gemm)");
  rc = lk_splitk_rope_kv(part.data_ptr<float>(), p.S, bp(qkv), qkv.stride(0), ip(positions), cos_sin.data_ptr<float>(),
                         p.M, (int)Hq, (int)Hkv, (int)D, bpo(k_cache), bpo(v_cache), ipo(slots), BS, neox ? 1 : 0,
                         write_k_inplace ? 1 : 0, cur_stream());
  CHECK_RC(rc, "ws_linear_rope_kv (rope)");
  return qkv;
}

// Weight-streaming GEMM whose workgroups compute their own X rows first (lk_wsgemm_pro):
//   kind 1: x (written) = RMSNorm(bf16(sum of pp's slabs) + res_in) * gamma; res_out = the summed
//           residual (a tensor other than res_in)
//   kind 2: x = the paged-decode output, rows with > 1 split merged from (po, pml) first
// Returns the f32 partial slabs [S, M, N] when S > 1 (reduce == false), else the bf16 (SwiGLU)
// output.
at::Tensor ws_pro(at::Tensor& x, const at::Tensor& w, bool swiglu, int64_t bn, int64_t splits, int64_t kind,
                  bool reduce, const c10::optional<at::Tensor>& pp, const c10::optional<at::Tensor>& res_in,
                  const c10::optional<at::Tensor>& res_out, const c10::optional<at::Tensor>& gamma, double eps,
                  const c10::optional<at::Tensor>& po, const c10::optional<at::Tensor>& pml,
                  const c10::optional<at::Tensor>& ctx, int64_t split, int64_t max_splits, int64_t Hq) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_CONTIG(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "ws_pro: x [M,K], w [N,K]");
  check_rows16(x, "x"); check_rows16(w, "w");
  const int M = x.size(0), K = x.size(1), N = w.size(0), S = (int)splits;
  TORCH_CHECK(M >= 1 && M <= 64 && S >= 1, "ws_pro: 1 <= M <= 64, splits >= 1");
  const int n_out = swiglu ? N / 2 : N;
  at::Tensor part, out;
  if (S > 1) part = at::empty({(long)S, M, N}, x.options().dtype(at::kFloat));
  if (kind == 0) {  // plain X: the partial slabs only (the producer of a kind-1 consumer)
    TORCH_CHECK(S > 1 && !swiglu, "ws_pro kind 0: split-K partials (splits > 1, no SwiGLU)");
    CHECK_RC(lk_wsgemm_part(bp(x), x.stride(0), bp(w), M, N, K, (int)bn, S, part.data_ptr<float>(), cur_stream()),
             "ws_pro (part)");
    return part;
  }
  if (S == 1 || reduce) out = at::empty({M, n_out}, x.options());
  const float* ppp = nullptr;
  int pS = 0;
  const bf16_t* rin = nullptr;
  bf16_t* rout = nullptr;
  long rs = 0;
  const bf16_t* g = nullptr;
  if (kind == 1) {
    TORCH_CHECK(pp && res_in && res_out && gamma, "ws_pro kind 1: pp, res_in, res_out, gamma");
    CHECK_CUDA(*pp); CHECK_F32(*pp); CHECK_CONTIG(*pp);
    TORCH_CHECK(pp->dim() == 3 && pp->size(1) == M && pp->size(2) == K, "pp must be [S, M, K]");
    CHECK_BF16(*res_in); CHECK_BF16(*res_out); CHECK_CONTIG(*res_in); CHECK_CONTIG(*res_out);
    TORCH_CHECK(res_in->size(0) == M && res_in->size(1) == K && res_out->sizes() == res_in->sizes(), "residual shapes");
    TORCH_CHECK(res_in->data_ptr() != res_out->data_ptr(), "res_out must not alias res_in");
    CHECK_BF16(*gamma); TORCH_CHECK(gamma->numel() == K && gamma->is_contiguous(), "gamma [K]");
    ppp = pp->data_ptr<float>();
    pS = pp->size(0);
    rin = bp(*res_in);
    rout = bp(*res_out);
    rs = res_in->stride(0);
    g = bp(*gamma);
  }
  const float* pop = nullptr;
  const float* pmp = nullptr;
  const int* cp = nullptr;
  int D = 0;
  if (kind == 2) {
    TORCH_CHECK(po && pml && ctx, "ws_pro kind 2: po, pml, ctx");
    CHECK_F32(*po); CHECK_F32(*pml); CHECK_CONTIG(*po); CHECK_CONTIG(*pml); CHECK_I32(*ctx); CHECK_CONTIG(*ctx);
    TORCH_CHECK(Hq > 0 && K % Hq == 0, "Hq");
    D = K / Hq;
    TORCH_CHECK(po->numel() >= (long)M * Hq * max_splits * D && pml->numel() >= (long)M * Hq * max_splits * 2 &&
                ctx->numel() >= M, "decode partials / ctx too small");
    pop = po->data_ptr<float>();
    pmp = pml->data_ptr<float>();
    cp = ctx->data_ptr<int>();
  }
  int rc = lk_wsgemm_pro((int)kind, bp(x), bp(w), M, N, K, (int)bn, S, swiglu ? 1 : 0,
                         out.defined() ? bp(out) : nullptr, out.defined() ? out.stride(0) : 0,
                         S > 1 ? part.data_ptr<float>() : nullptr, ppp, pS, rin, rout, rs, g, (float)eps, pop, pmp, cp,
                         (int)Hq, D, (int)max_splits, (int)split, cur_stream());
  CHECK_RC(rc, "ws_pro");
  return out.defined() ? out : part;
}

// rope_kv_ over the reduce of split-K QKV slabs part [S, M, N] (as ws_linear_rope_kv's second half)
at::Tensor splitk_rope_kv(const at::Tensor& part, const at::Tensor& positions, const at::Tensor& cos_sin, int64_t Hq,
                          int64_t Hkv, int64_t D, const c10::optional<at::Tensor>& k_cache,
                          const c10::optional<at::Tensor>& v_cache, const c10::optional<at::Tensor>& slots, bool neox,
                          bool write_k_inplace) {
  CHECK_CUDA(part); CHECK_F32(part); CHECK_CONTIG(part);
  TORCH_CHECK(part.dim() == 3 && part.size(2) == (Hq + 2 * Hkv) * D, "part must be [S, M, (Hq + 2 Hkv) * D]");
  const int S = part.size(0), M = part.size(1), N = part.size(2);
  CHECK_I32(positions); CHECK_F32(cos_sin); CHECK_CONTIG(cos_sin); CHECK_CONTIG(positions);
  TORCH_CHECK(positions.numel() == M, "positions");
  TORCH_CHECK(cos_sin.dim() == 2 && cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  int BS = 1;
  if (k_cache || v_cache) {
    TORCH_CHECK(k_cache && v_cache && slots, "k_cache, v_cache and slots go together");
    CHECK_BF16(*k_cache); CHECK_BF16(*v_cache); CHECK_CONTIG(*k_cache); CHECK_CONTIG(*v_cache);
    CHECK_I32(*slots); TORCH_CHECK(slots->numel() == M, "slots");
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == Hkv && k_cache->size(3) == D, "k_cache must be [NB, Hkv, BS, D]");
    TORCH_CHECK(v_cache->sizes() == k_cache->sizes(), "v_cache shape");
    BS = k_cache->size(2);
  }
  at::Tensor qkv = at::empty({M, N}, part.options().dtype(at::kBFloat16));
  int rc = lk_splitk_rope_kv(part.data_ptr<float>(), S, bp(qkv), qkv.stride(0), ip(positions), cos_sin.data_ptr<float>(),
                             M, (int)Hq, (int)Hkv, (int)D, bpo(k_cache), bpo(v_cache), ipo(slots), BS, neox ? 1 : 0,
                             write_k_inplace ? 1 : 0, cur_stream());
  CHECK_RC(rc, "splitk_rope_kv");
  return qkv;
}

// RMSNorm(bf16(sum of part's slabs) + residual) * w, residual updated in place (lk_splitk_rmsnorm)
at::Tensor splitk_rmsnorm(const at::Tensor& part, at::Tensor& residual, const at::Tensor& w, double eps) {
  CHECK_CUDA(part); CHECK_F32(part); CHECK_CONTIG(part);
  CHECK_BF16(residual); CHECK_LASTDIM(residual); CHECK_BF16(w); check_rows16(residual, "residual");
  TORCH_CHECK(part.dim() == 3 && part.size(1) == residual.size(0) && part.size(2) == residual.size(1), "part [S, M, H]");
  const long M = residual.size(0);
  const int H = residual.size(1);
  TORCH_CHECK(w.numel() == H && w.is_contiguous(), "w [H]");
  at::Tensor out = at::empty({M, H}, residual.options());
  CHECK_RC(lk_splitk_rmsnorm(bp(out), bp(residual), part.data_ptr<float>(), part.size(0), bp(w), M, H, (float)eps,
                             out.stride(0), residual.stride(0), cur_stream()), "splitk_rmsnorm");
  return out;
}

// Decode GEMV for M <= 2 rows (csrc/gemv_decode.hip).  mode 0: returns x.w^T; 1: res += x.w^T in
// place (returns res); 2: SwiGLU over w = [Wg; Wu] (returns [M, N/2]); 3: RoPE + paged-KV write of a
// packed QKV projection (returns the qkv rows).  gamma: RMSNorm(x) * gamma is the GEMV's input.
at::Tensor gemv_decode(int64_t mode, const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& gamma,
                       double eps, const c10::optional<at::Tensor>& res, const c10::optional<at::Tensor>& positions,
                       const c10::optional<at::Tensor>& cos_sin, int64_t Hq, int64_t Hkv, int64_t D,
                       const c10::optional<at::Tensor>& k_cache, const c10::optional<at::Tensor>& v_cache,
                       const c10::optional<at::Tensor>& slots, bool neox, const c10::optional<at::Tensor>& po,
                       const c10::optional<at::Tensor>& pml, const c10::optional<at::Tensor>& ctx,
                       int64_t max_splits, int64_t split) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "gemv_decode: x [M,K], w [N,K]");
  if (po) {  // the O projection merging the paged-decode split partials of x's rows
    TORCH_CHECK(mode == 1 && pml && ctx && !gamma, "gemv_decode merge prologue: mode 1 with pml, ctx, no gamma");
    CHECK_F32(*po); CHECK_F32(*pml); CHECK_I32(*ctx); CHECK_CONTIG(*po); CHECK_CONTIG(*pml);
    TORCH_CHECK(po->dim() == 4 && po->size(0) >= x.size(0) && po->size(1) == Hq && po->size(2) == max_splits &&
                    po->size(3) == D && Hq * D == x.size(1), "po [M, Hq, max_splits, D]");
    TORCH_CHECK(pml->dim() == 4 && pml->size(0) == po->size(0) && pml->size(1) == Hq && pml->size(2) == max_splits &&
                    pml->size(3) == 2, "pml [M, Hq, max_splits, 2]");
    TORCH_CHECK(ctx->numel() >= x.size(0) && split > 0, "ctx: one per row; split > 0");
  }
  check_rows16(x, "x"); check_rows16(w, "w");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(lk_gemv_supported(M, N, K, (int)mode), "gemv_decode: unsupported shape M", M, " N", N, " K", K);
  if (gamma) { CHECK_BF16(*gamma); TORCH_CHECK(gamma->numel() == K && gamma->is_contiguous(), "gamma [K]"); }
  at::Tensor out;
  bf16_t* rp = nullptr;
  long ldr = 0;
  const int *pos = nullptr, *sl = nullptr;
  const float* cs = nullptr;
  bf16_t *kc = nullptr, *vc = nullptr;
  int BS = 0;
  if (mode == 0) {
    out = at::empty({M, N}, x.options());
  } else if (mode == 1) {
    TORCH_CHECK(res.has_value(), "gemv_decode mode 1: res");
    CHECK_BF16(*res); CHECK_LASTDIM(*res);
    TORCH_CHECK(res->size(0) == M && res->size(1) == N && res->stride(0) % 2 == 0, "res [M, N]");
    out = *res;
    rp = bp(*res);
    ldr = res->stride(0);
  } else if (mode == 2) {
    out = at::empty({M, N / 2}, x.options());
  } else if (mode == 3) {
    TORCH_CHECK(positions && cos_sin && slots, "gemv_decode mode 3: positions, cos_sin, slots");
    CHECK_I32(*positions); CHECK_I32(*slots); CHECK_F32(*cos_sin); CHECK_CONTIG(*cos_sin);
    TORCH_CHECK(positions->numel() >= M && slots->numel() >= M, "positions / slots: one per row");
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == D, "cos_sin [P, D]");
    TORCH_CHECK(N == (Hq + 2 * Hkv) * D, "qkv rows = (Hq + 2 Hkv) D");
    out = at::empty({M, N}, x.options());
    pos = ip(*positions); sl = ip(*slots); cs = cos_sin->data_ptr<float>();
    if (k_cache) {
      TORCH_CHECK(v_cache.has_value(), "k_cache without v_cache");
      CHECK_BF16(*k_cache); CHECK_BF16(*v_cache); CHECK_CONTIG(*k_cache); CHECK_CONTIG(*v_cache);
      TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == Hkv && k_cache->size(3) == D &&
                  v_cache->sizes() == k_cache->sizes(), "cache [blocks, Hkv, BS, D]");
      kc = bp(*k_cache); vc = bp(*v_cache); BS = k_cache->size(2);
    }
  } else {
    TORCH_CHECK(false, "gemv_decode: mode 0..3");
  }
  CHECK_RC(lk_gemv_decode((int)mode, bp(x), x.stride(0), bpo(gamma), (float)eps, bp(w), M, N, K,
                          mode == 1 ? nullptr : bp(out), mode == 1 ? 0 : out.stride(0), rp, ldr, pos, cs, (int)Hq,
                          (int)Hkv, (int)D, kc, vc, sl, BS, neox ? 1 : 0, po ? po->data_ptr<float>() : nullptr,
                          pml ? pml->data_ptr<float>() : nullptr, ctx ? ip(*ctx) : nullptr, (int)max_splits,
                          (int)split, cur_stream()),
           "gemv_decode");
  return out;
}

// Prefill / encoder-regime linear (csrc/gemm.hip): epi(x [M, K] . w[N, K]^T (+ bias)).
// epi 0 none, 1 SwiGLU (w = [Wg; Wu], out [M, N/2]), 2 bias, 3 bias+GELU(erf), 4 bias+ReLU.
at::Tensor gemm(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias, int64_t epi,
                int64_t bn, const c10::optional<at::Tensor>& out_, int64_t variant, int64_t splits) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "x [M,K], w [N,K]");
  check_rows16(x, "x"); check_rows16(w, "w");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(gemm_shape_ok(M, N, K, (int)epi, (int)bn, (int)splits, (int)variant), "gemm: unsupported shape M", M, " N", N,
              " K", K, " epi", epi, " bn", bn, " splits", splits);
  if (epi >= 2) {
    TORCH_CHECK(bias.has_value(), "gemm: this epilogue needs a bias");
    CHECK_CUDA(*bias); CHECK_BF16(*bias); CHECK_CONTIG(*bias);
    TORCH_CHECK(bias->numel() == N && reinterpret_cast<uintptr_t>(bias->data_ptr()) % 16 == 0, "gemm: bias [N], 16-B aligned");
  }
  const int n_out = epi == 1 ? N / 2 : N;
  at::Tensor out = out_ ? *out_ : at::empty({M, n_out}, x.options());
  CHECK_BF16(out); CHECK_LASTDIM(out);
  TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == n_out, "out shape");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 && out.stride(0) % 8 == 0, "out alignment (16 B)");
  // split-K partials: fp32 [splits, M, N] from the caching allocator (stream-ordered reuse)
  at::Tensor ws;
  if (splits > 1) ws = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
  int rc = lk_gemm(bp(x), x.stride(0), bp(w), epi >= 2 ? bp(*bias) : nullptr, M, N, K, (int)epi, (int)bn, (int)variant, bp(out),
                   out.stride(0), cur_stream(), (int)splits, splits > 1 ? ws.data_ptr<float>() : nullptr);
  CHECK_RC(rc, "gemm");
  return out;
}


// The fused prefill chain (csrc/gemm.hip LkEpi): epi 0 / 1 / 7 with an optional folded-RMSNorm
// row scale from ss_in [nt, ld] f32, epi 6 (RESID) updating `resid` in place and writing the
// per-256-column partial sums of squares into ss_out [N / 256, ld].  Returns `out` (RESID: resid).
at::Tensor gemm_fused(const at::Tensor& x, const at::Tensor& w, int64_t epi, int64_t bn, const c10::optional<at::Tensor>& out_,
                      int64_t variant, int64_t splits, const c10::optional<at::Tensor>& ss_in, double eps,
                      const c10::optional<at::Tensor>& resid, const c10::optional<at::Tensor>& ss_out,
                      const c10::optional<at::Tensor>& positions, const c10::optional<at::Tensor>& cos_sin,
                      const c10::optional<at::Tensor>& slots, const c10::optional<at::Tensor>& k_cache,
                      const c10::optional<at::Tensor>& v_cache, int64_t hq, int64_t hkv, int64_t hd) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(w); CHECK_LASTDIM(x); CHECK_CONTIG(w);
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "x [M,K], w [N,K]");
  check_rows16(x, "x"); check_rows16(w, "w");
  const int M = x.size(0), K = x.size(1), N = w.size(0);
  TORCH_CHECK(epi == 0 || epi == 1 || epi == 6 || epi == 7, "gemm_fused: epi must be NONE / SWIGLU / RESID / QKV");
  TORCH_CHECK(gemm_shape_ok(M, N, K, (int)epi, (int)bn, (int)splits, (int)variant), "gemm_fused: unsupported shape M", M, " N", N,
              " K", K, " epi", epi, " bn", bn, " splits", splits);
  LkEpi ea;
  const int H = K;
  if (ss_in) {
    CHECK_CUDA(*ss_in); CHECK_F32(*ss_in); CHECK_CONTIG(*ss_in);
    TORCH_CHECK(ss_in->dim() == 2 && ss_in->size(0) >= 1 && ss_in->size(0) <= 32 && ss_in->size(1) >= M,
                "ss_in must be [nt <= 32, >= M] f32");
    ea.ss_in = ss_in->data_ptr<float>();
    ea.ss_nt = ss_in->size(0);
    ea.ss_ld = ss_in->size(1);
    ea.inv_h = 1.f / (float)H;
    ea.eps = (float)eps;
  }
  at::Tensor out;
  if (epi == 6) {
    TORCH_CHECK(resid && ss_out, "RESID needs resid and ss_out");
    CHECK_CUDA(*resid); CHECK_BF16(*resid); CHECK_LASTDIM(*resid); check_rows16(*resid, "resid");
    TORCH_CHECK(resid->dim() == 2 && resid->size(0) == M && resid->size(1) == N, "resid must be [M, N]");
    CHECK_CUDA(*ss_out); CHECK_F32(*ss_out); CHECK_CONTIG(*ss_out);
    TORCH_CHECK(ss_out->dim() == 2 && ss_out->size(0) == N / 256 && ss_out->size(1) >= M, "ss_out must be [N/256, >= M]");
    ea.resid = bp(*resid);
    ea.ldr = resid->stride(0);
    ea.ss_out = ss_out->data_ptr<float>();
    ea.ss_out_ld = ss_out->size(1);
    out = *resid;
  } else {
    const int n_out = epi == 1 ? N / 2 : N;
    out = out_ ? *out_ : at::empty({M, n_out}, x.options());
    CHECK_BF16(out); CHECK_LASTDIM(out);
    TORCH_CHECK(out.dim() == 2 && out.size(0) == M && out.size(1) == n_out, "out shape");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 && out.stride(0) % 8 == 0, "out alignment (16 B)");
  }
  if (epi == 7) {
    TORCH_CHECK(positions && cos_sin, "QKV needs positions and cos_sin");
    CHECK_I32(*positions); CHECK_CONTIG(*positions); CHECK_F32(*cos_sin); CHECK_CONTIG(*cos_sin);
    TORCH_CHECK(positions->numel() >= M, "positions [>= M]");
    TORCH_CHECK(cos_sin->dim() == 2 && cos_sin->size(1) == hd, "cos_sin [max_pos, hd]");
    TORCH_CHECK(N == (hq + 2 * hkv) * hd && hd % 16 == 0, "QKV: N must be (hq + 2 hkv) * hd");
    ea.pos = ip(*positions);
    ea.cos_sin = cos_sin->data_ptr<float>();
    ea.hq = hq; ea.hkv = hkv; ea.hd = hd;
    if (k_cache || v_cache) {
      TORCH_CHECK(k_cache && v_cache && slots, "QKV: k_cache, v_cache and slots together");
      CHECK_BF16(*k_cache); CHECK_BF16(*v_cache); CHECK_CONTIG(*k_cache); CHECK_CONTIG(*v_cache);
      CHECK_I32(*slots); CHECK_CONTIG(*slots);
      TORCH_CHECK(slots->numel() >= M, "slots [>= M]");
      TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == hkv && k_cache->size(3) == hd && k_cache->sizes() == v_cache->sizes(),
                  "caches [num_blocks, hkv, bs, hd]");
      ea.kc = bp(*k_cache); ea.vc = bp(*v_cache); ea.slots = ip(*slots); ea.bs = k_cache->size(2);
    }
  }
  at::Tensor ws;
  if (splits > 1) ws = at::empty({splits, M, N}, x.options().dtype(at::kFloat));
  int rc = lk_gemm(bp(x), x.stride(0), bp(w), nullptr, M, N, K, (int)epi, (int)bn, (int)variant, bp(out), out.stride(0),
                   cur_stream(), (int)splits, splits > 1 ? ws.data_ptr<float>() : nullptr, &ea);
  CHECK_RC(rc, "gemm_fused");
  return out;
}

// embedding rows from int32 ids (vocab shard [lo, lo + n_local) of a vocab-parallel table: others 0)
at::Tensor embed_rows(const at::Tensor& table, const at::Tensor& ids, int64_t lo, int64_t n_local) {
  CHECK_CUDA(table); CHECK_BF16(table); CHECK_CONTIG(table); CHECK_CUDA(ids); CHECK_I32(ids); CHECK_CONTIG(ids);
  const int strict = (lo == 0 && n_local < 0) ? 1 : 0;  // the whole table: an id outside it is an error
  if (n_local < 0) n_local = table.size(0);
  TORCH_CHECK(table.dim() == 2 && table.size(1) % 8 == 0 && n_local <= table.size(0), "table [V, H], H % 8");
  check_rows16(table, "table");
  at::Tensor out = at::empty({ids.numel(), table.size(1)}, table.options());
  CHECK_RC(lk_embed_rows(bp(out), bp(table), ip(ids), ids.numel(), table.size(1), lo, n_local, cur_stream(), strict),
           "embed_rows");
  return out;
}

// ids[dst] = prev[src] (in-flight decode inputs of a pipelined step)
void scatter_ids(at::Tensor& ids, const at::Tensor& dst, const at::Tensor& prev, const at::Tensor& src) {
  CHECK_CUDA(ids); CHECK_I32(ids); CHECK_CONTIG(ids); CHECK_I32(prev); CHECK_CONTIG(prev);
  TORCH_CHECK(dst.scalar_type() == at::kLong && src.scalar_type() == at::kLong && dst.is_contiguous() && src.is_contiguous() &&
              dst.numel() == src.numel(), "dst / src int64 of equal length");
  CHECK_RC(lk_scatter_ids(ids.data_ptr<int>(), dst.data_ptr<int64_t>(), prev.data_ptr<int>(), src.data_ptr<int64_t>(),
                          (int)dst.numel(), cur_stream()), "scatter_ids");
}

// out[r] = x[idx[r]] (bf16 rows)
at::Tensor gather_rows(const at::Tensor& x, const at::Tensor& idx) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_LASTDIM(x); check_rows16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 8 == 0, "x [T, H], H % 8");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_contiguous(), "idx int64");
  at::Tensor out = at::empty({idx.numel(), x.size(1)}, x.options());
  CHECK_RC(lk_gather_rows(bp(out), bp(x), x.stride(0), idx.data_ptr<int64_t>(), idx.numel(), x.size(1), cur_stream()),
           "gather_rows");
  return out;
}

int64_t gemm_streamk(int64_t mode) { return lk_gemm_streamk((int)mode); }

bool gemm_supported(int64_t M, int64_t N, int64_t K, int64_t epi, int64_t bn, int64_t splits, int64_t variant) {
  return gemm_shape_ok((int)M, (int)N, (int)K, (int)epi, (int)bn, (int)splits, (int)variant);
}

std::vector<int64_t> ws_plan(int64_t M, int64_t N, int64_t K, bool swiglu) {
  int bn = 64, s = 1;
  lk_wsgemm_plan((int)M, (int)N, (int)K, swiglu ? 1 : 0, &bn, &s);
  return {bn, s};
}

int64_t skinny_splits(int64_t M, int64_t N, int64_t K, bool swiglu) {
  return lk_skinny_splits((int)M, (int)N, (int)K, swiglu ? 1 : 0);
}

void activation_(at::Tensor& x, const c10::optional<at::Tensor>& bias, int64_t kind) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_LASTDIM(x);
  TORCH_CHECK(x.dim() == 2, "x must be 2-D");
  check_rows16(x, "x");
  if (bias) { CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == x.size(1), "bias shape"); }
  int rc = lk_activation(bp(x), bpo(bias), x.size(0), x.size(1), x.stride(0), (int)kind, cur_stream());
  CHECK_RC(rc, "activation");
}

void rope_kv_(at::Tensor& qkv, const at::Tensor& positions, const at::Tensor& cos_sin, int64_t Hq,
              int64_t Hkv, int64_t D, const c10::optional<at::Tensor>& k_cache,
              const c10::optional<at::Tensor>& v_cache, const c10::optional<at::Tensor>& slots,
              bool neox, bool write_k_inplace) {
  CHECK_CUDA(qkv); CHECK_BF16(qkv); CHECK_LASTDIM(qkv); CHECK_I32(positions); CHECK_F32(cos_sin);
  CHECK_CONTIG(cos_sin); CHECK_CONTIG(positions);
  TORCH_CHECK(qkv.dim() == 2 && qkv.size(1) >= (Hq + 2 * Hkv) * D, "qkv must be [T, >=(Hq+2Hkv)*D]");
  TORCH_CHECK(cos_sin.size(1) == D, "cos_sin must be [max_pos, D]");
  check_rows16(qkv, "qkv");
  const long T = qkv.size(0);
  TORCH_CHECK(positions.numel() == T, "positions");
  int BS = 1;
  if (k_cache || v_cache) {
    TORCH_CHECK(k_cache && v_cache && slots, "k_cache, v_cache and slots go together");
    CHECK_BF16(*k_cache); CHECK_BF16(*v_cache); CHECK_CONTIG(*k_cache); CHECK_CONTIG(*v_cache);
    CHECK_I32(*slots); TORCH_CHECK(slots->numel() == T, "slots");
    TORCH_CHECK(k_cache->dim() == 4 && k_cache->size(1) == Hkv && k_cache->size(3) == D, "k_cache must be [NB, Hkv, BS, D]");
    TORCH_CHECK(v_cache->sizes() == k_cache->sizes(), "v_cache shape");
    BS = k_cache->size(2);
  }
  int rc = lk_rope_kv(bp(qkv), qkv.stride(0), ip(positions), cos_sin.data_ptr<float>(), T, Hq, Hkv, D,
                      bpo(k_cache), bpo(v_cache), ipo(slots), BS, neox ? 1 : 0, write_k_inplace ? 1 : 0,
                      cur_stream());
  CHECK_RC(rc, "rope_kv");
}

void kv_write(const at::Tensor& k, const at::Tensor& v, at::Tensor& k_cache, at::Tensor& v_cache,
              const at::Tensor& slots) {
  CHECK_CUDA(k); CHECK_BF16(k); CHECK_BF16(v); CHECK_I32(slots);
  TORCH_CHECK(k.dim() == 3 && v.sizes() == k.sizes(), "k/v must be [T, Hkv, D]");
  TORCH_CHECK(k.stride(2) == 1 && k.stride(1) == k.size(2) && v.stride(2) == 1 && v.stride(1) == v.size(2), "k/v inner layout");
  const int Hkv = k.size(1), D = k.size(2);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.size(1) == Hkv && k_cache.size(3) == D && k_cache.is_contiguous() && v_cache.is_contiguous(), "cache layout");
  int rc = lk_kv_write(bp(k), k.stride(0), bp(v), v.stride(0), bp(k_cache), bp(v_cache), ip(slots),
                       k.size(0), Hkv, D, k_cache.size(2), cur_stream());
  CHECK_RC(rc, "kv_write");
}

int64_t decode_splits(int64_t max_context, int64_t split) { return lk_decode_splits((int)max_context, (int)split); }
int64_t decode_split_size(int64_t B, int64_t Hkv) { return lk_decode_split_size((int)B, (int)Hkv); }

// k_start: optional device int32 [1] -- keys [0, k_start) are a prefix shared by every row,
// attended separately (flash_prefill partial mode) into pp_o [B, Hq, D] / pp_ml [B, Hq, 2]
// and merged by the reduce kernel (cascade decode).
at::Tensor paged_decode(const at::Tensor& q, const at::Tensor& k_cache, const at::Tensor& v_cache,
                        const at::Tensor& block_tables, const at::Tensor& ctx_lens, int64_t max_splits,
                        int64_t split, double scale, const c10::optional<at::Tensor>& part_o,
                        const c10::optional<at::Tensor>& part_ml, const c10::optional<at::Tensor>& out_,
                        const c10::optional<at::Tensor>& k_start, const c10::optional<at::Tensor>& pp_o,
                        const c10::optional<at::Tensor>& pp_ml, const c10::optional<at::Tensor>& tickets,
                        bool reduce) {
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(k_cache); CHECK_BF16(v_cache);
  CHECK_I32(block_tables); CHECK_I32(ctx_lens); CHECK_CONTIG(ctx_lens);
  TORCH_CHECK(q.dim() == 3 && q.stride(2) == 1 && q.stride(1) == q.size(2), "q must be [B, Hq, D] (row-strided)");
  const int B = q.size(0), Hq = q.size(1), D = q.size(2);
  TORCH_CHECK(k_cache.dim() == 4 && k_cache.is_contiguous() && v_cache.is_contiguous() && v_cache.sizes() == k_cache.sizes(), "cache layout");
  const int Hkv = k_cache.size(1), BS = k_cache.size(2);
  TORCH_CHECK(k_cache.size(3) == D, "head dim mismatch");
  TORCH_CHECK(block_tables.dim() == 2 && block_tables.size(0) >= B && block_tables.stride(1) == 1, "block_tables");
  TORCH_CHECK(ctx_lens.numel() >= B, "ctx_lens");
  TORCH_CHECK(split >= 32 && split <= 2048 && split % 32 == 0 && split % BS == 0, "decode split must be a multiple of 32 and of the block size, <= 2048");
  TORCH_CHECK(max_splits >= 1 && (long)(max_splits - 1) * split < (long)block_tables.size(1) * BS, "max_splits exceeds block table capacity");
  check_rows16(q, "q");
  const bool cascade = pp_o.has_value();
  TORCH_CHECK(cascade == pp_ml.has_value() && cascade == k_start.has_value(), "cascade needs k_start, pp_o and pp_ml");
  if (cascade) {
    CHECK_CUDA(*k_start); CHECK_I32(*k_start); TORCH_CHECK(k_start->numel() >= 1, "k_start");
    CHECK_F32(*pp_o); CHECK_F32(*pp_ml); CHECK_CONTIG(*pp_o); CHECK_CONTIG(*pp_ml);
    TORCH_CHECK(pp_o->numel() >= (long)B * Hq * D && pp_ml->numel() >= (long)B * Hq * 2, "prefix partials too small");
  }
  at::Tensor out = out_ ? *out_ : at::empty({B, Hq, D}, q.options());
  TORCH_CHECK(out.size(0) == B && out.size(1) == Hq && out.size(2) == D && out.stride(2) == 1 && out.stride(1) == D, "out layout");
  at::Tensor po, pm;
  const bool parts = max_splits > 1 || cascade;
  if (parts) {
    po = part_o ? *part_o : at::empty({B, Hq, max_splits, D}, q.options().dtype(at::kFloat));
    pm = part_ml ? *part_ml : at::empty({B, Hq, max_splits, 2}, q.options().dtype(at::kFloat));
    TORCH_CHECK(po.numel() >= (long)B * Hq * max_splits * D && pm.numel() >= (long)B * Hq * max_splits * 2, "partials too small");
    CHECK_F32(po); CHECK_F32(pm);
  }
  if (tickets) {  // fused split merge: one zero-initialised int32 counter per (seq, kv head)
    CHECK_CUDA(*tickets); CHECK_I32(*tickets); CHECK_CONTIG(*tickets);
    TORCH_CHECK(tickets->numel() >= (long)B * Hkv, "tickets: one counter per (sequence, kv head)");
  }
  int rc = lk_paged_decode(bp(q), q.stride(0), bp(k_cache), bp(v_cache), ip(block_tables), block_tables.stride(0),
                           ip(ctx_lens), bp(out), out.stride(0), parts ? po.data_ptr<float>() : nullptr,
                           parts ? pm.data_ptr<float>() : nullptr, B, Hq, Hkv, D, BS, (int)max_splits,
                           (int)split, (float)scale, cascade ? ip(*k_start) : nullptr,
                           cascade ? pp_o->data_ptr<float>() : nullptr, cascade ? pp_ml->data_ptr<float>() : nullptr,
                           cur_stream(), tickets ? tickets->data_ptr<int>() : nullptr, reduce ? 1 : 0);
  CHECK_RC(rc, "paged_decode");
  return out;
}

int64_t prefill_rows_per_tile(int64_t G, int64_t D) { return lk_prefill_rows_per_tile((int)G, (int)D); }

at::Tensor flash_prefill(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
                         const c10::optional<at::Tensor>& block_tables, const at::Tensor& cu_q,
                         const c10::optional<at::Tensor>& ctx_lens, const at::Tensor& tile_seq,
                         const at::Tensor& tile_q0, int64_t Hq, int64_t Hkv, int64_t D, double scale,
                         bool causal, const c10::optional<at::Tensor>& out_,
                         const c10::optional<at::Tensor>& part_o, const c10::optional<at::Tensor>& part_ml,
                         const c10::optional<at::Tensor>& q_past) {
  CHECK_CUDA(q); CHECK_BF16(q); CHECK_BF16(k); CHECK_BF16(v); CHECK_LASTDIM(q);
  if (q_past) {
    CHECK_I32(*q_past);
    TORCH_CHECK(q_past->numel() >= cu_q.numel() - 1, "q_past: one entry per sequence");
  }
  CHECK_I32(cu_q); CHECK_I32(tile_seq); CHECK_I32(tile_q0);
  TORCH_CHECK(q.dim() == 2 && q.size(1) >= Hq * D, "q must be [T, >=Hq*D] (head-major rows)");
  check_rows16(q, "q");
  const long T = q.size(0);
  const bool paged = block_tables.has_value();
  int BS = 0, bt_stride = 0;
  long ks = 0, vs = 0;
  if (paged) {
    CHECK_I32(*block_tables);
    TORCH_CHECK(ctx_lens.has_value(), "ctx_lens required for paged prefill");
    TORCH_CHECK(k.dim() == 4 && k.size(1) == Hkv && k.size(3) == D && k.is_contiguous() && v.is_contiguous() && v.sizes() == k.sizes(), "cache layout");
    BS = k.size(2);
    bt_stride = block_tables->stride(0);
  } else {
    TORCH_CHECK(k.dim() == 2 && v.dim() == 2 && k.size(0) == T && v.size(0) == T && k.size(1) >= Hkv * D && v.size(1) >= Hkv * D, "dense k/v must be [T, >=Hkv*D]");
    CHECK_LASTDIM(k); CHECK_LASTDIM(v); check_rows16(k, "k"); check_rows16(v, "v");
    ks = k.stride(0);
    vs = v.stride(0);
  }
  if (ctx_lens) CHECK_I32(*ctx_lens);
  TORCH_CHECK(tile_seq.numel() == tile_q0.numel(), "tile arrays");
  const bool partial = part_o.has_value();
  TORCH_CHECK(partial == part_ml.has_value(), "partial mode needs part_o and part_ml");
  if (partial) {
    CHECK_F32(*part_o); CHECK_F32(*part_ml); CHECK_CONTIG(*part_o); CHECK_CONTIG(*part_ml);
    TORCH_CHECK(part_o->numel() >= T * Hq * D && part_ml->numel() >= T * Hq * 2, "partials too small");
    TORCH_CHECK(D % 4 == 0, "partial mode needs D % 4 == 0");
  }
  at::Tensor out = out_ ? *out_ : (partial ? *part_o : at::empty({T, Hq * D}, q.options()));
  if (!partial) {
    CHECK_LASTDIM(out); check_rows16(out, "out");
    TORCH_CHECK(out.size(0) == T && out.size(1) >= Hq * D, "out shape");
  }
  int rc = lk_flash_prefill(bp(q), q.stride(0), bp(k), bp(v), ks, vs, paged ? ip(*block_tables) : nullptr,
                            bt_stride, ip(cu_q), ipo(ctx_lens), ip(tile_seq), ip(tile_q0), tile_seq.numel(),
                            partial ? nullptr : bp(out), partial ? 0 : out.stride(0), Hq, Hkv, D, BS, (float)scale,
                            causal ? 1 : 0, paged ? 1 : 0, partial ? part_o->data_ptr<float>() : nullptr,
                            partial ? part_ml->data_ptr<float>() : nullptr, ipo(q_past), cur_stream());
  CHECK_RC(rc, "flash_prefill");
  return out;
}

std::vector<at::Tensor> knn_topk(const at::Tensor& corpus, const at::Tensor& cnorm, const at::Tensor& queries,
                                 const at::Tensor& qnorm, int64_t K, bool force_fused) {
  CHECK_CUDA(corpus); CHECK_BF16(corpus); CHECK_CONTIG(corpus); CHECK_F32(cnorm); CHECK_CONTIG(cnorm);
  CHECK_BF16(queries); CHECK_CONTIG(queries); CHECK_F32(qnorm); CHECK_CONTIG(qnorm);
  TORCH_CHECK(corpus.dim() == 2 && queries.dim() == 2 && corpus.size(1) == queries.size(1), "dimension mismatch");
  const long N = corpus.size(0);
  const int D = corpus.size(1), nq = queries.size(0);
  TORCH_CHECK(cnorm.numel() == N && qnorm.numel() == nq, "norm shapes");
  TORCH_CHECK(K >= 1 && K <= 64, "K in [1, 64]");
  auto fo = corpus.options().dtype(at::kFloat);
  auto io = corpus.options().dtype(at::kInt);
  const int kk = (int)std::min<long>(K, std::max<long>(N, 1));
  // the merge kernel writes every one of the K slots of every query (-inf / -1 pads)
  if (N == 0 || nq == 0) return {at::full({nq, (long)K}, -INFINITY, fo), at::full({nq, (long)K}, -1, io)};
  at::Tensor out_s = at::empty({nq, (long)K}, fo);
  at::Tensor out_i = at::empty({nq, (long)K}, io);
  if (D % 64 == 0 && nq <= 256 && !force_fused) {
    // corpus streamed once by the LDS-DMA weight-streaming GEMM (dots in f32), then a
    // normalise + chunked top-k pass and the shared merge
    at::Tensor scores = at::empty({nq, N}, fo);
    int rc = lk_ws_scores_f32(bp(queries), D, bp(corpus), nq, N, D, scores.data_ptr<float>(), N, cur_stream());
    CHECK_RC(rc, "knn scores");
    const int nc = lk_knn_score_chunks(N);
    at::Tensor ps = at::empty({nq, nc, kk}, fo);
    at::Tensor pi = at::empty({nq, nc, kk}, io);
    rc = lk_knn_score_topk(scores.data_ptr<float>(), N, cnorm.data_ptr<float>(), qnorm.data_ptr<float>(), N, nq, kk,
                           ps.data_ptr<float>(), pi.data_ptr<int>(), cur_stream());
    CHECK_RC(rc, "knn score_topk");
    rc = lk_knn_merge(ps.data_ptr<float>(), pi.data_ptr<int>(), nq, nc * kk, (int)K, out_s.data_ptr<float>(),
                      out_i.data_ptr<int>(), cur_stream());
    CHECK_RC(rc, "knn_merge");
    return {out_s, out_i};
  }
  const int nb = lk_knn_nblocks(N);
  at::Tensor ps = at::empty({nq, nb, kk}, fo);
  at::Tensor pi = at::empty({nq, nb, kk}, io);
  int rc = lk_knn_partial(bp(corpus), cnorm.data_ptr<float>(), N, D, bp(queries), qnorm.data_ptr<float>(), nq, kk,
                          ps.data_ptr<float>(), pi.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "knn_partial");
  rc = lk_knn_merge(ps.data_ptr<float>(), pi.data_ptr<int>(), nq, nb * kk, (int)K, out_s.data_ptr<float>(),
                    out_i.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "knn_merge");
  return {out_s, out_i};
}

std::vector<at::Tensor> knn_merge(const at::Tensor& cand_s, const at::Tensor& cand_i, int64_t K) {
  CHECK_CUDA(cand_s); CHECK_F32(cand_s); CHECK_I32(cand_i); CHECK_CONTIG(cand_s); CHECK_CONTIG(cand_i);
  TORCH_CHECK(cand_s.dim() == 2 && cand_s.sizes() == cand_i.sizes(), "candidates [nq, ncand]");
  const int nq = cand_s.size(0), nc = cand_s.size(1);
  at::Tensor out_s = at::empty({nq, K}, cand_s.options());
  at::Tensor out_i = at::empty({nq, K}, cand_i.options());
  int rc = lk_knn_merge(cand_s.data_ptr<float>(), cand_i.data_ptr<int>(), nq, nc, (int)K, out_s.data_ptr<float>(),
                        out_i.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "knn_merge");
  return {out_s, out_i};
}

// out: optional destination rows [B, H] (f32 or bf16, unit last stride, 16-byte rows), e.g. a
// slice of the caller's embedding matrix; default a new f32 [B, H]
at::Tensor pool_normalize(const at::Tensor& hidden, const at::Tensor& cu, int64_t mode, bool normalize,
                          const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(hidden); CHECK_BF16(hidden); CHECK_LASTDIM(hidden); CHECK_I32(cu); CHECK_CONTIG(cu);
  check_rows16(hidden, "hidden");
  const int B = cu.numel() - 1, H = hidden.size(1);
  at::Tensor out = out_ ? *out_ : at::empty({B, H}, hidden.options().dtype(at::kFloat));
  const bool obf = out.scalar_type() == at::kBFloat16;
  TORCH_CHECK(obf || out.scalar_type() == at::kFloat, "out must be f32 or bf16");
  CHECK_CUDA(out); CHECK_LASTDIM(out); check_rows16(out, "out");
  TORCH_CHECK(out.dim() == 2 && out.size(0) == B && out.size(1) == H, "out [B, H]");
  int rc = lk_pool_normalize(bp(hidden), hidden.stride(0), ip(cu), B, H, (int)mode, normalize ? 1 : 0,
                             out.data_ptr(), out.stride(0), obf ? 1 : 0, cur_stream());
  CHECK_RC(rc, "pool_normalize");
  return out;
}

at::Tensor row_norms(const at::Tensor& x) {
  CHECK_CUDA(x); CHECK_BF16(x); CHECK_CONTIG(x);
  at::Tensor out = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  int rc = lk_row_norms(bp(x), x.size(0), x.size(1), out.data_ptr<float>(), cur_stream());
  CHECK_RC(rc, "row_norms");
  return out;
}

at::Tensor select_tokens(const at::Tensor& logits, const c10::optional<at::Tensor>& temps, int64_t seed,
                         int64_t step, const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(logits); CHECK_LASTDIM(logits);
  TORCH_CHECK(logits.dim() == 2, "logits [B, V]");
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(is_bf16 || logits.scalar_type() == at::kFloat, "logits must be bf16 or f32");
  TORCH_CHECK(logits.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(logits.data_ptr()) % 32 == 0, "logits rows must be 32-byte aligned");
  const int B = logits.size(0), V = logits.size(1);
  if (temps) { CHECK_F32(*temps); TORCH_CHECK(temps->numel() >= B, "temps"); }
  at::Tensor out = out_ ? *out_ : at::empty({B}, logits.options().dtype(at::kInt));
  CHECK_I32(out);
  int rc = lk_select_tokens(logits.data_ptr(), is_bf16 ? 1 : 0, logits.stride(0), B, V,
                            temps ? temps->data_ptr<float>() : nullptr, (unsigned long long)seed, (int)step,
                            out.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "select_tokens");
  return out;
}

// vocab-parallel greedy (parallel/tp.py TPGroup.greedy_ids): per-row packed (value, id) keys
at::Tensor argmax_key(const at::Tensor& logits, int64_t vocab_lo) {
  CHECK_CUDA(logits); CHECK_LASTDIM(logits);
  TORCH_CHECK(logits.dim() == 2, "logits [B, V]");
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(is_bf16 || logits.scalar_type() == at::kFloat, "logits must be bf16 or f32");
  TORCH_CHECK(logits.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(logits.data_ptr()) % 32 == 0, "logits rows must be 32-byte aligned");
  TORCH_CHECK(vocab_lo >= 0 && vocab_lo + logits.size(1) < (1ll << 31), "vocab_lo");
  const int B = logits.size(0), V = logits.size(1);
  at::Tensor keys = at::empty({B}, logits.options().dtype(at::kLong));
  int rc = lk_argmax_key(logits.data_ptr(), is_bf16 ? 1 : 0, logits.stride(0), B, V, (int)vocab_lo,
                         reinterpret_cast<long long*>(keys.data_ptr<int64_t>()), cur_stream());
  CHECK_RC(rc, "argmax_key");
  return keys;
}

at::Tensor keys_to_ids(const at::Tensor& keys) {
  CHECK_CUDA(keys); CHECK_CONTIG(keys);
  TORCH_CHECK(keys.scalar_type() == at::kLong && keys.dim() == 2, "keys [W, R] int64");
  const int W = keys.size(0), R = keys.size(1);
  at::Tensor ids = at::empty({R}, keys.options().dtype(at::kInt));
  int rc = lk_keys_to_ids(reinterpret_cast<const long long*>(keys.data_ptr<int64_t>()), W, R, ids.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "keys_to_ids");
  return ids;
}

// token selection restricted per row to an allowed id list (grammar-constrained decoding)
at::Tensor select_allowed(const at::Tensor& logits, const at::Tensor& plan, const c10::optional<at::Tensor>& temps,
                          int64_t seed, int64_t step) {
  CHECK_CUDA(logits); CHECK_LASTDIM(logits); CHECK_CUDA(plan); CHECK_I32(plan); CHECK_CONTIG(plan);
  TORCH_CHECK(logits.dim() == 2, "logits [B, V]");
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(is_bf16 || logits.scalar_type() == at::kFloat, "logits must be bf16 or f32");
  TORCH_CHECK(logits.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(logits.data_ptr()) % 32 == 0, "logits rows must be 32-byte aligned");
  const int B = logits.size(0), V = logits.size(1);
  TORCH_CHECK(plan.numel() >= 2 * B + 1, "plan must hold [B flags | B+1 offsets | ids]");
  if (temps) { CHECK_F32(*temps); TORCH_CHECK(temps->numel() >= B, "temps"); }
  at::Tensor out = at::empty({B}, logits.options().dtype(at::kInt));
  int rc = lk_select_allowed(logits.data_ptr(), is_bf16 ? 1 : 0, logits.stride(0), B, V,
                             temps ? temps->data_ptr<float>() : nullptr, (unsigned long long)seed, (int)step,
                             plan.data_ptr<int>(), out.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "select_allowed");
  return out;
}

// Fused Ollama-default sampler (csrc/sampling.hip lk_sample): see kernels.h
at::Tensor sample(at::Tensor& logits, const at::Tensor& prm, at::Tensor& hist, at::Tensor& hist_len, int64_t seed,
                  const c10::optional<at::Tensor>& out_) {
  CHECK_CUDA(logits); CHECK_F32(logits); CHECK_LASTDIM(logits);
  TORCH_CHECK(logits.dim() == 2, "logits [B, V]");
  const int B = logits.size(0), V = logits.size(1);
  CHECK_I32(prm); CHECK_CONTIG(prm); TORCH_CHECK(prm.dim() == 2 && prm.size(0) == B && prm.size(1) == 8, "prm [B, 8]");
  CHECK_I32(hist); CHECK_CONTIG(hist); TORCH_CHECK(hist.dim() == 2, "hist [slots, W]");
  CHECK_I32(hist_len); CHECK_CONTIG(hist_len); TORCH_CHECK(hist_len.numel() == hist.size(0), "hist_len [slots]");
  TORCH_CHECK(prm.is_cuda() && hist.is_cuda() && hist_len.is_cuda(), "sampler state must be on the GPU");
  // slot ids / top_k are read by the kernel: checked here (one small D2H of the parameter rows is
  // avoided by the caller, which validates the host copy it uploads: ops.sample)
  at::Tensor out = out_ ? *out_ : at::empty({B}, logits.options().dtype(at::kInt));
  CHECK_I32(out);
  int rc = lk_sample(logits.data_ptr<float>(), logits.stride(0), B, V, ip(prm), hist.data_ptr<int>(),
                     hist_len.data_ptr<int>(), hist.size(1), (unsigned long long)seed, out.data_ptr<int>(), cur_stream());
  CHECK_RC(rc, "sample");
  return out;
}

void repeat_penalty_(at::Tensor& logits, const at::Tensor& window, const at::Tensor& penalty) {
  CHECK_CUDA(logits); CHECK_I32(window); CHECK_F32(penalty); CHECK_CONTIG(window);
  const bool is_bf16 = logits.scalar_type() == at::kBFloat16;
  TORCH_CHECK(window.dim() == 2 && window.size(0) == logits.size(0), "window [B, W]");
  int rc = lk_repeat_penalty(logits.data_ptr(), is_bf16 ? 1 : 0, logits.stride(0), logits.size(0), ip(window),
                             window.size(1), penalty.data_ptr<float>(), cur_stream());
  CHECK_RC(rc, "repeat_penalty");
}

// One-shot xGMI all-reduce state of one rank (K14): its IPC-exported staging + signal buffers
// and the peers' buffers opened in this process.  Python exchanges handles() over the TP
// control group, then calls open(); all_reduce() is hipGraph-capturable.
struct XgmiAr {
  int rank = 0, world = 1;
  size_t bytes = 0;
  void* data = nullptr;
  void* sig = nullptr;
  int* err = nullptr;
  std::vector<void*> pdata, psig;  // per rank, as mapped here
  std::vector<void*> opened;       // IPC mappings to close

  XgmiAr(int rank_, int world_, int64_t bytes_) : rank(rank_), world(world_), bytes((size_t)bytes_) {
    TORCH_CHECK(world >= 1 && world <= lk_xgmi_ar_max_ranks() && rank >= 0 && rank < world, "xgmi_ar: rank/world");
    TORCH_CHECK(bytes_ > 0 && bytes_ % 16 == 0, "xgmi_ar: staging bytes must be a positive multiple of 16");
    const size_t sig_bytes = (size_t)lk_xgmi_ar_sig_words() * sizeof(unsigned);
    // two regions of `bytes`: the staged inputs and (two-shot) the reduced slices
    TORCH_CHECK(hipMalloc(&data, 2 * bytes) == hipSuccess, "xgmi_ar: hipMalloc staging");
    TORCH_CHECK(hipExtMallocWithFlags(&sig, sig_bytes, hipDeviceMallocUncached) == hipSuccess, "xgmi_ar: signal alloc");
    TORCH_CHECK(hipMalloc(reinterpret_cast<void**>(&err), sizeof(int)) == hipSuccess, "xgmi_ar: hipMalloc err");
    TORCH_CHECK(hipMemset(sig, 0, sig_bytes) == hipSuccess && hipMemset(err, 0, sizeof(int)) == hipSuccess &&
                hipDeviceSynchronize() == hipSuccess, "xgmi_ar: init");
    pdata.assign(world, nullptr);
    psig.assign(world, nullptr);
    pdata[rank] = data;
    psig[rank] = sig;
  }
  ~XgmiAr() {
    for (void* p : opened) (void)hipIpcCloseMemHandle(p);
    if (data) (void)hipFree(data);
    if (sig) (void)hipFree(sig);
    if (err) (void)hipFree(err);
  }
  py::bytes handles() const {
    hipIpcMemHandle_t h[2];
    TORCH_CHECK(hipIpcGetMemHandle(&h[0], data) == hipSuccess, "xgmi_ar: hipIpcGetMemHandle(staging)");
    TORCH_CHECK(hipIpcGetMemHandle(&h[1], sig) == hipSuccess, "xgmi_ar: hipIpcGetMemHandle(signal)");
    return py::bytes(reinterpret_cast<const char*>(h), sizeof(h));
  }
  void open(const std::vector<py::bytes>& all) {
    TORCH_CHECK((int)all.size() == world, "xgmi_ar: one handle blob per rank");
    for (int r = 0; r < world; ++r) {
      if (r == rank) continue;
      std::string s = all[r];
      TORCH_CHECK(s.size() == 2 * sizeof(hipIpcMemHandle_t), "xgmi_ar: bad handle blob");
      hipIpcMemHandle_t h[2];
      memcpy(h, s.data(), sizeof(h));
      void *d = nullptr, *g = nullptr;
      TORCH_CHECK(hipIpcOpenMemHandle(&d, h[0], hipIpcMemLazyEnablePeerAccess) == hipSuccess,
                  "xgmi_ar: hipIpcOpenMemHandle(staging) of rank ", r);
      TORCH_CHECK(hipIpcOpenMemHandle(&g, h[1], hipIpcMemLazyEnablePeerAccess) == hipSuccess,
                  "xgmi_ar: hipIpcOpenMemHandle(signal) of rank ", r);
      opened.push_back(d);
      opened.push_back(g);
      pdata[r] = d;
      psig[r] = g;
    }
  }
  void all_reduce(const at::Tensor& in, at::Tensor& out) {
    CHECK_CUDA(in); CHECK_BF16(in); CHECK_BF16(out); CHECK_CONTIG(in); CHECK_CONTIG(out);
    TORCH_CHECK(in.numel() == out.numel(), "xgmi_ar: in/out size");
    TORCH_CHECK(in.numel() % 8 == 0 && (size_t)in.numel() * 2 <= bytes, "xgmi_ar: numel must be a multiple of 8 and fit the staging buffer");
    for (int r = 0; r < world; ++r) TORCH_CHECK(pdata[r] && psig[r], "xgmi_ar: open() not called");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "xgmi_ar: 16-B alignment");
    int rc = lk_xgmi_allreduce(reinterpret_cast<bf16_t* const*>(pdata.data()), reinterpret_cast<unsigned* const*>(psig.data()),
                               rank, world, bp(in), bp(out), in.numel(), err, cur_stream());
    CHECK_RC(rc, "xgmi_allreduce");
  }
  // out = RMSNorm(allreduce(x) + residual) * w with residual updated in place (one kernel)
  void all_reduce_rmsnorm(const at::Tensor& x, at::Tensor& residual, const at::Tensor& w, double eps, at::Tensor& out) {
    CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(residual); CHECK_BF16(w); CHECK_BF16(out);
    CHECK_CONTIG(x); CHECK_CONTIG(residual); CHECK_CONTIG(w); CHECK_CONTIG(out);
    TORCH_CHECK(x.dim() == 2 && residual.sizes() == x.sizes() && out.sizes() == x.sizes() && w.numel() == x.size(1),
                "xgmi_ar_rmsnorm: x / residual / out [T, H], w [H]");
    TORCH_CHECK(x.size(1) % 8 == 0 && (size_t)x.numel() * 2 <= bytes, "xgmi_ar_rmsnorm: H % 8 and the staging size");
    for (int r = 0; r < world; ++r) TORCH_CHECK(pdata[r] && psig[r], "xgmi_ar: open() not called");
    int rc = lk_xgmi_allreduce_rmsnorm(reinterpret_cast<bf16_t* const*>(pdata.data()),
                                       reinterpret_cast<unsigned* const*>(psig.data()), rank, world, bp(x), bp(residual),
                                       bp(w), bp(out), (int)x.size(0), (int)x.size(1), (float)eps, err, cur_stream());
    CHECK_RC(rc, "xgmi_allreduce_rmsnorm");
  }
  // two-shot (reduce-scatter + all-gather over the peer mappings) all-reduce of x [T, H] into
  // out, or with residual / w given: residual += sum, out = RMSNorm(residual) * w
  void all_reduce2(const at::Tensor& x, at::Tensor& out, const c10::optional<at::Tensor>& residual,
                   const c10::optional<at::Tensor>& w, double eps) {
    CHECK_CUDA(x); CHECK_BF16(x); CHECK_BF16(out); CHECK_CONTIG(x); CHECK_CONTIG(out);
    TORCH_CHECK(x.dim() == 2 && out.sizes() == x.sizes() && x.size(1) % 8 == 0, "xgmi_ar2: x / out [T, H], H % 8");
    TORCH_CHECK((size_t)x.numel() * 2 <= bytes, "xgmi_ar2: message larger than the staging region");
    TORCH_CHECK(residual.has_value() == w.has_value(), "xgmi_ar2: residual and w together");
    bf16_t* rp = nullptr;
    const bf16_t* wp = nullptr;
    if (residual.has_value()) {
      CHECK_BF16((*residual)); CHECK_CONTIG((*residual)); CHECK_BF16((*w)); CHECK_CONTIG((*w));
      TORCH_CHECK(residual->sizes() == x.sizes() && w->numel() == x.size(1), "xgmi_ar2: residual [T, H], w [H]");
      rp = bp(*residual);
      wp = bp(*w);
    }
    for (int r = 0; r < world; ++r) TORCH_CHECK(pdata[r] && psig[r], "xgmi_ar: open() not called");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0, "xgmi_ar2: 16-B alignment");
    int rc = lk_xgmi_allreduce2(reinterpret_cast<bf16_t* const*>(pdata.data()),
                                reinterpret_cast<unsigned* const*>(psig.data()), (long)(bytes / 2), rank, world, bp(x), rp,
                                wp, bp(out), (int)x.size(0), (int)x.size(1), (float)eps, rp != nullptr, err,
                                cur_stream());
    CHECK_RC(rc, "xgmi_allreduce2");
  }
  // raw-byte all-gather (root < 0: out = world x in) or broadcast from root (out = root's in)
  void gather(const at::Tensor& in, at::Tensor& out, int64_t root) {
    CHECK_CUDA(in); CHECK_CUDA(out); CHECK_CONTIG(in); CHECK_CONTIG(out);
    const long nb = in.numel() * in.element_size();
    TORCH_CHECK(nb % 16 == 0 && (size_t)nb <= bytes, "xgmi_gather: bytes must be a multiple of 16 and fit the staging buffer");
    TORCH_CHECK(out.numel() * out.element_size() == (root < 0 ? world * nb : nb), "xgmi_gather: out size");
    TORCH_CHECK(root < world, "xgmi_gather: root");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(in.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
                "xgmi_gather: 16-B alignment");
    for (int r = 0; r < world; ++r) TORCH_CHECK(pdata[r] && psig[r], "xgmi_ar: open() not called");
    int rc = lk_xgmi_gather(reinterpret_cast<bf16_t* const*>(pdata.data()), reinterpret_cast<unsigned* const*>(psig.data()),
                            rank, world, (int)root, in.data_ptr(), out.data_ptr(), nb, err, cur_stream());
    CHECK_RC(rc, "xgmi_gather");
  }
  int64_t max_bytes() const { return (int64_t)bytes; }
  int error() const {
    int h = 0;
    TORCH_CHECK(hipMemcpy(&h, err, sizeof(int), hipMemcpyDeviceToHost) == hipSuccess, "xgmi_ar: read error word");
    return h;
  }
};

}  // namespace

// build provenance: "LKSTAMP:<hash of sources + flags>", generated by csrc/build.py at link time
extern "C" const char lk_source_stamp[];

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("window_mark", [](int64_t id) { CHECK_RC(lk_window_mark((int)id, cur_stream()), "window_mark"); });
  m.def("debug_invalid_launch", []() { CHECK_RC(lk_debug_invalid_launch(cur_stream()), "debug_invalid_launch"); });
  // a HIP stream restricted to the CUs of a bit mask (32 CUs per word): two kernels that
  // would each fill the chip (a mixed step's flash prefill and paged decode) run side by side
  // on disjoint CU sets.  Returned as an integer handle for torch.cuda.ExternalStream; the
  // stream lives for the process.
  m.def("cu_mask_stream", [](std::vector<int64_t> words) {
    std::vector<uint32_t> w(words.size());
    for (size_t i = 0; i < words.size(); ++i) w[i] = (uint32_t)(words[i] & 0xffffffffLL);
    hipStream_t st = nullptr;
    TORCH_CHECK(hipExtStreamCreateWithCUMask(&st, (uint32_t)w.size(), w.data()) == hipSuccess,
                "hipExtStreamCreateWithCUMask failed");
    return (int64_t)reinterpret_cast<uintptr_t>(st);
  });
  m.def("stream_cu_mask", [](int64_t handle, int64_t nwords) {
    std::vector<uint32_t> w((size_t)nwords, 0u);
    TORCH_CHECK(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>((uintptr_t)handle), (uint32_t)nwords, w.data()) ==
                    hipSuccess, "hipExtStreamGetCUMask failed");
    return std::vector<int64_t>(w.begin(), w.end());
  });
  m.def("source_stamp", [] { return std::string(lk_source_stamp + 8); });
  py::class_<XgmiAr>(m, "XgmiAr")
      .def(py::init<int, int, int64_t>(), py::arg("rank"), py::arg("world"), py::arg("bytes"))
      .def("handles", &XgmiAr::handles)
      .def("open", &XgmiAr::open)
      .def("all_reduce", &XgmiAr::all_reduce)
      .def("all_reduce_rmsnorm", &XgmiAr::all_reduce_rmsnorm)
      .def("all_reduce2", &XgmiAr::all_reduce2, "", py::arg("x"), py::arg("out"), py::arg("residual") = py::none(),
           py::arg("w") = py::none(), py::arg("eps") = 1e-5)
      .def("gather", &XgmiAr::gather, "", py::arg("in"), py::arg("out"), py::arg("root") = -1)
      .def("max_bytes", &XgmiAr::max_bytes)
      .def("error", &XgmiAr::error)
      .def_readonly("bytes", &XgmiAr::bytes);
  m.doc() = "gfx950 (MI355X) HIP kernel library";
  m.def("rmsnorm", &rmsnorm, "", py::arg("x"), py::arg("w"), py::arg("eps"), py::arg("residual") = py::none(), py::arg("out") = py::none());
  m.def("layernorm", &layernorm, "", py::arg("x"), py::arg("w"), py::arg("b"), py::arg("eps"), py::arg("residual") = py::none(), py::arg("write_residual") = false);
  m.def("embed_layernorm", &embed_layernorm);
  m.def("skinny_linear", &skinny_linear, "", py::arg("x"), py::arg("w"), py::arg("swiglu") = false,
        py::arg("splits") = 0, py::arg("out") = py::none());
  m.def("skinny_splits", &skinny_splits);
  m.def("ws_linear", &ws_linear, "", py::arg("x"), py::arg("w"), py::arg("swiglu") = false, py::arg("bn") = 0,
        py::arg("splits") = 0, py::arg("out") = py::none());
  m.def("ws_plan", &ws_plan);
  m.def("gemm", &gemm, "", py::arg("x"), py::arg("w"), py::arg("bias") = py::none(), py::arg("epi") = 0,
        py::arg("bn") = 256, py::arg("out") = py::none(), py::arg("variant") = 1,
        py::arg("splits") = 1);
  m.def("gemm_fused", &gemm_fused, "", py::arg("x"), py::arg("w"), py::arg("epi"), py::arg("bn"), py::arg("out") = py::none(),
        py::arg("variant") = 2, py::arg("splits") = 1, py::arg("ss_in") = py::none(), py::arg("eps") = 1e-5,
        py::arg("resid") = py::none(), py::arg("ss_out") = py::none(), py::arg("positions") = py::none(),
        py::arg("cos_sin") = py::none(), py::arg("slots") = py::none(), py::arg("k_cache") = py::none(),
        py::arg("v_cache") = py::none(), py::arg("hq") = 0, py::arg("hkv") = 0, py::arg("hd") = 0);
  m.def("embed_rows", &embed_rows, "", py::arg("table"), py::arg("ids"), py::arg("lo") = 0, py::arg("n_local") = -1);
  m.def("embed_errors", []() { return (int64_t)lk_embed_errors(); },
        "token ids outside the (whole) embedding table seen since the last call (resets)");
  m.def("scatter_ids", &scatter_ids);
  m.def("gather_rows", &gather_rows);
  m.def("argmax_key", &argmax_key, "", py::arg("logits"), py::arg("vocab_lo") = 0);
  m.def("keys_to_ids", &keys_to_ids);
  m.def("gemm_streamk", &gemm_streamk,
        "stream-K policy of the prefill GEMM (mode 0 off / 1 on / -1 keep); returns the waits that gave up since the last call",
        py::arg("mode") = -1);
  m.def("gemm_supported", &gemm_supported, "", py::arg("M"), py::arg("N"), py::arg("K"), py::arg("epi"), py::arg("bn"),
        py::arg("splits") = 1, py::arg("variant") = -1);
  m.def("silu_mul", &silu_mul, "", py::arg("x"), py::arg("out") = py::none());
  m.def("activation_", &activation_);
  m.def("rope_kv_", &rope_kv_);
  m.def("ws_set_rot", [](int64_t r) { lk_wsgemm_set_rot((int)r); });
  m.def("ws_linear_rmsnorm", &ws_linear_rmsnorm, "", py::arg("x"), py::arg("w"), py::arg("residual"),
        py::arg("norm_w"), py::arg("eps"), py::arg("bn") = 0, py::arg("splits") = 0, py::arg("tickets") = py::none());
  m.def("ws_linear_rope_kv", &ws_linear_rope_kv, "", py::arg("x"), py::arg("w"), py::arg("positions"),
        py::arg("cos_sin"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"), py::arg("k_cache"), py::arg("v_cache"),
        py::arg("slots"), py::arg("neox") = true, py::arg("write_k_inplace") = false, py::arg("bn") = 0,
        py::arg("splits") = 0, py::arg("tickets") = py::none());
  m.def("kv_write", &kv_write);
  m.def("decode_splits", &decode_splits);
  m.def("decode_split_size", &decode_split_size);
  m.def("paged_decode", &paged_decode, "", py::arg("q"), py::arg("k_cache"), py::arg("v_cache"), py::arg("block_tables"), py::arg("ctx_lens"), py::arg("max_splits"), py::arg("split"), py::arg("scale"), py::arg("part_o") = py::none(), py::arg("part_ml") = py::none(), py::arg("out") = py::none(), py::arg("k_start") = py::none(), py::arg("pp_o") = py::none(), py::arg("pp_ml") = py::none(), py::arg("tickets") = py::none(), py::arg("reduce") = true);
  m.def("prefill_rows_per_tile", &prefill_rows_per_tile);
  m.def("ws_pro", &ws_pro, "", py::arg("x"), py::arg("w"), py::arg("swiglu"), py::arg("bn"), py::arg("splits"),
        py::arg("kind"), py::arg("reduce") = false, py::arg("pp") = py::none(), py::arg("res_in") = py::none(),
        py::arg("res_out") = py::none(), py::arg("gamma") = py::none(), py::arg("eps") = 0.0,
        py::arg("po") = py::none(), py::arg("pml") = py::none(), py::arg("ctx") = py::none(), py::arg("split") = 0,
        py::arg("max_splits") = 0, py::arg("Hq") = 0);
  m.def("splitk_rope_kv", &splitk_rope_kv);
  m.def("splitk_rmsnorm", &splitk_rmsnorm);
  m.def("gemv_decode", &gemv_decode, "", py::arg("mode"), py::arg("x"), py::arg("w"), py::arg("gamma") = py::none(),
        py::arg("eps") = 1e-5, py::arg("res") = py::none(), py::arg("positions") = py::none(),
        py::arg("cos_sin") = py::none(), py::arg("Hq") = 0, py::arg("Hkv") = 0, py::arg("D") = 0,
        py::arg("k_cache") = py::none(), py::arg("v_cache") = py::none(), py::arg("slots") = py::none(),
        py::arg("neox") = true, py::arg("po") = py::none(), py::arg("pml") = py::none(), py::arg("ctx") = py::none(),
        py::arg("max_splits") = 0, py::arg("split") = 0);
  m.def("gemv_supported", [](int64_t M, int64_t N, int64_t K, int64_t mode) {
    return lk_gemv_supported((int)M, (int)N, (int)K, (int)mode) != 0;
  });
  m.def("gemv_set_wgs", [](int64_t n) { lk_gemv_set_wgs((int)n); });
  m.def("gemv_set_ksplit", [](bool on) { lk_gemv_set_ksplit(on ? 1 : 0); });
  // read rows [r0, r1) of a contiguous 2-D tensor through the Infinity Cache (lk_l3_prefetch)
  m.def("l3_prefetch", [](const at::Tensor& t, int64_t r0, int64_t r1, int64_t wgs, at::Tensor& sink) {
    CHECK_CUDA(t); CHECK_CONTIG(t); CHECK_CUDA(sink);
    TORCH_CHECK(sink.scalar_type() == at::kInt && sink.numel() >= 1, "sink: int32 [>= 1]");
    TORCH_CHECK(t.dim() == 2 && 0 <= r0 && r0 <= r1 && r1 <= t.size(0), "rows out of range");
    const long row = t.size(1) * t.element_size();
    const char* base = reinterpret_cast<const char*>(t.data_ptr()) + r0 * row;
    CHECK_RC(lk_l3_prefetch(base, (r1 - r0) * row, (int)wgs, reinterpret_cast<unsigned*>(sink.data_ptr<int>()),
                            cur_stream()), "l3_prefetch");
  });
  m.def("ws_set_variant", [](int64_t M, int64_t N, int64_t K, bool swiglu, int64_t v) {
    CHECK_RC(lk_wsgemm_set_variant((int)M, (int)N, (int)K, swiglu ? 1 : 0, (int)v), "ws_set_variant");
  }, "weight-streaming GEMM kernel for this (M bucket, N, K, swiglu): 0 ring, 1 loader waves, -1 default",
        py::arg("M"), py::arg("N"), py::arg("K"), py::arg("swiglu"), py::arg("variant"));
  m.def("flash_prefill", &flash_prefill, "", py::arg("q"), py::arg("k"), py::arg("v"), py::arg("block_tables"), py::arg("cu_q"), py::arg("ctx_lens"), py::arg("tile_seq"), py::arg("tile_q0"), py::arg("Hq"), py::arg("Hkv"), py::arg("D"), py::arg("scale"), py::arg("causal"), py::arg("out") = py::none(), py::arg("part_o") = py::none(), py::arg("part_ml") = py::none(), py::arg("q_past") = py::none());
  m.def("knn_topk", &knn_topk, "", py::arg("corpus"), py::arg("cnorm"), py::arg("queries"), py::arg("qnorm"),
        py::arg("K"), py::arg("force_fused") = false);
  m.def("knn_merge", &knn_merge);
  m.def("pool_normalize", &pool_normalize, "", py::arg("hidden"), py::arg("cu"), py::arg("mode"), py::arg("normalize"),
        py::arg("out") = py::none());
  m.def("row_norms", &row_norms);
  m.def("select_allowed", &select_allowed, "", py::arg("logits"), py::arg("plan"), py::arg("temps") = py::none(),
        py::arg("seed") = 0, py::arg("step") = 0);
  m.def("select_tokens", &select_tokens, "", py::arg("logits"), py::arg("temps") = py::none(), py::arg("seed") = 0, py::arg("step") = 0, py::arg("out") = py::none());
  m.def("repeat_penalty_", &repeat_penalty_);
  m.def("sample", &sample, "", py::arg("logits"), py::arg("prm"), py::arg("hist"), py::arg("hist_len"),
        py::arg("seed") = 0, py::arg("out") = py::none());
}
