"""Plain-PyTorch fp32 reference implementations of every HIP kernel.

They define the numerics the kernels are tested against (tests compare the HIP op
with these on the same inputs) and they are the compute path for CPU runs (the
"Minimal_RAG on CPU" configuration).  Layouts match the kernels exactly:

* paged KV cache: ``[num_blocks, Hkv, block_size, D]``; ``slot = block * BS + off``
* packed QKV rows: ``[T, (Hq + 2*Hkv) * D]``
* cos/sin table: ``[max_pos, D]`` f32 = ``[cos(D/2) | sin(D/2)]``
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rmsnorm(x, w, eps, residual=None):
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
        residual.copy_(s)
        x = s
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return ((xf * inv).to(x.dtype).float() * w.float()).to(x.dtype)


def layernorm(x, w, b, eps, residual=None, write_residual=False):
    if residual is not None:
        s = (x.float() + residual.float()).to(x.dtype)
        if write_residual:
            residual.copy_(s)
        x = s
    y = F.layer_norm(x.float(), (x.shape[-1],), w.float(), None if b is None else b.float(), eps)
    return y.to(x.dtype)


def embed_layernorm(ids, pos_ids, type_ids, tok, pos, typ, w, b, eps):
    e = tok[ids.long()].float()
    if pos is not None:
        e = e + pos[pos_ids.long()].float()
    if typ is not None:
        tid = type_ids.long() if type_ids is not None else torch.zeros_like(ids, dtype=torch.long)
        e = e + typ[tid].float()
    return F.layer_norm(e, (e.shape[-1],), w.float(), b.float(), eps).to(tok.dtype)


def silu_mul(x):
    i = x.shape[-1] // 2
    g, u = x[..., :i], x[..., i:]
    return (F.silu(g.float()).to(x.dtype).float() * u.float()).to(x.dtype)


def activation_(x, bias=None, kind=0):
    v = x.float()
    if bias is not None:
        v = (v + bias.float()).to(x.dtype).float()
    if kind == 0:
        v = F.gelu(v)
    elif kind == 1:
        v = F.gelu(v, approximate="tanh")
    else:
        v = F.relu(v)
    x.copy_(v.to(x.dtype))
    return x


def rope_cos_sin(max_pos, D, theta=10000.0, scaling=None, device=None):
    """[max_pos, D] f32 table = [cos | sin] over D/2 frequencies (neox convention).

    ``scaling``: dict for Llama-3.1 ``rope_type == "llama3"`` (factor, low_freq_factor,
    high_freq_factor, original_max_position_embeddings).
    """
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lf, hf = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        low_wl, high_wl = old / lf, old / hf
        wl = 2 * math.pi / inv
        smooth = (old / wl - lf) / (hf - lf)
        scaled = torch.where(wl > low_wl, inv / factor, inv)
        mid = (1 - smooth) * inv / factor + smooth * inv
        is_mid = (wl <= low_wl) & (wl >= high_wl)
        inv = torch.where(is_mid, mid, scaled)
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return torch.cat([f.cos(), f.sin()], dim=-1).float().to(device)


def _rotate(x, cs, neox):
    # x [T, H, D] f32; cs [T, D]
    D = x.shape[-1]
    c, s = cs[:, None, : D // 2], cs[:, None, D // 2:]
    if neox:
        x1, x2 = x[..., : D // 2], x[..., D // 2:]
        return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)
    x1, x2 = x[..., 0::2], x[..., 1::2]
    y = torch.empty_like(x)
    y[..., 0::2] = x1 * c - x2 * s
    y[..., 1::2] = x2 * c + x1 * s
    return y


def rope_kv_(qkv, positions, cos_sin, Hq, Hkv, D, k_cache=None, v_cache=None, slots=None,
             neox=True, write_k_inplace=False):
    T = qkv.shape[0]
    cs = cos_sin[positions.long()]
    q = qkv[:, : Hq * D].reshape(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(T, Hkv, D)
    qr = _rotate(q.float(), cs, neox).to(qkv.dtype)
    kr = _rotate(k.float(), cs, neox).to(qkv.dtype)
    qkv[:, : Hq * D] = qr.reshape(T, Hq * D)
    if write_k_inplace:
        qkv[:, Hq * D:(Hq + Hkv) * D] = kr.reshape(T, Hkv * D)
    if k_cache is not None:
        kv_write(kr, v, k_cache, v_cache, slots)
    return qkv


def kv_write(k, v, k_cache, v_cache, slots):
    BS = k_cache.shape[2]
    sl = slots.long()
    keep = sl >= 0
    sl = sl[keep]
    blk, off = sl // BS, sl % BS
    k_cache[blk, :, off] = k[keep].to(k_cache.dtype)
    v_cache[blk, :, off] = v[keep].to(v_cache.dtype)


def gather_paged(cache, block_table, n):
    """Rows 0..n-1 of one sequence from a paged cache -> [n, Hkv, D]."""
    BS = cache.shape[2]
    idx = torch.arange(n, device=cache.device)
    blk = block_table.long()[idx // BS]
    return cache[blk, :, idx % BS]


def attention_ref(q, k, v, causal, past=0, scale=None):
    """q [Sq, Hq, D], k/v [Sk, Hkv, D] -> [Sq, Hq, D] (GQA by head repetition)."""
    Sq, Hq, D = q.shape
    Sk, Hkv, _ = k.shape
    g = Hq // Hkv
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    kf = k.float().repeat_interleave(g, dim=1)
    vf = v.float().repeat_interleave(g, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal:
        qpos = past + torch.arange(Sq, device=q.device)[:, None]
        kpos = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill((kpos > qpos)[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, vf)


def paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale):
    B, Hq, D = q.shape
    out = torch.empty_like(q)
    for b in range(B):
        n = int(ctx_lens[b])
        k = gather_paged(k_cache, block_tables[b], n)
        v = gather_paged(v_cache, block_tables[b], n)
        out[b] = attention_ref(q[b:b + 1], k, v, False, scale=scale)[0].to(q.dtype)
    return out


def flash_prefill(q, k, v, block_tables, cu_q, ctx_lens, Hq, Hkv, D, scale, causal):
    """q [T, >=Hq*D]; paged (block_tables given) or dense k/v [T, >=Hkv*D]."""
    T = q.shape[0]
    out = torch.empty(T, Hq * D, dtype=q.dtype, device=q.device)
    cu = [int(x) for x in cu_q]
    for b in range(len(cu) - 1):
        s, e = cu[b], cu[b + 1]
        if e == s:
            continue
        qb = q[s:e, : Hq * D].reshape(e - s, Hq, D)
        if block_tables is not None:
            n = int(ctx_lens[b])
            kb = gather_paged(k, block_tables[b], n)
            vb = gather_paged(v, block_tables[b], n)
        else:
            n = e - s
            kb = k[s:e, : Hkv * D].reshape(n, Hkv, D)
            vb = v[s:e, : Hkv * D].reshape(n, Hkv, D)
        o = attention_ref(qb, kb, vb, causal, past=n - (e - s), scale=scale)
        out[s:e] = o.reshape(e - s, Hq * D).to(q.dtype)
    return out


def cosine_scores(corpus, cnorm, queries, qnorm, eps=1e-9):
    dot = queries.double() @ corpus.double().T
    return dot / (qnorm.double()[:, None] * cnorm.double()[None, :] + eps)


def stable_topk(scores, K):
    """Descending scores, ties by ascending index (C# OrderByDescending is stable)."""
    nq, N = scores.shape
    K_eff = min(K, N)
    out_s = torch.full((nq, K), float("-inf"), dtype=torch.float32)
    out_i = torch.full((nq, K), -1, dtype=torch.int32)
    for i in range(nq):
        order = sorted(range(N), key=lambda j: (-float(scores[i, j]), j))[:K_eff]
        out_i[i, :K_eff] = torch.tensor(order, dtype=torch.int32)
        out_s[i, :K_eff] = scores[i, order].float()
    return out_s, out_i


def knn_topk(corpus, cnorm, queries, qnorm, K):
    sc = cosine_scores(corpus.float().cpu(), cnorm.cpu(), queries.float().cpu(), qnorm.cpu())
    return stable_topk(sc, K)


def pool_normalize(hidden, cu, mode, normalize):
    cu = [int(x) for x in cu]
    outs = []
    for b in range(len(cu) - 1):
        h = hidden[cu[b]:cu[b + 1]].float()
        v = h[0] if mode == 1 else h.mean(0)
        if normalize:
            v = v / v.norm().clamp_min(1e-12)
        outs.append(v)
    return torch.stack(outs) if outs else hidden.new_zeros((0, hidden.shape[1]), dtype=torch.float32)


def row_norms(x):
    return x.float().norm(dim=-1)


def select_tokens(logits, temps=None, seed=0, step=0):
    if temps is None:
        return logits.float().argmax(-1).int()
    out = []
    g = torch.Generator(device="cpu").manual_seed(int(seed) * 1000003 + int(step))
    for i in range(logits.shape[0]):
        t = float(temps[i])
        row = logits[i].float().cpu()
        if t <= 0:
            out.append(int(row.argmax()))
        else:
            u = torch.rand(row.shape, generator=g).clamp(1e-12, 1 - 1e-7)
            out.append(int((row / t - torch.log(-torch.log(u))).argmax()))
    return torch.tensor(out, dtype=torch.int32, device=logits.device)


def argmax_key(logits, vocab_lo: int = 0):
    """Order-preserving int64 (max value, ~(vocab_lo + first argmax)) key per row (the HIP
    kernel's encoding: csrc/sampling.hip select_kernel<..., KEY>)."""
    x = logits.float()
    idx = x.argmax(-1)
    best = x.gather(1, idx[:, None]).squeeze(1)
    best = torch.where(torch.isnan(best), torch.full_like(best, float("-inf")), best)
    fb = best.view(torch.int32).long() & 0xFFFFFFFF
    u = torch.where(fb >= 0x80000000, (~fb) & 0xFFFFFFFF, fb | 0x80000000)
    hi = (u ^ 0x80000000) - ((u ^ 0x80000000) >= 0x80000000).long() * (1 << 32)  # signed 32-bit
    lo = (~(idx + vocab_lo)) & 0xFFFFFFFF
    return hi * (1 << 32) + lo


def keys_to_ids(keys):
    k = keys.max(dim=0).values
    return ((~(k & 0xFFFFFFFF)) & 0xFFFFFFFF).int()


def repeat_penalty_(logits, window, penalty):
    for b in range(logits.shape[0]):
        p = float(penalty[b])
        toks = sorted({int(t) for t in window[b].tolist() if int(t) >= 0})
        if not toks:
            continue
        idx = torch.tensor(toks, device=logits.device)
        l = logits[b, idx].float()
        logits[b, idx] = torch.where(l > 0, l / p, l * p).to(logits.dtype)
    return logits


SAMPLE_KMAX = 1024  # csrc/sampling.hip kSampKMax


def sample(logits, prm, hist, hist_len, seed=0):
    """fp32 reference of lk_sample (csrc/sampling.hip): per row the repeat penalty over the
    unique tokens of the last min(len, last_n) ring entries, top-k by (value desc, index asc),
    softmax at the row's temperature, the top-p prefix (a token is kept while the mass before
    it is <= top_p), one draw; the token is appended to the ring.  Same distribution as the
    kernel (the random stream differs: torch's generator seeded per (seed, request seed,
    position))."""
    B, V = logits.shape
    W = hist.shape[1]
    out = torch.empty(B, dtype=torch.int32)
    P = prm.cpu()
    for r in range(B):
        row = P[r]
        temp = float(row[0:1].view(torch.float32)[0])
        top_p = float(row[1:2].view(torch.float32)[0])
        pen = float(row[2:3].view(torch.float32)[0])
        top_k, last_n, slot, reset, rseed = (int(x) for x in row[3:8])
        hl = 0 if reset else int(hist_len[slot])
        l = logits[r].float().clone()
        if pen != 1.0 and last_n != 0:
            n = min(hl, last_n if last_n > 0 else W, W)
            toks = {int(hist[slot, (hl - 1 - j) % W]) for j in range(n)}
            for t in toks:
                if t >= 0:
                    l[t] = l[t] / pen if l[t] > 0 else l[t] * pen
            logits[r] = l.to(logits.dtype)
        greedy = temp <= 0.0
        K = 1 if greedy else min(top_k if top_k > 0 else SAMPLE_KMAX, V, SAMPLE_KMAX)
        order = _topk_stable(l, K)
        if greedy or K == 1:
            tok = order[0]
        else:
            v = l[torch.tensor(order)].double()
            e = torch.exp((v - v[0]) / temp)
            incl = torch.cumsum(e, 0)
            keep = (incl - e) <= top_p * incl[-1]
            nkeep = int(keep.sum())
            g = torch.Generator().manual_seed((int(seed) * 1000003 + rseed * 7919 + hl) & ((1 << 62) - 1))
            u = float(torch.rand((), generator=g, dtype=torch.float64)) * float(incl[nkeep - 1])
            pick = int((incl[:nkeep] > u).nonzero()[0]) if bool((incl[:nkeep] > u).any()) else nkeep - 1
            tok = order[pick]
        out[r] = tok
        hist[slot, hl % W] = tok
        hist_len[slot] = hl + 1
    return out.to(logits.device)


def _topk_stable(l, K):
    """indices of the K largest (value desc, index asc)."""
    vals, idx = torch.sort(l, descending=True, stable=True)
    return idx[:K].tolist()


# ---------------------------------------------------------------- fused prefill chain
# (csrc/gemm.hip LkEpi: the decoder block's RMSNorm folded into its neighbouring GEMMs)
def ss_partials(r: torch.Tensor, cols: int = 256) -> torch.Tensor:
    """Per-``cols``-column partial sums of squares of r [M, N]: [N / cols, M] f32."""
    M, N = r.shape
    return r.float().pow(2).reshape(M, N // cols, cols).sum(-1).t().contiguous()


def row_scale(ss: torch.Tensor, H: int, eps: float) -> torch.Tensor:
    """[M] f32 rsqrt(mean of squares + eps) from the partials [nt, >= M]."""
    return torch.rsqrt(ss.float().sum(0) / H + eps)


def linear_resid(x, w, residual, ss_out):
    """residual = bf16(residual + bf16(x w^T)) in place; ss_out [N/256, >= M] = its partials."""
    y = (x.float() @ w.float().t()).to(x.dtype)
    residual.copy_((residual.float() + y.float()).to(residual.dtype))
    M = residual.shape[0]
    ss_out[:, :M] = ss_partials(residual)
    return residual


def gemm_scaled(x, w, ss, H, eps, swiglu=False):
    """x w^T with each row scaled by the folded norm's rsqrt (ss None: unscaled); SwiGLU:
    silu(g) * u on the scaled, bf16-rounded halves."""
    acc = x.float() @ w.float().t()
    if ss is not None:
        acc = acc * row_scale(ss, H, eps)[: x.shape[0], None]
    if not swiglu:
        return acc.to(x.dtype)
    I = w.shape[0] // 2
    g, u = acc[:, :I].to(x.dtype).float(), acc[:, I:].to(x.dtype).float()
    return ((g * torch.sigmoid(g)).to(x.dtype).float() * u).to(x.dtype)


def qkv_fused(x, w, ss, H, eps, positions, cos_sin, Hq, Hkv, D, k_cache=None, v_cache=None, slots=None):
    """The QKV GEMM's fused epilogue: scaled, bf16-rounded projection, interleaved-pair RoPE on
    q and k (written back into the row), K / V into the paged cache."""
    qkv = gemm_scaled(x, w, ss, H, eps)
    return rope_kv_(qkv, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox=False, write_k_inplace=True)
