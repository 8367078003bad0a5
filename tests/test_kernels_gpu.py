"""Numerics of every HIP kernel vs the plain-PyTorch fp32 reference (ops.reference)."""
import math

import numpy as np
import pytest
import torch

from llm_kubernetes_minikube_sharp4dev_amd import ops
from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item() if a.numel() else 0.0
    tol = atol + rtol * b.abs().max().item() if b.numel() else atol
    assert err <= tol, f"{msg} max abs err {err:.4g} > {tol:.4g}"


@pytest.mark.parametrize("H", [384, 768, 4096, 8192])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm(hip, H, with_res):
    torch.manual_seed(0)
    x = torch.randn(37, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    res = torch.randn(37, H, device=DEV, dtype=torch.bfloat16) if with_res else None
    res2 = res.clone() if with_res else None
    y = hip.rmsnorm(x, w, 1e-5, res, None)
    y_ref = ref.rmsnorm(x, w, 1e-5, res2)
    _close(y, y_ref, 0.05, 0.01, "rmsnorm")
    if with_res:
        _close(res, res2, 1e-2, 0, "residual")


@pytest.mark.parametrize("H", [384, 768, 1024])
def test_layernorm(hip, H):
    torch.manual_seed(1)
    x = torch.randn(29, H, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(29, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    r2 = r.clone()
    y = hip.layernorm(x, w, b, 1e-12, r, True)
    y_ref = ref.layernorm(x, w, b, 1e-12, r2, True)
    _close(y, y_ref, 0.05, 0.01, "layernorm")
    _close(r, r2, 1e-2, 0, "residual")


def test_embed_layernorm(hip):
    torch.manual_seed(2)
    V, P, H, T = 1000, 512, 768, 50
    tok = torch.randn(V, H, device=DEV, dtype=torch.bfloat16)
    pos = torch.randn(P, H, device=DEV, dtype=torch.bfloat16)
    typ = torch.randn(2, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, V, (T,), device=DEV, dtype=torch.int32)
    pids = torch.randint(0, P, (T,), device=DEV, dtype=torch.int32)
    tids = torch.randint(0, 2, (T,), device=DEV, dtype=torch.int32)
    y = hip.embed_layernorm(ids, pids, tids, tok, pos, typ, w, b, 1e-12)
    _close(y, ref.embed_layernorm(ids, pids, tids, tok, pos, typ, w, b, 1e-12), 0.05, 0.01)


def test_activations(hip):
    torch.manual_seed(3)
    x = torch.randn(33, 2 * 1536, device=DEV, dtype=torch.bfloat16)
    _close(hip.silu_mul(x, None), ref.silu_mul(x), 0.02, 0.01, "silu_mul")
    # 2-vector-per-thread path (I >= 4096), partial last segment, strided rows in and out
    for rows, I in ((130, 14336), (7, 4104), (3, 1792)):
        xw = torch.randn(rows, 2 * I + 64, device=DEV, dtype=torch.bfloat16)
        xv = xw[:, : 2 * I]
        ow = torch.full((rows, I + 32), 7.0, device=DEV, dtype=torch.bfloat16)
        hip.silu_mul(xv, ow[:, :I])
        _close(ow[:, :I], ref.silu_mul(xv), 0.02, 0.01, f"silu_mul rows{rows} I{I}")
        assert (ow[:, I:] == 7.0).all(), "silu_mul wrote past the row"
    for kind in (0, 1, 2):
        y = torch.randn(17, 3072, device=DEV, dtype=torch.bfloat16)
        bias = torch.randn(3072, device=DEV, dtype=torch.bfloat16)
        y2 = y.clone()
        hip.activation_(y, bias, kind)
        ref.activation_(y2, bias, kind)
        _close(y, y2, 0.02, 0.01, f"act{kind}")


@pytest.mark.parametrize("neox", [True, False])
def test_rope_kv(hip, neox):
    torch.manual_seed(4)
    T, Hq, Hkv, D, BS, NB = 45, 32, 8, 128, 16, 8
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(4096, D, 500000.0, device=DEV)
    kc = torch.zeros(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(NB * BS, device=DEV)[:T].int()
    slots[3] = -1
    qkv2, kc2, vc2 = qkv.clone(), kc.clone(), vc.clone()
    hip.rope_kv_(qkv, pos, cs, Hq, Hkv, D, kc, vc, slots, neox, True)
    ref.rope_kv_(qkv2, pos, cs, Hq, Hkv, D, kc2, vc2, slots, neox, True)
    _close(qkv, qkv2, 0.03, 0.0, "qkv")
    _close(kc, kc2, 0.03, 0.0, "k cache")
    _close(vc, vc2, 0.0, 0.0, "v cache")


def _paged_setup(B, ctx, Hkv, D, BS, seed=5):
    g = torch.Generator().manual_seed(seed)
    nblk = [(c + BS - 1) // BS for c in ctx]
    NB = sum(nblk) + 3
    kc = torch.randn(NB, Hkv, BS, D, generator=g).to(DEV, torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS, D, generator=g).to(DEV, torch.bfloat16)
    perm = torch.randperm(NB, generator=g).tolist()
    width = max(nblk)
    bt = torch.zeros(B, width, dtype=torch.int32)
    p = 0
    for b in range(B):
        for j in range(nblk[b]):
            bt[b, j] = perm[p]
            p += 1
    return kc, vc, bt.to(DEV)


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("D", [64, 128])
def test_paged_decode(hip, G, D):
    torch.manual_seed(6)
    Hkv, BS = 2, 16
    Hq = Hkv * G
    ctx = [1, 17, 511, 512, 513, 1500, 2100]
    B = len(ctx)
    kc, vc, bt = _paged_setup(B, ctx, Hkv, D, BS)
    q = torch.randn(B, Hq, D, device=DEV, dtype=torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    y_ref = ref.paged_decode(q, kc, vc, bt, cl, scale)
    tickets = torch.zeros(B * Hkv, dtype=torch.int32, device=DEV)
    for split in (128, 256, 2048):  # many partials / few partials / single pass
        max_splits = ops.decode_splits(bt.shape[1] * BS, split)
        y = hip.paged_decode(q, kc, vc, bt, cl, max_splits, split, scale, None, None, None)
        _close(y, y_ref, 0.02, 0.0, f"paged decode split={split}")
        # fused merge (the last split workgroup of each (seq, kv head) reduces): same output, and
        # every ticket back at 0 for the next launch
        for _ in range(2):
            yf = hip.paged_decode(q, kc, vc, bt, cl, max_splits, split, scale, None, None, None, None, None, None,
                                  tickets)
            _close(yf, y_ref, 0.02, 0.0, f"paged decode fused merge split={split}")
            assert int(tickets.abs().sum()) == 0


def test_paged_decode_fused_merge_empty_rows(hip):
    """Rows without keys (graph-bucket padding, ctx 0) get zeros from split 0 when no reduce
    kernel runs (the separate reduce kernel leaves such rows unwritten: nobody reads them); the
    rows with keys equal the reduce kernel's."""
    torch.manual_seed(16)
    Hkv, BS, G, D = 8, 16, 4, 128
    ctx = [0, 700, 0, 1, 3000]
    B = len(ctx)
    kc, vc, bt = _paged_setup(B, [max(c, 1) for c in ctx], Hkv, D, BS, seed=17)
    q = torch.randn(B, Hkv * G, D, device=DEV, dtype=torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    tickets = torch.zeros(B * Hkv, dtype=torch.int32, device=DEV)
    for split in (128, 512):
        ms = ops.decode_splits(bt.shape[1] * BS, split)
        want = hip.paged_decode(q, kc, vc, bt, cl, ms, split, 0.088, None, None, torch.full_like(q, 7.0))
        got = hip.paged_decode(q, kc, vc, bt, cl, ms, split, 0.088, None, None, torch.full_like(q, 7.0), None, None,
                               None, tickets)
        assert bool((got[0] == 0).all()) and bool((got[2] == 0).all())
        keep = [1, 3, 4]
        _close(got[keep], want[keep], 1e-3, 0.0, f"fused vs reduce kernel split={split}")
        assert int(tickets.abs().sum()) == 0


@pytest.mark.parametrize("G", [1, 4, 8])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("S", [0, 3, 18])
def test_cascade_decode(hip, G, D, S):
    """Cascade decode: the first S blocks are the same cache blocks in every row's table
    (a prefix-cached system prompt); the flash kernel attends them once for all rows into
    f32 partials, the split-K decode attends the rest and merges -- vs the fp32 reference
    over the whole context (S=0: empty prefix, merge of a no-key partial)."""
    torch.manual_seed(9)
    Hkv, BS = 2, 16
    Hq = Hkv * G
    ctx = [S * BS + e for e in (1, 17, 300, 16, 900, 1, 64, 2)]
    B = len(ctx)
    kc, vc, bt = _paged_setup(B, ctx, Hkv, D, BS, seed=10)
    if S:
        bt[:, :S] = bt[0, :S]  # shared prefix blocks
    q = torch.randn(B, Hq * D, device=DEV, dtype=torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    y_ref = ref.paged_decode(q.view(B, Hq, D), kc, vc, bt, cl, scale)
    k0 = torch.tensor([S * BS], dtype=torch.int32, device=DEV)
    rpt = ops.prefill_rows_per_tile(G, D)
    nt = (B + rpt - 1) // rpt
    tiles = (torch.zeros(nt, dtype=torch.int32, device=DEV),
             torch.arange(0, nt * rpt, rpt, dtype=torch.int32, device=DEV))
    pp_o = torch.empty(B, Hq, D, device=DEV)
    pp_ml = torch.empty(B, Hq, 2, device=DEV)
    cu = torch.tensor([0, B], dtype=torch.int32, device=DEV)
    for split in (128, 2048):
        ops.flash_prefill(q, kc, vc, cu, Hq, Hkv, D, scale, False, block_tables=bt[0:1], ctx_lens=k0,
                          tiles=tiles, part=(pp_o, pp_ml))
        max_splits = ops.decode_splits(bt.shape[1] * BS, split)
        y = ops.paged_decode(q.view(B, Hq, D), kc, vc, bt, cl, scale, max_splits, split=split, k_start=k0,
                             prefix=(pp_o, pp_ml))
        _close(y, y_ref, 0.02, 0.0, f"cascade decode S={S} split={split}")


@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("BS", [8, 16, 128])
def test_flash_prefill_paged(G, D, BS):
    """Paged K/V through the block table for cache blocks smaller than, equal to a wave's
    staged rows and larger than a key tile (BS 128: a scalar in-block offset on odd tiles)."""
    torch.manual_seed(7)
    Hkv = 2
    Hq = Hkv * G
    q_lens = [1, 33, 100, 257, 64]
    past = [0, 5, 0, 40, 700]
    ctx = [a + b for a, b in zip(q_lens, past)]
    B = len(q_lens)
    kc, vc, bt = _paged_setup(B, ctx, Hkv, D, BS, seed=8)
    T = sum(q_lens)
    q = torch.randn(T, Hq * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    y = ops.flash_prefill(q, kc, vc, cu, Hq, Hkv, D, scale, True, block_tables=bt, ctx_lens=cl,
                          q_lens_cpu=q_lens, ctx_lens_cpu=ctx)
    y_ref = ref.flash_prefill(q, kc, vc, bt, cu.cpu(), cl.cpu(), Hq, Hkv, D, scale, True)
    _close(y, y_ref, 0.02, 0.0, "flash prefill paged")


@pytest.mark.parametrize("D", [32, 64, 128])
def test_flash_encoder_dense(D):
    torch.manual_seed(9)
    H = 4
    q_lens = [7, 128, 300, 1]
    T = sum(q_lens)
    qkv = torch.randn(T, 3 * H * D, device=DEV, dtype=torch.bfloat16)
    q, k, v = qkv[:, : H * D], qkv[:, H * D: 2 * H * D], qkv[:, 2 * H * D:]
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    y = ops.flash_prefill(q, k, v, cu, H, H, D, scale, False, q_lens_cpu=q_lens)
    y_ref = ref.flash_prefill(q, k, v, None, cu.cpu(), None, H, H, D, scale, False)
    _close(y, y_ref, 0.02, 0.0, "encoder attention")


def test_flash_prefill_causal_dense_long():
    torch.manual_seed(10)
    Hq, Hkv, D = 8, 2, 128
    q_lens = [1030]
    T = sum(q_lens)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    q = qkv[:, : Hq * D]
    k = qkv[:, Hq * D:(Hq + Hkv) * D]
    v = qkv[:, (Hq + Hkv) * D:]
    cu = torch.tensor([0, T], dtype=torch.int32, device=DEV)
    y = ops.flash_prefill(q, k, v, cu, Hq, Hkv, D, 1 / math.sqrt(D), True, q_lens_cpu=q_lens)
    y_ref = ref.flash_prefill(q, k, v, None, cu.cpu(), None, Hq, Hkv, D, 1 / math.sqrt(D), True)
    _close(y, y_ref, 0.02, 0.0, "causal dense")


def test_flash_softmax_spike():
    """Force a large running-max jump mid-sequence (online rescale path)."""
    Hq = Hkv = 1
    D = 128
    T = 200
    q = torch.full((T, D), 0.1, device=DEV, dtype=torch.bfloat16)
    k = torch.randn(T, D, device=DEV, dtype=torch.bfloat16) * 0.1
    k[150] = 4.0
    v = torch.randn(T, D, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0, T], dtype=torch.int32, device=DEV)
    y = ops.flash_prefill(q, k, v, cu, Hq, Hkv, D, 1.0, True, q_lens_cpu=[T])
    y_ref = ref.flash_prefill(q, k, v, None, cu.cpu(), None, Hq, Hkv, D, 1.0, True)
    _close(y, y_ref, 0.03, 0.0, "spike")


@pytest.mark.parametrize("N,D", [(1, 384), (1000, 768), (70000, 768), (5000, 1024), (3000, 128), (777, 256), (2000, 512)])
@pytest.mark.parametrize("fused", [False, True])
def test_knn_topk(hip, N, D, fused):
    """fused=False: the GEMM-scores path (weight-streaming kernel + chunked top-k);
    fused=True: the single-pass MFMA kernel with in-LDS top-k."""
    torch.manual_seed(11)
    corpus = torch.randn(N, D, device=DEV).to(torch.bfloat16)
    if N > 10:
        corpus[7] = corpus[3]  # exact duplicate -> tie must keep insertion order
    qs = torch.randn(5, D, device=DEV).to(torch.bfloat16)
    if N > 10:
        qs[0] = corpus[3]
    cn = hip.row_norms(corpus)
    qn = hip.row_norms(qs)
    _close(cn, corpus.float().norm(dim=-1), 1e-2, 1e-3, "row norms")
    K = 10
    s, i = hip.knn_topk(corpus, cn, qs, qn, K, fused)
    sc = ref.cosine_scores(corpus.float().cpu(), cn.cpu(), qs.float().cpu(), qn.cpu())
    rs, ri = ref.stable_topk(sc, K)
    kk = min(K, N)
    _close(s[:, :kk], rs[:, :kk], 2e-3, 0.0, "knn scores")
    # indices agree wherever scores are separated by more than the fp32 accumulation noise
    for q in range(5):
        for j in range(kk):
            if int(i[q, j]) != int(ri[q, j]):
                assert abs(float(sc[q, int(i[q, j])]) - float(rs[q, j])) < 2e-3
    if N > 10:
        assert int(i[0, 0]) == 3 and int(i[0, 1]) == 7


def test_pool_normalize(hip):
    torch.manual_seed(12)
    lens = [3, 1, 40]
    T, H = sum(lens), 768
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0, 3, 4, 44], dtype=torch.int32, device=DEV)
    for mode in (0, 1):
        want = ref.pool_normalize(x, cu.cpu(), mode, True)
        _close(hip.pool_normalize(x, cu, mode, True), want, 1e-3, 0.0)
        # destination rows: a strided slice of a bigger f32 / bf16 matrix, written in place and
        # nothing else touched (the embed engine's rows, the bf16 kNN query operand)
        for dt in (torch.float32, torch.bfloat16):
            big = torch.full((6, H + 64), 7.0, device=DEV, dtype=dt)
            dst = big[2:5, :H]
            got = hip.pool_normalize(x, cu, mode, True, dst)
            assert got.data_ptr() == dst.data_ptr()
            _close(dst.float(), want, 1e-3 if dt == torch.float32 else 8e-3, 0.0)
            assert bool((big[:2] == 7).all()) and bool((big[5:] == 7).all()) and bool((big[:, H:] == 7).all())


def test_select_tokens(hip):
    torch.manual_seed(13)
    for dt in (torch.bfloat16, torch.float32):
        lg = torch.randn(9, 128256, device=DEV).to(dt)
        lg[2, 77] = 100.0
        lg[2, 5] = 100.0  # tie -> lowest index
        t = hip.select_tokens(lg, None, 0, 0, None)
        assert torch.equal(t.cpu(), lg.float().argmax(-1).int().cpu())
        temps = torch.zeros(9, device=DEV)
        t2 = hip.select_tokens(lg, temps, 123, 4, None)
        assert torch.equal(t2.cpu(), t.cpu())
        temps.fill_(1.0)
        t3 = hip.select_tokens(lg, temps, 123, 4, None)
        assert int(t3[2]) in (5, 77)


def test_select_tokens_distribution(hip):
    """Gumbel-max sampling follows softmax(logits / T)."""
    lg = torch.tensor([[0.0, 1.0, 2.0, -1.0] + [-1e9] * 4], device=DEV).repeat(4000, 1)
    temps = torch.full((4000,), 1.0, device=DEV)
    t = hip.select_tokens(lg, temps, 7, 1, None).cpu()
    freq = torch.bincount(t.long(), minlength=8)[:4].float() / 4000
    p = torch.softmax(torch.tensor([0.0, 1.0, 2.0, -1.0]), 0)
    assert (freq - p).abs().max() < 0.04


def test_repeat_penalty(hip):
    lg = torch.randn(3, 1000, device=DEV)
    win = torch.tensor([[1, 2, 2, -1], [5, 5, 5, 5], [-1, -1, -1, -1]], device=DEV, dtype=torch.int32)
    pen = torch.tensor([1.1, 2.0, 1.5], device=DEV)
    a, b = lg.clone(), lg.clone()
    hip.repeat_penalty_(a, win, pen)
    ref.repeat_penalty_(b, win.cpu(), pen.cpu())
    _close(a, b, 1e-6)


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 100, 128, 200, 256])
@pytest.mark.parametrize("NK", [(6144, 4096), (4096, 4096), (4096, 14336), (1280, 8192), (768, 768)])
def test_skinny_linear(hip, M, NK):
    """Decode-regime GEMM (split-K + reduce where chosen) vs an fp32 matmul."""
    N, K = NK
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    y = hip.skinny_linear(x, w)
    y_ref = x.float() @ w.float().t()
    _close(y, y_ref, 0.02, 0.01, f"skinny M{M} N{N} K{K}")
    for S in (1, 2):  # explicit split counts agree
        if K % (S * 256) == 0:
            _close(hip.skinny_linear(x, w, False, S), y_ref, 0.02, 0.01, f"skinny S{S}")


@pytest.mark.parametrize("M", [1, 5, 64, 128, 130])
@pytest.mark.parametrize("IK", [(14336, 4096), (3584, 8192), (1536, 512)])
def test_skinny_swiglu_matches_unfused(hip, M, IK):
    """GEMM with the fused SwiGLU epilogue == linear -> silu_mul, bit for bit modulo the
    GEMM accumulation order."""
    I, K = IK
    torch.manual_seed(1)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, K, device=DEV, dtype=torch.bfloat16) * 0.05
    a = hip.skinny_linear(x, w, True)
    gu = (x.float() @ w.float().t()).to(torch.bfloat16)
    a_ref = ref.silu_mul(gu)
    _close(a, a_ref, 0.03, 0.01, f"swiglu M{M} I{I}")
    if K % 512 == 0:
        _close(hip.skinny_linear(x, w, True, 2), a_ref, 0.03, 0.01, "swiglu split 2")


@pytest.fixture
def static_decode_routing():
    """The static decode rule, without measurements an engine in an earlier test recorded."""
    saved = dict(ops._DECODE_TABLE)
    ops._DECODE_TABLE.clear()
    yield
    ops._DECODE_TABLE.clear()
    ops._DECODE_TABLE.update(saved)


def test_linear_dispatch_decode_kernels(hip, static_decode_routing):
    """Decode-sized projections take the weight-streaming kernel (whose split-K reduce the
    consumer fuses) from M = 1; the LM head at M <= 16 the fragment-load kernel."""
    x = torch.randn(8, 4096, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(6144, 4096, device=DEV, dtype=torch.bfloat16) * 0.05
    assert ops._decode_gemm_kind(x, w, False) == "ws"
    _close(ops.linear(x, w), x.float() @ w.float().t(), 0.02, 0.01)
    head = torch.randn(128256, 4096, device=DEV, dtype=torch.bfloat16) * 0.05
    assert ops._decode_gemm_kind(x, head, False) == "skinny"
    _close(ops.linear(x, head), x.float() @ head.float().t(), 0.02, 0.01)
    assert ops._decode_gemm_kind(torch.randn(512, 4096, device=DEV, dtype=torch.bfloat16), w, False) is None
    x128 = torch.randn(128, 4096, device=DEV, dtype=torch.bfloat16)
    assert ops._decode_gemm_kind(x128, w, False) == "ws"
    _close(ops.linear(x128, w), x128.float() @ w.float().t(), 0.02, 0.01)


@pytest.mark.parametrize("M", [1, 2, 8, 16, 33, 64, 65, 100, 128, 129, 160, 192, 200, 256])
@pytest.mark.parametrize("NK", [(6144, 4096), (4096, 4096), (4096, 14336), (1280, 8192), (128256, 4096)])
def test_ws_linear(hip, M, NK):
    """LDS-DMA staged weight-streaming GEMM (every BN / split plan) vs an fp32 matmul."""
    N, K = NK
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    y_ref = x.float() @ w.float().t()
    _close(hip.ws_linear(x, w), y_ref, 0.02, 0.01, f"ws M{M} N{N} K{K}")
    if N <= 6144:
        for bn, S in ((64, 1), (128, 2), (64, 4), (96, 4)):
            if N % bn == 0 and K % (S * 64) == 0:
                _close(hip.ws_linear(x, w, False, bn, S), y_ref, 0.02, 0.01, f"ws bn{bn} S{S}")


@pytest.mark.parametrize("M", [1, 16, 64, 100, 129, 192, 256])
def test_ws_bn96_plan_and_variants(hip, M):
    """96-column weight-streaming tiles (the Llama-3-8B QKV projection: 64 tiles x 4 K-splits = 256
    blocks instead of 192 at 128 columns), ring and loader-wave kernels, plain and with the split-K
    partials reduced by the RoPE / KV consumer, vs an fp32 matmul."""
    N, K = 6144, 4096
    assert tuple(hip.ws_plan(M, N, K, False)) == (96, 4)
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    y_ref = x.float() @ w.float().t()
    try:
        for v in (0, 1):
            hip.ws_set_variant(M, N, K, False, v)
            _close(hip.ws_linear(x, w), y_ref, 0.02, 0.01, f"ws bn96 M{M} variant {v}")
            _close(hip.ws_linear(x, w, False, 96, 2), y_ref, 0.02, 0.01, f"ws bn96 S2 M{M} variant {v}")
    finally:
        hip.ws_set_variant(M, N, K, False, -1)


@pytest.mark.parametrize("M", [1, 8, 64, 128, 150, 192, 256])
@pytest.mark.parametrize("IK", [(14336, 4096), (3584, 8192)])
def test_ws_swiglu(hip, M, IK):
    I, K = IK
    torch.manual_seed(2)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, K, device=DEV, dtype=torch.bfloat16) * 0.05
    a_ref = ref.silu_mul((x.float() @ w.float().t()).to(torch.bfloat16))
    _close(hip.ws_linear(x, w, True), a_ref, 0.03, 0.01, f"ws swiglu M{M} I{I}")
    _close(hip.ws_linear(x, w, True, 64, 2), a_ref, 0.03, 0.01, "ws swiglu bn64 S2")


# (schedule, column tile): gemm.hip schedules 0-2, and variants 3 / 4 / 5 = csrc/gemm1w.hip (256-wide
# column tiles, 256 / 192 / 128-row tiles)
GEMM_CFGS = [(0, 256), (1, 256), (2, 256), (0, 192), (1, 192), (2, 192), (3, 256), (4, 256), (5, 256)]


@pytest.mark.parametrize("M", [1, 257, 1000, 3584])
@pytest.mark.parametrize("NK", [(6144, 4096), (4096, 14336), (768, 768), (1280, 8192), (1152, 384)])
def test_gemm(hip, M, NK):
    """Prefill-regime 256 x {256, 192} MFMA GEMM (csrc/gemm.hip), both K-loop schedules, vs an
    fp32 matmul, including M tails (rows past M read as zeros by the buffer descriptor)."""
    N, K = NK
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    y_ref = x.float() @ w.float().t()
    ran = 0
    for sched, bn in GEMM_CFGS:
        if hip.gemm_supported(M, N, K, 0, bn, 1, sched):
            _close(hip.gemm(x, w, None, 0, bn, None, sched), y_ref, 0.02, 0.01, f"gemm s{sched}/{bn} M{M} N{N} K{K}")
            ran += 1
    assert ran >= 2


@pytest.mark.parametrize("M,N,K", [(50001, 3072, 768), (40000, 2304, 768), (33000, 768, 1024)])
@pytest.mark.parametrize("epi", [0, 2, 3, 4])
def test_gemm1w_persistent_walk(hip, M, N, K, epi):
    """Short-K shapes with many tiles run gemm1w's persistent walk (one workgroup per CU, the next
    tile's first K-tiles DMA'd during the current tile's last two): every tile, M tails and the
    bias / GELU / ReLU epilogues vs fp32 (the encoder's K = 768 projections)."""
    torch.manual_seed(M + N + epi)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16) if epi else None
    y = x.float() @ w.float().t()
    if epi:
        y = (y + b.float()).to(torch.bfloat16).float()
    if epi == 3:
        y = torch.nn.functional.gelu(y)
    elif epi == 4:
        y = torch.relu(y)
    assert hip.gemm_supported(M, N, K, epi, 256, 1, 3)
    _close(hip.gemm(x, w, b, epi, 256, None, 3, 1), y, 0.03, 0.01, f"persistent epi{epi} M{M} N{N} K{K}")


@pytest.mark.parametrize("MNK", [(2048, 4096, 4096), (300, 1280, 8192), (1000, 768, 3072), (4096, 1280, 8192)])
@pytest.mark.parametrize("splits", [2, 3, 4])
@pytest.mark.parametrize("epi", [0, 2, 3, 4])
def test_gemm_splitk(hip, MNK, splits, epi):
    """Split-K (fp32 partials of `splits` K-ranges + a reduce kernel applying the epilogue) vs
    fp32 linear -> bf16 -> activation, with uneven K-ranges (K-tiles % splits != 0) and M tails."""
    M, N, K = MNK
    torch.manual_seed(M + N + splits + epi)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16) if epi else None
    y = x.float() @ w.float().t()
    if epi:
        y = (y + b.float()).to(torch.bfloat16).float()
    if epi == 3:
        y = torch.nn.functional.gelu(y)
    elif epi == 4:
        y = torch.relu(y)
    for sched in (0, 1, 3, 4, 5):
        for bn in (256, 192):
            if hip.gemm_supported(M, N, K, epi, bn, splits, sched):
                _close(hip.gemm(x, w, b, epi, bn, None, sched, splits), y, 0.03, 0.01,
                       f"gemm split{splits} epi{epi} s{sched}/{bn} M{M} N{N} K{K}")


@pytest.mark.parametrize("MNKE", [(4352, 4096, 4096, 0), (4300, 6144, 4096, 0), (4352, 28672, 4096, 1),
                                  (5000, 3072, 4096, 3), (4864, 4096, 14336, 0), (1536, 4096, 4096, 2),
                                  (5376, 4096, 14336, 2)])
def test_gemm_streamk(hip, MNKE):
    """Hybrid stream-K (persistent grid: whole waves of tiles data-parallel, a short last wave
    cut into K units over up to 4 workgroups per tile on the tile's XCD, fp32 partial tiles
    summed by the owner of each tile's first units) vs the plain tiling and the fp32
    reference, every epilogue and M tails; no wait ever gives up."""
    M, N, K, epi = MNKE
    torch.manual_seed(M + N + K + epi)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16) if epi >= 2 else None
    y = x.float() @ w.float().t()
    if epi == 1:
        y = ref.silu_mul(y.to(torch.bfloat16)).float()
    elif epi >= 2:
        y = (y + b.float()).to(torch.bfloat16).float()
        y = torch.nn.functional.gelu(y) if epi == 3 else y
    hip.gemm_streamk(0)
    ran = 0
    try:
        for sched, bn in GEMM_CFGS:
            if not hip.gemm_supported(M, N, K, epi, bn):
                continue
            hip.gemm_streamk(0)
            plain = hip.gemm(x, w, b, epi, bn, None, sched)
            hip.gemm_streamk(1)
            n0 = hip.gemm_streamk(-2)
            sk = hip.gemm(x, w, b, epi, bn, None, sched)
            engaged = hip.gemm_streamk(-2) > n0
            sk2 = hip.gemm(x, w, b, epi, bn, None, sched)  # flags reset by the consumers
            torch.cuda.synchronize()
            assert hip.gemm_streamk(-1) == 0, "a stream-K wait gave up"
            _close(sk, y, 0.03, 0.01, f"streamk epi{epi} s{sched}/{bn} M{M} N{N} K{K}")
            assert torch.equal(sk, sk2), "stream-K not deterministic"
            _close(sk, plain.float(), 0.02, 0.01, "streamk vs plain")
            ran += engaged
        assert ran or M < 2048, "no configuration engaged stream-K"
    finally:
        hip.gemm_streamk(1)


def test_gemm_streamk_layout(hip):
    """A = I with an asymmetric B on a stream-K grid (17 x 16 tiles: one whole wave, then 16
    tiles each cut over 4 workgroups): catches a misplaced partial tile or a wrong owner."""
    M, N, K = 4352, 4096, 4096
    x = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(N * K, device=DEV, dtype=torch.float32).view(N, K) % 97 - 48).to(torch.bfloat16)
    exp = torch.zeros(M, N)
    exp[:K] = w.float().t().cpu()
    hip.gemm_streamk(1)
    n0 = hip.gemm_streamk(-2)
    for sched in (0, 1, 2):
        assert torch.equal(hip.gemm(x, w, None, 0, 256, None, sched).float().cpu(), exp), sched
    assert hip.gemm_streamk(-2) == n0 + 3, "the stream-K grid did not engage"
    assert hip.gemm_streamk(-1) == 0


def test_gemm_splitk_dispatch(hip):
    """ops.gemm picks split-K for the low-tile-count shapes and stays on one pass elsewhere."""
    assert ops._gemm_default(2048, 4096, 4096, 0)[2] == 2
    assert ops._gemm_default(4096, 1280, 8192, 0)[2] == 3
    assert ops._gemm_default(8192, 4096, 4096, 0)[2] == 1
    assert ops._gemm_default(2048, 28672, 4096, 1)[2] == 1
    x = torch.randn(2048, 4096, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16) * 0.05
    _close(ops.gemm(x, w), x.float() @ w.float().t(), 0.02, 0.01, "ops.gemm split-K")


def test_gemm_asymmetric_layout(hip):
    """A = I with an asymmetric B catches a transposed C write (CDNA4 playbook §3)."""
    M = N = K = 256
    x = torch.eye(M, K, device=DEV, dtype=torch.bfloat16)
    w = (torch.arange(N * K, device=DEV, dtype=torch.float32).view(N, K) % 97 - 48).to(torch.bfloat16)
    for sched, bn in [(0, 256), (1, 256), (3, 256), (4, 256), (5, 256)]:
        y = hip.gemm(x, w, None, 0, bn, None, sched)
        assert torch.equal(y.float().cpu(), w.float().t().cpu()), f"s{sched}/{bn}"


@pytest.mark.parametrize("M", [300, 2048])
@pytest.mark.parametrize("IK", [(14336, 4096), (3584, 8192), (1536, 768)])
def test_gemm_swiglu_matches_unfused(hip, M, IK):
    I, K = IK
    torch.manual_seed(3)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(2 * I, K, device=DEV, dtype=torch.bfloat16) * 0.05
    a_ref = ref.silu_mul((x.float() @ w.float().t()).to(torch.bfloat16))
    for sched in (0, 1, 3, 4, 5):
        _close(hip.gemm(x, w, None, 1, 256, None, sched), a_ref, 0.03, 0.01, f"gemm s{sched} swiglu M{M} I{I}")


@pytest.mark.parametrize("M", [7, 300, 4000])
@pytest.mark.parametrize("NK", [(2304, 768), (3072, 768), (768, 3072), (1536, 384)])
@pytest.mark.parametrize("epi", [2, 3, 4])
def test_gemm_bias_epilogues(hip, M, NK, epi):
    """bias / bias+GELU(erf) / bias+ReLU epilogues vs fp32 linear -> bf16 -> activation."""
    N, K = NK
    torch.manual_seed(M * 7 + N + epi)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    y = (x.float() @ w.float().t() + b.float()).to(torch.bfloat16).float()
    if epi == 3:
        y = torch.nn.functional.gelu(y)
    elif epi == 4:
        y = torch.relu(y)
    for sched, bn in GEMM_CFGS:
        if hip.gemm_supported(M, N, K, epi, bn, 1, sched):
            _close(hip.gemm(x, w, b, epi, bn, None, sched), y, 0.03, 0.01, f"gemm epi{epi} s{sched}/{bn} M{M} N{N}")


def _model_gemms(name, tp_size):
    """(M values, [(fn, N, K, bias, act)]) of every projection one layer of ``name`` runs on
    TP rank 0 of ``tp_size``, plus its LM head, read off the model's own parameter shapes
    (meta device: no memory)."""
    from llm_kubernetes_minikube_sharp4dev_amd.models import configs
    from llm_kubernetes_minikube_sharp4dev_amd.models.bert import EncoderModel
    from llm_kubernetes_minikube_sharp4dev_amd.models.llama import LlamaModel
    from llm_kubernetes_minikube_sharp4dev_amd.models.opt import OPTModel
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup

    out = []
    if name in configs.ENCODERS:
        cfg = configs.encoder_config(name, num_layers=1)
        m = EncoderModel(cfg, torch.bfloat16, "meta")
        L = m.layers[0]
        out += [("linear", *L.qkv.shape, True, None), ("linear", *L.o.shape, True, None)]
        if L.fc1_b is None:
            out.append(("swiglu", *L.fc1.shape, False, None))
        else:
            out.append(("linear", *L.fc1.shape, True, "gelu"))
        out.append(("linear", *L.fc2.shape, True, None))
        return [16, 300, 2000, 8192], [], out
    cfg = configs.decoder_config(name, num_layers=1)
    tp = TPGroup(rank=0, size=tp_size)
    if cfg.arch == "llama":
        m = LlamaModel(cfg, tp, torch.bfloat16, "meta")
        L = m.layers[0]
        out = [("linear", *L.qkv.shape, False, None), ("linear", *L.o.shape, False, None),
               ("swiglu", *L.gate_up.shape, False, None), ("linear", *L.down.shape, False, None)]
    else:
        m = OPTModel(cfg, tp, torch.bfloat16, "meta")
        L = m.layers[0]
        out = [("linear", *L.qkv.shape, True, None), ("linear", *L.o.shape, True, None),
               ("linear", *L.fc1.shape, True, "relu"), ("linear", *L.fc2.shape, True, None)]
    head = [("linear", *m.lm_head.shape, False, None)]
    return [1, 16, 64, 160, 256, 1024, 4096, 8192], head, out


@pytest.mark.parametrize("name,tp_size", [("llama-3-8b", 1), ("llama-3-70b", 1), ("llama-3-70b", 8),
                                          ("opt-125m", 1), ("bge-base", 1), ("minilm-l6", 1),
                                          ("nomic-embed-text", 1)])
def test_serving_gemms_never_reach_the_library(hip, name, tp_size):
    """Every projection + LM-head shape of every config the engine serves (8B, 70B TP=1, the 70B
    TP=8 rank shard, OPT-125m, the encoders) at decode- and prefill-regime row counts goes to
    the hand-written kernels: no hipBLASLt fallback counted (VERDICT r2 weak #7 / missing #2)."""
    ms, head, body = _model_gemms(name, tp_size)
    ops.LIBRARY_FALLBACKS.clear()
    torch.manual_seed(0)
    for kind, N, K, has_b, act in body + head:
        w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
        bias = torch.zeros(N, device=DEV, dtype=torch.bfloat16) if has_b else None
        for M in (ms if (kind, N, K, has_b, act) not in head else [1, 16, 64, 128, 256]):
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            y = ops.linear_swiglu(x, w) if kind == "swiglu" else ops.linear(x, w, bias, act=act)
            assert y.shape == (M, N // 2 if kind == "swiglu" else N)
            if M <= 256:  # spot-check numerics of the decode-regime kernels on a few rows
                r = x[:4].float() @ w.float().t()
                if kind == "swiglu":
                    g, u = r.chunk(2, dim=1)
                    r = torch.nn.functional.silu(g) * u
                elif act == "relu":
                    r = torch.relu(r)
                elif act == "gelu":
                    r = torch.nn.functional.gelu(r)
                _close(y[:4], r, 0.03, 0.02, f"{name} tp{tp_size} {kind} M{M} N{N} K{K}")
        del w
    torch.cuda.synchronize()
    assert not ops.LIBRARY_FALLBACKS, ops.LIBRARY_FALLBACKS


@pytest.mark.parametrize("M", [1, 4, 16, 33, 64, 100, 128, 200, 256])
@pytest.mark.parametrize("NK", [(4096, 4096), (4096, 14336), (8192, 8192), (8192, 28672)])
def test_ws_linear_rmsnorm_matches_unfused(hip, M, NK):
    """Decode fusion: split-K weight-streaming GEMM -> (reduce + residual add + RMSNorm in one
    kernel) is bit-identical to ws_linear + rmsnorm with the same plan."""
    N, K = NK
    bn, S = hip.ws_plan(M, N, K, False)
    if S < 2:
        S = 2
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    g = torch.rand(N, device=DEV, dtype=torch.bfloat16) + 0.5
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    res2 = res.clone()
    y = hip.ws_linear_rmsnorm(x, w, res, g, 1e-5, bn, S)
    y2 = hip.rmsnorm(hip.ws_linear(x, w, False, bn, S), g, 1e-5, res2, None)
    assert torch.equal(res, res2), "residual"
    assert torch.equal(y, y2), "normed output"
    # and against fp32 math
    r32 = res2.float()  # already updated: x W^T + residual (bf16-rounded)
    y_ref = r32 * torch.rsqrt(r32.pow(2).mean(-1, keepdim=True) + 1e-5) * g.float()
    _close(y, y_ref, 0.05, 0.02, f"rmsnorm M{M} N{N}")


@pytest.mark.parametrize("M", [1, 3, 40, 128, 200])
@pytest.mark.parametrize("neox", [True, False])
@pytest.mark.parametrize("inplace", [False, True])
def test_ws_linear_rope_kv_matches_unfused(hip, M, neox, inplace):
    """Decode fusion: split-K QKV GEMM -> (reduce + RoPE + paged KV write in one kernel) leaves
    the qkv row and both caches exactly as ws_linear + rope_kv_ does."""
    Hq, Hkv, D, BS, NB, K = 32, 8, 128, 16, 32, 4096
    N = (Hq + 2 * Hkv) * D
    bn, S = hip.ws_plan(M, N, K, False)
    if S < 2:
        S = 2
    torch.manual_seed(M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    pos = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(4096, D, 500000.0, device=DEV)
    kc = torch.zeros(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(NB * BS, device=DEV)[:M].int()
    if M > 1:
        slots[1] = -1
    kc2, vc2 = kc.clone(), vc.clone()
    qkv = hip.ws_linear_rope_kv(x, w, pos, cs, Hq, Hkv, D, kc, vc, slots, neox, inplace, bn, S)
    qkv2 = hip.ws_linear(x, w, False, bn, S)
    hip.rope_kv_(qkv2, pos, cs, Hq, Hkv, D, kc2, vc2, slots, neox, inplace)
    assert torch.equal(qkv, qkv2), "qkv"
    assert torch.equal(kc, kc2), "k cache"
    assert torch.equal(vc, vc2), "v cache"


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("NK", [(4096, 4096), (4096, 14336), (8192, 28672)])
def test_ws_linear_rmsnorm_fused_tail(hip, M, NK):
    """Split-K GEMM whose LAST workgroup does residual + RMSNorm (WsTail kind 2: no reduce
    launch) == the two-launch path: residual bit for bit, the normed rows to a bf16 ulp (the
    sum of squares is reduced over another thread split); tickets back at 0."""
    N, K = NK
    bn, S = hip.ws_plan(M, N, K, False)
    if S < 2:
        S = 2
    torch.manual_seed(M * 7 + K)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    g = torch.rand(N, device=DEV, dtype=torch.bfloat16) + 0.5
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    res2 = res.clone()
    tickets = torch.zeros(64, dtype=torch.int32, device=DEV)
    for _ in range(2):
        y = hip.ws_linear_rmsnorm(x, w, res, g, 1e-5, bn, S, tickets)
        y2 = hip.ws_linear_rmsnorm(x, w, res2, g, 1e-5, bn, S)
        assert torch.equal(res, res2), "residual"
        _close(y, y2, 0.0, 2 ** -7, f"fused-tail rmsnorm M{M} N{N}")
        assert int(tickets.abs().sum()) == 0


@pytest.mark.parametrize("M", [1, 3, 40, 200])
@pytest.mark.parametrize("neox", [True, False])
@pytest.mark.parametrize("inplace", [False, True])
def test_ws_linear_rope_kv_fused_tail(hip, M, neox, inplace):
    """Split-K QKV GEMM whose last workgroup per head applies RoPE and writes the paged KV
    (WsTail kind 1: no reduce launch) == ws_linear + rope_kv_; tickets back at 0."""
    Hq, Hkv, D, BS, NB, K = 32, 8, 128, 16, 32, 4096
    N = (Hq + 2 * Hkv) * D
    bn, S = hip.ws_plan(M, N, K, False)
    if bn != 128 or S not in (2, 4, 8):
        bn, S = 128, 4
    torch.manual_seed(M + 100)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    pos = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(4096, D, 500000.0, device=DEV)
    kc = torch.zeros(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    slots = torch.randperm(NB * BS, device=DEV)[:M].int()
    if M > 1:
        slots[1] = -1
    kc2, vc2 = kc.clone(), vc.clone()
    tickets = torch.zeros(Hq + 2 * Hkv, dtype=torch.int32, device=DEV)
    qkv = hip.ws_linear_rope_kv(x, w, pos, cs, Hq, Hkv, D, kc, vc, slots, neox, inplace, bn, S, tickets)
    qkv2 = hip.ws_linear(x, w, False, bn, S)
    hip.rope_kv_(qkv2, pos, cs, Hq, Hkv, D, kc2, vc2, slots, neox, inplace)
    _close(qkv, qkv2, 0.0, 2 ** -8, "qkv")
    _close(kc, kc2, 0.0, 2 ** -8, "k cache")
    assert torch.equal(vc, vc2), "v cache"
    assert int(tickets.abs().sum()) == 0


def test_linear_add_rmsnorm_dispatch(hip):
    """ops.linear_add_rmsnorm takes the fused path on a split-K decode shape and matches the
    unfused dispatch (LK_DECODE_FUSION=0) bit for bit."""
    assert ops.DECODE_FUSION
    x = torch.randn(128, 4096, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(4096, 14336, device=DEV, dtype=torch.bfloat16) * 0.02
    a = torch.randn(128, 14336, device=DEV, dtype=torch.bfloat16)
    g = torch.ones(4096, device=DEV, dtype=torch.bfloat16)
    res, res2 = x.clone(), x.clone()
    y = ops.linear_add_rmsnorm(a, w, res, g, 1e-5)
    ops.DECODE_FUSION = False
    try:
        y2 = ops.linear_add_rmsnorm(a, w, res2, g, 1e-5)
    finally:
        ops.DECODE_FUSION = True
    assert torch.equal(y, y2) and torch.equal(res, res2)


@pytest.mark.parametrize("sample", [False, True])
def test_select_allowed_matches_masked_select(hip, sample):
    """Grammar-constrained selection over per-row allowed ids equals masking every other id
    to -inf and scanning the whole row (greedy and Gumbel sampling, ties included)."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import Sampler

    torch.manual_seed(11)
    B, V = 7, 128256
    logits = torch.randn(B, V, device=DEV)
    logits[2, 500] = logits[2, 77] = 50.0  # tie: the lower id wins on both paths
    g = torch.Generator().manual_seed(0)
    rows = {0: torch.randint(0, V, (3000,), generator=g).numpy(), 2: np.array([77, 500, 9, 128000]),
            3: np.array([5]), 5: torch.randint(0, V, (40,), generator=g).numpy(), 6: np.array([V - 1, 0])}
    rows = {i: a.astype(np.int64) for i, a in rows.items()}
    plan = Sampler(V)._plan(rows, B, torch.device(DEV))
    masked = logits.clone()
    for i, a in rows.items():
        m = torch.full((V,), float("-inf"), device=DEV)
        m[torch.from_numpy(a).to(DEV)] = 0.0
        masked[i] += m
    temps = torch.tensor([0.7, 1.0, 0.0, 1.3, 0.9, 0.5, 2.0], device=DEV) if sample else None
    a = hip.select_allowed(logits, plan, temps, 1234, 5)
    b = hip.select_tokens(masked, temps, 1234, 5, None)
    assert torch.equal(a, b)
    assert int(a[2]) == 77 or sample


def test_tune_decode_routes_by_measurement(hip):
    """ops.tune_decode fills the decode routing table from cold-weight timings, and
    _decode_gemm_kind / linear follow it for every bucket (results stay exact either way)."""
    w = torch.randn(7168, 8192, device=DEV, dtype=torch.bfloat16) * 0.02  # 70B TP=8 gate_up shard
    o = torch.randn(8192, 1024, device=DEV, dtype=torch.bfloat16) * 0.02   # 70B TP=8 o shard
    saved = dict(ops._DECODE_TABLE)
    saved_var = dict(ops._WS_VARIANTS)
    shapes = ((7168, 8192, True), (8192, 1024, False))
    variants = {}
    try:
        ops._DECODE_TABLE.clear()
        res = ops.tune_decode([(w, True), (o, False)], ms=(64, 192, 256), iters=3, cold_bytes=256 << 20)
        routes = {key: v for key, v in res.items() if len(key) == 4}
        variants = {key[:4]: v for key, v in res.items() if len(key) == 5}
        assert set(routes) == {(m, n, k, sw) for m in (64, 192, 256) for (n, k, sw) in shapes}
        # the weight-streaming kernel variant (one ring / loader waves) is measured per row tile too
        assert set(variants) == set(routes) and all(key[4] == "ws_variant" for key in res if len(key) == 5)
        for key, arms in variants.items():
            assert set(arms) == {"ring", "loader"}
            # the pick is the faster arm (the reported times are rounded to 0.1 us: ties allowed)
            assert arms[("ring", "loader")[ops._WS_VARIANTS[key]]] == min(arms.values())
        for (m, n, k, sw), arms in routes.items():
            assert set(arms) == {"ws", "gemm"} and all(v > 0 for v in arms.values())
            pick = ops._DECODE_TABLE[(m, n, k, sw)]
            assert arms[pick] == min(arms.values())
            x = torch.randn(m - 7, k, device=DEV, dtype=torch.bfloat16)  # same bucket
            kind = ops._decode_gemm_kind(x, w if sw else o, sw)
            assert kind == ("ws" if pick == "ws" else None)
            if sw:
                _close(ops.linear_swiglu(x, w), ref.silu_mul((x.float() @ w.float().t()).to(torch.bfloat16)), 0.03, 0.01)
            else:
                _close(ops.linear(x, o), x.float() @ o.float().t(), 0.02, 0.01)
    finally:
        ops._DECODE_TABLE.clear()
        ops._DECODE_TABLE.update(saved)
        for (m, n, k, sw) in variants:
            hip.ws_set_variant(m, n, k, sw, -1)
        ops.apply_ws_variants(saved_var)


# ---------------------------------------------------------------- fused prefill chain epilogues
def _qkv_setup(M, Hq=32, Hkv=8, D=128, H=4096, nb=600, bs=16, seed=0):
    torch.manual_seed(seed)
    x = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn((Hq + 2 * Hkv) * D, H, device=DEV, dtype=torch.bfloat16) * 0.02
    pos = torch.randint(0, 4000, (M,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(8192, D, 500000.0, device=DEV)
    perm = torch.randperm(nb * bs, device=DEV)[:M].to(torch.int32)
    slots = torch.where(torch.rand(M, device=DEV) < 0.1, torch.full_like(perm, -1), perm)
    kc = torch.zeros(nb, Hkv, bs, D, device=DEV, dtype=torch.bfloat16)
    return x, w, pos, cs, slots, kc, kc.clone()


@pytest.mark.parametrize("M,N,K,splits", [(300, 1024, 512, 1), (1000, 4096, 1024, 1), (2304, 4096, 14336, 3),
                                          (777, 2048, 4096, 2), (4352, 4096, 4096, 1), (2664, 4096, 4096, 1)])
@pytest.mark.parametrize("variant", [2, 3, 4, 5, 6])
def test_gemm_resid_epilogue(hip, M, N, K, splits, variant):
    """RESID (producer side of the folded norm): r = bf16(r + bf16(x W^T)) in place and the
    per-256-column partial sums of squares of the new r, in-kernel and through the split-K
    reduce, M tails; 4352 x 4096 engages stream-K (17 x 16 tiles)."""
    torch.manual_seed(M + N + splits)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    r = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    r_ref, ss_ref = r.clone(), torch.zeros(N // 256, M, device=DEV)
    ref.linear_resid(x, w, r_ref, ss_ref)
    ss = torch.full((N // 256, M), float("nan"), device=DEV)
    n0 = hip.gemm_streamk(-2)
    hip.gemm_fused(x, w, 6, 256, None, variant, splits, resid=r, ss_out=ss)
    torch.cuda.synchronize()
    _close(r, r_ref, 0.02, 0.01, f"resid M{M} N{N} K{K} s{splits} v{variant}")
    _close(ss, ss_ref, 0.5, 0.01, f"ss partials M{M} N{N}")
    assert hip.gemm_streamk(-1) == 0
    if M == 4352 and variant == 2:
        assert hip.gemm_streamk(-2) > n0, "stream-K did not engage"


@pytest.mark.parametrize("M", [300, 2048, 4352])
@pytest.mark.parametrize("scaled", [False, True])
@pytest.mark.parametrize("variant,H", [(2, 4096), (3, 4096), (3, 8192), (4, 4096), (5, 8192)])
def test_gemm_swiglu_row_scale(hip, M, scaled, variant, H):
    """SwiGLU epilogue with the folded post-norm's row scale s = rsqrt(sum(ss) / H + eps) (H 8192:
    32 partial planes, the 70B width)."""
    torch.manual_seed(M)
    I = 1792
    r = torch.randn(M, H, device=DEV, dtype=torch.bfloat16) * 3
    w = torch.randn(2 * I, H, device=DEV, dtype=torch.bfloat16) * 0.02
    ss = ref.ss_partials(r) if scaled else None
    y = hip.gemm_fused(r, w, 1, 256, None, variant, 1, ss_in=ss, eps=1e-5)
    y_ref = ref.gemm_scaled(r, w, ss, H, 1e-5, swiglu=True)
    _close(y, y_ref, 0.03, 0.02, f"swiglu scaled={scaled} M{M} v{variant} H{H}")


@pytest.mark.parametrize("M,bn,variant", [(300, 192, 2), (1111, 256, 2), (4352, 192, 2), (2560, 256, 2),
                                          (300, 256, 3), (1111, 256, 3), (4352, 256, 3), (2664, 256, 4),
                                          (300, 256, 4), (2664, 256, 5), (1111, 256, 5), (4352, 256, 6),
                                          (4000, 256, 7)])
@pytest.mark.parametrize("scaled", [False, True])
def test_gemm_qkv_epilogue(hip, M, bn, variant, scaled):
    """QKV epilogue: row scale, interleaved-pair RoPE on q / k, K / V into the paged cache at
    slots[row] (-1 skipped), the qkv row written back -- vs GEMM -> rope_kv_ in fp32; 4352 rows
    at bn 192 engage stream-K."""
    x, w, pos, cs, slots, kc, vc = _qkv_setup(M, seed=M + bn)
    ss = ref.ss_partials(x) if scaled else None
    kc2, vc2 = kc.clone(), vc.clone()
    out = hip.gemm_fused(x, w, 7, bn, None, variant, 1, ss_in=ss, eps=1e-5, positions=pos, cos_sin=cs, slots=slots,
                         k_cache=kc, v_cache=vc, hq=32, hkv=8, hd=128)
    want = ref.qkv_fused(x, w, ss, 4096, 1e-5, pos, cs, 32, 8, 128, kc2, vc2, slots)
    torch.cuda.synchronize()
    _close(out, want, 0.03, 0.02, f"qkv M{M} bn{bn} v{variant}")
    _close(kc, kc2, 0.03, 0.02, "k cache")
    _close(vc, vc2, 0.03, 0.02, "v cache")
    assert hip.gemm_streamk(-1) == 0


@pytest.mark.parametrize("variant", [6, 7])
@pytest.mark.parametrize("M,N,K,epi", [(4000, 6144, 512, 0), (4352, 4096, 768, 3), (600, 28672, 512, 1),
                                       (6000, 3072, 768, 2)])
def test_gemm1w_column_split(hip, variant, M, N, K, epi):
    """Variants 6 / 7: the column tiles that fill whole waves on 256-row tiles, the rest on 128 /
    192-row tiles (two launches, the second offset by tn0 column tiles) -- every column, bias and
    SwiGLU pair lands where the one-launch kernel puts it."""
    assert ops._split_applies(M, N, epi), "shape must engage the split"
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16) if epi >= 2 else None
    got = hip.gemm(x, w, b, epi, 256, None, variant, 1)
    y = x.float() @ w.float().t()
    if epi == 1:
        I = N // 2
        y = torch.nn.functional.silu(y[:, :I].bfloat16().float()) * y[:, I:].bfloat16().float()
    elif epi >= 2:
        y = y.bfloat16().float() + b.float()
        y = torch.nn.functional.gelu(y) if epi == 3 else y
    _close(got, y, 0.03, 0.02, f"split v{variant} epi{epi} M{M} N{N}")


@pytest.mark.parametrize("M,Hq,Hkv", [(1111, 32, 8), (2664, 32, 8)])
def test_linear_rope_kv_epilogue_matches_unfused(hip, monkeypatch, M, Hq, Hkv):
    """Prefill-sized QKV outside the fused chain (the TP block's path): RoPE and the paged-KV
    write run in the QKV GEMM's epilogue (128- / 192-row gemm1w tiles at these M), matching
    GEMM -> rope_kv_ (interleaved pairs)."""
    x, w, pos, cs, slots, kc, vc = _qkv_setup(M, Hq=Hq, Hkv=Hkv, H=4096, seed=M)
    kc2, vc2 = kc.clone(), vc.clone()
    assert ops._qkv_epilogue_ok(x, w, False, False, kc, slots)
    got = ops.linear_rope_kv(x, w, pos, cs, Hq, Hkv, 128, kc, vc, slots, neox=False)
    monkeypatch.setattr(ops, "PREFILL_CHAIN", False)
    want = ops.linear_rope_kv(x, w, pos, cs, Hq, Hkv, 128, kc2, vc2, slots, neox=False)
    torch.cuda.synchronize()
    qd, kd = Hq * 128, (Hq + Hkv) * 128  # k columns of the row: rotated by the epilogue, unused (K is read from the cache)
    _close(got[:, :qd], want[:, :qd], 0.02, 0.01, f"q: epilogue vs unfused M{M}")
    _close(got[:, kd:], want[:, kd:], 0.02, 0.01, f"v: epilogue vs unfused M{M}")
    _close(kc, kc2, 0.02, 0.01, "k cache")
    _close(vc, vc2, 0.02, 0.01, "v cache")


def test_gemm_qkv_epilogue_layout(hip):
    """Asymmetric exact data through the QKV epilogue: x = I-rows, W rows = distinct ramps, RoPE at
    position 0 (identity): every output column / cache element lands where the reference puts it."""
    M, Hq, Hkv, D, H = 512, 4, 2, 128, 1024
    x = torch.zeros(M, H, device=DEV, dtype=torch.bfloat16)
    x[torch.arange(M), torch.arange(M) % H] = 1
    N = (Hq + 2 * Hkv) * D
    w = ((torch.arange(N, device=DEV)[:, None] * 7 + torch.arange(H, device=DEV)[None, :]) % 251 - 125).to(torch.bfloat16)
    pos = torch.zeros(M, device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(16, D, 10000.0, device=DEV)
    slots = torch.arange(M, device=DEV, dtype=torch.int32)
    kc = torch.zeros(M // 16, Hkv, 16, D, device=DEV, dtype=torch.bfloat16)
    vc, kc2, vc2 = kc.clone(), kc.clone(), kc.clone()
    for variant in (2, 3, 4, 5):
        kc.zero_(), vc.zero_(), kc2.zero_(), vc2.zero_()
        out = hip.gemm_fused(x, w, 7, 256, None, variant, 1, positions=pos, cos_sin=cs, slots=slots, k_cache=kc,
                             v_cache=vc, hq=Hq, hkv=Hkv, hd=D)
        want = ref.qkv_fused(x, w, None, H, 1e-5, pos, cs, Hq, Hkv, D, kc2, vc2, slots)
        assert torch.equal(out.cpu(), want.cpu()) and torch.equal(kc.cpu(), kc2.cpu()) and torch.equal(vc.cpu(), vc2.cpu())


@pytest.mark.parametrize("lo,n_local", [(0, None), (0, 300), (300, 300), (600, 424)])
def test_embed_rows(hip, lo, n_local):
    """Token-embedding gather (full table, and a vocab-parallel shard: out-of-shard ids -> 0)."""
    V, H = 1024, 4096
    table = torch.randn(V if n_local is None else n_local, H, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, V, (777,), device=DEV, dtype=torch.int32)
    got = ops.embed_rows(table, ids, lo, n_local)
    local = ids.long() - lo
    n = table.shape[0]
    want = table[local.clamp(0, n - 1)].masked_fill(((local < 0) | (local >= n))[:, None], 0)
    assert torch.equal(got.cpu(), want.cpu())


def test_embed_rows_counts_out_of_vocab_ids(hip):
    """The whole-table lookup (no vocab shard) counts ids outside the table on the device, so a
    tokenizer / model vocab mismatch fails the engine's health check instead of passing as
    silent zero embeddings; a vocab-parallel shard's out-of-shard ids are not errors."""
    V, H = 512, 1024
    table = torch.randn(V, H, device=DEV, dtype=torch.bfloat16)
    hip.embed_errors()  # reset
    ids = torch.tensor([0, 5, V - 1, 3], device=DEV, dtype=torch.int32)
    ops.embed_rows(table, ids)
    torch.cuda.synchronize()
    assert hip.embed_errors() == 0
    bad = torch.tensor([1, V, V + 7, -2, 4], device=DEV, dtype=torch.int32)
    out = ops.embed_rows(table, bad)
    torch.cuda.synchronize()
    assert hip.embed_errors() == 3 and hip.embed_errors() == 0
    assert torch.equal(out[1].cpu(), torch.zeros(H, dtype=torch.bfloat16))
    ops.embed_rows(table, bad, 0, 256)  # shard [0, 256): out-of-shard ids are the TP contract
    torch.cuda.synchronize()
    assert hip.embed_errors() == 0


def test_scatter_ids_and_gather_rows(hip):
    ids = torch.arange(64, device=DEV, dtype=torch.int32)
    prev = torch.randint(0, 1000, (16,), device=DEV, dtype=torch.int32)
    dst = torch.tensor([3, 9, 40], device=DEV)
    src = torch.tensor([15, 0, 7], device=DEV)
    want = ids.clone()
    want[dst] = prev[src]
    ops.scatter_ids(ids, dst, prev, src)
    assert torch.equal(ids.cpu(), want.cpu())
    x = torch.randn(1000, 4096, device=DEV, dtype=torch.bfloat16)
    idx = torch.tensor([999, 0, 17, 17, 500], device=DEV)
    assert torch.equal(ops.gather_rows(x, idx).cpu(), x[idx].cpu())


@pytest.mark.parametrize("M", [1, 40, 64, 100, 128, 160, 192, 230, 256])
@pytest.mark.parametrize("NK,swiglu", [((6144, 4096), False), ((4096, 14336), False), ((28672, 4096), True),
                                        ((1280, 8192), False)])
def test_ws_loader_wave_variant_bit_identical(hip, M, NK, swiglu):
    """The loader-wave weight-streaming kernel (wsgemm_lw_kernel) computes every tile with the
    same MFMA sequence as the one-ring kernel: bit-identical output for each BN / split plan,
    the split-K partial path and SwiGLU, and within tolerance of the fp32 product."""
    N, K = NK
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    plans = [(None, None)] + ([(64, 1), (128, 2), (64, 4)] if not swiglu else [(128, 1), (64, 1)])
    try:
        for bn, S in plans:
            if bn is not None and ((N // 2 if swiglu else N) % (bn // 2 if swiglu else bn) or K % (S * 64)):
                continue
            outs = []
            for v in (0, 1):
                hip.ws_set_variant(M, N, K, swiglu, v)
                outs.append(hip.ws_linear(x, w, swiglu) if bn is None else hip.ws_linear(x, w, swiglu, bn, S))
            torch.cuda.synchronize()
            assert torch.equal(outs[0], outs[1]), (M, N, K, bn, S)
        y = x.float() @ w.float().t()
        if swiglu:
            g, u = y[:, : N // 2], y[:, N // 2:]
            y = torch.nn.functional.silu(g) * u
        _close(outs[1], y, 0.03, 0.02, f"lw M{M} N{N} K{K}")
    finally:
        hip.ws_set_variant(M, N, K, swiglu, -1)


def test_invalid_launch_raises(hip):
    """A launch the runtime rejects (2048 threads per workgroup) raises with the HIP error
    instead of returning as if it had run; the next op on the stream still works."""
    with pytest.raises(RuntimeError, match="kernel launch failed"):
        hip.debug_invalid_launch()
    x = torch.randn(4, 768, device=DEV, dtype=torch.bfloat16)
    w = torch.ones(768, device=DEV, dtype=torch.bfloat16)
    _close(hip.rmsnorm(x, w, 1e-5, None, None), ref.rmsnorm(x, w, 1e-5, None), 0.05, 0.01, "after a failed launch")


@pytest.mark.parametrize("fused", [False, True])
def test_knn_topk_config4_scale(hip, fused):
    """BASELINE config 4's index size: 1M runbook documents -> ~4.86M chunks x 768 (7.5 GB bf16,
    past every 32-bit byte offset and 4 GB buffer range), vs an fp32 reference computed in
    row chunks.  Exact duplicates planted far apart (different tiles, different halves of the
    corpus) must tie bit-identically and come back in id order; the last row (a partial tail
    tile) must be found."""
    N, D, K = 4_900_000, 768, 6
    g = torch.Generator(device=DEV).manual_seed(21)
    corpus = torch.empty(N, D, device=DEV, dtype=torch.bfloat16)
    for a in range(0, N, 1 << 20):
        b = min(N, a + (1 << 20))
        corpus[a:b] = torch.randn(b - a, D, device=DEV, generator=g).to(torch.bfloat16)
    dup = (123, 3_000_000, 4_800_000)
    for j in dup[1:]:
        corpus[j] = corpus[dup[0]]
    qs = torch.randn(8, D, device=DEV, generator=g).to(torch.bfloat16)
    qs[0] = corpus[dup[0]]
    qs[1] = corpus[N - 1]
    qs[2] = corpus[2_500_000] * 0.5 + qs[2] * 0.1
    cn, qn = hip.row_norms(corpus), hip.row_norms(qs)
    s, i = hip.knn_topk(corpus, cn, qs, qn, K, fused)
    torch.cuda.synchronize()
    # fp32 reference: per 1M-row chunk, the best 64 candidates, then a stable (score, id) merge
    qf = qs.float()
    cand_s, cand_i = [], []
    for a in range(0, N, 1 << 20):
        b = min(N, a + (1 << 20))
        sc = (qf @ corpus[a:b].float().T) / (qf.norm(dim=1, keepdim=True) * corpus[a:b].float().norm(dim=1)[None] + 1e-9)
        ts, ti = sc.topk(64, dim=1)
        cand_s.append(ts.cpu())
        cand_i.append((ti + a).cpu())
    cs, ci = torch.cat(cand_s, 1), torch.cat(cand_i, 1)
    s, i = s.cpu(), i.cpu().long()
    for q in range(8):
        order = sorted(range(cs.shape[1]), key=lambda j: (-float(cs[q, j]), int(ci[q, j])))[:K]
        want_i = [int(ci[q, j]) for j in order]
        want_s = [float(cs[q, j]) for j in order]
        ref_of = {int(ci[q, j]): float(cs[q, j]) for j in range(cs.shape[1])}
        assert bool((s[q, 1:] <= s[q, :-1]).all()), f"query {q}: scores not descending"
        for j in range(K):
            got = int(i[q, j])
            assert abs(float(s[q, j]) - want_s[j]) < 2e-3, (q, j, float(s[q, j]), want_s[j])
            if got != want_i[j]:  # only a near-tie may reorder
                assert got in ref_of and abs(ref_of[got] - want_s[j]) < 2e-3, (q, j, got, want_i[j])
    assert i[0, :3].tolist() == list(dup), i[0].tolist()
    assert float(s[0, 0]) == float(s[0, 1]) == float(s[0, 2])
    assert int(i[1, 0]) == N - 1 and int(i[2, 0]) == 2_500_000


# ---- consumer-side prologues of the weight-streaming GEMM (decode steps of few rows) ----
@pytest.mark.parametrize("M", [1, 4, 16])
@pytest.mark.parametrize("shape", ["qkv", "gate_up"])
def test_ws_pro_norm_matches_unfused(hip, M, shape):
    """ws_pro kind 1 (residual add + RMSNorm of the producer's split-K slabs computed by the GEMM's
    own workgroups) == splitk_rmsnorm followed by the same GEMM, bit for bit: the normed rows, the
    new residual (written by workgroup 0 into another buffer) and the GEMM output."""
    H, eps = 4096, 1e-5
    N, swiglu = (6144, False) if shape == "qkv" else (28672, True)
    torch.manual_seed(M + N)
    pp = torch.randn(4, M, H, device=DEV) * 0.5
    res = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    g = (torch.rand(H, device=DEV) + 0.5).to(torch.bfloat16)
    w = torch.randn(N, H, device=DEV, dtype=torch.bfloat16) * 0.02
    bn, S = hip.ws_plan(M, N, H, swiglu)
    hip.ws_set_variant(M, N, H, swiglu, 0)
    try:
        res_ref = res.clone()
        x_ref = hip.splitk_rmsnorm(pp, res_ref, g, eps)
        res_in, res_out, x = res.clone(), torch.full_like(res, 3.0), torch.empty_like(res)
        if swiglu:
            want = hip.ws_linear(x_ref, w, True, bn, S)
            got = hip.ws_pro(x, w, True, bn, S, 1, True, pp, res_in, res_out, g, eps)
        else:
            want = hip.ws_pro(x_ref, w, False, bn, S, 0)
            got = hip.ws_pro(x, w, False, bn, S, 1, False, pp, res_in, res_out, g, eps)
        torch.cuda.synchronize()
        assert torch.equal(x, x_ref) and torch.equal(res_out, res_ref) and torch.equal(res_in, res)
        assert torch.equal(got, want), (got.float() - want.float()).abs().max()
    finally:
        hip.ws_set_variant(M, N, H, swiglu, -1)


@pytest.mark.parametrize("M", [1, 3, 16])
def test_ws_pro_merge_matches_decode_reduce(hip, M):
    """ws_pro kind 2: the O projection's workgroups merge the split-K paged-decode partials of
    their K slice (paged_decode(reduce=False): no decode_reduce launch) -- the attention rows
    equal the reduce kernel's bit for bit (one-split rows written by the attention kernel itself)
    and the O partial slabs equal the plain GEMM's over the reduced rows."""
    Hkv, G, D, BS = 8, 4, 128, 16
    Hq = Hkv * G
    ctx = ([1, 700, 2100, 129, 5, 1000, 64, 3000, 17, 256, 900, 1500, 33, 2, 511, 800])[:M]
    kc, vc, bt = _paged_setup(M, ctx, Hkv, D, BS, seed=21)
    q = torch.randn(M, Hq, D, device=DEV, dtype=torch.bfloat16)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    split = 128
    ms = ops.decode_splits(bt.shape[1] * BS, split)
    w = torch.randn(4096, Hq * D, device=DEV, dtype=torch.bfloat16) * 0.02
    bn, S = hip.ws_plan(M, 4096, Hq * D, False)
    po = torch.empty(M, Hq, ms, D, device=DEV)
    pml = torch.empty(M, Hq, ms, 2, device=DEV)
    want_rows = hip.paged_decode(q, kc, vc, bt, cl, ms, split, 0.088, None, None, None).view(M, Hq * D)
    rows = torch.full((M, Hq * D), 5.0, device=DEV, dtype=torch.bfloat16)
    hip.paged_decode(q, kc, vc, bt, cl, ms, split, 0.088, po, pml, rows.view(M, Hq, D), None, None, None, None, False)
    got = hip.ws_pro(rows, w, False, bn, S, 2, False, None, None, None, None, 0.0, po, pml, cl, split, ms, Hq)
    want = hip.ws_pro(want_rows.contiguous(), w, False, bn, S, 0)
    torch.cuda.synchronize()
    assert torch.equal(rows, want_rows)
    assert torch.equal(got, want)
