"""Decode GEMV (csrc/gemv_decode.hip) vs plain-PyTorch fp32 references: every mode (plain, residual
add, SwiGLU, RoPE + paged-KV write) with and without the RMSNorm prologue, at the Llama-3-8B and
70B-TP8 projection shapes, and one decode step of a Llama-3-8B-shaped model through the GEMV block
vs the weight-streaming block on the same inputs."""
import copy

import pytest
import torch

from llm_kubernetes_minikube_sharp4dev_amd import ops
from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, K): QKV / O / gate_up / down of Llama-3-8B, and 70B TP=8 shards (K 8192, K 3584)
SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (1280, 8192), (8192, 3584)]


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item() if a.numel() else 0.0
    tol = atol + rtol * b.abs().max().item() if b.numel() else atol
    assert err <= tol, f"{msg} max abs err {err:.4g} > {tol:.4g}"


def _normed(x, g, eps):
    """rmsnorm_kernel's arithmetic: bf16(x * inv) * g, rounded to bf16."""
    xf = x.float()
    inv = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return ((xf * inv).to(torch.bfloat16).float() * g.float()).to(torch.bfloat16)


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("NK", SHAPES)
@pytest.mark.parametrize("norm", [False, True])
def test_gemv_plain(hip, M, NK, norm):
    N, K = NK
    assert hip.gemv_supported(M, N, K, 0)
    torch.manual_seed(N + K + M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    g = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16) if norm else None
    xin = _normed(x, g, 1e-5) if norm else x
    y = hip.gemv_decode(0, x, w, g, 1e-5)
    _close(y, xin.float() @ w.float().t(), 0.02, 0.01, f"gemv M{M} N{N} K{K} norm {norm}")


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("NK", [(4096, 4096), (4096, 14336), (8192, 3584)])
def test_gemv_residual(hip, M, NK):
    N, K = NK
    torch.manual_seed(3 * N + M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    res = torch.randn(M, N, device=DEV, dtype=torch.bfloat16)
    want = ((x.float() @ w.float().t()).to(torch.bfloat16).float() + res.float()).to(torch.bfloat16)
    out = hip.gemv_decode(1, x, w, res=res)
    assert out.data_ptr() == res.data_ptr()
    _close(res, want, 0.03, 0.01, f"gemv residual M{M} N{N}")


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("NK", [(4096, 14336), (1280, 8192)])
def test_gemv_ksplit_arms_agree(hip, M, NK):
    """Long-K shapes run two waves per pair (a K half each, joined in LDS); with the split off one
    wave walks all of K -- both against the fp32 reference and each other."""
    N, K = NK
    torch.manual_seed(N + M)
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.02
    want = x.float() @ w.float().t()
    try:
        outs = []
        for on in (True, False):
            hip.gemv_set_ksplit(on)
            outs.append(hip.gemv_decode(0, x, w))
    finally:
        hip.gemv_set_ksplit(ops.GEMV_KSPLIT)
    for y in outs:
        _close(y, want, 0.02, 0.01, f"gemv M{M} N{N} K{K}")
    _close(outs[0], outs[1], 0.01, 0.005, "ksplit arms")


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("IK", [(14336, 4096), (3584, 8192)])
def test_gemv_swiglu_norm(hip, M, IK):
    I, K = IK
    torch.manual_seed(I + M)
    res = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    g = (torch.rand(K, device=DEV) + 0.5).to(torch.bfloat16)
    w = torch.randn(2 * I, K, device=DEV, dtype=torch.bfloat16) * 0.02
    xin = _normed(res, g, 1e-5)
    a_ref = ref.silu_mul((xin.float() @ w.float().t()).to(torch.bfloat16))
    a = hip.gemv_decode(2, res, w, g, 1e-5)
    assert a.shape == (M, I)
    _close(a, a_ref, 0.03, 0.01, f"gemv swiglu M{M} I{I}")


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("neox", [True, False])
@pytest.mark.parametrize("heads", [(32, 8), (8, 1)])
def test_gemv_qkv_rope_kv(hip, M, neox, heads):
    """Mode 3 == GEMV -> rope_kv_ (fp32 reference): q rotated in the row, k unrotated in the row and
    rotated in the paged cache at the row's slot, v copied; a slot of -1 writes no cache."""
    Hq, Hkv = heads
    D, BS, H = 128, 16, 4096 if Hq == 32 else 8192
    N = (Hq + 2 * Hkv) * D
    torch.manual_seed(Hq + M + int(neox))
    res = torch.randn(M, H, device=DEV, dtype=torch.bfloat16)
    g = (torch.rand(H, device=DEV) + 0.5).to(torch.bfloat16)
    w = torch.randn(N, H, device=DEV, dtype=torch.bfloat16) * 0.02
    cos_sin = ops.rope_cos_sin(4096, D, 500000.0, None, device=DEV)
    pos = torch.tensor([37, 2049][:M], dtype=torch.int32, device=DEV)
    slots = torch.tensor([5 * BS + 3, -1][:M], dtype=torch.int32, device=DEV)
    kc = torch.zeros(12, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    kc_ref, vc_ref = kc.clone(), vc.clone()
    qkv_ref = (_normed(res, g, 1e-5).float() @ w.float().t()).to(torch.bfloat16)
    unrot = qkv_ref.clone()
    ref.rope_kv_(qkv_ref, pos, cos_sin, Hq, Hkv, D, kc_ref, vc_ref, slots, neox, False)
    qkv = hip.gemv_decode(3, res, w, g, 1e-5, None, pos, cos_sin, Hq, Hkv, D, kc, vc, slots, neox)
    _close(qkv[:, : Hq * D], qkv_ref[:, : Hq * D], 0.03, 0.01, "q rotated")
    _close(qkv[:, Hq * D:], unrot[:, Hq * D:], 0.03, 0.01, "k / v rows (k unrotated)")
    _close(kc, kc_ref, 0.03, 0.01, "k cache")
    _close(vc, vc_ref, 0.03, 0.01, "v cache")
    assert kc.float().abs().sum() > 0 and torch.count_nonzero(kc.float()) == Hkv * D


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("ctx", [(700, 100), (1000, 2000), (64, 90)])
def test_gemv_o_merges_decode_splits(hip, M, ctx):
    """Mode 1 with the split-merge prologue: paged_decode(reduce=False) leaves multi-split rows as
    partials, the O projection's GEMV merges them (decode_reduce_kernel's arithmetic) -- the new
    residual equals decode_reduce -> plain GEMV; one-split rows pass through unmerged."""
    Hkv, G, D, BS = 8, 4, 128, 16
    Hq = Hkv * G
    g = torch.Generator().manual_seed(sum(ctx) + M)
    ctx = list(ctx)[:M]
    nblk = [(c + BS - 1) // BS for c in ctx]
    NB = sum(nblk) + 2
    kc = torch.randn(NB, Hkv, BS, D, generator=g).to(DEV, torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS, D, generator=g).to(DEV, torch.bfloat16)
    width = 2048 // BS
    bt = torch.zeros(M, width, dtype=torch.int32)
    p = 0
    for b in range(M):
        for j in range(nblk[b]):
            bt[b, j] = p
            p += 1
    bt = bt.to(DEV)
    cl = torch.tensor(ctx, dtype=torch.int32, device=DEV)
    q = torch.randn(M, Hq, D, generator=g).to(DEV, torch.bfloat16)
    split = 128
    ms = ops.decode_splits(width * BS, split)
    w = (torch.randn(4096, Hq * D, generator=g) * 0.02).to(DEV, torch.bfloat16)
    res = torch.randn(M, 4096, generator=g).to(DEV, torch.bfloat16)
    scale = 1.0 / D ** 0.5
    po = torch.empty(M, Hq, ms, D, device=DEV)
    pml = torch.empty(M, Hq, ms, 2, device=DEV)
    attn_ref = torch.empty(M, Hq, D, device=DEV, dtype=torch.bfloat16)
    ops.paged_decode(q, kc, vc, bt, cl, scale, ms, po.clone(), pml.clone(), out=attn_ref, split=split)
    want = res.clone()
    hip.gemv_decode(1, attn_ref.view(M, Hq * D), w, res=want)
    attn = torch.full((M, Hq, D), 7.0, device=DEV, dtype=torch.bfloat16)
    ops.paged_decode(q, kc, vc, bt, cl, scale, ms, po, pml, out=attn, split=split, reduce=False)
    got = res.clone()
    hip.gemv_decode(1, attn.view(M, Hq * D), w, res=got, po=po, pml=pml, ctx=cl, max_splits=ms, split=split,
                    Hq=Hq, D=D)
    torch.cuda.synchronize()
    _close(got, want, 0.02, 0.005, f"merged O M{M} ctx{ctx}")


def test_gemv_rejects_unsupported(hip):
    x = torch.randn(3, 4096, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
    assert not hip.gemv_supported(3, 4096, 4096, 0)
    with pytest.raises(RuntimeError):
        hip.gemv_decode(0, x, w)
    assert not hip.gemv_supported(1, 4096, 4000, 0)


def _clone_meta(meta):
    m2 = copy.copy(meta)
    for k, v in vars(meta).items():
        if isinstance(v, torch.Tensor):
            setattr(m2, k, v.clone())
    return m2


@pytest.mark.parametrize("folded", [False, True])
def test_decode_step_gemv_equals_ws(monkeypatch, folded):
    """One batch-1 decode step of a 2-layer Llama-3-8B-shaped model (real projection shapes) through
    the GEMV block (models/llama.py _forward_decode_gemv) vs the weight-streaming block, on the same
    captured step inputs: final hidden states and the K/V written to the cache agree to bf16
    rounding; the engine's greedy decode runs the GEMV block, eager and in hipGraphs, with equal
    tokens."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder
    from llm_kubernetes_minikube_sharp4dev_amd.models import llama as llama_mod

    m = build_decoder("llama-3-8b", device=DEV, num_layers=2)
    if folded:
        m.fold_norms()
    else:  # non-trivial norm weights
        for L in m.layers:
            L.input_norm.copy_((torch.rand_like(L.input_norm.float()) + 0.5).to(torch.bfloat16))
            L.post_norm.copy_((torch.rand_like(L.post_norm.float()) + 0.5).to(torch.bfloat16))
    saved = {}
    calls = []
    real_fwd = llama_mod.LlamaModel.forward
    real_gemv = llama_mod.LlamaModel._forward_decode_gemv

    def spy_fwd(self, ids, meta, kv):
        if ids.shape[0] == 1 and "ids" not in saved and meta.num_prefill_tokens == 0 and len(calls) >= 3:
            saved.update(ids=ids.clone(), meta=_clone_meta(meta), kv=[(k.clone(), v.clone()) for k, v in kv])
        return real_fwd(self, ids, meta, kv)

    def spy_gemv(self, *a, **kw):
        calls.append(a[0].shape[0])
        return real_gemv(self, *a, **kw)

    monkeypatch.setattr(llama_mod.LlamaModel, "forward", spy_fwd)
    monkeypatch.setattr(llama_mod.LlamaModel, "_forward_decode_gemv", spy_gemv)
    prompt = list(range(100, 160))
    toks = {}
    for graphs in (False, True):
        calls.clear()
        eng = LLMEngine(m, None, block_size=16, max_model_len=2048, max_num_seqs=4, eos_ids=set(), num_blocks=512,
                        use_graphs=graphs)
        toks[graphs] = eng.generate([prompt], SamplingParams.greedy(24))[0].output_ids
        assert calls, f"GEMV block not used (graphs={graphs})"
    assert toks[True] == toks[False]
    assert saved, "no decode step captured"
    outs, kvs = {}, {}
    for on in (True, False):
        monkeypatch.setattr(ops, "GEMV", on)
        kv = [(k.clone(), v.clone()) for k, v in saved["kv"]]
        outs[on] = real_fwd(m, saved["ids"].clone(), _clone_meta(saved["meta"]), kv)
        kvs[on] = kv
    monkeypatch.setattr(ops, "GEMV", True)
    monkeypatch.setattr(ops, "GEMV_L3_MB", 16)  # Infinity-Cache prefetch beside the attention: same values
    kv = [(k.clone(), v.clone()) for k, v in saved["kv"]]
    pf = real_fwd(m, saved["ids"].clone(), _clone_meta(saved["meta"]), kv)
    torch.cuda.synchronize()
    assert torch.equal(pf, outs[True])
    _close(outs[True], outs[False], 0.06, 0.02, "final hidden")
    for (k1, v1), (k2, v2) in zip(kvs[True], kvs[False]):
        _close(k1, k2, 0.05, 0.01, "k cache")
        _close(v1, v2, 0.05, 0.01, "v cache")
