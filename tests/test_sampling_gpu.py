"""Fused Ollama-default sampler (csrc/sampling.hip lk_sample) vs the fp32 torch reference:
the sampled distribution, the top-k / top-p support, greedy ties, the repeat penalty read
from the device history ring, and the exact radix-select fallback on adversarial rows."""
import math

import numpy as np
import pytest
import torch

from llm_kubernetes_minikube_sharp4dev_amd import ops
from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _prm(B, temp=0.8, top_k=40, top_p=0.9, pen=1.0, last_n=64, slots=None, reset=1, seeds=None):
    prm = np.zeros((B, 8), dtype=np.int32)
    f = prm.view(np.float32)
    f[:, 0], f[:, 1], f[:, 2] = temp, top_p, pen
    prm[:, 3], prm[:, 4] = top_k, last_n
    prm[:, 5] = np.arange(B) if slots is None else slots
    prm[:, 6] = reset
    prm[:, 7] = np.arange(B) if seeds is None else seeds
    return torch.from_numpy(prm)


def _expected(row, temp, top_k, top_p):
    """fp64 probabilities of the reference chain over one logits row."""
    v, idx = torch.sort(row.double(), descending=True, stable=True)
    v, idx = v[:top_k], idx[:top_k]
    e = torch.exp((v - v[0]) / temp)
    incl = torch.cumsum(e, 0)
    keep = (incl - e) <= top_p * incl[-1]
    p = torch.zeros_like(row, dtype=torch.float64)
    p[idx[keep]] = e[keep] / e[keep].sum()
    return p


@pytest.mark.parametrize("temp,top_k,top_p", [(0.8, 40, 0.9), (1.0, 8, 1.0), (0.5, 1000, 0.5)])
def test_sampled_distribution_matches_reference(hip, temp, top_k, top_p):
    torch.manual_seed(0)
    V, B = 4096, 16384
    base = torch.randn(V) * 2.0
    logits = base.repeat(B, 1).to(DEV)
    hist = torch.zeros(B, 64, dtype=torch.int32, device=DEV)
    hl = torch.zeros(B, dtype=torch.int32, device=DEV)
    out = ops.sample(logits, _prm(B, temp, top_k, top_p).to(DEV), hist, hl, seed=123)
    counts = torch.bincount(out.long().cpu(), minlength=V).double()
    p = _expected(base, temp, top_k, top_p)
    assert counts[p == 0].sum() == 0, "token outside the top-k / top-p support"
    # per-token binomial check at 5 sigma, and total variation distance
    sigma = torch.sqrt(B * p * (1 - p)) + 1.0
    assert ((counts - B * p).abs() <= 5 * sigma).all()
    tv = 0.5 * (counts / B - p).abs().sum().item()
    assert tv < 0.03, tv
    # the ring got every row's token at position 0, length 1
    assert torch.equal(hist[:, 0].cpu(), out.cpu()) and (hl == 1).all()


def test_full_vocab_support_and_greedy_ties(hip):
    torch.manual_seed(1)
    V, B = 128256, 64
    logits = torch.randn(B, V, device=DEV) * 3
    logits[3, 100] = logits[3, 5000] = logits[3].max() + 1.0  # tie at the max: lowest index wins
    hist = torch.zeros(B, 64, dtype=torch.int32, device=DEV)
    hl = torch.zeros(B, dtype=torch.int32, device=DEV)
    greedy = ops.sample(logits.clone(), _prm(B, temp=0.0).to(DEV), hist, hl)
    exp_g = logits.float().argmax(-1).int()
    exp_g[3] = 100
    assert torch.equal(greedy.cpu(), exp_g.cpu())
    hl.zero_()
    samp = ops.sample(logits.clone(), _prm(B).to(DEV), hist, hl, seed=7).cpu()
    for r in range(B):
        p = _expected(logits[r].cpu(), 0.8, 40, 0.9)
        assert p[int(samp[r])] > 0


def test_repeat_penalty_from_device_ring(hip):
    """Step 1 picks the max; step 2 (same logits, penalty 2.0 over the ring) must not pick it
    again when the runner-up beats max / 2; the kernel appended both tokens."""
    V, B = 1000, 4
    logits = torch.full((B, V), -5.0, device=DEV)
    logits[:, 10] = 8.0
    logits[:, 20] = 5.0
    hist = torch.full((B, 64), -1, dtype=torch.int32, device=DEV)
    hl = torch.zeros(B, dtype=torch.int32, device=DEV)
    a = ops.sample(logits.clone(), _prm(B, temp=0.0, pen=2.0).to(DEV), hist, hl)
    assert (a == 10).all() and (hl == 1).all()
    b = ops.sample(logits.clone(), _prm(B, temp=0.0, pen=2.0, reset=0).to(DEV), hist, hl)
    assert (b == 20).all() and (hl == 2).all()
    assert (hist[:, :2].cpu() == torch.tensor([10, 20], dtype=torch.int32)).all()
    # a new sequence in the same slot (reset) starts with an empty window
    c = ops.sample(logits.clone(), _prm(B, temp=0.0, pen=2.0, reset=1).to(DEV), hist, hl)
    assert (c == 10).all() and (hl == 1).all()


def test_kernel_matches_reference_chain_exactly_on_greedy_penalty(hip):
    """Same parameter rows and ring through the kernel and the CPU reference: identical ids
    for greedy rows with a repeat penalty over a pre-filled ring."""
    torch.manual_seed(3)
    V, B, W = 32000, 32, 64
    logits = torch.randn(B, V) * 4
    hist = torch.randint(0, 200, (B, W), dtype=torch.int32)
    hl = torch.randint(0, 90, (B,), dtype=torch.int32)
    logits[:, :200] += 6.0  # make the penalised tokens matter
    prm = _prm(B, temp=0.0, pen=1.3, last_n=48, reset=0)
    h_ref, l_ref = hist.clone(), hl.clone()
    exp = ref.sample(logits.clone(), prm, h_ref, l_ref)
    hd, ld = hist.to(DEV), hl.to(DEV)
    got = ops.sample(logits.to(DEV), prm.to(DEV), hd, ld)
    assert torch.equal(got.cpu(), exp.cpu())
    assert torch.equal(hd.cpu(), h_ref) and torch.equal(ld.cpu(), l_ref)


def test_radix_fallback_on_plateau_rows(hip):
    """More than 4096 values tie above the per-thread-max bound: the exact radix select
    picks the top K with the lowest indices among ties (greedy and sampled)."""
    V, B = 128256, 2
    logits = torch.zeros(B, V, device=DEV)
    logits[:, 70000:] = 1.0  # 58256 tied maxima
    hist = torch.zeros(B, 64, dtype=torch.int32, device=DEV)
    hl = torch.zeros(B, dtype=torch.int32, device=DEV)
    g = ops.sample(logits.clone(), _prm(B, temp=0.0).to(DEV), hist, hl)
    assert (g == 70000).all()
    s = ops.sample(logits.clone(), _prm(B, temp=1.0, top_k=40, top_p=1.0).to(DEV), hist, hl)
    assert ((s >= 70000) & (s < 70040)).all()


def test_sampler_engine_path_uses_the_kernel(hip):
    """engine.sampling.Sampler with Ollama's default parameters lands on ops.sample and keeps
    one ring per sequence key across calls."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import Sampler, SamplingParams

    s = Sampler(1000, seed=5)
    logits = torch.randn(3, 1000, device=DEV)
    p = SamplingParams()  # temperature 0.8, top-k 40, top-p 0.9, repeat penalty 1.1
    ids1 = s(logits.clone(), [p, p, p], [[], [], []], ["a", "b", "c"])
    ids2 = s(logits.clone(), [p, p, p], [[], [], []], ["a", "b", "c"])
    assert ids1.is_cuda and ids1.dtype == torch.int32
    slots = [s._slot_of[k][0] for k in "abc"]
    assert (s._hist_len[slots] == 2).all()
    assert torch.equal(s._hist[slots, 0].cpu(), ids1.cpu()) and torch.equal(s._hist[slots, 1].cpu(), ids2.cpu())
    s.release("a")
    assert "a" not in s._slot_of
    assert math.isfinite(float(logits.sum()))


@pytest.mark.parametrize("last_n", [-1, 600])
def test_repeat_penalty_window_longer_than_256(hip, last_n):
    """repeat_last_n = -1 (Ollama: whole context) and > 256 penalise the whole generated
    history: a 1000-entry ring with every token repeated, greedy rows, kernel == reference."""
    torch.manual_seed(4)
    V, B, W = 128256, 8, 1024
    logits = torch.randn(B, V) * 2
    hist = torch.randint(0, 700, (B, W), dtype=torch.int32)
    hl = torch.full((B,), 1000, dtype=torch.int32)
    logits[:, :700] += 8.0  # the penalised ids dominate: a missed penalty changes the argmax
    prm = _prm(B, temp=0.0, pen=3.0, last_n=last_n, reset=0)
    h_ref, l_ref = hist.clone(), hl.clone()
    exp = ref.sample(logits.clone(), prm, h_ref, l_ref)
    got = ops.sample(logits.to(DEV), prm.to(DEV), hist.to(DEV), hl.to(DEV))
    assert torch.equal(got.cpu(), exp.cpu())
    # an entry 549 tokens back (outside a 256 ring) flips the choice
    only_old = torch.randint(700, 800, (B, W), dtype=torch.int32)
    only_old[:, 450] = 5
    lg = torch.full((B, V), -10.0)
    lg[:, 5] = 9.0
    lg[:, 950] = 4.0  # not in the ring (700-799): unpenalised
    got2 = ops.sample(lg.to(DEV), _prm(B, temp=0.0, pen=3.0, last_n=last_n, reset=0).to(DEV),
                      only_old.to(DEV), torch.full((B,), 1000, dtype=torch.int32, device=DEV))
    assert (got2.cpu() == 950).all()  # token 5 sits 549 entries back in the window: penalised


def test_sampler_ring_covers_max_model_len(hip):
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import Sampler, SamplingParams

    s = Sampler(1000, seed=5, history_len=4000)
    assert s.RING >= 4000
    p = SamplingParams(temperature=0.0, top_k=0, top_p=1.0, repeat_penalty=5.0, repeat_last_n=-1)
    lg = torch.zeros(1, 1000, device=DEV)
    lg[0, :600] = torch.linspace(10.0, 9.0, 600, device=DEV)
    seen = []
    for _ in range(600):  # greedy + a strong whole-history penalty walks 600 distinct ids
        seen.append(int(s(lg.clone(), [p], [[]], ["x"])[0]))
    assert len(set(seen)) == 600


def test_grammar_masked_rows_with_penalty(hip):
    """rows where a grammar mask leaves fewer finite logits than top_k (a literal
    state: 1-3 allowed ids) under Ollama's default chain sample only allowed ids (no -inf
    flood of the candidate list / radix fallback); an all -inf row yields id 0."""
    torch.manual_seed(6)
    V, B = 128256, 64
    logits = torch.full((B, V), float("-inf"), device=DEV)
    allowed = torch.randint(0, V, (B, 3), device=DEV)
    for j in range(3):
        logits[torch.arange(B, device=DEV), allowed[:, j]] = torch.randn(B, device=DEV)
    logits[B - 1] = float("-inf")
    hist = torch.randint(0, V, (B, 64), dtype=torch.int32, device=DEV)
    hl = torch.full((B,), 64, dtype=torch.int32, device=DEV)
    hist[:, 0] = allowed[:, 0].int()  # one allowed id is in the penalty window
    out = ops.sample(logits.clone(), _prm(B, temp=0.8, top_k=40, top_p=0.9, pen=1.1, reset=0).to(DEV),
                     hist, hl, seed=11)
    ok = (out[:, None].long() == allowed).any(1)
    assert ok[: B - 1].all()
    assert int(out[B - 1]) == 0
    g = ops.sample(logits.clone(), _prm(B, temp=0.0, top_k=40, pen=1.1, reset=0).to(DEV), hist, hl)
    assert ((g[: B - 1, None].long() == allowed[: B - 1]).any(1)).all() and int(g[B - 1]) == 0
