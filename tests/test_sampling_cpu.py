"""Sampler semantics on the CPU (ops.reference.sample, the oracle of csrc/sampling.hip):
Ollama's default chain, the per-sequence history ring, slot reuse and seeds."""
import numpy as np
import torch

from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import Sampler, SamplingParams
from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref


def _support(row, temp, top_k, top_p):
    v, idx = torch.sort(row.double(), descending=True, stable=True)
    v, idx = v[:top_k], idx[:top_k]
    e = torch.exp((v - v[0]) / temp)
    incl = torch.cumsum(e, 0)
    return set(idx[(incl - e) <= top_p * incl[-1]].tolist())


def test_default_params_are_ollamas():
    p = SamplingParams()
    assert (p.temperature, p.top_k, p.top_p, p.repeat_penalty, p.repeat_last_n) == (0.8, 40, 0.9, 1.1, 64)
    assert SamplingParams.from_ollama(None).top_k == 40


def test_sampler_support_ring_and_release():
    torch.manual_seed(0)
    s = Sampler(500, seed=1)
    base = torch.randn(500) * 3
    p = SamplingParams()
    keys = ["x", "y"]
    for step in range(5):
        logits = base.repeat(2, 1).clone()
        ids = s(logits, [p, p], [[], []], keys)
        for t in ids.tolist():
            assert t in _support(base, 0.8, 40, 0.9) or step > 0  # later steps: penalised row
    slots = [s._slot_of[k][0] for k in keys]
    assert s._hist_len[slots].tolist() == [5, 5]
    s.release("x")
    assert "x" not in s._slot_of and slots[0] in s._free


def test_repeat_penalty_counts_generated_tokens_once():
    """Duplicates in the window are penalised once (llama.cpp / Ollama semantics)."""
    V = 10
    logits = torch.zeros(1, V)
    logits[0, 3] = 4.0
    hist = torch.tensor([[3, 3, 3, 3] + [0] * 60], dtype=torch.int32)
    hl = torch.tensor([4], dtype=torch.int32)
    prm = np.zeros((1, 8), dtype=np.int32)
    f = prm.view(np.float32)
    f[0, 0], f[0, 1], f[0, 2] = 0.0, 1.0, 2.0
    prm[0, 3:8] = [0, 64, 0, 0, 0]
    ref.sample(logits, torch.from_numpy(prm), hist, hl)
    assert float(logits[0, 3]) == 2.0  # 4 / 2 once, not 4 / 16


def test_seeded_requests_are_reproducible():
    base = torch.randn(1, 300) * 2
    outs = []
    for _ in range(2):
        s = Sampler(300, seed=9)
        p = SamplingParams(seed=42)
        outs.append([int(s(base.clone(), [p], [[]], ["r"])[0]) for _ in range(4)])
    assert outs[0] == outs[1]


def test_whole_history_window_is_not_clamped_to_256():
    """repeat_last_n = -1 / > 256: the engine sizes the ring to max_model_len, so a token
    generated 500 steps back is still penalised (it used to be capped at 256)."""
    s = Sampler(50, seed=0, history_len=2048)
    assert s.RING == 2048
    p = SamplingParams(temperature=0.0, top_k=0, top_p=1.0, repeat_penalty=4.0, repeat_last_n=-1)
    lg = torch.zeros(1, 50)
    lg[0, 7] = 3.0
    lg[0, 9] = 1.0
    assert int(s(lg.clone(), [p], [[]], ["k"])[0]) == 7
    flat = torch.zeros(1, 50)
    flat[0, 11] = 0.5
    for _ in range(500):  # 500 more tokens, none of them 7
        assert int(s(flat.clone(), [p], [[]], ["k"])[0]) != 7
    # token 7 is 500 entries back: 3.0 / 4 = 0.75 < 1.0, so 9 wins
    assert int(s(lg.clone(), [p], [[]], ["k"])[0]) == 9
