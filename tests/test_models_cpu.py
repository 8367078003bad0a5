"""Model parity vs HuggingFace transformers (same random weights, fp32, CPU) and
engine consistency (paged KV, chunked prefill, prefix caching, preemption)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder, build_encoder
from llm_kubernetes_minikube_sharp4dev_amd.models.configs import DecoderConfig, EncoderConfig


def _hf_llama():
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024,
                                   rope_theta=10000.0, rms_norm_eps=1e-5, tie_word_embeddings=False)
    torch.manual_seed(0)
    m = transformers.LlamaForCausalLM(cfg).eval()
    ours = DecoderConfig("t", "llama", 2, 128, 4, 2, 32, 256, 512, max_position=1024, rope_theta=10000.0)
    return m, ours


def _engine(model, **kw):
    kw.setdefault("num_blocks", 128)
    kw.setdefault("eos_ids", set())
    return LLMEngine(model, None, block_size=16, max_model_len=512, max_num_seqs=8, **kw)


def test_llama_matches_hf():
    hf, cfg = _hf_llama()
    m = build_decoder(cfg, dtype=torch.float32)
    m.load_hf_state_dict(hf.state_dict())
    prompt = [5, 17, 99, 3, 250, 7, 7, 1, 400, 33, 21, 8, 2, 9, 11, 60, 61, 62, 63]
    with torch.no_grad():
        ref = hf.generate(torch.tensor([prompt]), max_new_tokens=12, do_sample=False)[0, len(prompt):].tolist()
        hf_logits = hf(torch.tensor([prompt])).logits[0, -1]
    eng = _engine(m)
    seq = eng.generate([prompt], SamplingParams.greedy(12))[0]
    assert seq.output_ids == ref
    # logits of the first step
    eng2 = _engine(m)
    s2 = eng2.add_request(prompt, SamplingParams.greedy(1))
    eng2._drain_inbox()
    batch = eng2.scheduler.schedule()
    rows, lg = eng2.runner.forward_logits(batch.items)
    assert torch.allclose(lg[0], hf_logits, atol=1e-4, rtol=1e-4)


def test_opt_matches_hf():
    cfg = transformers.OPTConfig(vocab_size=512, hidden_size=64, ffn_dim=128, num_hidden_layers=2,
                                 num_attention_heads=2, max_position_embeddings=256, word_embed_proj_dim=64,
                                 do_layer_norm_before=True, enable_bias=True)
    torch.manual_seed(1)
    hf = transformers.OPTForCausalLM(cfg).eval()
    ours = DecoderConfig("t", "opt", 2, 64, 2, 2, 32, 128, 512, max_position=256, tie_word_embeddings=True,
                         activation="relu", bias=True)
    m = build_decoder(ours, dtype=torch.float32)
    m.load_hf_state_dict(hf.state_dict())
    prompt = [2, 45, 100, 7, 8, 300, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22]
    with torch.no_grad():
        ref = hf.generate(torch.tensor([prompt]), max_new_tokens=10, do_sample=False)[0, len(prompt):].tolist()
    seq = _engine(m).generate([prompt], SamplingParams.greedy(10))[0]
    assert seq.output_ids == ref


@pytest.mark.parametrize("pooling", ["cls", "mean"])
def test_bert_matches_hf(pooling):
    cfg = transformers.BertConfig(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=2,
                                  intermediate_size=128, max_position_embeddings=128, hidden_act="gelu")
    torch.manual_seed(2)
    hf = transformers.BertModel(cfg, add_pooling_layer=False).eval()
    ours = EncoderConfig("t", "bert", 2, 64, 2, 128, 300, max_position=128, pooling=pooling)
    m = build_encoder(ours, dtype=torch.float32)
    m.load_hf_state_dict(hf.state_dict())
    seqs = [[1, 5, 9, 22, 2], [1, 7, 2], [1, 100, 101, 102, 103, 104, 105, 2]]
    ids = torch.tensor(sum(seqs, []), dtype=torch.int32)
    cu = torch.tensor([0, 5, 8, 16], dtype=torch.int32)
    pos = torch.tensor(sum([list(range(len(s))) for s in seqs], []), dtype=torch.int32)
    emb = m(ids, cu, pos, [len(s) for s in seqs])
    for i, s in enumerate(seqs):
        with torch.no_grad():
            h = hf(torch.tensor([s])).last_hidden_state[0]
        v = h[0] if pooling == "cls" else h.mean(0)
        v = v / v.norm()
        assert torch.allclose(emb[i], v, atol=1e-4), (i, (emb[i] - v).abs().max())


def test_chunked_prefill_prefix_cache_and_preemption_consistent():
    m = build_decoder("llama-tiny", dtype=torch.float32)
    prompts = [list(range(3, 3 + n)) for n in (70, 33, 5, 100)]
    ref = [s.output_ids for s in _engine(m).generate(prompts, SamplingParams.greedy(10))]
    # tiny token budget -> chunked prefill interleaved with decode
    chunked = _engine(m, max_num_batched_tokens=24)
    assert [s.output_ids for s in chunked.generate(prompts, SamplingParams.greedy(10))] == ref
    # prefix cache: a second request sharing 64 tokens reuses 4 blocks
    eng = _engine(m)
    eng.generate([prompts[0]], SamplingParams.greedy(10))
    s = eng.generate([prompts[0][:64] + [7, 8, 9]], SamplingParams.greedy(4))[0]
    assert s.num_cached_prefix == 64
    fresh = _engine(m, max_num_batched_tokens=4096).generate([prompts[0][:64] + [7, 8, 9]],
                                                              SamplingParams.greedy(4))[0]
    assert s.output_ids == fresh.output_ids
    # KV pool too small for all sequences at once -> preemption + recompute, same answers
    ref30 = [s.output_ids for s in _engine(m).generate(prompts, SamplingParams.greedy(30))]
    small = _engine(m, num_blocks=10)
    out = small.generate(prompts, SamplingParams.greedy(30))
    assert [x.output_ids for x in out] == ref30
    assert sum(x.num_preemptions for x in out) > 0


def test_unified_mixed_attention_matches_split(monkeypatch):
    """LK_UNIFIED_ATTN: a mixed step's decode rows join the prompt chunks as one-token sequences
    of ONE flash-attention call (combined cu / ctx / block tables built by ModelRunner._meta);
    tokens equal the split path (flash for the chunks + paged decode for the rows), with
    chunked prefill interleaved with decode and jump-forward-free greedy decoding."""
    from llm_kubernetes_minikube_sharp4dev_amd.models import attention

    m = build_decoder("llama-tiny", dtype=torch.float32)
    prompts = [list(range(3, 3 + n)) for n in (70, 33, 5, 100, 17)]
    ref = [s.output_ids for s in _engine(m, max_num_batched_tokens=24).generate(prompts, SamplingParams.greedy(12))]
    seen = []
    real = attention.ops.flash_prefill

    def spy(q, *a, **kw):
        seen.append(q.shape[0])
        return real(q, *a, **kw)

    monkeypatch.setattr(attention, "UNIFIED_ATTN", True)
    monkeypatch.setattr(attention.ops, "flash_prefill", spy)
    eng = _engine(m, max_num_batched_tokens=24)
    out = [s.output_ids for s in eng.generate(prompts, SamplingParams.greedy(12))]
    assert out == ref
    # some steps were mixed and ran as one launch covering prompt and decode rows
    assert getattr(eng.runner, "unified_attn_steps", 0) > 0 and seen and max(seen) <= 24


def _run_pipelined(eng, prompts, params_fn, stagger: int = 0):
    """Drive eng with step_pipelined (requests i >= 2 admitted `stagger` iterations apart)."""
    seqs, pending, it = [], list(enumerate(prompts)), 0
    while pending or eng.has_work():
        while pending and (not stagger or it >= stagger * pending[0][0] or pending[0][0] < 2):
            i, p = pending.pop(0)
            seqs.append((i, eng.add_request(p, params_fn())))
        if eng.has_work():
            eng.step_pipelined()
        else:
            eng.flush()
        it += 1
    eng.flush()
    return [s.output_ids for _, s in sorted(seqs, key=lambda x: x[0])]


def test_pipelined_steps_match_synchronous():
    """step_pipelined (step N+1 launched before step N's ids reach the host, decode
    inputs gathered on the device) gives exactly the synchronous engine's tokens:
    chunked prefill, staggered admission, EOS stops mid-flight, a history-dependent
    logits processor, and preemption under a tiny KV pool."""
    m = build_decoder("llama-tiny", dtype=torch.float32)
    prompts = [list(range(3, 3 + n)) for n in (70, 33, 5, 100, 17)]

    def proc(hist):  # history-dependent constraint (like the tool-call grammar)
        return list(range(1 + (len(hist) % 5), m.cfg.vocab_size, 3))

    cases = [
        (lambda: SamplingParams.greedy(12), {}),
        (lambda: SamplingParams.greedy(12, logits_processor=proc), {"max_num_batched_tokens": 24}),
        (lambda: SamplingParams.greedy(30), {"num_blocks": 10}),
    ]
    for params_fn, kw in cases:
        ref = [s.output_ids for s in _engine(m, **kw).generate(prompts, params_fn())]
        assert _run_pipelined(_engine(m, **kw), prompts, params_fn) == ref
        assert _run_pipelined(_engine(m, **kw), prompts, params_fn, stagger=3) == ref
    # EOS stop: pick a token the reference emits mid-sequence
    base = [s.output_ids for s in _engine(m).generate(prompts, SamplingParams.greedy(12))]
    eos = base[0][4]
    ref = [s.output_ids for s in _engine(m, eos_ids={eos}).generate(prompts, SamplingParams.greedy(12))]
    assert any(len(r) < 12 for r in ref)
    eng = LLMEngine(m, None, block_size=16, max_model_len=512, max_num_seqs=8, eos_ids={eos}, num_blocks=128)
    assert _run_pipelined(eng, prompts, lambda: SamplingParams.greedy(12)) == ref
    assert eng.allocator.usage() == 0.0 or not eng.scheduler.running


@pytest.mark.parametrize("ext_as_decode", [16, 0])
def test_jump_forward_matches_step_by_step(monkeypatch, ext_as_decode):
    """Grammar jump-forward (tokens with a one-id mask appended by the host and run as an
    extend chunk -- as causal decode rows, or as a prefill chunk) gives exactly the
    step-by-step tokens, synchronous and pipelined, under chunked prefill and preemption,
    with fewer engine steps per request; the last token of every request is still sampled."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine import llm_engine, model_runner

    monkeypatch.setattr(model_runner, "EXTEND_AS_DECODE", ext_as_decode)

    m = build_decoder("llama-tiny", dtype=torch.float32)
    V = m.cfg.vocab_size
    prompts = [list(range(3, 3 + n)) for n in (70, 33, 5, 100, 17)]

    def proc(hist):  # runs of forced tokens (a literal) between free choices
        n = len(hist)
        if n % 7 in (2, 3, 4) or (n % 11 == 5):
            return [(n * 37 + 11) % V]
        return list(range(1 + (n % 5), V, 3))

    cases = [
        (lambda: SamplingParams.greedy(20, logits_processor=proc), {}),
        (lambda: SamplingParams.greedy(20, logits_processor=proc), {"max_num_batched_tokens": 24}),
        (lambda: SamplingParams.greedy(30, logits_processor=proc), {"num_blocks": 10}),
    ]
    for params_fn, kw in cases:
        monkeypatch.setattr(llm_engine, "JUMP_FORWARD", False)
        off = _engine(m, **kw).generate(prompts, params_fn())
        ref = [s.output_ids for s in off]
        assert all(s.jumped == 0 for s in off)
        monkeypatch.setattr(llm_engine, "JUMP_FORWARD", True)
        on = _engine(m, **kw).generate(prompts, params_fn())
        assert [s.output_ids for s in on] == ref
        assert all(s.jumped > 0 for s in on)
        assert sum(s.steps_run for s in on) < sum(s.steps_run for s in off)
        assert _run_pipelined(_engine(m, **kw), prompts, params_fn) == ref
        assert _run_pipelined(_engine(m, **kw), prompts, params_fn, stagger=3) == ref
    # a forced final token is not appended by the host: with every token forced the request
    # still takes its last token from the sampler (no forward pass of the step-by-step run skipped)
    eng = _engine(m)
    s = eng.generate([prompts[2]], SamplingParams.greedy(6, logits_processor=lambda h: [9]))[0]
    assert s.output_ids == [9] * 6 and s.jumped == 4  # first sampled, 4 jumped, last sampled
    assert eng.allocator.usage() == 0.0 or not eng.scheduler.running


def test_prefill_hold_back_same_tokens_fuller_steps(monkeypatch):
    """Prefill hold-back (LK_PREFILL_HOLD): with enough decode rows running, new prompts wait
    until they fill the step's token budget (or the hold limit expires): same greedy tokens
    as the eager scheduler, and every step that carries prefill is full unless the hold
    expired or nothing else was running."""
    m = build_decoder("llama-tiny", dtype=torch.float32)
    monkeypatch.setenv("LK_HOLD_MIN_DECODE", "2")
    prompts = [list(range(3, 3 + n)) for n in (40, 33, 25, 30, 17, 22, 35, 28)]

    def run(hold):
        eng = _engine(m, max_num_batched_tokens=64, prefill_hold=hold, token_align=0)
        eng.step_trace = []
        seqs = [eng.add_request(p, SamplingParams.greedy(12)) for p in prompts[:3]]
        it = 0
        while eng.has_work() or len(seqs) < len(prompts):
            if it % 3 == 2 and len(seqs) < len(prompts):  # arrivals while others decode
                seqs.append(eng.add_request(prompts[len(seqs)], SamplingParams.greedy(12)))
            eng.step()
            it += 1
        return [s.output_ids for s in seqs], eng.step_trace

    ref, tr0 = run(0)
    got, tr1 = run(4)
    assert got == ref
    part0 = sum(1 for t in tr0 if 0 < t[0] and t[0] + t[1] < 64)
    part1 = sum(1 for t in tr1 if 0 < t[0] and t[0] + t[1] < 64)
    assert part1 < part0, (part0, part1)


def test_prefill_hold_small_fill_same_tokens(monkeypatch):
    """LK_HOLD_SMALL: a held step still takes prompt tokens up to hold_small rows in total -- same
    greedy tokens as the eager scheduler, no held step past hold_small rows, and prompt tokens do
    ride in steps the plain hold-back leaves decode-only."""
    m = build_decoder("llama-tiny", dtype=torch.float32)
    monkeypatch.setenv("LK_HOLD_MIN_DECODE", "2")
    prompts = [list(range(3, 3 + n)) for n in (40, 33, 25, 30, 17, 22, 35, 28)]

    def run(hold, small):
        monkeypatch.setenv("LK_HOLD_SMALL", str(small))
        eng = _engine(m, max_num_batched_tokens=64, prefill_hold=hold, token_align=0)
        eng.step_trace = []
        seqs = [eng.add_request(p, SamplingParams.greedy(12)) for p in prompts[:3]]
        it, held_sizes = 0, []
        while eng.has_work() or len(seqs) < len(prompts):
            if it % 3 == 2 and len(seqs) < len(prompts):
                seqs.append(eng.add_request(prompts[len(seqs)], SamplingParams.greedy(12)))
            held_before = eng.scheduler._held
            eng.step()
            if eng.scheduler._held > held_before:  # this step held prefill back
                held_sizes.append(eng.step_trace[-1][0] + eng.step_trace[-1][1])
            it += 1
        return [s.output_ids for s in seqs], eng.step_trace, held_sizes

    ref, _, _ = run(0, 0)
    got0, tr0, held0 = run(4, 0)
    got1, tr1, held1 = run(4, 8)
    assert got0 == ref and got1 == ref
    assert held1 and max(held1) <= 8, held1
    small0 = sum(t[0] for t in tr0 if t[0] + t[1] <= 8)
    small1 = sum(t[0] for t in tr1 if t[0] + t[1] <= 8)
    assert small1 > small0, (small0, small1)


def test_small_step_bucket_alignment_same_tokens(monkeypatch):
    """LK_SMALL_STEP_ALIGN: a weight-streaming step (<= the largest bucket in rows) with decode
    rows trims prompt prefill to the row bucket its decode rows need (the trimmed tokens lead the
    next step): same greedy tokens as without it, and no step mixes decode rows with prefill
    past that bucket."""
    m = build_decoder("llama-tiny", dtype=torch.float32)
    prompts = [list(range(3, 3 + n)) for n in (40, 33, 25, 30, 17, 22, 35, 28)]

    def run(buckets):
        monkeypatch.setenv("LK_SMALL_STEP_ALIGN", buckets)
        eng = _engine(m, max_num_batched_tokens=64, token_align=0)
        eng.step_trace = []
        seqs = [eng.add_request(p, SamplingParams.greedy(12)) for p in prompts[:3]]
        it = 0
        while eng.has_work() or len(seqs) < len(prompts):
            if it % 3 == 2 and len(seqs) < len(prompts):
                seqs.append(eng.add_request(prompts[len(seqs)], SamplingParams.greedy(12)))
            eng.step()
            it += 1
        return [s.output_ids for s in seqs], eng.step_trace

    ref, _ = run("0")
    got, tr = run("4,8,16")
    assert got == ref
    trimmed = 0
    for npre, ndec, *_ in tr:  # (prefill tokens, decode rows, ...)
        if npre and ndec and npre + ndec <= 16:  # a step the alignment applies to
            cap = next(b for b in (4, 8, 16) if b >= ndec)
            assert npre + ndec <= cap, (npre, ndec)
            trimmed += npre + ndec == cap
    assert trimmed  # the policy engaged


def test_fused_decode_ops_cpu_fallback():
    """ops.linear_add_rmsnorm / ops.linear_rope_kv on CPU tensors are the unfused
    reference ops (the HIP fusions only exist for split-K decode shapes on the GPU)."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    torch.manual_seed(0)
    x, w = torch.randn(5, 64), torch.randn(32, 64) * 0.1
    g, res = torch.rand(32) + 0.5, torch.randn(5, 32)
    r1, r2 = res.clone(), res.clone()
    y = ops.linear_add_rmsnorm(x, w, r1, g, 1e-5)
    y2 = ops.rmsnorm(ops.linear(x, w), g, 1e-5, residual=r2)
    assert torch.equal(y, y2) and torch.equal(r1, r2)

    Hq, Hkv, D, BS, NB = 4, 2, 16, 4, 8
    wq = torch.randn((Hq + 2 * Hkv) * D, 64) * 0.1
    pos = torch.arange(5, dtype=torch.int32)
    cs = ops.rope_cos_sin(64, D, 10000.0)
    kc, vc = torch.zeros(NB, Hkv, BS, D), torch.zeros(NB, Hkv, BS, D)
    kc2, vc2 = kc.clone(), vc.clone()
    slots = torch.tensor([0, 1, 2, 5, 9], dtype=torch.int32)
    q1 = ops.linear_rope_kv(x, wq, pos, cs, Hq, Hkv, D, kc, vc, slots)
    q2 = ops.linear(x, wq)
    ops.rope_kv_(q2, pos, cs, Hq, Hkv, D, kc2, vc2, slots)
    assert torch.equal(q1, q2) and torch.equal(kc, kc2) and torch.equal(vc, vc2)


def test_gemm_split_k_policy():
    """Prefill-GEMM dispatch (pure host logic): split-K only where the 256-row tile grid covers
    at most half of the 256 CUs, never for SwiGLU, at most 4 splits of >= 8 K-tiles each
    (profiles/r2_gemm_splitk.md)."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    assert ops._gemm_default(1024, 4096, 4096, 0) == (ops._gemm_sched(4096), 256, 4)
    if ops.GEMM_SCHED is None:  # default schedule policy: static-priority 4-phase for the decoder's K
        assert ops._gemm_sched(4096) == 2 and ops._gemm_sched(14336) == 2 and ops._gemm_sched(768) == 0
    assert ops._gemm_default(2048, 4096, 14336, 0)[2] == 2
    assert ops._gemm_default(1024, 6144, 4096, 0)[1:] == (192, 2)
    assert ops._gemm_default(4096, 1280, 8192, 0)[2] == 3
    assert ops._gemm_default(8192, 4096, 4096, 0)[2] == 1
    assert ops._gemm_default(2560, 4096, 4096, 2)[2] == 1
    assert ops._gemm_default(2560, 4096, 14336, 0)[2] == 3  # 160 tiles, long K
    assert ops._gemm_default(2816, 4096, 14336, 0)[2] == 1  # 176 tiles
    assert ops._gemm_default(512, 28672, 4096, 1)[2] == 1  # SwiGLU: single pass
    assert ops._gemm_default(256, 768, 768, 2)[2] == 1  # 12 K-tiles: < 8 per split at S 2


def test_gemm1w_default_policy(monkeypatch):
    """Fallback policy (shapes without a measured entry): 256-wide prefill tiles go to the
    one-wave-per-SIMD kernel (variant 3, csrc/gemm1w.hip) once they fill a wave of 256 CUs, its
    192-row tiles (variant 4) where 256-row tiles would leave over a third of one wave idle; QKV
    at M 4096 keeps gemm.hip's 192-wide tiles (2 whole waves), split-K shapes stay on gemm.hip;
    LK_GEMM1W=0 turns it off."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    monkeypatch.setattr(ops, "GEMM1W", True)
    assert ops._gemm_default(4096, 4096, 4096, 0) == (3, 256, 1)      # O
    assert ops._gemm_default(4096, 4096, 14336, 6) == (3, 256, 1)     # down, RESID
    assert ops._gemm_default(4096, 28672, 4096, 1) == (3, 256, 1)     # gate_up + SwiGLU
    assert ops._gemm_default(4096, 6144, 4096, 7)[:2] == (ops._gemm_sched(4096), 192)  # QKV: 2 whole waves
    assert ops._gemm_default(8192, 6144, 4096, 0) == (3, 256, 1)      # tie on waves -> 256
    assert ops._gemm_default(2664, 4096, 4096, 0) == (4, 256, 1)      # 176 tiles -> 224 of 192 rows
    assert ops._gemm_default(1024, 4096, 4096, 0)[0] not in ops.GEMM1W_BM  # 64 tiles: split-K on gemm.hip
    assert {(3, 256), (4, 256), (5, 256)} <= set(ops._gemm_configs(4096, 0))
    assert (3, 256) in ops._gemm_configs(28672, 1)
    assert all(c[0] not in ops.GEMM1W_BM for c in ops._gemm_configs(1152, 0))  # no 256-wide tile
    monkeypatch.setattr(ops, "GEMM1W", False)
    assert ops._gemm_default(4096, 4096, 4096, 0)[0] == ops._gemm_sched(4096)
    assert all(c[0] not in ops.GEMM1W_BM for c in ops._gemm_configs(4096, 0))


def test_static_gemm_table_is_well_formed(monkeypatch):
    """The shipped measured dispatch table (benchmarks/gemm_table.py on an MI355X): every entry a
    kernel / tile / split the dispatch knows, looked up by _cfg_of before the fallback policy,
    and ignored under LK_GEMM1W=0 where it names a gemm1w variant."""
    import json
    import os

    from llm_kubernetes_minikube_sharp4dev_amd import ops

    if not os.path.exists(ops.GEMM_TABLE_FILE):
        pytest.skip("no measured table shipped")
    doc = json.load(open(ops.GEMM_TABLE_FILE))
    assert doc["arch"] == "gfx950" and doc["entries"]
    for mb, n, k, epi, v, bn, ks in doc["entries"]:
        assert v in (0, 1, 2, 3, 4, 5, 6, 7) and bn in (192, 256) and 1 <= ks <= 4 and epi in (0, 1, 2, 3, 4)
        assert bn == 256 or v not in ops.GEMM1W_BM
        assert ks == 1 or v not in ops.GEMM1W_BM
        assert k % 64 == 0 and n % bn == 0
    mb, n, k, epi, v, bn, ks = doc["entries"][0]
    monkeypatch.setattr(ops, "_GEMM_TABLE", {})
    monkeypatch.setattr(ops, "GEMM1W", True)
    assert ops._cfg_of(mb * 256, n, k, epi) == (v, bn, ks)
    monkeypatch.setattr(ops, "GEMM1W", False)
    assert ops._cfg_of(mb * 256, n, k, epi)[0] not in ops.GEMM1W_BM


def test_lib_path_ab_knob_loads_the_named_build():
    """LK_LIB_PATH (same-box A/B of two builds of the kernel library) loads the extension from
    the given file instead of the in-tree one."""
    import glob
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    so = glob.glob(os.path.join(root, "llm_kubernetes_minikube_sharp4dev_amd", "_C.*.so"))
    if not so:
        pytest.skip("kernel library not built")
    code = ("from llm_kubernetes_minikube_sharp4dev_amd.ops import _ext; m = _ext.try_lib(); "
            "print(m.__file__ if m is not None else 'ERR ' + repr(_ext._err))")
    env = {**os.environ, "LK_LIB_PATH": so[0]}
    out = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True,
                         timeout=300).stdout.strip().splitlines()[-1]
    assert out == so[0], out


def _first_step_logits(m, prompts):
    eng = _engine(m)
    for p in prompts:
        eng.add_request(p, SamplingParams.greedy(1))
    eng._drain_inbox()
    rows, lg = eng.runner.forward_logits(eng.scheduler.schedule().items)
    return lg


def test_folded_norms_and_fused_chain_match_hf(monkeypatch):
    """fold_norms (norm weights into qkv / gate_up, q / k rows to adjacent RoPE pairs) is the same
    model, and the fused prefill chain (_forward_chain: scale-in-epilogue GEMMs, RESID partial
    sums of squares, RoPE + KV write in the QKV epilogue) computes the same logits and greedy
    tokens as HF -- fp32 reference ops on the CPU (the GPU test runs the HIP epilogues)."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    hcfg = transformers.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                    num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024,
                                    rope_theta=10000.0, rms_norm_eps=1e-5, tie_word_embeddings=False)
    torch.manual_seed(0)
    hf = transformers.LlamaForCausalLM(hcfg).eval()
    cfg = DecoderConfig("t", "llama", 2, 256, 4, 2, 64, 512, 512, max_position=1024, rope_theta=10000.0)
    sd = hf.state_dict()
    for k in list(sd):  # non-trivial norm weights, so the fold is exercised
        if k.endswith("norm.weight"):
            sd[k] = 1 + 0.1 * torch.randn_like(sd[k])
    hf.load_state_dict(sd)
    prompts = [[5, 17, 99, 3, 250, 7, 7, 1, 400, 33, 21, 8, 2, 9, 11, 60, 61, 62, 63], list(range(30, 70))]
    m = build_decoder(cfg, dtype=torch.float32)
    m.load_hf_state_dict(sd)
    assert not m.folded  # CPU: checkpoint layout
    with torch.no_grad():
        want = torch.stack([hf(torch.tensor([p])).logits[0, -1] for p in prompts])
    plain = _first_step_logits(m, prompts)
    m.fold_norms()
    assert m.folded and not m.rope_neox and torch.all(m.layers[0].input_norm == 1)
    folded = _first_step_logits(m, prompts)
    calls = []
    real = m._forward_chain

    def spy(*a, **k):
        calls.append(1)
        return real(*a, **k)

    monkeypatch.setattr(ops, "prefill_chain_ok", lambda *a: True)
    monkeypatch.setattr(m, "_forward_chain", spy)
    chained = _first_step_logits(m, prompts)
    assert calls, "the fused chain did not run"
    for got in (plain, folded, chained):
        assert torch.allclose(got, want, atol=2e-4, rtol=2e-4), (got - want).abs().max()
    seqs = _engine(m).generate(prompts, SamplingParams.greedy(8))
    with torch.no_grad():
        for p, s in zip(prompts, seqs):
            ref = hf.generate(torch.tensor([p]), max_new_tokens=8, do_sample=False)[0, len(p):].tolist()
            assert s.output_ids == ref


def test_fused_chain_reference_ops():
    """The CPU oracles of the fused epilogues: RESID partial sums of squares per 256 columns and
    the consumer's row scale reproduce RMSNorm; the QKV oracle is GEMM -> interleaved rope_kv_."""
    from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as R

    torch.manual_seed(1)
    M, H = 37, 512
    r = torch.randn(M, H)
    x = torch.randn(M, 256)
    w = torch.randn(H, 256) * 0.05
    ss = torch.zeros(H // 256, 64)
    r2 = r.clone()
    R.linear_resid(x, w, r2, ss)
    assert torch.allclose(r2, r + x @ w.t(), atol=1e-5)
    s = R.row_scale(ss, H, 1e-5)[:M]
    assert torch.allclose(s, torch.rsqrt(r2.pow(2).mean(-1) + 1e-5), rtol=1e-5)
    wg = torch.randn(64, H) * 0.05
    y = R.gemm_scaled(r2, wg, ss, H, 1e-5)
    normed = r2 * torch.rsqrt(r2.pow(2).mean(-1, keepdim=True) + 1e-5)
    assert torch.allclose(y, normed @ wg.t(), atol=1e-4)


def test_gemm1w_column_split_plan():
    """Variants 6 / 7 split the column tiles: whole waves of 256-row tiles first (mirrors
    lk_gemm1w_split_cols in csrc/gemm1w.hip)."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    assert ops.gemm1w_split_cols(4096, 6144, 0) == 16  # 16 x 24 = 1.5 waves -> 16 x 16, then 8 columns
    assert ops._split_applies(4096, 6144, 0)
    assert not ops._split_applies(4096, 4096, 0)  # 16 x 16: exactly one wave
    assert not ops._split_applies(8192, 6144, 0)  # 32 x 24: three waves
    assert not ops._split_applies(1024, 4096, 0)  # under a wave: nothing to split
    assert ops.gemm1w_split_cols(600, 28672, 1) == 85  # SwiGLU: 3 x 112 tiles
