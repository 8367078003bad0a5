"""End-to-end GPU paths (every op on the HIP kernel library): Llama / BERT forwards vs
HuggingFace fp32 on the CPU, hipGraph decode == eager decode, the RAG pipeline on a
GPU index, and the loud failure when the kernel library is forced off."""
import os

import pytest
import torch

transformers = pytest.importorskip("transformers")

from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder, build_encoder  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models.configs import DecoderConfig, EncoderConfig  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
PROMPTS = [[5, 17, 99, 3, 250, 7, 7, 1, 400, 33, 21, 8, 2, 9, 11, 60, 61, 62, 63], [7, 8, 9],
           list(range(10, 90)), [300, 301], list(range(200, 237))]


def _hf_llama(random_norms: bool = False):
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024,
                                   rope_theta=10000.0, rms_norm_eps=1e-5, tie_word_embeddings=False)
    torch.manual_seed(0)
    hf = transformers.LlamaForCausalLM(cfg).eval()
    if random_norms:  # HF initialises RMSNorm weights to 1: real checkpoints do not
        g = torch.Generator().manual_seed(11)
        with torch.no_grad():
            for mod in hf.modules():
                if isinstance(mod, transformers.models.llama.modeling_llama.LlamaRMSNorm):
                    mod.weight.copy_(torch.rand(mod.weight.shape, generator=g) * 1.5 + 0.25)
    ours = DecoderConfig("t", "llama", 2, 256, 4, 2, 64, 512, 512, max_position=1024, rope_theta=10000.0)
    return hf, ours


def _gpu_llama(random_norms: bool = False):
    hf, cfg = _hf_llama(random_norms)
    m = build_decoder(cfg, device=DEV, dtype=torch.bfloat16)
    m.load_hf_state_dict(hf.state_dict())
    return hf, m


def _engine(m, **kw):
    kw.setdefault("num_blocks", 256)
    return LLMEngine(m, None, block_size=16, max_model_len=512, max_num_seqs=8, eos_ids=set(), **kw)


def test_llama_gpu_logits_match_hf_fp32():
    hf, m = _gpu_llama()
    eng = _engine(m, use_graphs=False)
    for p in PROMPTS:
        eng.add_request(p, SamplingParams.greedy(1))
    eng._drain_inbox()
    batch = eng.scheduler.schedule()
    rows, lg = eng.runner.forward_logits(batch.items)
    for (seq, _), got in zip(rows, lg):
        with torch.no_grad():
            want = hf(torch.tensor([seq.prompt_ids])).logits[0, -1]
        got = got.float().cpu()
        err = (got - want).abs().max().item()
        assert err < 0.05 * want.abs().max().item() + 0.05, err
        assert torch.nn.functional.cosine_similarity(got, want, dim=0) > 0.999


def test_graph_decode_equals_eager():
    _, m = _gpu_llama()
    eager = [s.output_ids for s in _engine(m, use_graphs=False).generate(PROMPTS, SamplingParams.greedy(12))]
    eng = _engine(m, use_graphs=True)
    eng.runner.capture_all(max_batch=8)
    graphed = [s.output_ids for s in eng.generate(PROMPTS, SamplingParams.greedy(12))]
    assert graphed == eager


@pytest.mark.parametrize("graphs", [False, True])
def test_pipelined_steps_equal_synchronous(graphs):
    """step_pipelined (step N+1 enqueued before step N's ids reach the host; decode
    inputs gathered on the device, from the graph's static output buffer when graphed)
    == synchronous stepping, greedy and with a history-dependent logits processor."""
    _, m = _gpu_llama()

    def proc(hist):
        return list(range(1 + (len(hist) % 5), 512, 3))

    def drive(pipelined, mk):
        eng = _engine(m, use_graphs=graphs)
        if graphs:
            eng.runner.capture_all(max_batch=8)
        seqs = [eng.add_request(p, mk()) for p in PROMPTS[:2]]
        it = 0
        while eng.has_work() or len(seqs) < len(PROMPTS):
            if it == 3:  # staggered admission: mixed prefill + in-flight decode steps
                seqs += [eng.add_request(p, mk()) for p in PROMPTS[2:]]
            eng.step_pipelined() if pipelined else eng.step()
            it += 1
        eng.flush()
        return [s.output_ids for s in seqs]

    for mk in (lambda: SamplingParams.greedy(12), lambda: SamplingParams.greedy(12, logits_processor=proc)):
        ref = drive(False, mk)
        assert all(len(r) == 12 for r in ref)
        assert drive(True, mk) == ref


@pytest.mark.parametrize("graphs", [False, True])
def test_bf16_logits_same_tokens_as_fp32(monkeypatch, graphs):
    """Sampled-logits steps hand the LM head's bf16 output to the HIP select kernels (no fp32
    copy, extend-row logits gathered by the step_ops kernel): the same tokens as fp32 logits for
    grammar-constrained greedy rows and for temperature sampling (the conversion is exact and
    the kernels draw from the same values)."""
    _, m = _gpu_llama()

    def proc(hist):
        return list(range(1 + (len(hist) % 5), 512, 3))

    def run(lowp, mk):
        monkeypatch.setenv("LK_LOWP_LOGITS", "1" if lowp else "0")
        eng = _engine(m, use_graphs=graphs)  # decode graphs captured on first use
        assert (eng.runner.logits_dtype is None) == lowp
        return [s.output_ids for s in eng.generate(PROMPTS, mk())]

    for mk in (lambda: SamplingParams.greedy(12, logits_processor=proc),
               lambda: SamplingParams(max_tokens=12, temperature=0.8, top_k=0, top_p=1.0, repeat_penalty=1.0,
                                      seed=7),
               lambda: SamplingParams(max_tokens=12, seed=7)):  # Ollama defaults: the fused sampler
        assert run(True, mk) == run(False, mk)


def _assert_same_or_near_tie(hf, prompts, got, ref):
    """Greedy sequences from two bf16 paths that sum attention in a different order: equal,
    or first apart at a step where the fp32 model itself rates the two tokens within the
    engine's logit error (0.05 * max|logit|, test_llama_gpu_logits_match_hf_fp32) -- a tie
    the rounding may break either way, not a wrong attention result."""
    for p, g, r in zip(prompts, got, ref):
        if g == r:
            continue
        k = next(i for i, (a, b) in enumerate(zip(g, r)) if a != b)
        with torch.no_grad():
            want = hf(torch.tensor([p + r[:k]])).logits[0, -1]
        gap = abs(want[g[k]] - want[r[k]]).item()
        assert gap < 0.05 * want.abs().max().item() + 0.05, (k, g[k], r[k], gap)


def test_cascade_decode_engine_matches_plain(monkeypatch):
    """Requests sharing a long prompt prefix (prefix-cache hits on the same blocks) decode
    with the cascade path (shared blocks attended once per step) -- eager and graphed --
    to the same tokens as engines with cascade off (up to a near-tie, see
    _assert_same_or_near_tie)."""
    hf, m = _gpu_llama()
    base = list(range(40, 40 + 70))
    prompts = [base + [300 + i, 7, 9 + i] for i in range(6)]

    def run(cascade, graphs):
        monkeypatch.setenv("LK_CASCADE", "1" if cascade else "0")
        eng = _engine(m, use_graphs=graphs)
        if graphs:
            eng.runner.capture_all(max_batch=8)
        eng.generate([prompts[0]], SamplingParams.greedy(2))  # publish the shared prefix blocks
        seqs = [eng.add_request(p, SamplingParams.greedy(10)) for p in prompts]
        eng.run_until_done(seqs)
        assert cascade == eng.runner.cascade
        assert all(s.num_cached_prefix >= 64 for s in seqs)
        return [s.output_ids for s in seqs]

    ref = run(False, False)
    _assert_same_or_near_tie(hf, prompts, run(True, False), ref)
    _assert_same_or_near_tie(hf, prompts, run(True, True), ref)


@pytest.mark.parametrize("ext_as_decode", [16, 0])
def test_jump_forward_matches_step_by_step_gpu(monkeypatch, ext_as_decode):
    """Grammar jump-forward on the GPU path (hipGraph decode + pipelined steps): forced
    tokens appended by the host and run as extend chunks -- causal paged-decode rows, or a
    flash-prefill chunk -- give the step-by-step tokens (up to a near-tie: the extend's
    attention sums in another kernel) in fewer engine steps."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine import llm_engine, model_runner

    hf, m = _gpu_llama()
    monkeypatch.setattr(model_runner, "EXTEND_AS_DECODE", ext_as_decode)

    def proc(hist):  # literal runs between free choices, like the tool-call grammar
        n = len(hist)
        return [(n * 37 + 11) % 512] if n % 7 in (2, 3, 4) else list(range(1 + (n % 5), 512, 3))

    def run(jf):
        monkeypatch.setattr(llm_engine, "JUMP_FORWARD", jf)
        eng = _engine(m, use_graphs=True)
        eng.runner.capture_all(max_batch=8)
        seqs = [eng.add_request(p, SamplingParams.greedy(20, logits_processor=proc)) for p in PROMPTS]
        while eng.has_work():
            eng.step_pipelined()
        eng.flush()
        return seqs

    off, on = run(False), run(True)
    assert all(s.jumped > 0 for s in on) and all(len(s.output_ids) == 20 for s in on)
    assert sum(s.steps_run for s in on) < sum(s.steps_run for s in off)
    _assert_same_or_near_tie(hf, PROMPTS, [s.output_ids for s in on], [s.output_ids for s in off])


def test_bert_gpu_matches_hf_fp32():
    cfg = transformers.BertConfig(vocab_size=300, hidden_size=256, num_hidden_layers=2, num_attention_heads=4,
                                  intermediate_size=1024, max_position_embeddings=128, hidden_act="gelu")
    torch.manual_seed(2)
    hf = transformers.BertModel(cfg, add_pooling_layer=False).eval()
    ours = EncoderConfig("t", "bert", 2, 256, 4, 1024, 300, max_position=128, pooling="cls")
    m = build_encoder(ours, device=DEV, dtype=torch.bfloat16)
    m.load_hf_state_dict(hf.state_dict())
    seqs = [[1, 5, 9, 22, 2], [1, 7, 2], [1] + list(range(100, 160)) + [2]]
    ids = torch.tensor(sum(seqs, []), dtype=torch.int32, device=DEV)
    cu = torch.tensor([0, 5, 8, 8 + len(seqs[2])], dtype=torch.int32, device=DEV)
    pos = torch.tensor(sum([list(range(len(s))) for s in seqs], []), dtype=torch.int32, device=DEV)
    emb = m(ids, cu, pos, [len(s) for s in seqs]).float().cpu()
    for i, s in enumerate(seqs):
        with torch.no_grad():
            v = hf(torch.tensor([s])).last_hidden_state[0][0]
        v = v / v.norm()
        assert torch.nn.functional.cosine_similarity(emb[i], v, dim=0) > 0.995


def test_rag_pipeline_on_gpu_index():
    import numpy as np

    from llm_kubernetes_minikube_sharp4dev_amd.agent.rag_pipeline import ContinuousLoad, RagAgentPipeline
    from llm_kubernetes_minikube_sharp4dev_amd.config import Config
    from llm_kubernetes_minikube_sharp4dev_amd.engine.embed_engine import EmbeddingEngine
    from llm_kubernetes_minikube_sharp4dev_amd.k8s.fake import FakeCluster
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer
    from llm_kubernetes_minikube_sharp4dev_amd.rag.corpus import build_chunks
    from llm_kubernetes_minikube_sharp4dev_amd.rag.embedder import LocalEmbedder
    from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagIndex
    from llm_kubernetes_minikube_sharp4dev_amd.rag.synthetic import make_queries

    tok = builtin_tokenizer()
    enc = build_encoder("bert-tiny", device=DEV, seed=0)
    emb = EmbeddingEngine(enc, tok, name="bert-tiny")
    chunks = build_chunks(200, 0, workers=1)
    idx = RagIndex(LocalEmbedder(emb), backend="gpu", device=DEV)
    vecs = emb.embed([c[2] for c in chunks]).float().cpu().numpy()
    idx.add([c[0] for c in chunks], [c[1] for c in chunks], [c[2] for c in chunks], np.asarray(vecs))
    # GPU kNN must agree with the exact (reference-semantics) scan on the same vectors
    exact = RagIndex(idx.embedder, backend="exact")
    exact.add([c[0] for c in chunks], [c[1] for c in chunks], [c[2] for c in chunks], np.asarray(vecs))
    q = emb.embed(make_queries(4, seed=5)).float().cpu().numpy()
    g, e = idx.search_vectors(q, 6), exact.search_vectors(q, 6)
    for gr, er in zip(g, e):
        assert [i for i, _ in gr][:3] == [i for i, _ in er][:3]
    llm = build_decoder("llama-tiny", device=DEV, seed=0)
    eng = LLMEngine(llm, tok, max_model_len=4096, max_num_seqs=8, num_blocks=1024, max_num_batched_tokens=2048,
                    eos_ids=set())
    pipe = RagAgentPipeline(idx, eng, tok, FakeCluster.default(), Config())
    counter = [0]

    def nq(k):
        counter[0] += 1
        return make_queries(k, seed=counter[0])

    for deferred in (False, True):
        load = ContinuousLoad(pipe, nq, SamplingParams.greedy(6, ignore_eos=True), concurrency=6, admit_chunk=3,
                              deferred=deferred)
        out = load.run(12)
        load.drain()
        assert len(out) >= 12 and all(r.status in (200, 400, 404, 500) for r in out)
        # the kNN's device time was measured in situ (events on the side stream)
        assert all("knn_gpu_s" in r.timings for r in out if r.timings)


def test_forced_reference_fails_loudly_not_silently():
    """LK_FORCE_REFERENCE routes ops to the torch reference; the bench entry point must
    refuse to run rather than measure that fallback, and without the flag a GPU op must
    go through the HIP library (the forced path really changes the dispatch)."""
    import subprocess
    import sys

    from llm_kubernetes_minikube_sharp4dev_amd import ops

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "bench.py", "--steps", "1", "--warmup", "0", "--docs", "10"], cwd=root,
                       env=dict(os.environ, LK_FORCE_REFERENCE="1"), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "LK_FORCE_REFERENCE" in (r.stderr + r.stdout)
    x = torch.randn(4, 768, device="cuda", dtype=torch.bfloat16)
    assert ops.use_hip(x)
    os.environ["LK_FORCE_REFERENCE"] = "1"
    try:
        assert not ops.use_hip(x)
    finally:
        del os.environ["LK_FORCE_REFERENCE"]


@pytest.mark.parametrize("random_norms,gemm1w", [(False, False), (True, False), (True, True)])
def test_fused_prefill_chain_matches_hf(monkeypatch, random_norms, gemm1w):
    """A folded GPU model runs prefill-sized steps (> 256 rows) as the fused GEMM chain (RoPE +
    KV write in the QKV epilogue, norms folded into the GEMMs) -- logits vs HF fp32 -- and the
    same greedy tokens as the unfused path (LK_PREFILL_CHAIN=0), up to near-ties.  With
    non-unit RMSNorm weights (folded into the bf16 QKV / gate_up weights, as a real checkpoint's
    are) and on either prefill GEMM (gemm.hip, or gemm1w.hip forced past its tile-count gate)."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    hf, m = _gpu_llama(random_norms)
    assert m.folded and not m.rope_neox
    # the toy QKV GEMM has 4 tiles, which the default dispatch would split over K (and a split
    # QKV GEMM has no in-kernel epilogue, so the chain would not be taken)
    monkeypatch.setattr(ops, "GEMM_SPLITK", False)
    monkeypatch.setattr(ops, "GEMM1W", gemm1w)
    if gemm1w:
        monkeypatch.setattr(ops, "GEMM1W_MIN_TILES", 0)
        assert ops._gemm_default(512, 1024, 256, 1)[0] == 3
    # 512 prefill rows in one step (a multiple of the scheduler's 256-row alignment, so no chunk
    # is trimmed and every prompt's last row is in this step)
    prompts = [list(range(3 + i, 3 + i + 128)) for i in range(4)]
    calls = []
    real = m._forward_chain
    monkeypatch.setattr(m, "_forward_chain", lambda *a, **k: calls.append(1) or real(*a, **k))
    eng = _engine(m, use_graphs=False)
    for p in prompts:
        eng.add_request(p, SamplingParams.greedy(1))
    eng._drain_inbox()
    rows, lg = eng.runner.forward_logits(eng.scheduler.schedule().items)
    assert calls, "prefill chain not taken"
    for (seq, _), got in zip(rows, lg):
        with torch.no_grad():
            want = hf(torch.tensor([seq.prompt_ids])).logits[0, -1]
        got = got.float().cpu()
        assert (got - want).abs().max().item() < 0.05 * want.abs().max().item() + 0.05
        assert torch.nn.functional.cosine_similarity(got, want, dim=0) > 0.999
    fused = [s.output_ids for s in _engine(m, use_graphs=True).generate(prompts, SamplingParams.greedy(10))]
    monkeypatch.setattr(ops, "PREFILL_CHAIN", False)
    plain = [s.output_ids for s in _engine(m, use_graphs=True).generate(prompts, SamplingParams.greedy(10))]
    _assert_same_or_near_tie(hf, prompts, fused, plain)


def test_folded_norms_greedy_parity_long_decode(monkeypatch):
    """Folding the RMSNorm weights into the bf16 QKV / gate_up weights (LK_FOLD_NORMS, the GPU
    default) rounds w * g back to bf16: over 200 greedy decode steps per prompt the folded model
    emits the unfolded model's tokens, up to near-ties (checked in fp32 against HF)."""
    from llm_kubernetes_minikube_sharp4dev_amd.models import llama as llama_mod

    hf, cfg = _hf_llama(random_norms=True)
    monkeypatch.setattr(llama_mod, "FOLD_NORMS", False)
    plain_m = build_decoder(cfg, device=DEV, dtype=torch.bfloat16)
    plain_m.load_hf_state_dict(hf.state_dict())
    monkeypatch.setattr(llama_mod, "FOLD_NORMS", True)
    fold_m = build_decoder(cfg, device=DEV, dtype=torch.bfloat16)
    fold_m.load_hf_state_dict(hf.state_dict())
    assert fold_m.folded and not getattr(plain_m, "folded", False)
    prompts = [p for p in PROMPTS[:3]]
    a = [s.output_ids for s in _engine(fold_m, use_graphs=True).generate(prompts, SamplingParams.greedy(200))]
    b = [s.output_ids for s in _engine(plain_m, use_graphs=True).generate(prompts, SamplingParams.greedy(200))]
    _assert_same_or_near_tie(hf, prompts, a, b)


def test_bulk_embedding_two_streams_bit_identical(monkeypatch):
    """Index-build embedding with micro-batches alternating over two HIP streams writes exactly
    the vectors of the one-stream build (same kernels, same inputs; every stream-K / split-K
    workspace is per stream or per call)."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine import embed_engine
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer
    from llm_kubernetes_minikube_sharp4dev_amd.rag.corpus import build_chunks

    tok = builtin_tokenizer()
    enc = build_encoder("bge-base", device=DEV, seed=0)
    chunks = [c[2] for c in build_chunks(1500, 0, workers=1)][:9000]
    assert len(chunks) > 4096  # more than one tokenisation group: the bulk path engages
    outs = []
    for n in (1, 2):
        monkeypatch.setattr(embed_engine, "BUILD_STREAMS", n)
        eng = embed_engine.EmbeddingEngine(enc, tok, name="bge", max_tokens_per_batch=65536)
        outs.append(eng.embed(chunks))
        torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


def test_query_encoder_graphs_equal_eager():
    """Single-query embeddings replayed from the per-length encoder hipGraphs
    (EmbeddingEngine.capture_queries) equal the eager encoder's, f32 and bf16 rows, also from
    several threads at once (replays are serialised on the engine's graph stream)."""
    import threading

    from llm_kubernetes_minikube_sharp4dev_amd.engine.embed_engine import EmbeddingEngine
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer

    enc = build_encoder("bge-base", device=DEV, dtype=torch.bfloat16)
    tok = builtin_tokenizer()
    eager = EmbeddingEngine(enc, tok, name="e")
    graphed = EmbeddingEngine(enc, tok, name="g")
    assert graphed.capture_queries(max_len=24) == 48
    texts = ["scale the api deployment in staging", "logs of pod web-1", "x", "how do I restart the worker",
             "namespace dev replicas 3 please now quickly"]
    for t in texts:
        for dt in (torch.float32, torch.bfloat16):
            want = eager.embed([t], dtype=dt)
            got = graphed.embed([t], dtype=dt)
            assert torch.equal(got, want), (t, dt)
    res = {}

    def worker(i):
        res[i] = [graphed.embed_cpu([t]) for t in texts]

    ths = [threading.Thread(target=worker, args=(i,)) for i in range(3)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    ref = [eager.embed_cpu([t]) for t in texts]
    for i in range(3):
        assert all(torch.equal(a, b) for a, b in zip(res[i], ref)), i


def test_decode_xpro_tokens_equal(monkeypatch):
    """Batch-1 / few-row decode steps with the consumer-side GEMM prologues (O merges the
    attention splits, gate_up / QKV add + RMSNorm the previous projection's split-K slabs:
    models/llama.py _forward_decode_xpro) emit exactly the tokens of the unfused step, eager and
    in the decode hipGraphs, on a 2-layer Llama-3-8B-shaped model (the real projection shapes)."""
    from llm_kubernetes_minikube_sharp4dev_amd import ops
    from llm_kubernetes_minikube_sharp4dev_amd.models import llama as llama_mod

    m = build_decoder("llama-3-8b", device=DEV, num_layers=2)
    used = []
    real = llama_mod.LlamaModel._forward_decode_xpro

    def spy(self, *a, **kw):
        used.append(a[0].shape[0])
        return real(self, *a, **kw)

    monkeypatch.setattr(llama_mod.LlamaModel, "_forward_decode_xpro", spy)
    monkeypatch.setattr(ops, "GEMV", False)  # (steps of <= 2 rows would take the GEMV block first)
    prompts = [list(range(100, 160)), [7, 8, 9, 10, 11], list(range(1000, 1400, 3))]
    for graphs in (False, True):
        outs = {}
        for on in (True, False):
            monkeypatch.setattr(ops, "XPRO", on)
            used.clear()
            eng = LLMEngine(m, None, block_size=16, max_model_len=2048, max_num_seqs=4, eos_ids=set(), num_blocks=512,
                            use_graphs=graphs)
            outs[on] = [[s.output_ids for s in eng.generate([p], SamplingParams.greedy(40))][0] for p in prompts]
            assert bool(used) == on
        assert outs[True] == outs[False], graphs
