"""Multi-process (gloo, world_size 2) tests of the distributed paths: tensor-parallel
Llama/OPT generation == single process, sharded kNN == unsharded, TP engine driver /
worker lockstep, DP router over two replicas."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

transformers = pytest.importorskip("transformers")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _hf_llama(seed=0):
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=1024,
                                   rope_theta=10000.0, tie_word_embeddings=False)
    torch.manual_seed(seed)
    return transformers.LlamaForCausalLM(cfg).eval()


def _ours_cfg(arch):
    from llm_kubernetes_minikube_sharp4dev_amd.models.configs import DecoderConfig

    if arch == "llama":
        return DecoderConfig("t", "llama", 2, 128, 4, 2, 32, 256, 512, max_position=1024, rope_theta=10000.0)
    return DecoderConfig("t", "opt", 2, 64, 2, 2, 32, 128, 512, max_position=256, tie_word_embeddings=True,
                         activation="relu", bias=True)


def _hf(arch):
    if arch == "llama":
        return _hf_llama()
    cfg = transformers.OPTConfig(vocab_size=512, hidden_size=64, ffn_dim=128, num_hidden_layers=2,
                                 num_attention_heads=2, max_position_embeddings=256, word_embed_proj_dim=64)
    torch.manual_seed(1)
    return transformers.OPTForCausalLM(cfg).eval()


PROMPTS = [[5, 17, 99, 3, 250, 7, 7, 1, 400, 33, 21, 8, 2, 9, 11, 60, 61, 62, 63], [7, 8, 9], list(range(10, 60))]


def _proc(hist):  # history-dependent constraint: non-greedy path (driver-side sampling), with
    # one-choice runs so grammar jump-forward sends extend chunks through the TP step messages
    n = len(hist)
    if n % 7 in (2, 3):
        return [(n * 37 + 11) % 512]
    return list(range(1 + (n % 5), 512, 3))


def _drive(eng, pipelined: bool, constrained: bool):
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams

    mk = (lambda: SamplingParams.greedy(10, logits_processor=_proc)) if constrained else (lambda: SamplingParams.greedy(10))
    seqs = [eng.add_request(p, mk()) for p in PROMPTS[:2]]
    it = 0
    while eng.has_work() or len(seqs) < len(PROMPTS):
        if it == 3:
            seqs += [eng.add_request(p, mk()) for p in PROMPTS[2:]]
        eng.step_pipelined() if pipelined else eng.step()
        it += 1
    eng.flush()
    return [s.output_ids for s in seqs]


def _tp_pipelined_worker(rank, world, port, out_path):
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import make_tp_engine, run_tp_worker, shutdown_tp

    tp = TPGroup(rank, world, dist.group.WORLD)
    m = build_decoder(_ours_cfg("llama"), dtype=torch.float32, tp=tp)
    m.load_hf_state_dict(_hf("llama").state_dict())
    kw = dict(block_size=16, max_model_len=512, max_num_seqs=8, num_blocks=96)
    if rank == 0:
        eng = make_tp_engine(m, tp, None, engine_kw={"eos_ids": set(), "max_num_batched_tokens": 40}, **kw)
        got = [_drive(eng, True, c) for c in (False, True)]
        shutdown_tp(eng)
        torch.save(got, out_path)
    else:
        run_tp_worker(m, tp, **kw)
    dist.destroy_process_group()


def test_tp2_pipelined_steps_match_synchronous_single_process():
    """Pipelined stepping under TP=2 (workers gather in-flight inputs from their greedy ids,
    or from the driver's sampled ids broadcast over the TP group) == one process, sync."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder

    m = build_decoder(_ours_cfg("llama"), dtype=torch.float32)
    m.load_hf_state_dict(_hf("llama").state_dict())
    ref = [_drive(LLMEngine(m, None, max_model_len=512, max_num_seqs=8, num_blocks=96, eos_ids=set(),
                            max_num_batched_tokens=40), False, c) for c in (False, True)]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.spawn(_tp_pipelined_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        got = torch.load(out, weights_only=True)
    assert got == ref


def _tp_worker(rank, world, port, arch, out_path, sp_min_tokens=None):
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import make_tp_engine, run_tp_worker, shutdown_tp

    tp = TPGroup(rank, world, dist.group.WORLD)
    m = build_decoder(_ours_cfg(arch), dtype=torch.float32, tp=tp)
    m.load_hf_state_dict(_hf(arch).state_dict())
    if sp_min_tokens == "overlap":
        # chunked row-parallel tails (models/llama.py _post_attn_pipelined) on every step of >= 2 rows:
        # 3 chunks of any size, so odd and uneven splits occur
        from llm_kubernetes_minikube_sharp4dev_amd.models import llama

        llama.TP_OVERLAP_MIN_ROWS, llama.TP_OVERLAP_ALIGN, llama.TP_OVERLAP_CHUNKS = 2, 1, 3
        assert llama.overlap_chunks(7) == [(0, 3), (3, 6), (6, 7)]
    elif sp_min_tokens is not None:
        m.sp_min_tokens = sp_min_tokens
    kw = dict(block_size=16, max_model_len=512, max_num_seqs=8, num_blocks=96)
    if rank == 0:
        eng = make_tp_engine(m, tp, None, engine_kw={"eos_ids": set(), "max_num_batched_tokens": 40}, **kw)
        seqs = eng.generate(PROMPTS, SamplingParams.greedy(10))
        shutdown_tp(eng)
        torch.save([s.output_ids for s in seqs], out_path)
    else:
        run_tp_worker(m, tp, **kw)
    dist.destroy_process_group()


@pytest.mark.parametrize("arch,sp", [("llama", None), ("opt", None), ("llama", 2), ("llama", "overlap")])
def test_tp2_generation_matches_single_process(arch, sp):
    """TP=2 == one process; ("llama", 2): sequence parallel on every step of >= 2 rows
    (odd row counts exercise the padding); ("llama", "overlap"): the chunked row-parallel
    tails of TP prefill (each chunk's all-reduce + norm overlapping the next chunk's GEMM)."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder

    m = build_decoder(_ours_cfg(arch), dtype=torch.float32)
    m.load_hf_state_dict(_hf(arch).state_dict())
    eng = LLMEngine(m, None, max_model_len=512, max_num_seqs=8, num_blocks=96, eos_ids=set())
    ref = [s.output_ids for s in eng.generate(PROMPTS, SamplingParams.greedy(10))]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.spawn(_tp_worker, args=(2, _free_port(), arch, out, sp), nprocs=2, join=True)
        got = torch.load(out, weights_only=True)
    assert got == ref


def _knn_worker(rank, world, port, out_path):
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.sharded_index import ShardedKnnIndex

    g = torch.Generator().manual_seed(0)
    corpus = torch.randn(301, 32, generator=g)
    corpus[200] = corpus[5]  # duplicate across shards -> tie resolved by global id
    q = torch.randn(4, 32, generator=g)
    q[0] = corpus[5]
    idx = ShardedKnnIndex.from_full(corpus)
    s, i = idx.search(q, 7)
    if rank == 0:
        torch.save((s, i), out_path)
    dist.destroy_process_group()


def test_sharded_knn_equals_single():
    from llm_kubernetes_minikube_sharp4dev_amd import ops

    g = torch.Generator().manual_seed(0)
    corpus = torch.randn(301, 32, generator=g)
    corpus[200] = corpus[5]
    q = torch.randn(4, 32, generator=g)
    q[0] = corpus[5]
    rs, ri = ops.knn_topk(corpus, ops.row_norms(corpus), q, ops.row_norms(q), 7)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "knn.pt")
        mp.spawn(_knn_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        s, i = torch.load(out, weights_only=True)
    assert torch.equal(i.int(), ri.int())
    assert torch.allclose(s.float(), rs.float(), atol=1e-6)
    assert int(i[0, 0]) == 5 and int(i[0, 1]) == 200


def test_router_balances_two_replicas():
    from fastapi.testclient import TestClient

    from llm_kubernetes_minikube_sharp4dev_amd.parallel.router import ReplicaPool

    pool = ReplicaPool(["http://a", "http://b"])
    a = pool.pick()
    a.inflight += 1
    b = pool.pick()
    assert a.url != b.url
    b.inflight += 1
    pool.mark_failed(a)
    assert pool.pick().url == b.url


def _tp_dp_worker(rank, world, port, out_path):
    """world 4 = 2 replicas x TP 2: the bench.py protocol (leaders drive, followers run
    run_tp_worker and join the driver's world barriers through the control group)."""
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import new_tp_groups
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import (make_tp_engine, run_tp_worker, shutdown_tp,
                                                                          tp_barrier)

    tpg = new_tp_groups(2)
    m = build_decoder(_ours_cfg("llama"), dtype=torch.float32, tp=tpg)
    m.load_hf_state_dict(_hf("llama").state_dict())
    kw = dict(block_size=16, max_model_len=512, max_num_seqs=8, num_blocks=96)
    got = None
    if tpg.rank == 0:
        eng = make_tp_engine(m, tpg, None, engine_kw={"eos_ids": set(), "max_num_batched_tokens": 40}, **kw)
        tp_barrier(eng)
        prompts = PROMPTS if rank == 0 else PROMPTS[::-1]
        got = [s.output_ids for s in eng.generate(prompts, SamplingParams.greedy(6))]
        tp_barrier(eng)
        shutdown_tp(eng)
    else:
        run_tp_worker(m, tpg, **kw)
    objs = [None] * world
    dist.all_gather_object(objs, got)
    if rank == 0:
        torch.save(objs, out_path)
    dist.destroy_process_group()


def test_tp2_dp2_driver_worker_barrier_protocol():
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder

    m = build_decoder(_ours_cfg("llama"), dtype=torch.float32)
    m.load_hf_state_dict(_hf("llama").state_dict())
    eng = LLMEngine(m, None, max_model_len=512, max_num_seqs=8, num_blocks=96, eos_ids=set())
    ref = [s.output_ids for s in eng.generate(PROMPTS, SamplingParams.greedy(6))]
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "out.pt")
        mp.spawn(_tp_dp_worker, args=(4, _free_port(), out), nprocs=4, join=True)
        objs = torch.load(out, weights_only=True)
    assert objs[1] is None and objs[3] is None
    assert objs[0] == ref and objs[2] == ref[::-1]


def _rand_step(B=128, width=512, live=60, prefill=2, seed=0):
    import numpy as np

    from llm_kubernetes_minikube_sharp4dev_amd.engine.model_runner import StepInputs

    rng = np.random.default_rng(seed)
    T = B + 300 * prefill
    td = np.zeros((B, width), dtype=np.int32)
    td[:, :live] = rng.integers(1, 20000, (B, live))
    tp_ = np.zeros((prefill, width), dtype=np.int32)
    tp_[:, :70] = rng.integers(1, 20000, (prefill, 70))
    return StepInputs(ids=rng.integers(0, 128256, T).astype(np.int32), positions=rng.integers(0, 4000, T).astype(np.int32),
                      slots=rng.integers(-1, 300000, T).astype(np.int32), num_decode=B, decode_graph=B,
                      q_lens=[300] * prefill, ctx_lens=[950] * prefill, tables_p=tp_, ctx_d=rng.integers(1, 4000, B).astype(np.int32),
                      tables_d=td, logits_rows=np.arange(B + prefill, dtype=np.int64), greedy=True,
                      gather=(np.arange(B, dtype=np.int64), np.arange(B, dtype=np.int64)[::-1].copy()),
                      shared_len=17, prev_bcast=3)


def test_control_message_roundtrip():
    """encode_msg / decode_msg reproduce every StepInputs field bit for bit (block tables are
    sent at their live width and re-padded with the zeros they had)."""
    import numpy as np

    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import decode_msg, encode_msg

    si = _rand_step()
    h, payload = encode_msg("step", si)
    assert payload.size < si.tables_d.size  # the 512-wide tables do not travel whole
    cmd, got = decode_msg(h, payload)
    assert cmd == "step"
    for f in ("ids", "positions", "slots", "tables_p", "ctx_d", "tables_d", "logits_rows"):
        a, b = getattr(si, f), getattr(got, f)
        assert a.dtype == b.dtype and np.array_equal(a, b), f
    assert got.q_lens == si.q_lens and got.ctx_lens == si.ctx_lens
    assert all(np.array_equal(x, y) and x.dtype == y.dtype for x, y in zip(si.gather, got.gather))
    assert (got.num_decode, got.decode_graph, got.greedy, got.shared_len, got.prev_bcast) == (128, 128, True, 17, 3)
    assert decode_msg(*encode_msg("capture", (64, True))) == ("capture", (64, True))
    assert decode_msg(*encode_msg("stop")) == ("stop", None)


def _ctrl_timing_worker(rank, world, port, out_path):
    _init(rank, world, port)
    import time

    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import _Ctrl

    ctrl = _Ctrl(TPGroup(rank, world, dist.group.WORLD))
    si = _rand_step()
    n, trials = 100, 3  # best of 3 windows: a loaded CI host (pytest -n) preempts the spinning ranks
    if rank == 0:
        for _ in range(20):
            ctrl.send("step", si)
        best = float("inf")
        for _ in range(trials):
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(n):
                ctrl.send("step", si)
            dist.barrier()
            best = min(best, (time.perf_counter() - t0) / n)
        torch.save(best, out_path)
        ctrl.send("stop")
    else:
        for _ in range(20):
            ctrl.recv()
        for _ in range(trials):
            dist.barrier()
            for _ in range(n):
                cmd, got = ctrl.recv()
                assert cmd == "step" and got.num_decode == 128
            dist.barrier()
        assert ctrl.recv()[0] == "stop"
    dist.destroy_process_group()


def test_control_hop_cost_world2_b128():
    """Per-step driver -> worker control hop at B = 128 decode rows + 2 prefill chunks
    (tensor header + payload over gloo): recorded, and far below a step's GPU time."""
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "t.pt")
        mp.spawn(_ctrl_timing_worker, args=(2, _free_port(), out), nprocs=2, join=True)
        per_step = torch.load(out, weights_only=True)
    print(f"control hop per step (world 2, B128): {per_step * 1e6:.1f} us")
    assert per_step < 1e-3


def _cfg70(tp_size):
    """70B-shaped miniature: GQA 8:1 with 8 KV heads -> one KV head per rank at TP=8."""
    from llm_kubernetes_minikube_sharp4dev_amd.models.configs import DecoderConfig

    return DecoderConfig("t70", "llama", 2, 512, 64, 8, 8, 512, 512, max_position=1024, rope_theta=10000.0)


def _hf70():
    cfg = transformers.LlamaConfig(vocab_size=512, hidden_size=512, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=64, num_key_value_heads=8, head_dim=8,
                                   max_position_embeddings=1024, rope_theta=10000.0, tie_word_embeddings=False)
    torch.manual_seed(70)
    return transformers.LlamaForCausalLM(cfg).eval()


def _tp8_worker(rank, world, port, out_path, sp=False):
    _init(rank, world, port)
    torch.set_num_threads(1)
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import make_tp_engine, run_tp_worker, shutdown_tp

    tp = TPGroup(rank, world, dist.group.WORLD)
    m = build_decoder(_cfg70(world), dtype=torch.float32, tp=tp)
    assert m.hkv == 1  # one KV head per rank
    m.load_hf_state_dict(_hf70().state_dict())
    if sp:
        m.sp_min_tokens = 2  # every step of >= 2 rows sequence-parallel (reduce-scatter / all-gather)
    kw = dict(block_size=16, max_model_len=512, max_num_seqs=8, num_blocks=96)
    if rank == 0:
        out = {}
        eng = make_tp_engine(m, tp, None, engine_kw={"eos_ids": set(), "max_num_batched_tokens": 40}, **kw)
        if sp:
            out["sp"] = [_drive(eng, False, False), _drive(eng, True, True)]
        else:
            out["plain"] = [_drive(eng, False, False)]
            out["pipelined"] = [_drive(eng, True, c) for c in (False, True)]
        out["ctrl_us_per_msg"] = eng.tp_ctrl.seconds / max(1, eng.tp_ctrl.messages) * 1e6
        shutdown_tp(eng)
        torch.save(out, out_path)
    else:
        run_tp_worker(m, tp, **kw)
    dist.destroy_process_group()


def test_tp8_70b_shaped_plain_sp_pipelined_match_single_process():
    """World 8 on gloo: the Llama-3-70B TP=8 layout (GQA 8:1, one KV head per rank) with plain
    TP, sequence-parallel steps and pipelined stepping (greedy, and driver-sampled under a
    history-dependent grammar) == one process, synchronous."""
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder

    m = build_decoder(_cfg70(1), dtype=torch.float32)
    m.load_hf_state_dict(_hf70().state_dict())

    def eng():
        return LLMEngine(m, None, max_model_len=512, max_num_seqs=8, num_blocks=96, eos_ids=set(),
                         max_num_batched_tokens=40)

    ref_plain = _drive(eng(), False, False)
    ref_c = _drive(eng(), False, True)
    got = {}
    with tempfile.TemporaryDirectory() as d:
        for sp in (False, True):
            out = os.path.join(d, f"out{sp}.pt")
            mp.spawn(_tp8_worker, args=(8, _free_port(), out, sp), nprocs=8, join=True)
            got.update(torch.load(out, weights_only=True))
    assert got["plain"] == [ref_plain]
    assert got["pipelined"] == [ref_plain, ref_c]
    assert got["sp"] == [ref_plain, ref_c]
    print(f"TP8 control hop: {got['ctrl_us_per_msg']:.0f} us per message")


# ---- context parallelism: paged_attention(cp_group=...) over contiguous KV shards
_CP_SEQS = [("prefill", 37, 9), ("prefill", 13, 13), ("decode", 50, 1), ("decode", 5, 1)]  # (kind, ctx, q)
_CP_H = (4, 2, 16)  # Hq, Hkv, D
_CP_BS = 4


def _cp_problem(C: int, rank: int):
    """The same attention problem on every rank; rank r's cache holds the r-th contiguous
    shard of every sequence's keys (C = 1: the whole context)."""
    from llm_kubernetes_minikube_sharp4dev_amd.models.attention import AttnMeta

    Hq, Hkv, D = _CP_H
    g = torch.Generator().manual_seed(7)
    keys = [(torch.randn(n, Hkv, D, generator=g), torch.randn(n, Hkv, D, generator=g)) for _, n, _ in _CP_SEQS]
    q = [torch.randn(ql, Hq, D, generator=g) for _, _, ql in _CP_SEQS]
    kc = torch.zeros(64, Hkv, _CP_BS, D)
    vc = torch.zeros_like(kc)
    nxt = 0
    tables, lens, starts = [], [], []
    for (k, v), (_, n, _) in zip(keys, _CP_SEQS):
        per = -(-n // C)
        a, b = min(n, rank * per), min(n, (rank + 1) * per)
        nb = max(1, -(-(b - a) // _CP_BS))
        blocks = list(range(nxt, nxt + nb))
        nxt += nb
        for j in range(b - a):
            kc[blocks[j // _CP_BS], :, j % _CP_BS] = k[a + j]
            vc[blocks[j // _CP_BS], :, j % _CP_BS] = v[a + j]
        tables.append(blocks + [0] * (16 - nb))
        lens.append(b - a)
        starts.append(a)
    pre = [i for i, s in enumerate(_CP_SEQS) if s[0] == "prefill"]
    dec = [i for i, s in enumerate(_CP_SEQS) if s[0] == "decode"]
    qrows = torch.cat([q[i] for i in pre + dec])
    T = qrows.shape[0]
    qkv = torch.zeros(T, (Hq + 2 * Hkv) * D)
    qkv[:, : Hq * D] = qrows.reshape(T, -1)
    pos = []
    for i in pre:
        n, ql = _CP_SEQS[i][1], _CP_SEQS[i][2]
        pos += list(range(n - ql, n))
    pos += [_CP_SEQS[i][1] - 1 for i in dec]
    cu = [0]
    for i in pre:
        cu.append(cu[-1] + _CP_SEQS[i][2])
    meta = AttnMeta(positions=torch.tensor(pos, dtype=torch.int32), slots=torch.full((T,), -1, dtype=torch.int32),
                    num_prefill_tokens=cu[-1], num_prefill_seqs=len(pre), num_decode=len(dec),
                    cu_q=torch.tensor(cu, dtype=torch.int32),
                    ctx_lens_p=torch.tensor([lens[i] for i in pre], dtype=torch.int32),
                    block_tables_p=torch.tensor([tables[i] for i in pre], dtype=torch.int32),
                    q_lens_cpu=[_CP_SEQS[i][2] for i in pre], ctx_lens_cpu=[lens[i] for i in pre],
                    block_tables_d=torch.tensor([tables[i] for i in dec], dtype=torch.int32),
                    ctx_lens_d=torch.tensor([lens[i] for i in dec], dtype=torch.int32),
                    cp_key_start_p=[starts[i] for i in pre], cp_key_start_d=[starts[i] for i in dec])
    return qkv, kc, vc, meta


def _cp_worker(rank, world, port, out_path):
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.models.attention import paged_attention

    Hq, Hkv, D = _CP_H
    qkv, kc, vc, meta = _cp_problem(world, rank)
    out = paged_attention(qkv, kc, vc, meta, Hq, Hkv, D, D ** -0.5, cp_group=dist.group.WORLD)
    torch.save(out, f"{out_path}.{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_context_parallel_attention_matches_single_process(world):
    """Every CP rank holds one contiguous shard of each sequence's keys (some shards empty
    for the 5-key sequence at world 3); partial attention + one all-gather + LSE merge must
    equal unsharded paged attention for chunked-prefill rows (causal by global position)
    and decode rows."""
    from llm_kubernetes_minikube_sharp4dev_amd.models.attention import paged_attention

    Hq, Hkv, D = _CP_H
    qkv, kc, vc, meta = _cp_problem(1, 0)
    meta.cp_key_start_p = meta.cp_key_start_d = None
    ref = paged_attention(qkv, kc, vc, meta, Hq, Hkv, D, D ** -0.5)
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "cp")
        mp.spawn(_cp_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        for r in range(world):
            got = torch.load(f"{out}.{r}", weights_only=True)
            torch.testing.assert_close(got, ref, atol=2e-5, rtol=2e-5)


def _serve_in_thread(app):
    """uvicorn on a free 127.0.0.1 port in a daemon thread; returns (url, server)."""
    import socket
    import threading
    import time

    import uvicorn

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(app, host="127.0.0.1", port=port, log_level="warning"))
    threading.Thread(target=srv.run, daemon=True).start()
    t0 = time.time()
    while not srv.started:
        assert time.time() - t0 < 20, "replica did not start"
        time.sleep(0.02)
    return f"http://127.0.0.1:{port}", srv


def test_router_proxies_streams_and_fails_over():
    """The router in front of one live replica and one dead URL: NDJSON streams pass through
    chunk by chunk, JSON routes are answered, the dead replica leaves the rotation after its
    first failed request and in-flight counts return to zero."""
    import json
    import socket

    from fastapi import FastAPI
    from fastapi.responses import StreamingResponse
    from fastapi.testclient import TestClient

    from llm_kubernetes_minikube_sharp4dev_amd.parallel.router import create_router_app

    rep = FastAPI()

    @rep.get("/api/version")
    async def version():
        return {"version": "0.0-test"}

    @rep.post("/api/generate")
    async def generate(body: dict):
        async def gen():
            for i in range(3):
                yield json.dumps({"response": f"{body['prompt']}{i}", "done": False}) + "\n"
            yield json.dumps({"response": "", "done": True}) + "\n"
        return StreamingResponse(gen(), media_type="application/x-ndjson")

    live, srv = _serve_in_thread(rep)
    with socket.socket() as so:  # a port nobody listens on
        so.bind(("127.0.0.1", 0))
        dead = f"http://127.0.0.1:{so.getsockname()[1]}"
    try:
        app = create_router_app([dead, live], probe_interval_s=3600)
        with TestClient(app) as c:
            for k in range(4):
                r = c.post("/api/generate", json={"model": "m", "prompt": f"p{k}"})
                assert r.status_code == 200 and "ndjson" in r.headers["content-type"]
                lines = [json.loads(x) for x in r.text.splitlines()]
                assert [x["response"] for x in lines] == [f"p{k}0", f"p{k}1", f"p{k}2", ""] and lines[-1]["done"]
            assert c.get("/api/version").json() == {"version": "0.0-test"}
            st = {x["url"]: x for x in c.get("/router/status").json()["replicas"]}
            assert not st[dead]["healthy"] and st[dead]["failures"] == 1
            assert st[live]["served"] == 5 and st[live]["inflight"] == 0 and st[dead]["inflight"] == 0
    finally:
        srv.should_exit = True


def test_shm_control_send_fails_when_a_worker_stops_acknowledging(monkeypatch):
    """the driver's send() must not spin forever behind a dead TP worker."""
    import numpy as np

    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import _ShmChannel

    monkeypatch.setenv("LK_TP_CTRL_TIMEOUT_S", "0.5")
    name = f"lk_test_ctrl_{os.getpid()}"
    drv = _ShmChannel(name, True, n_workers=1)
    wk = _ShmChannel(name, False, worker_index=0, n_workers=1)
    try:
        h = np.zeros(8, dtype=np.int64)
        p = np.zeros(4, dtype=np.int32)
        drv.send(h, p)
        drv.send(h, p)
        wk.recv()  # the worker takes message 1, then "dies"
        drv.send(h, p)  # slot of message 1 is free
        with pytest.raises(RuntimeError, match="did not take message 2"):
            drv.send(h, p)  # needs message 2 acknowledged: never happens
    finally:
        wk.close()
        drv.close()


# ---------------------------------------------------------------- IPC self-check / packed greedy
def test_route_table_respects_self_check_vetoes():
    """A (bucket, algorithm) the self-check failed is never routed, whatever its timing; a bucket
    with every IPC form failed goes to RCCL when the group has a communicator."""
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import route_table

    timings = {1: {"ipc1": 5.0, "ipc2": 9.0, "rccl": 30.0}, 64: {"ipc1": 20.0, "ipc2": 12.0, "rccl": 25.0},
               4096: {"ipc1": 900.0, "ipc2": 300.0, "rccl": 200.0}}
    assert route_table(timings, {}, True) == {1: "ipc1", 64: "ipc2", 4096: "rccl"}
    assert route_table(timings, {1: {"ipc1"}, 64: {"ipc2"}}, True) == {1: "ipc2", 64: "ipc1", 4096: "rccl"}
    assert route_table(timings, {1: {"ipc1", "ipc2"}}, True)[1] == "rccl"
    # no communicator: rccl is never chosen
    no_rccl = {T: {a: v for a, v in d.items() if a != "rccl"} for T, d in timings.items()}
    assert route_table(no_rccl, {64: {"ipc2"}}, False) == {1: "ipc1", 64: "ipc1", 4096: "ipc2"}


class _FakeIpcState:
    """CPU stand-in for the HIP IPC state (xgmi_ar): gloo sums; ``broken`` corrupts one
    algorithm on THIS rank only (the group must still agree to veto it)."""

    def __init__(self, tp, broken=None, gather_broken=False):
        self.tp, self.broken, self.gather_broken = tp, broken, gather_broken

    def _sum(self, x):
        y = x.float().clone()
        dist.all_reduce(y)
        return y

    def all_reduce(self, inp, out):
        y = self._sum(inp)
        if self.broken in ("ipc1", "both"):
            y[0, 0] += 1
        out.copy_(y.to(out.dtype))

    def all_reduce2(self, inp, out, residual=None, w=None, eps=None):
        y = self._sum(inp)
        if self.broken in ("ipc2", "both"):
            y.view(-1)[-1] += 2
        if residual is None:
            out.copy_(y.to(out.dtype))
            return
        residual.copy_((residual.float() + y).to(residual.dtype))
        from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref

        out.copy_(ref.rmsnorm(residual.clone(), w, eps))

    def all_reduce_rmsnorm(self, x, residual, w, eps, out):
        y = self._sum(x)
        if self.broken in ("ipc1", "both"):
            y[0, 0] += 1
        residual.copy_((residual.float() + y).to(residual.dtype))
        from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref

        out.copy_(ref.rmsnorm(residual.clone(), w, eps))

    def gather(self, src, out, root):
        parts = [torch.empty_like(src) for _ in range(self.tp.size)]
        dist.all_gather(parts, src)
        if self.gather_broken:
            parts[0] = parts[0].flip(0)
        out.copy_(torch.cat(parts))

    def error(self):
        return 0


def _selfcheck_worker(rank, world, port, out_path, broken_rank, broken_algo, gather_broken):
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce, route_table

    tp = TPGroup(rank, world, dist.group.WORLD, dist.group.WORLD, list(range(world)))
    x = XgmiAllReduce.__new__(XgmiAllReduce)
    x.tp, x.max_bytes, x.two_shot, x.two_shot_min, x.rccl = tp, 1 << 20, None, 1 << 20, False
    x.table, x.timings, x.bad, x.gather_ok, x.check = {}, {}, {}, True, {}
    x.state = _FakeIpcState(tp, broken_algo if rank == broken_rank else None, gather_broken and rank == broken_rank)
    rep = x.self_check(64, rows=(1, 4, 16))
    try:
        table = route_table({T: {"ipc1": 1.0, "ipc2": 2.0} for T in (1, 4, 16)}, x.bad, False)
    except RuntimeError as e:
        table = str(e)
    # the staging-sized chunked all-reduce honours the vetoes too (or refuses)
    t = torch.full((3, 8), float(rank + 1)).to(torch.bfloat16)
    try:
        chunked = bool(torch.equal(x._all_reduce_chunked(t), torch.full((3, 8), 3.0).to(torch.bfloat16)))
    except RuntimeError as e:
        chunked = str(e)
    torch.save((rep, {T: sorted(s) for T, s in x.bad.items()}, x.gather_ok, table, chunked), f"{out_path}.{rank}")
    dist.destroy_process_group()


@pytest.mark.parametrize("broken_algo,gather_broken", [(None, False), ("ipc1", False), ("ipc2", False), (None, True),
                                                       ("both", False)])
def test_ipc_self_check_agrees_and_vetoes(broken_algo, gather_broken):
    """The start-up self-check (xgmi_ar.XgmiAllReduce.self_check) on a gloo world of 2 with a
    fake IPC state: a collective that is wrong on ONE rank is vetoed on BOTH (MAX agreement),
    the routing table and the chunked all-reduce then avoid it, a broken all-gather takes the
    group off the IPC path, and a group with no RCCL whose every IPC all-reduce failed is
    reported unusable (tune_collectives raises on ``ipc_disabled``) instead of routed."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "sc")
        mp.spawn(_selfcheck_worker, args=(2, port, path, 1, broken_algo, gather_broken), nprocs=2, join=True)
        res = [torch.load(f"{path}.{r}", weights_only=False) for r in range(2)]
    (rep0, bad0, g0, t0, c0), (rep1, bad1, g1, t1, c1) = res
    assert bad0 == bad1 and g0 == g1 and t0 == t1 and c0 == c1  # every rank routes alike
    if broken_algo == "both":
        assert bad0 == {T: ["ipc1", "ipc2"] for T in (1, 4, 16)}
        assert rep0["unusable_buckets"] == [1, 4, 16] and rep0["ipc_disabled"] is True
        assert isinstance(t0, str) and "no RCCL" in t0          # route_table refuses
        assert isinstance(c0, str) and "self-check" in c0       # chunked all-reduce refuses
        return
    want = {T: ([broken_algo] if broken_algo else []) for T in (1, 4, 16)}
    assert bad0 == want and rep0["unusable_buckets"] == []
    assert c0 is True
    if broken_algo:
        other = "ipc2" if broken_algo == "ipc1" else "ipc1"
        assert set(t0.values()) == {other}
        assert rep0["vetoed_buckets"] == [1, 4, 16] and not rep0["ipc_disabled"]
        assert all(v[broken_algo] == "FAILED" for v in rep0["buckets"].values())
    assert g0 is (not gather_broken) and rep0["ipc_disabled"] is gather_broken
    assert rep0["reference"].startswith("gloo")


def _greedy_worker(rank, world, port, out_path):
    _init(rank, world, port)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup

    tp = TPGroup(rank, world, dist.group.WORLD)
    torch.manual_seed(3)
    V = 64
    full = torch.randn(9, world * V)
    full[1, 5] = 7.0
    full[1, V + 5] = 7.0      # tie across shards: the lower id wins
    full[2] = -1.5            # all equal: id 0
    full[3, world * V - 1] = 50.0
    shard = full[:, rank * V:(rank + 1) * V].clone()
    ids = tp.greedy_ids(shard, vocab_lo=rank * V)
    torch.save((ids, full.argmax(-1).int()), f"{out_path}.{rank}")
    dist.destroy_process_group()


def test_vocab_parallel_greedy_one_packed_all_gather():
    """TPGroup.greedy_ids: ONE all-gather of packed (value, id) keys over the vocab shards picks
    exactly torch.argmax over the full row (ties -> lowest global id), on every rank."""
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "g")
        mp.spawn(_greedy_worker, args=(2, port, path), nprocs=2, join=True)
        for r in range(2):
            ids, want = torch.load(f"{path}.{r}", weights_only=True)
            assert torch.equal(ids, want), (r, ids, want)


def test_same_host_gate(monkeypatch):
    """Auto IPC attach only when every rank of the group is on this host (IPC handles do not map
    across nodes): the host names come from an all-gather over the control group."""
    from llm_kubernetes_minikube_sharp4dev_amd.parallel import tp as tpmod

    calls = []

    def fake_gather(out, obj, group=None):
        calls.append(obj)
        out[0], out[1] = obj, "other-node" if fake_gather.split else obj

    monkeypatch.setattr(tpmod.dist, "all_gather_object", fake_gather)
    g = tpmod.TPGroup(0, 2, None, None, [0, 1])
    fake_gather.split = False
    assert tpmod._same_host(g)
    fake_gather.split = True
    assert not tpmod._same_host(g)
