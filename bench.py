#!/usr/bin/env python3
"""Headline benchmark: RAG queries/sec (whole node) + p50 end-to-end latency,
Llama-3-8B (BASELINE.json config 2: bge-base embedder + Llama-3-8B bf16 TP=1 per
MI355X, 100k-document synthetic corpus).

One rank per GPU.  Default: DP replicas (TP=1, weak scaling: per-GPU concurrency
fixed as N grows).  Each request is the full ``/agent_rag`` pipeline of
``Minimal_RAG/Program.cs:106-316``:

  bge-base query embeddings -> cosine top-6 over the HBM-resident corpus (HIP kNN)
  -> citation gating -> evidence JSON prompt -> Llama-3-8B (flash prefill, prefix
  cache, hipGraph decode, greedy, ``--max-new-tokens`` per request) -> JSON
  extraction -> typed tool call -> RAG gating -> (fake) Kubernetes action.

Default load is closed-loop continuous batching (``--batch`` requests in flight per
replica; a step = ``--batch`` completions per replica).  Other BASELINE configs:
  --workload agent        Minimal_Agent /agent tool-call loop (config 3)
  --workload mixed        concurrent agent + RAG sessions on one engine (config 5)
  --model llama-3-70b --tp 8 --docs 1000000   70B TP=8 over RCCL, 1M-doc kNN (config 4)
With ``--tp T`` the world is split into TP groups of T ranks: the group's rank 0
drives the engine (scheduler, retrieval, sampling) and the others follow in lockstep.

Weights are random-init (no checkpoints offline), data synthetic.  Decoding is greedy
under the tool-call grammar (so the random model's output is a valid, allowlisted tool
call and the k8s action / gating path runs for every request), with EOS ignored so
every request generates exactly ``--max-new-tokens`` tokens (the reference's tool call
is ~20-60 tokens; default 48).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node 8 bench.py --gpus 8 ...

``--gpus N`` decides the world: under torchrun it must equal ``WORLD_SIZE`` (a mismatch is
refused); without a launcher (no ``WORLD_SIZE`` in the environment) and N > 1 this process
makes no HIP call, starts N fresh rank processes itself (``parallel/launch.py`` rank env,
one per local device) and relays rank 0's JSON line -- so ``python bench.py --gpus 8`` is a
whole-node run either way.  Ranks must land on N distinct devices (``--one-device`` aside).
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRICS = {
    "rag": "RAG queries/sec (whole node) + p50 end-to-end latency, {model}",
    "agent": "Agent tool-call requests/sec (whole node) + p50 end-to-end latency, {model}",
    "mixed": "Mixed agent+RAG requests/sec (whole node) + p50 end-to-end latency, {model}",
}
MODEL_NAMES = {"llama-3-8b": "Llama-3-8B", "llama-3-70b": "Llama-3-70B", "opt-125m": "OPT-125m"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks) of the job; default: WORLD_SIZE under a launcher, else 1.  Without a "
                         "launcher, N > 1 spawns the N rank processes itself")
    ap.add_argument("--steps", type=int, default=8, help="timed steps (continuous mode: a step = --batch completions per replica; 8 x 128 keeps the window-boundary noise of in-flight requests under 1%%)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128,
                    help="requests per replica per step (= in-flight concurrency in continuous mode)")
    ap.add_argument("--mode", choices=["continuous", "batch"], default="continuous",
                    help="continuous: closed-loop load, `batch` requests always in flight, a step = `batch` "
                         "completions; batch: a step = one synchronous batch of `batch` requests")
    ap.add_argument("--workload", choices=sorted(METRICS), default="rag")
    ap.add_argument("--docs", type=int, default=100_000, help="synthetic runbook documents in the knowledge base")
    ap.add_argument("--long-evidence", action="store_true",
                    help="corpus of ~1150-char sections (one chunk each): /agent_rag prompts of 6 evidence chunks "
                         "near the 1500-char evidence cap, ~3k tokens (SURVEY 3.3)")
    ap.add_argument("--max-new-tokens", type=int, default=48)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--embedder", default="bge-base")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree (ranks per replica)")
    ap.add_argument("--tp-sim", type=int, default=1,
                    help="one GPU runs rank 0's shard of a TP group of this size with local stand-in "
                         "collectives (parallel.tp.SimulatedTPGroup): per-rank compute of e.g. 70B TP=8; "
                         "the JSON reports the all-reduce bytes the real group would move")
    ap.add_argument("--kv-gb", type=float, default=48.0)
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="token budget per engine step (default: continuous 64 x --batch capped at 8192, "
                         "batch mode 65536)")
    ap.add_argument("--free-pods", action="store_true",
                    help="round-2 tool-call grammar: pod names free-form, deployment names not tied to the "
                         "chosen namespace (more requests end in the reference's 404 -> 500 branch)")
    ap.add_argument("--admit-chunk", type=int, default=None,
                    help="continuous mode: requests retrieved + admitted together (batched embed/kNN); "
                         "default --batch / 8")
    ap.add_argument("--unconstrained", dest="constrained", action="store_false",
                    help="decode without the tool-call grammar.  Default: the grammar (engine/constrained.py) makes "
                         "the random-init model emit valid tool calls, so every request also runs the k8s dispatch "
                         "and RAG gating path (same token counts; measured at the same speed)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--sp-min-tokens", type=int, default=None,
                    help="with --tp > 1: steps of at least this many rows run sequence-parallel "
                         "(reduce-scatter / all-gather around the norms); default off")
    ap.add_argument("--token-align", type=int, default=256,
                    help="trim mixed steps' prefill chunks to a multiple of this many rows (0: off)")
    ap.add_argument("--token-align-wave", type=int, default=0,
                    help="steps longer than this many rows are trimmed to a multiple of it (4096: whole "
                         "waves of 256x256 tiles on the N=4096 projections); 0: off")
    ap.add_argument("--admission", choices=["deferred", "inline", "threaded"], default="deferred",
                    help="continuous mode, how retrieval for newly freed slots runs on the engine thread: "
                         "deferred (default) launches query encoder + kNN on a side stream and admits the "
                         "requests at the first loop iteration after their top-k landed -- the host never "
                         "blocks on the device; inline waits for the top-k before the next step "
                         "(measured on MI355X, 2 runs each: 98.7/98.8 q/s either way, deferred p50 +3 ms, "
                         "host kNN wait 0.2 vs 3.8 ms); threaded plans on a planner thread")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--device", choices=["cuda", "cpu"], default="cuda",
                    help="cpu: BASELINE config 1 plumbing run (fp32 torch reference ops, gloo), e.g. "
                         "--device cpu --model opt-125m --embedder minilm-l6 --docs 1000")
    ap.add_argument("--sampling", choices=["greedy", "ollama"], default="greedy",
                    help="greedy (default; with the tool-call grammar unless --unconstrained) or Ollama's server "
                         "defaults (temperature 0.8, top-k 40, top-p 0.9, repeat penalty 1.1: what the .NET client "
                         "gets, no grammar) -- the in-process arm of the --via-http comparison")
    ap.add_argument("--via-http", action="store_true",
                    help="the .NET-facing path: Ollama-compatible server + Minimal_RAG app as separate processes, "
                         "/agent_rag driven over HTTP at concurrency 1, 8, 128 (benchmarks/http_bench.py)")
    ap.add_argument("--frontends", type=int, default=0,
                    help="with --via-http: split server, this many HTTP front-end processes before the GPU engine core")
    ap.add_argument("--http-levels", default=None, help="with --via-http: concurrency levels (default 1,8,128)")
    ap.add_argument("--http-requests", default=None, help="with --via-http: requests per level")
    ap.add_argument("--tokenizer", default=None,
                    help="tokenizer.json to use instead of the built-in one (e.g. benchmarks/data/"
                         "bpe_runbooks_r1.json, the round-1 tokenizer trained on the synthetic corpus itself, "
                         "for like-for-like comparisons with round-1 numbers)")
    ap.add_argument("--one-device", action="store_true",
                    help="every rank on cuda:0 (several ranks share ONE GPU): gloo process group, the TP "
                         "collectives on the IPC kernels only (LK_TP_COLLECTIVES=ipc) -- runs the multi-rank "
                         "TP engine (e.g. --tp 8, 70B shards of 17.6 GB each) on a one-GPU box; a correctness "
                         "and collective-table run, not a throughput figure")
    ap.add_argument("--collective-floor", default=None,
                    help="with --tp-sim: JSON of the measured per-call TP tail collective floor "
                         "(benchmarks/xgmi_floor.py --world 2; default profiles/r4_tp_collectives/floor_tp2_h<H>.json)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.admit_chunk is None:  # 1/8 of the in-flight requests per retrieval batch (16 at 128)
        args.admit_chunk = max(1, args.batch // 8)
    if args.via_http:  # before any GPU use: the servers are child processes
        import subprocess

        cmd = [sys.executable, os.path.join(ROOT, "benchmarks", "http_bench.py"), "--docs", str(args.docs),
               "--max-new-tokens", str(args.max_new_tokens), "--model", args.model, "--embedder", args.embedder,
               "--kv-gb", str(args.kv_gb)] + (["--json-out", args.json_out] if args.json_out else []) + \
            (["--frontends", str(args.frontends)] if args.frontends else []) + \
            (["--concurrency", args.http_levels, "--requests", args.http_requests] if args.http_levels else [])
        raise SystemExit(subprocess.call(cmd))
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus is not None and args.gpus > 1:
            raise SystemExit(_launch_ranks(args.gpus))  # no HIP call in this process
        args.gpus = 1
    elif args.gpus is None:
        args.gpus = int(env_world)
    elif int(env_world) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={env_world} ranks; "
                         f"refusing to report a {env_world}-rank run as {args.gpus} GPUs")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world % args.tp:
        raise SystemExit(f"--tp {args.tp} must divide the world size {world}")
    if args.tp_sim > 1 and (args.tp > 1 or world > 1):
        raise SystemExit("--tp-sim runs one rank's shard in a single process (no --tp, WORLD_SIZE 1)")
    if args.device == "cuda" and os.environ.get("LK_FORCE_REFERENCE", "0") not in ("", "0", "false", "False"):
        # the flag routes GPU tensors to the torch reference ops: never measure that as the framework
        raise SystemExit("bench.py: LK_FORCE_REFERENCE is set -- refusing to time the torch reference path "
                         "instead of the HIP kernels")
    t_setup = time.perf_counter()

    # ---- corpus chunks (CPU, before any GPU init: the pool forks)
    from llm_kubernetes_minikube_sharp4dev_amd.rag.corpus import build_chunks

    ncpu = os.cpu_count() or 8
    chunks = build_chunks(args.docs, args.seed, workers=max(1, min(16, ncpu) // max(1, world)),  # (at most 16 workers over all ranks)
                          section_chars=1150 if args.long_evidence else 0)
    log(rank, f"corpus: {args.docs} docs -> {len(chunks)} chunks ({time.perf_counter() - t_setup:.1f}s)")

    import torch
    import torch.distributed as dist

    from llm_kubernetes_minikube_sharp4dev_amd.agent.agent_pipeline import AgentPipeline, MixedPipeline
    from llm_kubernetes_minikube_sharp4dev_amd.agent.rag_pipeline import ContinuousLoad, RagAgentPipeline
    from llm_kubernetes_minikube_sharp4dev_amd.config import Config
    from llm_kubernetes_minikube_sharp4dev_amd.engine.embed_engine import EmbeddingEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.k8s.fake import FakeCluster
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder, build_encoder
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer
    from llm_kubernetes_minikube_sharp4dev_amd import ops
    from llm_kubernetes_minikube_sharp4dev_amd.ops import _ext
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import SINGLE, SimulatedTPGroup, new_tp_groups
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import (make_tp_engine, run_tp_worker,
                                                                          shutdown_tp, tp_barrier, tp_capture_all)
    from llm_kubernetes_minikube_sharp4dev_amd.rag.embedder import LocalEmbedder
    from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagChunk, RagIndex
    from llm_kubernetes_minikube_sharp4dev_amd.rag.synthetic import make_queries

    on_gpu = args.device == "cuda"
    if on_gpu and args.one_device:
        # several processes' hardware queues share the device: at 4 per process the scheduler
        # time-slices 8 ranks and every all-reduce waits for its peers' turn (0.08 vs 2.46 q/s at
        # 2 per process, profiles/r4_tp8_onedev/); read when HIP initialises, so set it first
        # (LK_ONE_DEVICE_HW_QUEUES: another cap, e.g. 4 for a 2-rank trace whose comm stream
        # needs a hardware queue of its own to overlap the compute stream)
        cap = int(os.environ.get("LK_ONE_DEVICE_HW_QUEUES", "2"))
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) > cap:
            os.environ["GPU_MAX_HW_QUEUES"] = str(cap)
    if on_gpu:
        assert torch.cuda.is_available(), "bench.py needs an MI355X (or --device cpu)"
        if args.one_device:
            # RCCL refuses several ranks on one device: gloo for the host-side collectives, the
            # IPC kernels for every TP collective, a capped grid so all ranks' spinning
            # workgroups stay co-resident on the one GPU
            local = 0
            os.environ["LK_TP_COLLECTIVES"] = "ipc"
            os.environ.setdefault("LK_XGMI_AR_BLOCKS", "16")
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        _ext.lib()  # fail loudly if the HIP library is not built
        if world > 1:
            if args.one_device:
                dist.init_process_group("gloo")
            else:
                dist.init_process_group("nccl", device_id=dev)
                # one rank per GPU: N ranks on fewer than N devices would time shared GPUs
                import socket

                where = [None] * world
                dist.all_gather_object(where, (socket.gethostname(), torch.cuda.current_device()))
                if len(set(where)) != world:
                    raise SystemExit(f"bench.py: {world} ranks landed on {len(set(where))} distinct devices "
                                     f"{sorted(set(where))}; --gpus {args.gpus} needs one device per rank "
                                     f"(--one-device shares one GPU on purpose)")
    else:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")

    def sync():
        if on_gpu:
            torch.cuda.synchronize()

    wdtype = torch.bfloat16 if on_gpu else torch.float32
    tpg = new_tp_groups(args.tp) if args.tp > 1 else SINGLE
    if args.tp_sim > 1:
        tpg = SimulatedTPGroup(rank=0, size=args.tp_sim)
    leader = tpg.rank == 0
    n_replicas = world // args.tp

    cfg = Config()
    if args.tokenizer:
        from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import load_tokenizer

        tok = load_tokenizer(args.tokenizer)
    else:
        tok = builtin_tokenizer()

    # ---- embedder + index build (embedding work sharded over ALL ranks, all-gather over RCCL;
    # every replica driver then holds the whole corpus in HBM: 1M x 768 bf16 = 1.5 GB)
    enc = build_encoder(args.embedder, device=dev, seed=args.seed, dtype=wdtype)
    emb_engine = EmbeddingEngine(enc, tok, name=args.embedder, max_tokens_per_batch=262144)
    n = len(chunks)
    per = (n + world - 1) // world
    lo, hi = min(n, rank * per), min(n, (rank + 1) * per)
    t0 = time.perf_counter()
    mine = emb_engine.embed([c[2] for c in chunks[lo:hi]])
    full = torch.zeros((per * world, enc.cfg.hidden), dtype=wdtype, device=dev)
    shard = torch.zeros((per, enc.cfg.hidden), dtype=wdtype, device=dev)
    shard[: hi - lo] = mine.to(wdtype)
    if world > 1 and args.one_device:  # gloo: through the host
        full = torch.cat([t.to(dev) for t in _gather_cpu(shard.cpu(), world)])
    elif world > 1:
        dist.all_gather_into_tensor(full, shard)
    else:
        full = shard
    corpus = full[:n].contiguous()
    del full, shard, mine
    sync()
    t_index = time.perf_counter() - t0
    if on_gpu:  # the encoder's micro-batch activations go back to the device before the KV pool is sized
        torch.cuda.empty_cache()
    if on_gpu and not args.no_graphs and args.admit_chunk == 1:
        # one query per retrieval (batch 1): its encoder pass replays a hipGraph per length
        t_cap = time.perf_counter()
        ncap = emb_engine.capture_queries(dtypes=(torch.bfloat16,))
        log(rank, f"query encoder: {ncap} hipGraphs captured in {time.perf_counter() - t_cap:.1f}s")
    index = RagIndex(LocalEmbedder(emb_engine), backend="gpu", device=str(dev))
    index.chunks = [RagChunk(i, s, t) for i, s, t in chunks]
    index.set_gpu_corpus(corpus)
    del chunks
    log(rank, f"index: {n} chunks x {enc.cfg.hidden} embedded in {t_index:.1f}s")

    # ---- generator + engine
    t0 = time.perf_counter()
    llm = build_decoder(args.model, device=dev, seed=args.seed, tp=tpg, dtype=wdtype)
    if args.sp_min_tokens is not None and hasattr(llm, "sp_min_tokens"):
        llm.sp_min_tokens = args.sp_min_tokens
    sync()
    log(rank, f"{args.model} random-init (tp={args.tp}{f', tp-sim {args.tp_sim}' if args.tp_sim > 1 else ''}) "
              f"in {time.perf_counter() - t0:.1f}s")
    # continuous: 4096-token steps.  Round 2 (step-by-step decoding) measured 8192-token steps
    # 2 % ahead of 4096 (profiles/r2_sched_sweep.md); with grammar jump-forward requests finish
    # in 22 % fewer steps, admissions arrive in smaller pieces, and 4096-token steps -- prefill
    # spread over more steps, fewer decode-only weight-streaming steps -- read 98.85 / 100.15
    # q/s vs 98.27 / 98.63 at 8192 and 93.7 at 3072 on one box (profiles/r3_mbt/); scaled with
    # the in-flight count below 64 requests (4096 at 64 for the 70B config, where 8192-token
    # steps measured 9 % slower)
    # Long-evidence prompts (~2.4k uncached tokens) queue behind a 4096-token budget (31 steps
    # queued per request): 8192 read 33.0 vs 32.2 q/s there, while the mixed agent + RAG
    # workload keeps 4096 (148.1 vs 143.3; profiles/r3_budget_wl/)
    cap = 8192 if args.long_evidence else 4096
    mbt = args.max_batched_tokens or (min(cap, 64 * max(args.batch, 32)) if args.mode == "continuous" else 65536)
    runner_kw = dict(block_size=16, max_model_len=8192, max_num_seqs=max(args.batch, 64), kv_cache_gb=args.kv_gb,
                     use_graphs=on_gpu and not args.no_graphs)
    if not on_gpu:
        runner_kw.pop("kv_cache_gb")
        runner_kw["num_blocks"] = max(256, args.batch * 80)
    engine_kw = dict(max_num_batched_tokens=mbt, enable_prefix_caching=not args.no_prefix_cache, eos_ids=set(),
                     token_align=args.token_align, token_align_wave=args.token_align_wave)
    if args.sampling == "ollama":
        params = SamplingParams(max_tokens=args.max_new_tokens, ignore_eos=True)  # Ollama defaults
        args.constrained = False
    else:
        params = SamplingParams.greedy(args.max_new_tokens, ignore_eos=True)
    if args.constrained:
        from llm_kubernetes_minikube_sharp4dev_amd.engine.constrained import tool_call_processor

        # namespaces from the RAG allowlist; deployment and pod names those of the chosen
        # namespace in the (fake) cluster, as a model reading the cluster context would pick them
        # (round 2 let pod names run free: 17 % of requests then ended in the reference's
        # get_logs 500 branch on invented pods); other strings free-form (<= 16 chars)
        from llm_kubernetes_minikube_sharp4dev_amd.k8s.fake import FakeCluster as _FC

        snap, by_ns = _FC.default(), {}
        for (ns, pod) in sorted(snap.pods):
            by_ns.setdefault(ns, {"pod": [], "name": []})["pod"].append(pod)
        for (ns, dep) in sorted(snap.deployments):
            by_ns.setdefault(ns, {"pod": [], "name": []})["name"].append(dep)
        enums = {"namespace": list(cfg.agent.allowed_namespaces) + ["default"]}
        for field in ("pod", "name"):
            enums[field] = {"__by__": "namespace", **{ns: v[field] for ns, v in by_ns.items()}}
        if args.free_pods:  # round-2 grammar: deployment names from a flat list, pods free-form
            enums = {"namespace": enums["namespace"], "name": ["echoserver", "api", "web", "worker"]}
        params.logits_processor = tool_call_processor(tok, max_str=16, enums=enums)
    results, trace, elapsed, tim_setup = [], [], 0.0, 0.0
    load, load_host, tp_ctrl, prompt_len = None, {}, {}, {}

    # --tp T: the corpus is sharded over the TP group (each rank scans 1/T of it; SURVEY 2.4
    # "sharded kNN index"), the leader merges the per-rank top-k
    knn_shard = None
    if args.tp > 1:
        from llm_kubernetes_minikube_sharp4dev_amd.parallel.sharded_index import ShardedKnnIndex

        knn_shard = ShardedKnnIndex.for_tp(corpus, tpg)
    if not leader:
        # TP follower: execute the driver's steps (and its barriers, sharded searches) until it says stop
        del corpus, index
        run_tp_worker(llm, tpg, knn=knn_shard, **runner_kw)
    else:
        # decode-graph buckets: one row per running request, plus the rows of jump-forward
        # extend chunks under the tool-call grammar
        graph_rows = max(args.batch, 1) * (2 if args.constrained and args.sampling == "greedy" else 1)
        if args.tp > 1:
            engine = make_tp_engine(llm, tpg, tok, engine_kw=engine_kw, **runner_kw)
            if runner_kw["use_graphs"]:
                tp_capture_all(engine, max_batch=graph_rows, variants=(args.sampling == "greedy" and not args.constrained,))
        else:
            engine = LLMEngine(llm, tok, **runner_kw, **engine_kw)
            if runner_kw["use_graphs"]:
                engine.runner.capture_all(max_batch=graph_rows, variants=(args.sampling == "greedy" and not args.constrained,))
        knn_info = {"mode": "single"}
        if knn_shard is not None:
            from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp_engine import tp_knn_search

            # the sharded search must return exactly the single-scan top-k (ties by id)
            qv = corpus[torch.arange(0, min(64, n)) * max(1, n // 64)].clone()
            qv[1:8] += 0.01 * torch.randn_like(qv[1:8])
            cs, ci = ops.knn_topk(corpus, index.gpu_tensors()[1], qv, ops.row_norms(qv), 6)
            ss, si = tp_knn_search(engine, knn_shard, qv, 6)
            knn_info = {"mode": f"sharded over tp{args.tp} ({knn_shard.corpus.shape[0]} rows per rank)",
                        "matches_single_scan": bool(torch.equal(si.cpu().long(), ci.cpu().long()))}
            index.set_sharded(lambda q, k: tp_knn_search(engine, knn_shard, q, k), dim=corpus.shape[1])
            log(rank, f"kNN: {knn_info}")
        k8s = FakeCluster.default()
        rag = RagAgentPipeline(index, engine, tok, k8s, cfg)
        agent = AgentPipeline(engine, tok, k8s, cfg)
        pipe = {"rag": rag, "agent": agent, "mixed": MixedPipeline(rag, agent)}[args.workload]
        replica = rank // args.tp
        qcount = [0]

        def next_queries(k):
            qcount[0] += 1
            return make_queries(k, seed=args.seed * 100003 + replica * 7919 + qcount[0])

        def batch_step():
            reqs, tim = pipe.plan_requests(next_queries(args.batch))
            todo = {}
            for i, (p, ids, ctx) in enumerate(reqs):
                if ids is not None:
                    todo[i] = engine.add_request(ids, params.__class__(**{**params.__dict__}))
            ts = time.perf_counter()
            engine.run_until_done(list(todo.values()))
            out = []
            for i, (p, ids, ctx) in enumerate(reqs):
                if i not in todo:
                    out.append(pipe.finish_request(p, [], None))
                    continue
                r = pipe.finish_request(p, todo[i].output_ids, ctx)
                r.prompt_tokens = len(ids)
                r.timings = {**tim, **todo[i].metrics(), "e2e_s": time.perf_counter() - ts}
                out.append(r)
            return out

        # progress on stderr every LK_BENCH_HEARTBEAT seconds (default 30; 0 = off): long
        # runs (70B, several ranks sharing one GPU) show where they are
        hb_s = float(os.environ.get("LK_BENCH_HEARTBEAT", "30"))
        if hb_s > 0:
            import threading

            def _beat():
                t_hb = time.perf_counter()
                while True:
                    time.sleep(hb_s)
                    # host-side counters only: no HIP call from this thread (a graph capture may be open)
                    log(rank, f"alive {time.perf_counter() - t_hb:.0f}s: engine steps {engine.steps}, launches "
                              f"{engine.launches}, timed completions {len(results)}")

            threading.Thread(target=_beat, name="bench-heartbeat", daemon=True).start()
        load = None
        if args.mode == "continuous":
            # warm-up fills the pipeline and reaches the steady prefill/decode mix; the timed
            # window continues the same stream (in-flight requests carry over)
            load = ContinuousLoad(pipe, next_queries, params, args.batch, admit_chunk=args.admit_chunk,
                                  threaded=args.admission == "threaded",
                                  deferred=args.admission == "deferred")
            load.run(max(args.warmup, 1) * args.batch)
        else:
            for _ in range(args.warmup):
                batch_step()
        tim_setup = time.perf_counter() - t_setup
        log(rank, f"setup {tim_setup:.1f}s; timing {args.steps} steps x {args.batch} req/replica")

        if world > 1:
            tp_barrier(engine)
        sync()
        engine.step_trace = []
        kv_keys0 = engine.runner.decode_kv_keys
        load_host0 = dict(load.host_s) if load is not None else {}
        chars0 = (rag.planned_chars, rag.planned_tokens, rag.planned_requests, rag.planned_evidence)
        ctrl0 = (engine.tp_ctrl.seconds, engine.tp_ctrl.messages) if args.tp > 1 else None
        prof = None
        if os.environ.get("LK_PROFILE_TIMED"):  # host-side cProfile of the timed window only
            import cProfile

            prof = cProfile.Profile()
            prof.enable()
        # LK_TRACE_WINDOW=1: marker kernels at both ends of the timed window, so a kernel trace
        # is summarised over exactly the timed steps (scripts/summarize_trace.py --window)
        mark = on_gpu and os.environ.get("LK_TRACE_WINDOW", "0") == "1"
        if mark:
            _ext.lib().window_mark(1)
        t0 = time.perf_counter()
        if load is not None:
            results.extend(load.run(args.steps * args.batch))
        else:
            for _ in range(args.steps):
                results.extend(batch_step())
        if mark:
            _ext.lib().window_mark(2)
        sync()
        if world > 1:
            tp_barrier(engine)
        elapsed = time.perf_counter() - t0
        if prof is not None:
            prof.disable()
            prof.dump_stats(f"{os.environ['LK_PROFILE_TIMED']}.rank{rank}")
        trace, engine.step_trace = engine.step_trace, None
        if os.environ.get("LK_STEP_TRACE_OUT"):  # every timed step's trace tuple, for offline analysis
            with open(os.environ["LK_STEP_TRACE_OUT"], "w") as f:
                json.dump({"fields": ["prefill_tokens", "decode_rows", "step_s", "schedule_s", "prepare_launch_s",
                                      "sample_sync_s", "post_s", "gpu_s", "idle_before_s", "tag", "starved", "rows"],
                           "steps": [list(t) for t in trace]}, f)
        # K / V bytes the decode attention read in the timed window (this rank's shard): over the
        # paged-decode kernel time of a timed-window trace, its in-situ bandwidth
        decode_kv_bytes = (engine.runner.decode_kv_keys - kv_keys0) * llm.kv_bytes_per_token()
        if ctrl0 is not None:  # driver -> TP worker control hop inside the timed window
            tp_ctrl = {"tp_ctrl_s": round(engine.tp_ctrl.seconds - ctrl0[0], 4),
                       "tp_ctrl_us_per_msg": round((engine.tp_ctrl.seconds - ctrl0[0]) * 1e6
                                                   / max(1, engine.tp_ctrl.messages - ctrl0[1]), 1),
                       "tp_ctrl_transport": "shm" if engine.tp_ctrl.shm is not None else "gloo"}
        dc, dt, dn, de = (a - b for a, b in zip(
            (rag.planned_chars, rag.planned_tokens, rag.planned_requests, rag.planned_evidence), chars0))
        if dn:  # RAG prompts planned inside the timed window
            prompt_len = {"prompt_chars": round(dc / dn, 1), "prompt_tokens": round(dt / dn, 1),
                          "chars_per_token": round(dc / dt, 3), "evidence_chunks": round(de / dn, 2)}
        if load is not None:
            load_host = {k: v - load_host0[k] for k, v in load.host_s.items()}
            load.drain()
        if args.tp > 1:
            shutdown_tp(engine)

    # ---- aggregate (every rank; followers contribute zero requests)
    lat = [r.timings.get("e2e_s", 0.0) for r in results if r.timings]
    ptok = [r.prompt_tokens for r in results if r.prompt_tokens]
    pre = [r.timings.get("cached_prefix_tokens", 0) for r in results if r.timings]
    stats = torch.tensor([elapsed, float(len(results)), float(sum(ptok)), float(len(ptok)),
                          float(torch.cuda.current_device() if on_gpu else -1)],
                         dtype=torch.float64, device=dev)
    if world > 1:
        if args.one_device:
            allst = torch.stack(_gather_cpu(stats.cpu(), world))
        else:
            allst = [torch.zeros_like(stats) for _ in range(world)]
            dist.all_gather(allst, stats)
            allst = torch.stack(allst).cpu()
        objs = [None] * world
        dist.all_gather_object(objs, lat)
        lat_all = [x for o in objs for x in o]
    else:
        allst = stats[None].cpu()
        lat_all = lat
    if rank == 0:
        t_max = float(allst[:, 0].max())
        total_req = float(allst[:, 1].sum())
        qps = total_req / t_max
        p50 = statistics.median(lat_all) * 1000 if lat_all else None
        lat_sorted = sorted(lat_all)
        p90 = lat_sorted[int(0.9 * (len(lat_sorted) - 1))] * 1000 if lat_sorted else None
        p99 = lat_sorted[int(0.99 * (len(lat_sorted) - 1))] * 1000 if lat_sorted else None
        avg_prompt = float(allst[:, 2].sum() / max(1.0, float(allst[:, 3].sum())))
        statuses = {}
        for r in results:
            statuses[str(r.status)] = statuses.get(str(r.status), 0) + 1
        dec_only = [t for t in trace if t[0] == 0]
        mixed = [t for t in trace if t[0] > 0]
        host = {}
        if trace:
            host = {k: round(sum(t[i] for t in trace), 3) for k, i in
                    (("schedule_s", 3), ("prepare_launch_s", 4), ("sample_sync_s", 5), ("post_s", 6))}
        if load is not None:
            host.update({f"load_{k}_s": round(v, 3) for k, v in load_host.items()})
        host.update(tp_ctrl)
        step_mix = {
            "host_breakdown": host,
            "steps": len(trace),
            "decode_only_steps": len(dec_only), "decode_only_gpu_s": round(sum(t[7] for t in dec_only), 3),
            "mixed_steps": len(mixed), "mixed_gpu_s": round(sum(t[7] for t in mixed), 3),
            # GPU time inside steps (first kernel -> ids copy) over the timed wall time: the rest is
            # device idle between steps
            "gpu_step_busy_frac": round(sum(t[7] for t in trace) / elapsed, 3) if trace and elapsed else None,
            "avg_prefill_tokens_mixed": round(statistics.mean(t[0] for t in mixed), 1) if mixed else 0,
            "avg_decode_rows": round(statistics.mean(t[1] for t in trace), 1) if trace else 0,
            "decode_attention_kv_gb": round(decode_kv_bytes / 1e9, 2),
            # device idle between a step's ids copy and the next step's start marker, i.e. the
            # host reached the launch after the device ran dry; by what the host did just before
            "idle_before_launch": _idle_summary(trace),
            # mixed steps by total rows (256-row buckets): where the prefill GEMMs run
            "mixed_rows_hist": {str(k * 256): v for k, v in sorted(collections.Counter(
                (t[0] + t[1] + 255) // 256 for t in mixed).items())},
        }
        tim = {k: statistics.mean(r.timings.get(k, 0.0) for r in results if r.timings)
               for k in ("embed_s", "knn_s", "knn_gpu_s", "prompt_s")
               if any(r.timings and k in r.timings for r in results)} if results else {}
        steps_acct = {k: round(statistics.mean(r.timings[k] for r in results if r.timings and r.timings.get(k) is not None), 2)
                      for k in ("steps_queued", "steps_in_system", "steps_run", "jumped_tokens")
                      if any(r.timings and r.timings.get(k) is not None for r in results)}
        # what the slowest decile of requests did differently from the median one (engine steps
        # waited / lived / ran, grammar-jumped tokens, prompt length, time to first token)
        tail = {}
        tim_res = [r for r in results if r.timings and r.timings.get("e2e_s") is not None]
        if len(tim_res) >= 20:
            cut = sorted(r.timings["e2e_s"] for r in tim_res)[int(0.9 * (len(tim_res) - 1))]
            for name, grp in (("p90_plus", [r for r in tim_res if r.timings["e2e_s"] >= cut]), ("all", tim_res)):
                tail[name] = {k: round(statistics.mean(r.timings[k] for r in grp if r.timings.get(k) is not None), 3)
                              for k in ("e2e_s", "ttft_s", "steps_queued", "steps_in_system", "steps_run",
                                        "jumped_tokens", "prompt_tokens", "preemptions")
                              if any(r.timings.get(k) is not None for r in grp)}
        par = f"dp{n_replicas}" if args.tp == 1 else f"tp{args.tp}" + (f"xdp{n_replicas}" if n_replicas > 1 else "")
        # what the process group really was, and what every replica (its TP leader) contributed:
        # a scaling record can show that all N ranks ran and every replica completed requests
        import socket

        dist_info = {
            "initialized": dist.is_initialized(),
            "world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "backend": dist.get_backend() if dist.is_initialized() else None,
            "env_world_size": world,
            "visible_devices": torch.cuda.device_count() if on_gpu else 0,
            "devices_used": sorted({int(d) for d in allst[:, 4].tolist()}) if on_gpu else [],
            "host": socket.gethostname(),
            "per_replica": [{"replica": rk // args.tp, "rank": rk, "completions": int(allst[rk, 1]),
                             "elapsed_s": round(float(allst[rk, 0]), 3),
                             "qps": round(float(allst[rk, 1]) / float(allst[rk, 0]), 3) if float(allst[rk, 0]) else None}
                            for rk in range(allst.shape[0]) if rk % args.tp == 0],
        }
        sim = {}
        if args.tp > 1 and getattr(tpg, "xgmi", None) is not None:
            # the measured collective table the TP group routes by (parallel/xgmi_ar.py tune)
            sim["tp_collectives"] = {"routes": {str(k): v for k, v in tpg.xgmi.table.items()},
                                     "us_by_rows": {str(k): v for k, v in tpg.xgmi.timings.items()},
                                     "mode": "ipc-only" if tpg.ipc_only else "auto (ipc1 / ipc2 / rccl measured)",
                                     # the start-up check of every IPC collective against the reference
                                     "self_check": tpg.xgmi.check,
                                     # handshakes that hit the bounded spin (a peer late by > ~4 s)
                                     "handshake_timeouts": int(tpg.xgmi.error())}
        elif args.tp > 1:
            sim["tp_collectives"] = {"mode": "rccl", "self_check": getattr(tpg, "xgmi_check", None)}
        if args.tp_sim > 1:
            par = f"tp{args.tp_sim}-sim (rank-0 shard on one GPU, collectives elided)"
            # what the real group moves per rank: every step's rows through 2 all-reduces per layer
            # (o / down row-parallel outputs) + the vocab-parallel embedding all-reduce, bf16
            lc = llm.cfg
            rows = sum(t[0] + t[1] for t in trace)
            ar_calls = (2 * lc.num_layers + 1) * len(trace)
            sim = {"tp_sim": args.tp_sim,
                   "allreduce_calls_per_step": 2 * lc.num_layers + 1,
                   "allreduce_bytes_per_step": round(rows * (2 * lc.num_layers + 1) * lc.hidden * 2 / max(1, len(trace))),
                   "allreduce_calls": ar_calls,
                   "rows_per_step": round(rows / max(1, len(trace)), 1),
                   "decode_only_steps": len(dec_only), "mixed_steps": len(mixed)}
            floor = _collective_floor(args.collective_floor, lc.hidden)
            if floor is not None:
                # per-step collective time the real group would add: per call the faster of
                # one-shot / two-shot = the measured kernel + handshake floor at that row count
                # (2 ranks sharing one device, benchmarks/xgmi_floor.py) + the xGMI link time of its
                # bytes at XGMI_LINK_GBPS per link (a model figure); 2 tails per layer + the
                # vocab-parallel embedding all-reduce
                W, Hd, n_ar = args.tp_sim, lc.hidden, 2 * lc.num_layers + 1
                est = {"floor_source": floor["_path"], "link_GBps_model": XGMI_LINK_GBPS, "hbm_GBps_model": HBM_GBPS,
                       "gemm_TFLOPs_model": GEMM_TFLOPS,
                       # prefill-sized steps run their o / down tails in row chunks overlapped with
                       # the next chunk's GEMM (models/llama.py _post_attn_pipelined): only the exposed part counts
                       "overlap": "prefill-sized steps: post-attention half of each layer pipelined over row "
                                  "chunks (compute o / mlp, comm tails); exposed = pipeline makespan - compute"}
                for name, up in (("upper", True), ("latency_floor_plus_bytes", False)):
                    per_step = [_exposed_step_us(floor, t[0] + t[1], lc, W, up) for t in trace]
                    tot_s = sum(per_step) / 1e6
                    est[name] = {
                        "ms_per_step": round(1e3 * tot_s / max(1, len(trace)), 3),
                        "timed_window_s": round(tot_s, 3), "vs_elapsed": round(tot_s / elapsed, 3) if elapsed else None,
                        "decode_only_ms_per_step": round(sum(p for p, t in zip(per_step, trace) if t[0] == 0) / 1e3
                                                         / max(1, len(dec_only)), 3),
                        "per_call_us": {str(r): round(_per_call_us(floor, r, Hd, W, up), 1)
                                        for r in (1, 64, 128, 256, 4096)}}
                sim["collective_estimate"] = est
        out = {
            "metric": METRICS[args.workload].format(model=MODEL_NAMES.get(args.model, args.model)),
            "value": round(qps, 3),
            "unit": "queries/s" if args.workload == "rag" else "requests/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1000, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if on_gpu else "fp32",
            "data": f"synthetic ({args.docs} runbook docs{', ~1150-char sections (long evidence)' if args.long_evidence else ''} "
                    f"-> {n} chunks; random-init weights)",
            "p50_latency_ms": round(p50, 1) if p50 is not None else None,
            "p90_latency_ms": round(p90, 1) if p90 is not None else None,
            "p99_latency_ms": round(p99, 1) if p99 is not None else None,
            # completions whose tool call executed (HTTP 200) per second: with random weights the
            # rest end in the reference's own 400 / 500 branches after the same generation work
            "success_qps": round(statuses.get("200", 0) * (total_req / max(1, len(results))) / t_max, 3),
            "config": {
                "model": f"{args.model} ({'bf16' if on_gpu else 'fp32, CPU'}, TP={args.tp}) + {args.embedder} embedder",
                "workload": args.workload,
                "global_batch": args.batch * n_replicas,
                "seq_len": round(avg_prompt, 1),
                # RAG prompt bodies planned in the timed window: characters, tokens (chat template
                # included) and their ratio under the built-in tokenizer (models/tokenizer.py)
                **prompt_len,
                "tokenizer": (os.path.basename(args.tokenizer) if args.tokenizer
                              else f"built-in byte-level BPE, llama-3 split, {tok.vocab_size} vocab"),
                "parallelism": par,
                "load": (f"continuous batching, closed loop, {args.batch} requests in flight per replica, "
                         f"step = {args.batch} completions per replica" if args.mode == "continuous"
                         else f"synchronous batches of {args.batch}"),
                "max_batched_tokens": mbt,
                "admit_chunk": args.admit_chunk if args.mode == "continuous" else None,
                "admission": args.admission if args.mode == "continuous" else None,
                "corpus_chunks": n,
                "max_new_tokens": args.max_new_tokens,
                "decoding": ("Ollama defaults (T 0.8, top-k 40, top-p 0.9, repeat penalty 1.1), ignore_eos"
                             if args.sampling == "ollama" else
                             "greedy, ignore_eos" + (", tool-call grammar" if args.constrained else "")),
                "prefix_caching": not args.no_prefix_cache,
                "hip_graphs": not args.no_graphs,
                # grammar-forced tokens appended by the host and run as extend chunks (every
                # token still gets its forward pass; LK_JUMP_FORWARD=0 steps them one by one)
                "jump_forward": bool(args.constrained and args.sampling == "greedy" and _jump_forward_on()),
                "avg_cached_prefix_tokens": round(statistics.mean(pre), 1) if pre else 0,
                "stage_means_s": {k: round(v, 4) for k, v in tim.items()},
                "engine_steps_per_request": steps_acct,
                "latency_tail": tail,
                "step_mix_rank0": step_mix,
                "index_build_s": round(t_index, 2),
                "knn": knn_info,
                "setup_s": round(tim_setup, 1),
                "http_status_counts_rank0": statuses,
                "distributed": dist_info,
                **sim,
            },
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


def _launch_ranks(n: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start N fresh rank processes (this
    process has made no HIP call, so nothing GPU-initialised forks or execs), rank r on local
    device r with the torchrun environment of ``parallel/launch.py:rank_env``.  Rank 0's stdout
    (the one JSON line) is relayed to this stdout; the other ranks' stdout goes to stderr.  The
    first rank to fail ends the job: the others are terminated and its exit code returned."""
    import signal
    import subprocess
    import threading

    from llm_kubernetes_minikube_sharp4dev_amd.parallel.launch import free_port, rank_env

    port = int(os.environ.get("MASTER_PORT") or free_port())
    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs = []
    for r in range(n):
        procs.append(subprocess.Popen(argv, env=rank_env(r, n, r, port),
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno(), text=True))
    print(f"[bench] launched {n} ranks (pids {[p.pid for p in procs]}, master 127.0.0.1:{port})",
          file=sys.stderr, flush=True)

    def relay():
        for line in procs[0].stdout:
            (sys.stdout if line.startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()

    th = threading.Thread(target=relay, daemon=True)
    th.start()

    def stop_all(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()

    signal.signal(signal.SIGTERM, lambda *a: (stop_all(), sys.exit(143)))
    rc = 0
    while any(p.poll() is None for p in procs):
        bad = [p for p in procs if p.poll() not in (None, 0)]
        if bad:
            rc = bad[0].returncode
            print(f"[bench] rank {procs.index(bad[0])} exited with {rc}: stopping the other ranks",
                  file=sys.stderr, flush=True)
            stop_all()
            break
        time.sleep(0.2)
    for p in procs:
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    th.join(timeout=10)
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode), 0)
    return rc if rc >= 0 else 128 - rc


def _idle_summary(trace) -> dict:
    """Device idle before each traced launch (engine step_trace element 8), in total and for
    gaps > 1 ms / > 0.1 ms, split by the host work tag of the launch (element 9: "plan" = a
    retrieval batch was launched, "admit" = planned requests were added, "" = neither)."""
    if not trace or len(trace[0]) < 10:
        return {}
    out = {"total_ms": round(1e3 * sum(t[8] for t in trace), 1)}
    if len(trace[0]) > 10:
        # launches that began with the device already idle: their schedule + input preparation
        # (host seconds 3 and 4) is device idle too, by step kind
        st = [t for t in trace if t[10]]
        out["starved_launches"] = {"count": len(st), "decode_only": sum(1 for t in st if t[0] == 0),
                                   "host_prep_ms": round(1e3 * sum(t[3] + t[4] for t in st), 1),
                                   "by_tag": dict(collections.Counter(t[9] or "-" for t in st))}
    for lim, key in ((1e-3, "gt_1ms"), (1e-4, "gt_0.1ms")):
        big = [t for t in trace if t[8] > lim]
        by = collections.Counter(t[9] or "-" for t in big)
        ms = collections.defaultdict(float)
        for t in big:
            ms[t[9] or "-"] += 1e3 * t[8]
        out[key] = {"count": len(big), "ms": round(1e3 * sum(t[8] for t in big), 1),
                    "by_tag": {k: [by[k], round(ms[k], 1)] for k in by},
                    "decode_only": sum(1 for t in big if t[0] == 0)}
    return out


def _gather_cpu(t, world: int) -> list:
    """all_gather of a host tensor over the (gloo) default group; bf16 travels as raw bytes
    (gloo has no 16-bit integer or bf16 all-gather)."""
    import torch
    import torch.distributed as dist

    src = t.contiguous().view(torch.uint8) if t.dtype == torch.bfloat16 else t
    out = [torch.empty_like(src) for _ in range(world)]
    dist.all_gather(out, src.contiguous())
    return [o.view(t.dtype) for o in out]


XGMI_LINK_GBPS = 153.0  # per xGMI link, per direction (MI355X: 7 links per GPU)


def _collective_floor(path, hidden: int):
    path = path or os.path.join(ROOT, "profiles", "r4_tp_collectives", f"floor_tp2_h{hidden}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        d = json.load(f)
    d["_path"] = os.path.relpath(path, ROOT)
    return d


def _floor_us(floor: dict, rows: int, algo: str) -> float:
    """Measured per-call floor (us) of ``algo`` at ``rows`` rows: the smallest measured bucket
    >= rows, linear in rows past the largest."""
    tab = {int(k): v for k, v in floor["us_by_rows"].items()}
    for b in sorted(tab):
        if rows <= b:
            return tab[b][algo]
    b = max(tab)
    return tab[b][algo] * rows / b


HBM_GBPS = 5000.0  # streaming rate of one MI355X's HBM3E under these kernels (model figure)
GEMM_TFLOPS = 1300.0  # in-situ prefill GEMM rate (profiles/r5_prof_window: ~1.3-1.5 PF/s; model figure)


def _exposed_step_us(floor: dict, rows: int, lc, world: int, upper: bool = True) -> float:
    """Collective time one TP step exposes: the vocab-parallel embedding all-reduce, then per
    layer the o and down tails -- whole (decode-sized steps), or, for steps models/llama.py
    chunks, the makespan of its pipeline (compute stream o(c) | mlp(c-1) | ..., communication
    stream tail_o(c), tail_down(c-1), ...; GEMMs at their shard FLOPs / GEMM_TFLOPS) minus
    the compute it contains."""
    from llm_kubernetes_minikube_sharp4dev_amd.models.llama import overlap_chunks

    H = lc.hidden
    total = _per_call_us(floor, rows, H, world, upper)  # embedding all-reduce (not chunked)
    chunks = overlap_chunks(rows)
    if chunks is None:
        return total + lc.num_layers * 2 * _per_call_us(floor, rows, H, world, upper)
    k_o, inter = lc.num_heads * lc.head_dim // world, lc.intermediate // world
    rate = GEMM_TFLOPS * 1e6  # flop per us
    t_main = t_comm = busy = 0.0
    ev_o, prev = {}, None

    def tail(c):
        nonlocal t_comm
        t_comm = max(t_comm, t_main) + _per_call_us(floor, c[1] - c[0], H, world, upper)
        return t_comm

    def mlp(c):
        nonlocal t_main, busy
        g = 2.0 * (c[1] - c[0]) * H * 3 * inter / rate  # gate_up (2 I / W) + down (I / W)
        t_main = max(t_main, ev_o[c]) + g
        busy += g
        tail(c)

    for c in chunks:
        g = 2.0 * (c[1] - c[0]) * k_o * H / rate
        t_main += g
        busy += g
        ev_o[c] = tail(c)
        if prev is not None:
            mlp(prev)
        prev = c
    mlp(prev)
    return total + lc.num_layers * (max(t_main, t_comm) - busy)


def _per_call_us(floor: dict, rows: int, hidden: int, world: int, upper: bool = True) -> float:
    """One fused all-reduce + norm tail of ``rows`` x ``hidden`` bf16 on ``world`` ranks: the
    faster of one-shot (every peer's S bytes over its own link, in parallel) and two-shot
    (2 S / world bytes per link).  ``upper``: measured floor at ``rows`` + link time -- the floor
    was measured with 2 ranks sharing one device, so past a few hundred rows it also carries
    both ranks' HBM passes through one HBM (an upper bound).  Otherwise: the measured floor at
    <= 64 rows (kernel + handshake latency) + link time + this rank's own HBM passes (one-shot:
    read W copies, write 2 (out + residual); two-shot: ~5 S / W + 2 S)."""
    S = rows * hidden * 2
    link = {"ipc1": S / (XGMI_LINK_GBPS * 1e3), "ipc2": 2 * S / world / (XGMI_LINK_GBPS * 1e3)}
    if upper:
        return min(_floor_us(floor, rows, a) + link[a] for a in ("ipc1", "ipc2"))
    hbm = {"ipc1": (world + 2) * S / (HBM_GBPS * 1e3), "ipc2": (5 * S / world + 2 * S) / (HBM_GBPS * 1e3)}
    return min(_floor_us(floor, min(rows, 64), a) + link[a] + hbm[a] for a in ("ipc1", "ipc2"))


def _jump_forward_on() -> bool:
    from llm_kubernetes_minikube_sharp4dev_amd.engine import llm_engine

    return llm_engine.JUMP_FORWARD


if __name__ == "__main__":
    main()
