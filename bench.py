#!/usr/bin/env python3
"""Headline benchmark: RAG queries/sec (whole node) + p50 end-to-end latency,
Llama-3-8B (BASELINE.json config 2: bge-base embedder + Llama-3-8B bf16 TP=1 per
MI355X, 100k-document synthetic corpus).

One rank per GPU (DP replicas, weak scaling: per-GPU batch fixed as N grows).  A
step = one batch of ``--batch`` concurrent ``/agent_rag`` requests per GPU through
the full pipeline of ``Minimal_RAG/Program.cs:106-316``:

  bge-base query embeddings -> cosine top-6 over the HBM-resident corpus (HIP kNN)
  -> citation gating -> evidence JSON prompt -> Llama-3-8B (flash prefill, prefix
  cache, hipGraph decode, greedy, ``--max-new-tokens`` per request) -> JSON
  extraction -> typed tool call -> RAG gating -> (fake) Kubernetes action.

Weights are random-init (no checkpoints offline), data synthetic; random weights
never emit EOS on purpose, so every request generates exactly ``--max-new-tokens``
tokens (the reference's tool call is ~20-60 tokens; default 48).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node 8 bench.py --gpus 8 ...
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=128,
                    help="requests per GPU per step (= in-flight concurrency in continuous mode)")
    ap.add_argument("--mode", choices=["continuous", "batch"], default="continuous",
                    help="continuous: closed-loop load, `batch` requests always in flight, a step = `batch` "
                         "completions; batch: a step = one synchronous batch of `batch` requests")
    ap.add_argument("--docs", type=int, default=100_000, help="synthetic runbook documents in the knowledge base")
    ap.add_argument("--max-new-tokens", type=int, default=48)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--embedder", default="bge-base")
    ap.add_argument("--kv-gb", type=float, default=48.0)
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="token budget per engine step (default: 4096 continuous, 65536 batch)")
    ap.add_argument("--admit-chunk", type=int, default=8,
                    help="continuous mode: requests retrieved + admitted together (batched embed/kNN)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def log(rank, *a):
    if rank == 0:
        print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    t_setup = time.perf_counter()

    # ---- corpus chunks (CPU, before any GPU init: the pool forks)
    from llm_kubernetes_minikube_sharp4dev_amd.rag.corpus import build_chunks

    ncpu = os.cpu_count() or 8
    chunks = build_chunks(args.docs, args.seed, workers=max(1, min(16, ncpu // max(1, world))))
    log(rank, f"corpus: {args.docs} docs -> {len(chunks)} chunks ({time.perf_counter() - t_setup:.1f}s)")

    import torch
    import torch.distributed as dist

    from llm_kubernetes_minikube_sharp4dev_amd.agent.rag_pipeline import RagAgentPipeline
    from llm_kubernetes_minikube_sharp4dev_amd.config import Config
    from llm_kubernetes_minikube_sharp4dev_amd.engine.embed_engine import EmbeddingEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.k8s.fake import FakeCluster
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder, build_encoder
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer
    from llm_kubernetes_minikube_sharp4dev_amd.ops import _ext
    from llm_kubernetes_minikube_sharp4dev_amd.rag.embedder import LocalEmbedder
    from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagChunk, RagIndex
    from llm_kubernetes_minikube_sharp4dev_amd.rag.synthetic import make_queries

    assert torch.cuda.is_available(), "bench.py needs an MI355X"
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    _ext.lib()  # fail loudly if the HIP library is not built
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    cfg = Config()
    tok = builtin_tokenizer()

    # ---- embedder + index build (embedding work sharded over ranks, all-gather over RCCL)
    enc = build_encoder(args.embedder, device=dev, seed=args.seed)
    emb_engine = EmbeddingEngine(enc, tok, name=args.embedder, max_tokens_per_batch=131072)
    n = len(chunks)
    per = (n + world - 1) // world
    lo, hi = min(n, rank * per), min(n, (rank + 1) * per)
    t0 = time.perf_counter()
    mine = emb_engine.embed([c[2] for c in chunks[lo:hi]])
    full = torch.zeros((per * world, enc.cfg.hidden), dtype=torch.bfloat16, device=dev)
    shard = torch.zeros((per, enc.cfg.hidden), dtype=torch.bfloat16, device=dev)
    shard[: hi - lo] = mine.to(torch.bfloat16)
    if world > 1:
        dist.all_gather_into_tensor(full, shard)
    else:
        full = shard
    corpus = full[:n].contiguous()
    torch.cuda.synchronize()
    t_index = time.perf_counter() - t0
    index = RagIndex(LocalEmbedder(emb_engine), backend="gpu", device=str(dev))
    index.chunks = [RagChunk(i, s, t) for i, s, t in chunks]
    index.set_gpu_corpus(corpus)
    del chunks
    log(rank, f"index: {n} chunks x {enc.cfg.hidden} embedded in {t_index:.1f}s")

    # ---- generator + engine
    t0 = time.perf_counter()
    llm = build_decoder(args.model, device=dev, seed=args.seed)
    torch.cuda.synchronize()
    log(rank, f"{args.model} random-init in {time.perf_counter() - t0:.1f}s")
    # continuous: ~4k-token steps keep most steps mixed (decode rows ride on the prefill
    # GEMMs) without starving decode (profiles/r1_sched_sweep.md)
    mbt = args.max_batched_tokens or (4096 if args.mode == "continuous" else 65536)
    engine = LLMEngine(llm, tok, block_size=16, max_model_len=8192, max_num_seqs=max(args.batch, 64),
                       max_num_batched_tokens=mbt,
                       enable_prefix_caching=not args.no_prefix_cache, use_graphs=not args.no_graphs,
                       kv_cache_gb=args.kv_gb, eos_ids=set())
    k8s = FakeCluster.default()
    pipe = RagAgentPipeline(index, engine, tok, k8s, cfg)
    params = SamplingParams.greedy(args.max_new_tokens, ignore_eos=True)
    if not args.no_graphs:
        engine.runner.capture_all(max_batch=max(args.batch, 1))

    qcount = [0]

    def next_queries(n):
        qcount[0] += 1
        return make_queries(n, seed=args.seed * 100003 + rank * 7919 + qcount[0])

    def step(i):
        if args.mode == "batch":
            return pipe.run_batch(next_queries(args.batch), params)
        return pipe.run_continuous(next_queries, params, args.batch, args.batch)

    if args.mode == "continuous":
        from llm_kubernetes_minikube_sharp4dev_amd.agent.rag_pipeline import ContinuousLoad

        # warm-up fills the pipeline and reaches the steady prefill/decode mix; the timed
        # window continues the same stream (in-flight requests carry over)
        load = ContinuousLoad(pipe, next_queries, params, args.batch, admit_chunk=args.admit_chunk)

        def run_steps(n):
            return load.run(n * args.batch)

        run_steps(max(args.warmup, 1))
    else:
        for w in range(args.warmup):
            step(-1 - w)
    log(rank, f"setup {time.perf_counter() - t_setup:.1f}s; timing {args.steps} steps x {args.batch} req/GPU")

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    engine.step_trace = []
    t0 = time.perf_counter()
    results = []
    step_times = []
    if args.mode == "continuous":
        results.extend(run_steps(args.steps))
    else:
        for i in range(args.steps):
            ts = time.perf_counter()
            results.extend(step(i))
            step_times.append(time.perf_counter() - ts)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    trace, engine.step_trace = engine.step_trace, None
    if args.mode == "continuous":
        load.drain()

    lat = [r.timings.get("e2e_s", 0.0) for r in results]
    ptok = [r.prompt_tokens for r in results if r.prompt_tokens]
    pre = [r.timings.get("cached_prefix_tokens", 0) for r in results if r.timings]
    gen = [r.output_tokens for r in results]
    stats = torch.tensor([elapsed, float(len(results)), float(sum(ptok)), float(len(ptok)), float(sum(gen))],
                         dtype=torch.float64, device=dev)
    lat_t = torch.tensor(lat, dtype=torch.float64, device=dev)
    if world > 1:
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)
        alll = [torch.zeros_like(lat_t) for _ in range(world)]
        dist.all_gather(alll, lat_t)
        allst = torch.stack(allst).cpu()
        lat_all = torch.cat(alll).cpu().tolist()
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
        avg_prompt = float(allst[:, 2].sum() / max(1.0, float(allst[:, 3].sum())))
        statuses = {}
        for r in results:
            statuses[str(r.status)] = statuses.get(str(r.status), 0) + 1
        dec_only = [t for t in trace if t[0] == 0]
        mixed = [t for t in trace if t[0] > 0]
        step_mix = {
            "steps": len(trace),
            "decode_only_steps": len(dec_only), "decode_only_s": round(sum(t[2] for t in dec_only), 3),
            "mixed_steps": len(mixed), "mixed_s": round(sum(t[2] for t in mixed), 3),
            "avg_prefill_tokens_mixed": round(statistics.mean(t[0] for t in mixed), 1) if mixed else 0,
            "avg_decode_rows": round(statistics.mean(t[1] for t in trace), 1) if trace else 0,
        }
        tim = {k: statistics.mean(r.timings.get(k, 0.0) for r in results) for k in ("embed_s", "knn_s", "prompt_s",
                                                                                   "generate_s")}
        out = {
            "metric": "RAG queries/sec (whole node) + p50 end-to-end latency, Llama-3-8B",
            "value": round(qps, 3),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1000, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": f"synthetic ({args.docs} runbook docs -> {n} chunks; random-init weights)",
            "p50_latency_ms": round(p50, 1) if p50 is not None else None,
            "p90_latency_ms": round(p90, 1) if p90 is not None else None,
            "config": {
                "model": f"{args.model} (bf16, TP=1) + {args.embedder} embedder",
                "global_batch": args.batch * world,
                "seq_len": round(avg_prompt, 1),
                "parallelism": f"dp{world}",
                "load": (f"continuous batching, closed loop, {args.batch} requests in flight per GPU, "
                         f"step = {args.batch} completions" if args.mode == "continuous"
                         else f"synchronous batches of {args.batch}"),
                "max_batched_tokens": mbt,
                "corpus_chunks": n,
                "max_new_tokens": args.max_new_tokens,
                "decoding": "greedy, ignore_eos",
                "prefix_caching": not args.no_prefix_cache,
                "hip_graphs": not args.no_graphs,
                "avg_cached_prefix_tokens": round(statistics.mean(pre), 1) if pre else 0,
                "stage_means_s": {k: round(v, 4) for k, v in tim.items()},
                "step_mix_rank0": step_mix,
                "admit_chunk": args.admit_chunk if args.mode == "continuous" else None,
                "index_build_s": round(t_index, 2),
                "http_status_counts": statuses,
            },
        }
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
