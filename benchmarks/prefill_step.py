#!/usr/bin/env python3
"""GPU time of a prefill-only engine step on Llama-3-8B (random init, bf16), no profiler attached:
S fresh prompts of L tokens (M = S x L rows in one step, greedy, one output token each), the
step's GPU span from the engine's step trace (first kernel -> ids copy), median over back-to-back
steps -- the sustained, DVFS-steady cost of the prefill GEMM chain that the rocprofv3 kernel trace
(which idles the device between dispatches) can misstate.

Arms run as separate processes (each arm's env is read at import), interleaved A B A B:

    python benchmarks/prefill_step.py --arms "gemm1w:LK_GEMM1W=1,lib2:LK_GEMM_LIBRARY=2" [--rounds 2]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(a):
    sys.path.insert(0, ROOT)
    import torch

    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder

    torch.cuda.set_device(0)
    m = build_decoder(a.model, device="cuda", seed=0)
    M = a.seqs * a.len
    eng = LLMEngine(m, None, max_model_len=8192, max_num_seqs=a.decode_rows + a.seqs + 8,
                    max_num_batched_tokens=M + a.decode_rows, enable_prefix_caching=False, use_graphs=False,
                    kv_cache_gb=32, eos_ids=set(), token_align=1)
    eng.step_trace = []
    g = torch.Generator().manual_seed(1)
    gpu = []
    # --decode-rows R: R long-running requests (context --ctx) decode in every measured step beside
    # the new prompts' prefill, as in the serving bench's mixed steps
    for _ in range(a.decode_rows):
        eng.add_request(torch.randint(10, 120000, (a.ctx,), generator=g).tolist(),
                        SamplingParams.greedy(8000 - a.ctx, ignore_eos=True))
    while any(s.num_computed < len(s.prompt_ids) for s in eng.scheduler.running) or eng.scheduler.waiting:
        eng.step()
    eng.step_trace.clear()
    for it in range(a.warmup + a.iters):
        for _ in range(a.seqs):
            eng.add_request(torch.randint(10, 120000, (a.len,), generator=g).tolist(), SamplingParams.greedy(1))
        eng.step()  # the new prompts' prefill (+ one decode row per running request)
        while a.decode_rows == 0 and eng.has_work():
            eng.step()
        if it >= a.warmup:
            gpu += [t[7] for t in eng.step_trace if t[0] == M]
        eng.step_trace.clear()
    late = gpu[len(gpu) * 2 // 3:]  # the last third: after seconds of sustained load
    print(json.dumps({"median_ms": round(statistics.median(gpu) * 1e3, 3), "min_ms": round(min(gpu) * 1e3, 3),
                      "late_median_ms": round(statistics.median(late) * 1e3, 3), "steps": len(gpu)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arms", default="gemm1w:LK_GEMM1W=1,lib2:LK_GEMM_LIBRARY=2")
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--seqs", type=int, default=4)
    ap.add_argument("--len", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--decode-rows", type=int, default=0)
    ap.add_argument("--ctx", type=int, default=900)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        return child(a)
    arms = []
    for spec in a.arms.split(","):
        name, _, env = spec.partition(":")
        arms.append((name, dict(kv.split("=", 1) for kv in env.split() if kv)))
    res = {n: [] for n, _ in arms}
    for r in range(a.rounds):
        for name, env in arms:
            t0 = time.time()
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "--model", a.model,
                                  "--seqs", str(a.seqs), "--len", str(a.len), "--iters", str(a.iters),
                                  "--warmup", str(a.warmup), "--decode-rows", str(a.decode_rows), "--ctx", str(a.ctx)],
                                 env=dict(os.environ, **env), capture_output=True,
                                 text=True, timeout=600)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-4000:], flush=True)
                raise SystemExit(f"arm {name} failed rc={out.returncode}")
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[name].append(d["median_ms"])
            print(f"round {r} {name:10s} M={a.seqs * a.len}: step GPU median {d['median_ms']:.2f} ms "
                  f"(min {d['min_ms']:.2f}, last third {d['late_median_ms']:.2f}, {d['steps']} steps, "
                  f"{time.time() - t0:.0f} s)", flush=True)
    base = statistics.median(res[arms[0][0]])
    for name, v in res.items():
        print(f"{name:10s} {statistics.median(v):.2f} ms  ({base / statistics.median(v):.3f}x of {arms[0][0]})")


if __name__ == "__main__":
    main()
