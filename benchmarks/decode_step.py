#!/usr/bin/env python3
"""One hipGraph-captured Llama-3-8B decode step at the RAG operating point (B rows,
~`ctx` tokens of context each, a shared `prefix`-token system prompt), timed with HIP
events; run under ``rocprofv3 --kernel-trace --stats`` for the per-kernel split.

    python benchmarks/decode_step.py [--batch 120] [--ctx 950] [--prefix 288] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import LLMEngine  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=120)
    ap.add_argument("--ctx", type=int, default=950)
    ap.add_argument("--prefix", type=int, default=288)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = build_decoder(a.model, device=dev)
    eng = LLMEngine(m, None, max_model_len=4096, max_num_seqs=256, kv_cache_gb=40, eos_ids=set())
    eng.runner.capture_all(max_batch=a.batch, variants=(True,))
    g = torch.Generator().manual_seed(0)
    shared = torch.randint(10, 100000, (a.prefix,), generator=g).tolist()
    seqs = []
    first = shared + torch.randint(10, 100000, (a.ctx - a.prefix,), generator=g).tolist()
    eng.generate([first], SamplingParams.greedy(1))  # publish the shared prefix blocks
    for i in range(a.batch):
        tail = torch.randint(10, 100000, (a.ctx - a.prefix,), generator=g).tolist()
        seqs.append(eng.add_request(shared + tail, SamplingParams.greedy(10_000, ignore_eos=True)))
    while any(not s.output_ids for s in seqs):  # prefill everything (prefix cache shares the prompt)
        eng.step()
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    times = []
    for _ in range(a.iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        eng.step()
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    times.sort()
    print(json.dumps({"case": f"decode step {a.model} B{a.batch} ctx{a.ctx} prefix{a.prefix}",
                      "ms_median": round(times[len(times) // 2], 3), "ms_min": round(times[0], 3),
                      "shared_prefix_tokens": min(s.num_cached_prefix for s in seqs[1:]) if a.batch > 1 else 0}))


if __name__ == "__main__":
    main()
