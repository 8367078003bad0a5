#!/usr/bin/env python3
"""Measure the prefill GEMM dispatch table for the shipped models on this MI355X: for every
projection (Llama-3-8B, Llama-3-70B, its TP=8 shard) and every 256-row M bucket from 512 to 8192
rows, time each candidate kernel (gemm.hip schedules 0-2 at 256 / 192-wide tiles with their
split-K, gemm1w.hip at 256 / 192 / 128-row tiles) with cold weights (ops.tune_gemm) and keep the
fastest.  Writes llm_kubernetes_minikube_sharp4dev_amd/ops/gemm_table_mi355x.json (the dispatch
default) and the per-candidate timings.

    python benchmarks/gemm_table.py [--out PATH] [--models llama-3-8b,llama-3-70b,llama-3-70b/tp8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models.configs import DECODERS, ENCODERS  # noqa: E402


def shapes(name: str):
    if name in ENCODERS:  # bias epilogues; M = the encoder's token-budget batches
        c = ENCODERS[name]
        return [(3 * c.hidden, c.hidden, 2), (c.hidden, c.hidden, 2), (c.intermediate, c.hidden, 3),
                (c.hidden, c.intermediate, 2)]
    base, _, tp = name.partition("/tp")
    c = DECODERS[base]
    t = int(tp) if tp else 1
    D = c.hidden // c.num_heads
    qkv = (c.num_heads // t + 2 * max(1, c.num_kv_heads // t)) * D
    return [(qkv, c.hidden, 0), (c.hidden, c.num_heads // t * D, 0), (2 * c.intermediate // t, c.hidden, 1),
            (c.hidden, c.intermediate // t, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=ops.GEMM_TABLE_FILE)
    ap.add_argument("--models", default="llama-3-8b,llama-3-70b,llama-3-70b/tp8")
    ap.add_argument("--min-m", type=int, default=512)
    ap.add_argument("--max-m", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=7)
    ap.add_argument("--encoders", default="bge-base", help="encoder presets, measured at --encoder-ms rows")
    ap.add_argument("--encoder-ms", default="16384,65536,131072")
    a = ap.parse_args()
    torch.manual_seed(0)
    t0 = time.time()
    ops._GEMM_TABLE.clear()
    timings = {}
    seen = set()
    for m in a.models.split(","):
        for N, K, epi in shapes(m):
            if (N, K, epi) in seen:
                continue
            seen.add((N, K, epi))
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            res = ops.tune_gemm([(w, epi)], a.max_m, a.min_m, iters=a.iters)
            for key, arms in res.items():
                timings[",".join(map(str, key))] = arms
                best = ops._GEMM_TABLE[key]
                print(f"{m:16s} M{key[0] * 256:5d} N{N:5d} K{K:5d} e{epi}: v{best[0]}/{best[1]}/k{best[2]} "
                      f"{arms[f'v{best[0]}/{best[1]}/k{best[2]}']:.1f} us  ({len(arms)} candidates)", flush=True)
            del w
    for m in [e for e in a.encoders.split(",") if e]:
        for N, K, epi in shapes(m):
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            res = ops.tune_gemm([(w, epi)], 0, iters=3, ms=[int(v) for v in a.encoder_ms.split(",")])
            for key, arms in res.items():
                timings[",".join(map(str, key))] = arms
                best = ops._GEMM_TABLE[key]
                print(f"{m:16s} M{key[0] * 256:6d} N{N:5d} K{K:5d} e{epi}: v{best[0]}/{best[1]}/k{best[2]} "
                      f"{arms[f'v{best[0]}/{best[1]}/k{best[2]}']:.1f} us  ({len(arms)} candidates)", flush=True)
            del w
    entries = sorted([list(k) + list(v) for k, v in ops._GEMM_TABLE.items()])
    doc = {"device": torch.cuda.get_device_name(), "arch": "gfx950", "cus": ops.device_cus(), "created": time.strftime("%Y-%m-%d"),
           "source": "benchmarks/gemm_table.py (ops.tune_gemm: cold weights, median of round-robin timings)",
           "key": "[M bucket = ceil(M / 256), N, K, epilogue, variant, column tile, splits]",
           "entries": entries, "timings_us": timings}
    with open(a.out, "w") as f:
        json.dump(doc, f, indent=0)
    print(f"{len(entries)} entries -> {a.out} in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
