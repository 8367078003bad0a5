#!/usr/bin/env python3
"""Decode-regime GEMM routing data: for every projection of the served models (Llama-3-8B,
Llama-3-70B TP=1, the 70B TP=8 rank shard, the LM heads) and decode batch sizes M 64..256,
time the weight-streaming kernel (csrc/skinny_gemm.hip ``ws``), the prefill kernel
(csrc/gemm.hip with the dispatch policy's tile / split-K) and hipBLASLt, with COLD weights
(each launch reads the next of enough copies to overflow the 256 MB MALL, as in a decode
step) and back-to-back launches (as in a captured decode graph).  ops._decode_gemm_kind's
rule is checked against the fastest arm.

    python benchmarks/decode_route.py [--json out.json] [--ms 64,128,160,192,224,256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

SHAPES = [  # (name, N, K, swiglu)
    ("8b qkv", 6144, 4096, False), ("8b o", 4096, 4096, False), ("8b gate_up", 28672, 4096, True),
    ("8b down", 4096, 14336, False), ("8b lm_head", 128256, 4096, False),
    ("70b qkv", 10240, 8192, False), ("70b o", 8192, 8192, False), ("70b gate_up", 57344, 8192, True),
    ("70b down", 8192, 28672, False), ("70b lm_head", 128256, 8192, False),
    ("70b/tp8 qkv", 1280, 8192, False), ("70b/tp8 o", 8192, 1024, False), ("70b/tp8 gate_up", 7168, 8192, True),
    ("70b/tp8 down", 8192, 3584, False), ("70b/tp8 lm_head", 16128, 8192, False),
]
REPS = 12


def run_arm(fn, copies, x):
    for i in range(3):
        fn(x, copies[i % len(copies)])
    torch.cuda.synchronize()
    best = None
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(REPS):
            fn(x, copies[i % len(copies)])
        b.record()
        b.synchronize()
        t = a.elapsed_time(b) * 1e3 / REPS
        best = t if best is None else min(best, t)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--ms", default="64,128,160,192,224,256")
    ap.add_argument("--only", default=None, help="substring filter on the shape name")
    a = ap.parse_args()
    L = ops.lib()
    rows = []
    for name, N, K, sw in SHAPES:
        if a.only and a.only not in name:
            continue
        ncopy = max(2, -(-(640 << 20) // (N * K * 2)))
        copies = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
        for M in (int(m) for m in a.ms.split(",")):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            rec = {"shape": name, "M": M, "N": N, "K": K, "swiglu": sw, "MB": round(N * K * 2 / 2**20, 1)}
            arms = {}
            if M <= 256 and (not sw or (N // 2) % 64 == 0):
                arms["ws"] = lambda x, w: L.ws_linear(x, w, sw)
            cfg = ops._gemm_default(M, N, K, 1 if sw else 0)
            if cfg is not None and L.gemm_supported(M, N, K, 1 if sw else 0, cfg[1], cfg[2]):
                arms["gemm"] = lambda x, w, cfg=cfg: L.gemm(x, w, None, 1 if sw else 0, cfg[1], None, cfg[0], cfg[2])
            if sw:
                arms["hipblaslt"] = lambda x, w: ops.silu_mul(torch.nn.functional.linear(x, w))
            else:
                arms["hipblaslt"] = lambda x, w: torch.nn.functional.linear(x, w)
            for k, fn in arms.items():
                rec[k + "_us"] = round(run_arm(fn, copies, x), 2)
            own = {k: rec[k + "_us"] for k in ("ws", "gemm") if k + "_us" in rec}
            rec["best_own"] = min(own, key=own.get) if own else None
            kind = ops._decode_gemm_kind(x, copies[0], sw)
            rec["policy"] = kind or "gemm"
            pol_us = own.get("ws" if kind == "ws" else "gemm")
            rec["policy_vs_hipblaslt"] = round(rec["hipblaslt_us"] / pol_us, 3) if pol_us else None
            rec["policy_vs_best_own"] = round(min(own.values()) / pol_us, 3) if pol_us else None
            if pol_us:
                rec["policy_TBps"] = round(N * K * 2 / pol_us / 1e6, 2)
            print(json.dumps(rec), flush=True)
            rows.append(rec)
        del copies
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"note": "cold weights, back-to-back launches, best of 3 x 12", "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
