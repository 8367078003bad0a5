#!/usr/bin/env python3
"""Batch-1 decode projections: the decode GEMV (csrc/gemv_decode.hip, with its prologue /
epilogue) against the weight-streaming path it replaces (split-K GEMM + its reduce / norm / RoPE
consumer), weights cold (each launch reads the next of enough weight copies to overflow the
256 MB MALL), medians of interleaved rounds, per workgroup-count setting of the GEMV.  Prints
microseconds and TB/s of weight bytes.

    python benchmarks/gemv_bench.py [--m 1] [--wgs 256,512,1024,2048] [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

# name: (N, K, gemv mode, norm prologue)
SHAPES = {"qkv": (6144, 4096, 3, True), "o": (4096, 4096, 1, False), "gate_up": (28672, 4096, 2, True),
          "down": (4096, 14336, 1, False), "lm_head": (128256, 4096, 0, False)}


def timed(fn, copies, iters=20):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn(copies[0])
    torch.cuda.synchronize()
    ev[0].record()
    for i in range(iters):
        fn(copies[i % len(copies)])
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--wgs", default="256,512,768,1024,2048")
    ap.add_argument("--shapes", default="qkv,o,gate_up,down,lm_head")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--md", default=None)
    ap.add_argument("--ksplit", default="1,0", help="GEMV two waves per pair on long-K shapes: arms")
    a = ap.parse_args()
    L = ops.lib()
    M, dev, eps = a.m, "cuda", 1e-5
    Hq, Hkv, D, BS = 32, 8, 128, 16
    cos_sin = ops.rope_cos_sin(8192, D, 500000.0, None, device=dev)
    pos = torch.full((M,), 700, dtype=torch.int32, device=dev)
    slots = torch.arange(M, dtype=torch.int32, device=dev) + 5 * BS
    kc = torch.zeros(64, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    arms = [(w, pf) for pf in a.ksplit.split(",") for w in a.wgs.split(",")]
    lines = ["| shape | MB | ws path us (TB/s) | " + " | ".join(f"gemv wgs {w} ksplit {pf} us (TB/s)" for w, pf in arms) + " |",
             "|---|---|---|" + "---|" * len(arms)]
    for name in a.shapes.split(","):
        N, K, mode, norm = SHAPES[name]
        wb = N * K * 2
        copies = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
                  for _ in range(max(2, -(-600 * 2**20 // wb)))]
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        res = torch.randn(M, N if mode == 1 else K, device=dev, dtype=torch.bfloat16)
        g = torch.ones(K, device=dev, dtype=torch.bfloat16)
        gn = torch.ones(N, device=dev, dtype=torch.bfloat16)

        def ws(w):  # the weight-streaming step this GEMV replaces
            if mode == 3:
                xn = ops.rmsnorm(res, g, eps)
                ops.linear_rope_kv(xn, w, pos, cos_sin, Hq, Hkv, D, kc, vc, slots, False, False)
            elif mode == 2:
                xn = ops.rmsnorm(res, g, eps)
                ops.linear_swiglu(xn, w)
            elif mode == 1:
                ops.linear_add_rmsnorm(x, w, res, gn, eps)
            else:
                ops.linear(x, w)

        def gv(w):
            if mode == 3:
                L.gemv_decode(3, res, w, g, eps, None, pos, cos_sin, Hq, Hkv, D, kc, vc, slots, False)
            elif mode == 2:
                L.gemv_decode(2, res, w, g, eps)
            elif mode == 1:
                L.gemv_decode(1, x, w, None, eps, res)
            else:
                L.gemv_decode(0, x, w)

        arms = [(w, pf) for pf in a.ksplit.split(",") for w in a.wgs.split(",")]
        t_ws, t_gv = [], {arm: [] for arm in arms}
        for _ in range(a.rounds):
            t_ws.append(timed(ws, copies))
            for wg, pf in t_gv:
                L.gemv_set_wgs(int(wg))
                L.gemv_set_ksplit(pf == "1")
                t_gv[(wg, pf)].append(timed(gv, copies))
        L.gemv_set_wgs(0)
        L.gemv_set_ksplit(True)
        mb = wb / 2**20

        def fmt(ts):
            us = statistics.median(ts)
            return f"{us:.1f} ({wb / us / 1e6:.2f})"

        lines.append(f"| {name} | {mb:.0f} | {fmt(t_ws)} | " + " | ".join(fmt(t_gv[w]) for w in t_gv) + " |")
        print(lines[-1], flush=True)
        del copies
        torch.cuda.empty_cache()
    out = "\n".join(lines)
    print(out)
    if a.md:
        with open(a.md, "w") as f:
            f.write(f"M = {M}, weights cold, median of {a.rounds} interleaved rounds x 20 launches\n\n{out}\n")


if __name__ == "__main__":
    main()
