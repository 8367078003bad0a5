#!/usr/bin/env python3
"""Per-tile fixed cost of the prefill GEMM (csrc/gemm.hip): time the kernel at fixed M, N
over a K sweep and fit t(K) = a + b * K per (schedule, tile width).  With one tile per CU
(M 4096 x N 4096 at BN 256 = 256 tiles) the intercept ``a`` is the launch + prologue +
epilogue cost of one tile; with several waves of tiles (N 28672: 7 per CU) it is paid per tile.

    python benchmarks/gemm_overhead.py [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd.ops import _ext  # noqa: E402


def timeit(fn, iters=15):
    ts = []
    for _ in range(3):
        fn()
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--Ns", default="4096,28672")
    ap.add_argument("--Ks", default="256,1024,2048,4096,8192,14336")
    ap.add_argument("--scheds", default="0,1,2")
    args = ap.parse_args()
    L = _ext.lib()
    dev = torch.device("cuda", 0)
    rows = []
    for N in [int(n) for n in args.Ns.split(",")]:
        for sched in [int(v) for v in args.scheds.split(",")]:
            pts = []
            for K in [int(k) for k in args.Ks.split(",")]:
                x = torch.randn(args.M, K, device=dev).bfloat16()
                w = torch.randn(N, K, device=dev).bfloat16() * 0.05
                out = torch.empty(args.M, N, device=dev, dtype=torch.bfloat16)
                us = timeit(lambda: L.gemm(x, w, None, 0, 256, out, sched))
                lib_us = timeit(lambda: torch.nn.functional.linear(x, w))
                tf = 2.0 * args.M * N * K / us / 1e6
                pts.append((K, us))
                r = {"M": args.M, "N": N, "K": K, "sched": sched, "us": round(us, 2), "tflops": round(tf, 1),
                     "lib_us": round(lib_us, 2)}
                rows.append(r)
                print(json.dumps(r), flush=True)
                del x, w, out
            # least-squares fit over K >= 1024
            fit = [(k, t) for k, t in pts if k >= 1024]
            n = len(fit)
            if n < 2:
                continue
            mk = sum(k for k, _ in fit) / n
            mt = sum(t for _, t in fit) / n
            b = sum((k - mk) * (t - mt) for k, t in fit) / sum((k - mk) ** 2 for k, _ in fit)
            a = mt - b * mk
            tiles = ((args.M + 255) // 256) * (N // 256)
            waves = -(-tiles // 256)
            steady = 2.0 * args.M * N / (b * 1e-6) / 1e15  # PF/s of the K-proportional part
            r = {"fit": True, "N": N, "sched": sched, "intercept_us": round(a, 2), "us_per_k64": round(b * 64, 3),
                 "tile_waves": waves, "intercept_per_tile_us": round(a / waves, 2), "steady_pflops": round(steady, 3)}
            rows.append(r)
            print(json.dumps(r), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
