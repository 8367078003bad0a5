#!/usr/bin/env python3
"""Stream-K vs plain tiling of the prefill GEMM at the serving step sizes (one MI355X).

For every Llama-3-8B projection at M = 256 t (the mixed-step row counts the scheduler
produces) the dispatch policy's own (schedule, column tile, splits) runs with the stream-K
policy off and on, interleaved in one process (rounds x variants, median), random operands.
Prints one JSON line per (M, projection) and a per-layer summary (sum over the 4 projections).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

PROJ = {"qkv": (6144, 4096, 0), "o": (4096, 4096, 0), "gate_up": (28672, 4096, 1), "down": (4096, 14336, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1280,2304,2816,3328,3840,4352,4864,5376,5888,6400,7168,8192")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=6)
    args = ap.parse_args()
    lib = ops.lib()
    torch.manual_seed(0)
    W = {k: torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02 for k, (n, kk, _) in PROJ.items()}
    per_layer = {}
    for M in [int(m) for m in args.ms.split(",")]:
        for name, (N, K, epi) in PROJ.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            times = {0: [], 1: []}
            for _ in range(args.rounds):
                for mode in (0, 1):
                    lib.gemm_streamk(mode)
                    for _ in range(2):
                        ops.gemm(x, W[name], None, epi)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(args.iters):
                        ops.gemm(x, W[name], None, epi)
                    b.record()
                    torch.cuda.synchronize()
                    times[mode].append(a.elapsed_time(b) * 1e3 / args.iters)
            lib.gemm_streamk(1)
            t0, t1 = statistics.median(times[0]), statistics.median(times[1])
            flops = 2.0 * M * N * K
            cfg = ops._gemm_default(M, N, K, epi)
            tiles = ((M + 255) // 256) * ((N // 2 // 128) if epi == 1 else N // cfg[1])
            print(json.dumps({"M": M, "proj": name, "cfg": cfg, "tiles": tiles, "plain_us": round(t0, 1),
                              "streamk_us": round(t1, 1), "speedup": round(t0 / t1, 3),
                              "plain_tflops": round(flops / t0 / 1e6, 1), "streamk_tflops": round(flops / t1 / 1e6, 1)}),
                  flush=True)
            pl = per_layer.setdefault(M, [0.0, 0.0])
            pl[0] += t0
            pl[1] += t1
    assert lib.gemm_streamk(-1) == 0, "a stream-K wait gave up"
    for M, (t0, t1) in per_layer.items():
        print(json.dumps({"M": M, "layer_plain_us": round(t0, 1), "layer_streamk_us": round(t1, 1),
                          "layer_speedup": round(t0 / t1, 3)}), flush=True)


if __name__ == "__main__":
    main()
