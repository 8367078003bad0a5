#!/usr/bin/env python3
"""Weight-streaming GEMM probe: K-step rotation per column tile (0 = off) on the Llama-3-8B
decode shapes, with COLD weights (a ring of copies larger than the 256 MB Infinity Cache,
as in a real decode step where 15 GB of other weights pass between two uses of one)."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

L = ops.lib()
SHAPES = [(6144, 4096, False), (4096, 4096, False), (28672, 4096, True), (4096, 14336, False)]


def bench(M, N, K, sw, rot, cold=True, iters=24):
    copies = max(2, (1 << 30) // (N * K * 2)) if cold else 1
    ws = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) for _ in range(copies)]
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    L.ws_set_rot(rot)
    for i in range(4):
        L.ws_linear(x, ws[i % copies], sw)
    torch.cuda.synchronize()
    ts = []
    for i in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        L.ws_linear(x, ws[i % copies], sw)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    L.ws_set_rot(-1)
    del ws
    return statistics.median(ts)


for M in (64, 128, 256):
    for N, K, sw in SHAPES:
        if sw and M > 160:
            continue
        r = {f"rot{rot}": round(bench(M, N, K, sw, rot), 1) for rot in (0, 1, 5, -1)}
        r["hot_rot0"] = round(bench(M, N, K, sw, 0, cold=False), 1)
        bn, S = L.ws_plan(M, N, K, sw)
        print(json.dumps({"case": f"M{M} N{N} K{K}{' swiglu' if sw else ''} BN{bn} S{S}", **r,
                          "GB/s_rot0": round(N * K * 2 / r["rot0"] / 1e3, 0)}), flush=True)
