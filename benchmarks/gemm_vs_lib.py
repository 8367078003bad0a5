#!/usr/bin/env python3
"""Prefill GEMM (the serving dispatch: ops.linear / ops.linear_swiglu) vs hipBLASLt (F.linear,
+ the silu_mul pass a SwiGLU projection needs after it) at the Llama-3-8B projections, with the
weights hot (one copy, MALL-resident where it fits) and cold (each launch reads the next of
enough copies to overflow the 256 MB MALL -- a serving step reads every layer's weights once),
interleaved rounds in one process, medians.

    python benchmarks/gemm_vs_lib.py [--ms 2048,4096,8192] [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

SHAPES = [("QKV", 6144, 4096, False), ("O", 4096, 4096, False), ("gate_up+SwiGLU", 28672, 4096, True),
          ("down", 4096, 14336, False)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="4096")
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    L = ops.lib()
    lines = ["| projection | M | weights | ours us | hipBLASLt us | ours / lib speed | ours TF/s |",
             "|---|---|---|---|---|---|---|"]
    for name, N, K, sw in SHAPES:
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        n_cold = max(2, -(-(640 << 20) // (N * K * 2)))
        copies = [w] + [w.clone() for _ in range(n_cold - 1)]
        for M in [int(v) for v in a.ms.split(",")]:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            arms = {
                "ours": (lambda c: ops.linear_swiglu(x, c)) if sw else (lambda c: ops.linear(x, c)),
                "lib": (lambda c: L.silu_mul(F.linear(x, c))) if sw else (lambda c: F.linear(x, c)),
            }
            for fn in arms.values():
                fn(w)
            torch.cuda.synchronize()
            for temp, seq in (("hot", [w] * 8), ("cold", copies[1:] + copies[:1])):
                ts = {k: [] for k in arms}
                for _ in range(a.rounds):
                    for k, fn in arms.items():
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        for c in seq:
                            fn(c)
                        e1.record()
                        e1.synchronize()
                        ts[k].append(e0.elapsed_time(e1) * 1e3 / len(seq))
                med = {k: statistics.median(v) for k, v in ts.items()}
                lines.append(f"| {name} | {M} | {temp} | {med['ours']:.1f} | {med['lib']:.1f} | "
                             f"{med['lib'] / med['ours']:.3f}x | {2 * M * N * K / (med['ours'] * 1e-6) / 1e12:.0f} |")
                print(lines[-1], flush=True)
        del copies
    if a.md:
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
