#!/usr/bin/env python3
"""Weight-streaming GEMM (csrc/skinny_gemm.hip) at decode-sized M: the one-ring kernel vs the
loader-wave kernel (and hipBLASLt, F.linear + silu_mul for SwiGLU, as a reference), Llama-3-8B projections, weights arriving from HBM (each launch reads the next
of enough copies to overflow the 256 MB MALL, as in a decode step), launches back to back,
interleaved rounds, medians.  Reports us and the weight stream rate (W bytes / time).

    python benchmarks/ws_variant_ab.py [--md out.md]
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
    ap.add_argument("--ms", default="64,128,192,256")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    L = ops.lib()
    lines = ["| projection | M | plan BN/S | ring us | loader us | ring TB/s | loader TB/s | loader speedup | hipBLASLt us |",
             "|---|---|---|---|---|---|---|---|---|"]
    for name, N, K, sw in SHAPES:
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        copies = [w] + [w.clone() for _ in range(max(1, -(-(640 << 20) // (N * K * 2)) - 1))]
        for M in [int(v) for v in a.ms.split(",")]:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            ts = {0: [], 1: [], "lib": []}
            lib = (lambda c: L.silu_mul(F.linear(x, c))) if sw else (lambda c: F.linear(x, c))
            for v in (0, 1):
                L.ws_set_variant(M, N, K, sw, v)
                L.ws_linear(x, copies[0], sw)
            lib(copies[0])
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for v in (0, 1, "lib"):
                    if v != "lib":
                        L.ws_set_variant(M, N, K, sw, v)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for c in copies[1:] + copies[:1]:
                        lib(c) if v == "lib" else L.ws_linear(x, c, sw)
                    e1.record()
                    e1.synchronize()
                    ts[v].append(e0.elapsed_time(e1) * 1e3 / len(copies))
            L.ws_set_variant(M, N, K, sw, -1)
            med = {v: statistics.median(t) for v, t in ts.items()}
            bn, S = L.ws_plan(M, N, K, sw)
            tb = {v: N * K * 2 / (med[v] * 1e-6) / 1e12 for v in med}
            lines.append(f"| {name} | {M} | {bn}/{S} | {med[0]:.1f} | {med[1]:.1f} | {tb[0]:.2f} | {tb[1]:.2f} | "
                         f"{med[0] / med[1]:.3f}x | {med['lib']:.1f} |")
            print(lines[-1], flush=True)
        del copies
    if a.md:
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
