#!/usr/bin/env python3
"""Cost of the prefill GEMM epilogues at the encoder's shapes (bge-base, K 768 / 3072, M 131072):
the same GEMM with no epilogue, bias, bias + GELU, bias + ReLU, timed back to back (hot weights,
medians of interleaved rounds).  The GELU-minus-bias difference is the erf epilogue's cost.

    python benchmarks/epi_cost.py [--M 131072]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=131072)
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    L = ops.lib()
    for N, K in ((3072, 768), (2304, 768), (768, 3072)):
        x = torch.randn(a.M, K, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        b = torch.randn(N, device="cuda", dtype=torch.bfloat16)
        out = torch.empty(a.M, N, device="cuda", dtype=torch.bfloat16)
        arms = {e: (lambda e=e: L.gemm(x, w, None if e == 0 else b, e, 256, out, 3, 1)) for e in (0, 2, 3, 4)}
        for f in arms.values():
            f()
        torch.cuda.synchronize()
        ts = {e: [] for e in arms}
        for _ in range(a.rounds):
            for e, f in arms.items():
                s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(5):
                    f()
                t.record()
                t.synchronize()
                ts[e].append(s.elapsed_time(t) * 1e3 / 5)
        med = {e: statistics.median(v) for e, v in ts.items()}
        tf = 2 * a.M * N * K / 1e12
        print(f"M{a.M} N{N} K{K}: " + "  ".join(f"{ {0: 'none', 2: 'bias', 3: 'gelu', 4: 'relu'}[e]} {v:.1f} us "
                                                   f"({tf / (v * 1e-6) / 1e3:.2f} PF/s)" for e, v in med.items()), flush=True)


if __name__ == "__main__":
    main()
