#!/usr/bin/env python3
"""Row-tile choice of the prefill GEMM: gemm1w.hip at 256 / 192 / 128-row tiles (lk_gemm variants
3 / 4 / 5) vs the serving default (ops.linear's dispatch) vs hipBLASLt (F.linear), the Llama-3-8B
projections at the mixed-step row counts of the serving bench (prefill rows + ~105 decode rows),
weights cold (rotated copies past the 256 MB MALL), interleaved rounds, medians.

    python benchmarks/gemm_tiles.py [--ms 2664,2816,3328,4096] [--shapes O,down,QKV]
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

SHAPES = {"QKV": (6144, 4096), "O": (4096, 4096), "down": (4096, 14336), "gate_up": (28672, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1280,2304,2664,2816,3328,3840,4096,4200")
    ap.add_argument("--shapes", default="QKV,O,down")
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    L = ops.lib()
    torch.manual_seed(0)
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        n_cold = max(2, -(-(640 << 20) // (N * K * 2)))
        copies = [w] + [w.clone() for _ in range(n_cold - 1)]
        for M in [int(v) for v in a.ms.split(",")]:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            arms = {}
            for v, bm in ((3, 256), (4, 192), (5, 128)):
                if L.gemm_supported(M, N, K, 0, 256, 1, v):
                    arms[f"g1w{bm}"] = lambda c, v=v: L.gemm(x, c, None, 0, 256, out, v, 1)
            arms["default"] = lambda c: ops.linear(x, c)
            arms["lib"] = lambda c: F.linear(x, c)
            ref = (x.float() @ w.float().t())
            for k, f in arms.items():
                y = f(w).float()
                err = (y - ref).abs().max().item()
                assert err < 0.05 * ref.abs().max().item() + 0.02, (name, M, k, err)
            torch.cuda.synchronize()
            seq = copies[1:] + copies[:1]
            ts = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, f in arms.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for c in seq:
                        f(c)
                    e1.record()
                    e1.synchronize()
                    ts[k].append(e0.elapsed_time(e1) * 1e3 / len(seq))
            med = {k: statistics.median(v) for k, v in ts.items()}
            best = min((k for k in med if k.startswith("g1w")), key=med.get)
            parts = " ".join(f"{k} {v:.1f}" for k, v in med.items())
            print(f"{name:8s} M{M:5d} N{N:5d} K{K:5d} | {parts} us | best {best}: {med['lib'] / med[best]:.3f}x lib, "
                  f"{med['default'] / med[best]:.3f}x default", flush=True)
        del copies


if __name__ == "__main__":
    main()
