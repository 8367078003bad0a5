#!/usr/bin/env python3
"""One GEMM shape, one implementation, N back-to-back launches (for rocprofv3 PMC passes).

    python benchmarks/gemm_one.py --M 4096 --N 4096 --K 14336 --impl ours|lib [--epi none] [--bn 256]
"""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

EPI = {"none": 0, "swiglu": 1, "bias": 2, "gelu": 3, "relu": 4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=14336)
    ap.add_argument("--epi", default="none")
    ap.add_argument("--bn", type=int, default=256)
    ap.add_argument("--impl", default="ours", help="ours (gemm.hip) | 4w (gemm4w.hip) | lib (hipBLASLt)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--variant", type=int, default=0, help="K-loop schedule (0: 4-phase, 1: 2-phase)")
    a = ap.parse_args()
    x = torch.randn(a.M, a.K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.N, a.K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(a.N, device="cuda", dtype=torch.bfloat16) if a.epi not in ("none", "swiglu") else None
    if a.impl == "ours":
        L = ops.lib()
        fn = lambda: L.gemm(x, w, b, EPI[a.epi], a.bn, None, a.variant)  # noqa: E731
    elif a.impl == "4w":  # csrc/gemm4w.hip
        L = ops.lib()
        fn = lambda: L.gemm4w(x, w, b, EPI[a.epi])  # noqa: E731
    else:
        fn = lambda: F.linear(x, w, b)  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        fn()
    e.record()
    e.synchronize()
    print(f"{a.impl} M{a.M} N{a.N} K{a.K} {a.epi}: {s.elapsed_time(e) / a.iters * 1e3:.1f} us/launch")


if __name__ == "__main__":
    main()
