#!/usr/bin/env python3
"""One GEMM shape, one implementation, N back-to-back launches (for rocprofv3 PMC passes).

    python benchmarks/gemm_one.py --M 4096 --N 4096 --K 14336 --impl ours|prod|lib [--epi none] [--bn 256]

ours = gemm.hip at the given tile / schedule; prod = the serving dispatch (ops.linear /
ops.linear_swiglu: the policy's tile, schedule, split and stream-K choice); lib = hipBLASLt
(F.linear; for SwiGLU the GEMM alone, without the silu * mul pass it would need).
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
    ap.add_argument("--impl", default="ours", help="ours (gemm.hip) | prod (serving dispatch) | lib (hipBLASLt)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--variant", type=int, default=0, help="K-loop schedule (0: 4-phase, 1: 2-phase)")
    a = ap.parse_args()
    x = torch.randn(a.M, a.K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.N, a.K, device="cuda", dtype=torch.bfloat16) * 0.02
    b = torch.randn(a.N, device="cuda", dtype=torch.bfloat16) if a.epi not in ("none", "swiglu") else None
    if a.impl == "ours":
        L = ops.lib()
        fn = lambda: L.gemm(x, w, b, EPI[a.epi], a.bn, None, a.variant)  # noqa: E731
    elif a.impl == "prod":
        if a.epi == "swiglu":
            fn = lambda: ops.linear_swiglu(x, w)  # noqa: E731
        else:
            act = {"none": None, "bias": None, "gelu": "gelu", "relu": "relu"}[a.epi]
            fn = lambda: ops.linear(x, w, b, act)  # noqa: E731
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
