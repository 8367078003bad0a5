#!/usr/bin/env python3
"""A/B of two builds of the prefill GEMM on one box: times each shape's dispatch-policy config
(cold weights) with the in-tree library, or with another build of the same extension loaded
from ``--lib`` (e.g. the previous commit's _C .so; pybind11 cannot hold both in one process,
so run the arms as alternating processes).

    python benchmarks/gemm_ab_lib.py [--lib path/to/_C.so] --tag old|new
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

SHAPES = {"llama": [(6144, 4096, 0), (4096, 4096, 0), (28672, 4096, 1), (4096, 14336, 0)],
          "bge": [(2304, 768, 2), (768, 768, 2), (3072, 768, 3), (768, 3072, 2)]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=None)
    ap.add_argument("--tag", default="new")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--sets", default="llama:4096,8192;bge:32768,131072")
    a = ap.parse_args()
    if a.lib:
        spec = importlib.util.spec_from_file_location("_C", a.lib)
        L = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(L)
    else:
        L = ops.lib()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for part in a.sets.split(";"):
        name, ms = part.split(":")
        for M in [int(v) for v in ms.split(",")]:
            for N, K, epi in SHAPES[name]:
                x = torch.randn(M, K, device=dev).bfloat16()
                nco = max(1, -(-(600 << 20) // (N * K * 2)))
                ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(nco)]
                b = torch.randn(N, device=dev).bfloat16() if epi >= 2 else None
                rot = [0]

                def wn():
                    rot[0] = (rot[0] + 1) % nco
                    return ws[rot[0]]
                cfg = ops._gemm_default(M, N, K, epi)
                fns = {a.tag: (lambda: L.gemm(x, wn(), b, epi, cfg[1], None, cfg[0], cfg[2]))}
                y = L.gemm(x, ws[0], b, epi, cfg[1], None, cfg[0], cfg[2])
                chk = float(y[:64].float().sum())  # same operands in both arms: equal sums = same result
                ts = {k: [] for k in fns}
                for f in fns.values():
                    f()
                torch.cuda.synchronize()
                for _ in range(a.rounds):
                    for k, f in fns.items():
                        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        s.record()
                        f()
                        e.record()
                        e.synchronize()
                        ts[k].append(s.elapsed_time(e) * 1e3)
                med = {k: round(statistics.median(v), 1) for k, v in ts.items()}
                print(json.dumps({"M": M, "N": N, "K": K, "epi": epi, "cfg": list(cfg), **med, "checksum": chk}), flush=True)
                del x, ws, b


if __name__ == "__main__":
    main()
