#!/usr/bin/env python3
"""Probe: does splitting one prefill GEMM into row halves on two HIP streams desynchronise the
tile-wave write bursts (profiles/r2_gemm_tile_overhead.md) enough to pay?  Times, per shape,
the single launch vs the two row halves launched on two streams (event-joined), cold weights.

    python benchmarks/gemm_2stream.py [--ms 4096,8192]
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

SHAPES = [(6144, 4096, 0), (4096, 4096, 0), (28672, 4096, 1), (4096, 14336, 0)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="4096,8192")
    ap.add_argument("--rounds", type=int, default=11)
    ap.add_argument("--parts", default="2,4")
    a = ap.parse_args()
    L = ops.lib()
    dev = torch.device("cuda", 0)
    main_s = torch.cuda.current_stream()
    sides = [torch.cuda.Stream(dev) for _ in range(3)]
    for M in [int(v) for v in a.ms.split(",")]:
        for N, K, epi in SHAPES:
            x = torch.randn(M, K, device=dev).bfloat16()
            nco = max(1, -(-(600 << 20) // (N * K * 2)))
            ws = [(torch.randn(N, K, device=dev) * 0.02).bfloat16() for _ in range(nco)]
            rot = [0]

            def wn():
                rot[0] = (rot[0] + 1) % nco
                return ws[rot[0]]
            cfg = ops._gemm_default(M, N, K, epi)
            n_out = N // 2 if epi == 1 else N
            out = torch.empty(M, n_out, device=dev, dtype=torch.bfloat16)

            def single():
                L.gemm(x, wn(), None, epi, cfg[1], out, cfg[0], cfg[2])

            def split(p):
                w = wn()
                rows = M // p
                ev = torch.cuda.Event()
                ev.record(main_s)
                joins = []
                for i in range(p):
                    st = main_s if i == 0 else sides[i - 1]
                    if i:
                        st.wait_event(ev)
                    with torch.cuda.stream(st):
                        L.gemm(x[i * rows:(i + 1) * rows], w, None, epi, cfg[1], out[i * rows:(i + 1) * rows], cfg[0],
                               cfg[2])
                    if i:
                        e = torch.cuda.Event()
                        e.record(st)
                        joins.append(e)
                for e in joins:
                    main_s.wait_event(e)

            fns = {"single": single}
            for p in [int(v) for v in a.parts.split(",")]:
                if M % (256 * p) == 0:
                    fns[f"split{p}"] = (lambda p=p: split(p))
            ts = {k: [] for k in fns}
            for k, f in fns.items():
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
            print(json.dumps({"M": M, "N": N, "K": K, "epi": epi, **{k: round(statistics.median(v), 1) for k, v in ts.items()}}),
                  flush=True)
            del x, ws, out


if __name__ == "__main__":
    main()
