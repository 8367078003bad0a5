#!/usr/bin/env python3
"""Does launching a hipGraph block the host?  A decode-step-shaped graph (N small kernels,
~5-7 ms of GPU work) is replayed K times back to back; the host time of each replay() call is
compared with the GPU time.  A launch that returns only when the graph is nearly done leaves
the device idle while the host does the next step's work (the engine's per-step gap,
profiles/r3_gaps/).  Also times N eager launches of the same kernels.

    python benchmarks/graph_launch_probe.py [--kernels 290] [--size 2048]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", type=int, default=290)
    ap.add_argument("--size", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(a.size, a.size, device=dev, dtype=torch.bfloat16)
    w = torch.randn(a.size, a.size, device=dev, dtype=torch.bfloat16) * 0.01
    bufs = [torch.empty_like(x) for _ in range(2)]

    def body():
        y = x
        for i in range(a.kernels):
            y = torch.mm(y, w, out=bufs[i % 2])

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        body()
    torch.cuda.synchronize()
    res = {"env": {k: os.environ[k] for k in sorted(os.environ) if k.startswith(("DEBUG_", "HIP_", "AMD_", "GPU_"))},
           "kernels": a.kernels}
    for mode in ("graph", "eager"):
        host = []
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            t = time.perf_counter()
            if mode == "graph":
                g.replay()
            else:
                body()
            host.append((time.perf_counter() - t) * 1e3)
        e1.record()
        t = time.perf_counter()
        e1.synchronize()
        tail = (time.perf_counter() - t) * 1e3
        res[mode] = {"host_ms_per_launch_median": round(statistics.median(host), 3),
                     "host_ms_first": round(host[0], 3), "gpu_ms_per_rep": round(e0.elapsed_time(e1) / a.reps, 3),
                     "host_wait_after_last_launch_ms": round(tail, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
