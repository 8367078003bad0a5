#!/usr/bin/env python3
"""Does PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution search) beat the
default hipBLASLt heuristic on the Llama-3-8B projection shapes?  Times each shape
with the default heuristic, then with TunableOp tuning enabled (results written to
gpurun_out/tunableop_results.csv)."""
import json
import os
import statistics
import sys

import torch

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
MS = [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else ["8192", "4096", "128"])]


def timeit(fn, iters=20):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return statistics.median(ts)


def run(tag):
    out = {}
    for M in MS:
        for N, K in SHAPES:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
            t = timeit(lambda: torch.nn.functional.linear(x, w))
            out[f"M{M} N{N} K{K}"] = t
            print(json.dumps({"tag": tag, "shape": f"M{M} N{N} K{K}", "us": round(t * 1e6, 1),
                              "TFLOP/s": round(2 * M * N * K / t / 1e12, 1)}), flush=True)
    return out


base = run("default")
import torch.cuda.tunable as tn  # noqa: E402

tn.enable(True)
tn.tuning_enable(True)
tn.set_filename(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "tunableop_results.csv"))
tn.set_max_tuning_duration(200)
tuned = run("tunableop")
tn.write_file()
for k in base:
    print(f"{k}: default {base[k]*1e6:.1f}us tuned {tuned[k]*1e6:.1f}us speedup {base[k]/tuned[k]:.3f}")
