#!/usr/bin/env python3
"""Weight-streaming GEMM plan sweep at the decode shapes: every (column tile BN, K-split S,
kernel variant) against the plan ``lk_wsgemm_plan`` picks, per row count, weights cold (each
launch reads the next of enough weight copies to overflow the 256 MB MALL), medians of
interleaved rounds.  Prints TB/s of weight bytes and the best candidate per (M, shape).

    python benchmarks/ws_plan_sweep.py [--ms 1,64,128,192] [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096, False), "o": (4096, 4096, False), "gate_up": (28672, 4096, True),
          "down": (4096, 14336, False)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,16,64,128,160,192")
    ap.add_argument("--shapes", default="qkv,o,down,gate_up")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    L = ops.lib()
    lines = ["| M | shape | plan (BN, S) | plan TB/s | best (BN, S, variant) | best TB/s |", "|---|---|---|---|---|---|"]
    detail = []
    for name in a.shapes.split(","):
        N, K, sw = SHAPES[name]
        wb = N * K * 2
        copies = [torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
                  for _ in range(max(2, -(-600 * 2**20 // wb)))]
        for M in [int(m) for m in a.ms.split(",")]:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            plan = tuple(L.ws_plan(M, N, K, sw))
            cands = []
            for bn in (64, 96, 128):
                per = bn // 2 if sw else bn
                cols = N // 2 if sw else N
                if (sw and bn == 96) or cols % per:
                    continue
                for S in (1, 2, 4, 8):
                    if K % (S * 64) or S * (cols // per) > 1024:
                        continue
                    for v in (0, 1):
                        cands.append((bn, S, v))
            rot = [0]

            def run(c):
                bn, S, v = c
                L.ws_set_variant(M, N, K, sw, v)
                rot[0] = (rot[0] + 1) % len(copies)
                L.ws_linear(x, copies[rot[0]], sw, bn, S)

            ts = {c: [] for c in cands}
            for c in cands:
                run(c)
            torch.cuda.synchronize()
            for _ in range(a.rounds):
                for c in cands:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(3):
                        run(c)
                    e1.record()
                    e1.synchronize()
                    ts[c].append(e0.elapsed_time(e1) * 1e3 / 3)
            L.ws_set_variant(M, N, K, sw, -1)
            med = {c: statistics.median(v) for c, v in ts.items()}
            best = min(med, key=med.get)
            plan_best = min((c for c in med if c[:2] == plan), key=med.get)
            tb = lambda us: wb / us / 1e6  # noqa: E731
            lines.append(f"| {M} | {name} | {plan} v{plan_best[2]} | {tb(med[plan_best]):.2f} ({med[plan_best]:.1f} us) | "
                         f"{best} | {tb(med[best]):.2f} ({med[best]:.1f} us) |")
            detail.append(f"{name} M{M}: " + ", ".join(f"{c}:{med[c]:.1f}" for c in sorted(med, key=med.get)[:6]))
            print(lines[-1], flush=True)
        del copies
        torch.cuda.empty_cache()
    out = "\n".join(lines) + "\n\nfastest six per case (BN, S, variant): us\n\n" + "\n".join(f"- {d}" for d in detail) + "\n"
    print(out, flush=True)
    if a.md:
        with open(a.md, "w") as f:
            f.write(out)


if __name__ == "__main__":
    main()
