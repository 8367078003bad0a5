#!/usr/bin/env python3
"""Cost of the prefill GEMM epilogues at the encoder's shapes (bge-base, K 768 / 3072, M 131072):
the same GEMM with no epilogue, bias, bias + GELU, bias + ReLU, timed back to back (hot weights,
medians of interleaved rounds).  The GELU-minus-bias difference is the erf epilogue's cost.

    python benchmarks/epi_cost.py [--M 131072]
    python benchmarks/epi_cost.py --llama [--M 4096]   # Llama-3-8B chain epilogues, cold weights

--llama: each Llama-3-8B projection plain vs with its chain epilogue (QKV: row scale + RoPE + KV
write; O / down: residual add + sums of squares; gate_up: row scale + SwiGLU), per row tile
(gemm1w 256 / 192 / 128 rows), weights rotated over copies larger than the 256 MB MALL.
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402


def _time(arms: dict, rounds: int, reps: int = 5) -> dict:
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    ts = {k: [] for k in arms}
    for _ in range(rounds):
        for k, f in arms.items():
            s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                f()
            t.record()
            t.synchronize()
            ts[k].append(s.elapsed_time(t) * 1e3 / reps)
    return {k: statistics.median(v) for k, v in ts.items()}


def llama(M: int, rounds: int):
    from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref

    L = ops.lib()
    dev = "cuda"
    H, Hq, Hkv, D, F = 4096, 32, 8, 128, 14336
    copies = 8
    x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    a14 = torch.randn(M, F, device=dev, dtype=torch.bfloat16)
    ss = ref.ss_partials(x)
    pos = torch.randint(0, 8000, (M,), device=dev, dtype=torch.int32)
    cs = ref.rope_cos_sin(8192, D, 500000.0, device=dev)
    slots = torch.arange(M, device=dev, dtype=torch.int32)
    kc = torch.zeros(M // 16 + 8, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    res = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
    ss_out = ops.ss_buffer(M, H, dev)
    shapes = {"qkv": ((Hq + 2 * Hkv) * D, H), "o": (H, H), "gate_up": (2 * F, H), "down": (H, F)}
    ws = {n: [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
          for n, (N, K) in shapes.items()}
    ctr = {"i": 0}

    def w_of(n):
        ctr["i"] += 1
        return ws[n][ctr["i"] % copies]

    for name, (N, K) in shapes.items():
        inp = a14 if name == "down" else x
        arms = {}
        for v in (3, 4, 5, 6, 7):
            bm = ops.GEMM1W_BM[v] if v not in ops.GEMM1W_SPLIT else f"256+{ops.GEMM1W_SPLIT[v]}"
            if name == "gate_up":
                out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
                arms[f"plain/{bm}"] = lambda v=v, out=out: L.gemm(inp, w_of("gate_up"), None, 1, 256, out, v, 1)
                arms[f"epi/{bm}"] = lambda v=v: L.gemm_fused(inp, w_of("gate_up"), 1, 256, None, v, 1, ss_in=ss, eps=1e-5)
            else:
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                arms[f"plain/{bm}"] = lambda v=v, out=out, n=name: L.gemm(inp, w_of(n), None, 0, 256, out, v, 1)
                if name == "qkv":
                    arms[f"epi/{bm}"] = lambda v=v: L.gemm_fused(
                        inp, w_of("qkv"), ops.EPI_QKV, 256, None, v, 1, ss_in=ss, eps=1e-5, positions=pos,
                        cos_sin=cs, slots=slots, k_cache=kc, v_cache=vc, hq=Hq, hkv=Hkv, hd=D)
                else:
                    arms[f"epi/{bm}"] = lambda v=v, n=name: L.gemm_fused(inp, w_of(n), ops.EPI_RESID, 256, None, v, 1,
                                                                        resid=res, ss_out=ss_out)
        med = _time(arms, rounds)
        tf = 2 * M * N * K / 1e12
        print(f"M{M} {name} N{N} K{K}: " + "  ".join(f"{k} {v:.1f} us ({tf / (v * 1e-6) / 1e3:.2f} PF/s)"
                                                    for k, v in med.items()), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--llama", action="store_true")
    a = ap.parse_args()
    if a.llama:
        for M in ((a.M,) if a.M else (4096, 2664)):
            llama(M, a.rounds)
        return
    a.M = a.M or 131072
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
