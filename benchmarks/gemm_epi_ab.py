#!/usr/bin/env python3
"""In-process A/B of the prefill GEMM's fused epilogue work (csrc/gemm.hip), cold weights (rotated
through > 600 MB of copies, as in serving), HIP events, interleaved rounds, medians.  (Round 4's
LDS-staged-store arm was removed with the variant: profiles/r4_kernels/gemm_epi_ab.md.)

* ``chain``: one decoder block's unfused prefill tail (QKV GEMM -> rope_kv_; O GEMM -> add+RMSNorm;
  gate_up+SwiGLU; down GEMM -> add+RMSNorm) vs the fused chain (QKV epilogue with RoPE + KV
  write and the input-norm scale; O / down RESID epilogues with partial sums of squares;
  SwiGLU with the post-norm scale), Llama-3-8B shapes.

    python benchmarks/gemm_epi_ab.py [--ms 2048,4096] [--md out.md]
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.ops import reference as ref  # noqa: E402

def _time(fns: dict, rounds: int = 7) -> dict:
    ts = {k: [] for k in fns}
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            b.synchronize()
            ts[k].append(a.elapsed_time(b) * 1e3)
    return {k: statistics.median(v) for k, v in ts.items()}


def _copies(w, cold=600 << 20):
    n = max(1, -(-cold // (w.numel() * 2)))
    return [w] + [w.clone() for _ in range(n - 1)]


def chain(ms, lines):
    """One Llama-3-8B block's projections + their tails, unfused vs fused (cold weights)."""
    H, I, Hq, Hkv, D = 4096, 14336, 32, 8, 128
    dev = "cuda"
    wq = torch.randn((Hq + 2 * Hkv) * D, H, device=dev, dtype=torch.bfloat16) * 0.02
    wo = torch.randn(H, Hq * D, device=dev, dtype=torch.bfloat16) * 0.02
    wgu = torch.randn(2 * I, H, device=dev, dtype=torch.bfloat16) * 0.02
    wd = torch.randn(H, I, device=dev, dtype=torch.bfloat16) * 0.02
    g = torch.ones(H, device=dev, dtype=torch.bfloat16)
    cs = ref.rope_cos_sin(8192, D, 500000.0, device=dev)
    nb = 4096
    kc = torch.zeros(nb, Hkv, 16, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros_like(kc)
    lines.append("")
    lines.append("| M | unfused block us (4 GEMMs + rope_kv + 2 add+norm) | fused chain us (4 GEMMs) | speedup |")
    lines.append("|---|---|---|---|")
    for M in ms:
        x = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
        res = torch.randn(M, H, device=dev, dtype=torch.bfloat16)
        attn = torch.randn(M, Hq * D, device=dev, dtype=torch.bfloat16)
        pos = torch.randint(0, 4000, (M,), device=dev, dtype=torch.int32)
        slots = torch.randperm(nb * 16, device=dev)[:M].to(torch.int32)
        ss_a, ss_b = ops.ss_buffer(M, H, dev), ops.ss_buffer(M, H, dev)
        ss_b.copy_(ref.ss_partials(res))

        def unfused():
            qkv = ops.linear(x, wq)
            ops.rope_kv_(qkv, pos, cs, Hq, Hkv, D, kc, vc, slots, False, False)
            y = ops.rmsnorm(ops.linear(attn, wo), g, 1e-5, residual=res)
            a = ops.linear_swiglu(y, wgu)
            ops.rmsnorm(ops.linear(a, wd), g, 1e-5, residual=res)

        def fused():
            ops.linear_qkv_fused(res, wq, ss_b, 1e-5, pos, cs, Hq, Hkv, D, kc, vc, slots)
            ops.linear_resid(attn, wo, res, ss_a)
            a = ops.linear_swiglu_scaled(res, wgu, ss_a, 1e-5)
            ops.linear_resid(a, wd, res, ss_b)

        t = _time({"unfused": unfused, "fused": fused})
        lines.append(f"| {M} | {t['unfused']:.1f} | {t['fused']:.1f} | {t['unfused'] / t['fused']:.3f} |")
        print(lines[-1], flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="2048,3072,4096,8192")
    ap.add_argument("--only", default="chain")
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    ms = [int(v) for v in a.ms.split(",")]
    lines = []
    if "chain" in a.only:
        chain(ms, lines)
    if a.md:
        os.makedirs(os.path.dirname(os.path.abspath(a.md)), exist_ok=True)
        with open(a.md, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
