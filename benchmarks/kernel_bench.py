#!/usr/bin/env python3
"""Per-kernel microbenchmarks on one MI355X vs. their rooflines.

Each case is timed with HIP events (median over iterations, after warm-up) on
random data, and reported as achieved GB/s (bandwidth-bound kernels) or TFLOP/s
(MFMA-bound kernels).  Output: one JSON line per case (+ a markdown table with
``--md``).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

DEV = "cuda"


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
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


def paged_setup(B, ctx, Hkv, D, BS=16):
    nblk = (ctx + BS - 1) // BS
    NB = B * nblk + 1
    kc = torch.randn(NB, Hkv, BS, D, device=DEV, dtype=torch.bfloat16)
    vc = torch.randn_like(kc)
    bt = torch.randperm(NB - 1, device=DEV)[: B * nblk].int().view(B, nblk)
    return kc, vc, bt


def case_decode(B=64, ctx=1000, Hq=32, Hkv=8, D=128, BS=16):
    kc, vc, bt = paged_setup(B, ctx, Hkv, D, BS)
    q = torch.randn(B, Hq, D, device=DEV, dtype=torch.bfloat16)
    cl = torch.full((B,), ctx, dtype=torch.int32, device=DEV)
    bt_full = torch.zeros(B, 8192 // BS, dtype=torch.int32, device=DEV)
    bt_full[:, : bt.shape[1]] = bt
    t = timeit(lambda: ops.paged_decode(q, kc, vc, bt_full, cl, 1 / math.sqrt(D)))
    byts = B * ctx * Hkv * D * 2 * 2
    bs = "" if BS == 16 else f" BS{BS}"
    return {"case": f"paged_decode B{B} ctx{ctx} Hq{Hq} Hkv{Hkv} D{D}{bs}", "us": t * 1e6, "GB/s": byts / t / 1e9}


def case_prefill(B=32, L=1024, Hq=32, Hkv=8, D=128):
    kc, vc, bt = paged_setup(B, L, Hkv, D)
    T = B * L
    q = torch.randn(T, Hq * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=DEV)
    cl = torch.full((B,), L, dtype=torch.int32, device=DEV)
    ts, tq = ops.prefill_tiles([L] * B, [L] * B, Hq // Hkv, True)
    tiles = (torch.from_numpy(ts).to(DEV), torch.from_numpy(tq).to(DEV))
    t = timeit(lambda: ops.flash_prefill(q, kc, vc, cu, Hq, Hkv, D, 1 / math.sqrt(D), True, block_tables=bt,
                                         ctx_lens=cl, tiles=tiles))
    flops = B * 4 * (L * L / 2) * D * Hq
    return {"case": f"flash_prefill causal B{B} L{L} Hq{Hq} Hkv{Hkv} D{D}", "us": t * 1e6, "TFLOP/s": flops / t / 1e12}


def case_prefill_chunk(B=6, q=643, ctx=930, Hq=32, Hkv=8, D=128):
    """The in-situ shape of a mixed serving step: B prompts whose first ctx-q tokens are a
    cached prefix (the shared system prompt), q new tokens each, K/V from the paged cache."""
    kc, vc, bt = paged_setup(B, ctx, Hkv, D)
    T = B * q
    qq = torch.randn(T, Hq * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.arange(0, T + 1, q, dtype=torch.int32, device=DEV)
    cl = torch.full((B,), ctx, dtype=torch.int32, device=DEV)
    ts, tq = ops.prefill_tiles([q] * B, [ctx] * B, Hq // Hkv, True)
    tiles = (torch.from_numpy(ts).to(DEV), torch.from_numpy(tq).to(DEV))
    t = timeit(lambda: ops.flash_prefill(qq, kc, vc, cu, Hq, Hkv, D, 1 / math.sqrt(D), True, block_tables=bt,
                                         ctx_lens=cl, tiles=tiles))
    keys = sum(ctx - q + i + 1 for i in range(q))
    flops = B * 4 * keys * D * Hq
    return {"case": f"flash_prefill chunk B{B} q{q} ctx{ctx} Hq{Hq} Hkv{Hkv} D{D}", "us": t * 1e6,
            "TFLOP/s": flops / t / 1e12}


def case_encoder_attn(B=1600, L=80, H=12, D=64):
    T = B * L
    qkv = torch.randn(T, 3 * H * D, device=DEV, dtype=torch.bfloat16)
    cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=DEV)
    ts, tq = ops.prefill_tiles([L] * B, [L] * B, 1, False)
    tiles = (torch.from_numpy(ts).to(DEV), torch.from_numpy(tq).to(DEV))
    t = timeit(lambda: ops.flash_prefill(qkv[:, : H * D], qkv[:, H * D: 2 * H * D], qkv[:, 2 * H * D:], cu, H, H, D,
                                         1 / math.sqrt(D), False, tiles=tiles))
    flops = B * 4 * L * L * D * H
    # q, k, v read + o written once each: at L <= 128 the kernel is bounded by these bytes
    return {"case": f"encoder_attn B{B} L{L} H{H} D{D}", "us": t * 1e6, "TFLOP/s": flops / t / 1e12,
            "GB/s": T * H * D * 2 * 4 / t / 1e9}


def case_rmsnorm(T=8192, H=4096):
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    r = torch.randn_like(x)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    t = timeit(lambda: ops.rmsnorm(x, w, 1e-5, residual=r))
    return {"case": f"rmsnorm+res T{T} H{H}", "us": t * 1e6, "GB/s": T * H * 2 * 4 / t / 1e9}


def case_silu(T=8192, I=14336):
    x = torch.randn(T, 2 * I, device=DEV, dtype=torch.bfloat16)
    t = timeit(lambda: ops.silu_mul(x))
    return {"case": f"silu_mul T{T} I{I}", "us": t * 1e6, "GB/s": T * I * 2 * 3 / t / 1e9}


def case_gelu(T=32768, N=3072):
    """Encoder FFN activation: in-place GELU(erf) with the fused bias, bge-base width."""
    x = torch.randn(T, N, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, device=DEV, dtype=torch.bfloat16)
    t = timeit(lambda: ops.lib().activation_(x, b, 0))
    return {"case": f"gelu+bias T{T} N{N}", "us": t * 1e6, "GB/s": T * N * 2 * 2 / t / 1e9}


def case_layernorm(T=32768, H=768):
    """Encoder post-LN with the residual add fused (bge-base / MiniLM widths)."""
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    r = torch.randn_like(x)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    t = timeit(lambda: ops.layernorm(x, w, b, 1e-12, residual=r))
    return {"case": f"layernorm+res T{T} H{H}", "us": t * 1e6, "GB/s": T * H * 2 * 3 / t / 1e9}


def case_silu_down(T=4096, I=14336, H=4096):
    """SwiGLU followed by the down projection that consumes its output (how the engine
    runs them), so a store policy that evicts the activation shows up in the GEMM."""
    x = torch.randn(T, 2 * I, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, I, device=DEV, dtype=torch.bfloat16) * 0.02
    t = timeit(lambda: torch.nn.functional.linear(ops.silu_mul(x), w))
    return {"case": f"silu_mul+down T{T} I{I} H{H}", "us": t * 1e6, "TFLOP/s": 2 * T * I * H / t / 1e12}


def case_knn(N=485_000, D=768, nq=64):
    c = torch.randn(N, D, device=DEV, dtype=torch.bfloat16)
    q = torch.randn(nq, D, device=DEV, dtype=torch.bfloat16)
    cn, qn = ops.row_norms(c), ops.row_norms(q)
    t = timeit(lambda: ops.knn_topk(c, cn, q, qn, 6))
    tf = timeit(lambda: ops.lib().knn_topk(c, cn, q, qn, 6, True))
    return {"case": f"knn_topk N{N} D{D} nq{nq} k6 (fused single-pass kernel: {tf * 1e6:.0f} us)", "us": t * 1e6,
            "GB/s": N * D * 2 / t / 1e9}


def case_gemm(M, N, K, layout="NT"):
    """hipBLASLt via torch: NT = x @ W^T with W [N,K] (nn.Linear layout), NN = x @ W with W [K,N]."""
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    if layout == "NT":
        b = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
        fn = lambda: torch.nn.functional.linear(a, b)  # noqa: E731
    else:
        b = torch.randn(K, N, device=DEV, dtype=torch.bfloat16)
        fn = lambda: a @ b  # noqa: E731
    t = timeit(fn)
    return {"case": f"hipBLASLt {layout} M{M} N{N} K{K}", "us": t * 1e6, "TFLOP/s": 2 * M * N * K / t / 1e12,
            "GB/s": (M * K + N * K + M * N) * 2 / t / 1e9}


def case_prefill_gemm(M, N, K, swiglu=False):
    """Hand-written prefill GEMM (csrc/gemm.hip, best schedule / column tile) vs hipBLASLt
    (+ silu_mul when swiglu); benchmarks/gemm_bench.py is the full interleaved sweep."""
    L = ops.lib()
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) * 0.05
    epi = 1 if swiglu else 0
    cfgs = [(sc, bn, 1) for sc, bn in ops._gemm_configs(N, epi)]
    dflt = ops._gemm_default(M, N, K, epi)  # the dispatch policy's pick, split-K included
    if dflt is not None and dflt not in cfgs:
        cfgs.append(dflt)
    ts = {c: timeit(lambda c=c: L.gemm(x, w, None, epi, c[1], None, c[0], c[2])) for c in cfgs}
    c, t = min(ts.items(), key=lambda kv: kv[1])
    if swiglu:
        tb = timeit(lambda: L.silu_mul(torch.nn.functional.linear(x, w)))
    else:
        tb = timeit(lambda: torch.nn.functional.linear(x, w))
    return {"case": f"gemm M{M} N{N} K{K}{' swiglu' if swiglu else ''} s{c[0]}/{c[1]}" + (f"/k{c[2]}" if c[2] > 1 else ""),
            "us": t * 1e6,
            "TFLOP/s": 2 * M * N * K / t / 1e12, "hipblaslt_us": tb * 1e6, "speedup": tb / t}


def case_skinny(M, N, K, swiglu=False):
    """Hand-written decode-regime GEMM vs hipBLASLt (+ silu_mul when swiglu) at the same shape."""
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    L = ops.lib()
    t = timeit(lambda: L.skinny_linear(a, b, swiglu))
    if swiglu:
        tb = timeit(lambda: ops.silu_mul(torch.nn.functional.linear(a, b)))
    else:
        tb = timeit(lambda: torch.nn.functional.linear(a, b))
    byts = (N * K + M * K + M * N) * 2
    return {"case": f"skinny{'+swiglu' if swiglu else ''} M{M} N{N} K{K} S{L.skinny_splits(min(M, 128), N, K, swiglu)}",
            "us": t * 1e6, "GB/s": byts / t / 1e9, "hipblaslt_us": tb * 1e6, "speedup": tb / t}


def case_ws(M, N, K, swiglu=False):
    """LDS-DMA weight-streaming GEMM vs the fragment-load skinny kernel vs hipBLASLt."""
    a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
    L = ops.lib()
    t = timeit(lambda: L.ws_linear(a, b, swiglu))
    tsk = timeit(lambda: L.skinny_linear(a, b, swiglu))
    if swiglu:
        tb = timeit(lambda: ops.silu_mul(torch.nn.functional.linear(a, b)))
    else:
        tb = timeit(lambda: torch.nn.functional.linear(a, b))
    byts = (N * K + M * K + M * N) * 2
    bn, S = L.ws_plan(M, N, K, swiglu)
    return {"case": f"ws{'+swiglu' if swiglu else ''} M{M} N{N} K{K} BN{bn} S{S}", "us": t * 1e6,
            "GB/s": byts / t / 1e9, "TFLOP/s": 2 * M * N * K / t / 1e12, "skinny_us": tsk * 1e6,
            "hipblaslt_us": tb * 1e6, "speedup": tb / t}


def case_ws_sweep():
    """Every (BN, split) plan of the weight-streaming GEMM per shape: the data the
    planner (lk_wsgemm_plan) is calibrated on."""
    L = ops.lib()
    rows = []
    shapes = LLAMA8B_SHAPES + [(10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672)]
    for M in (64, 128, 192, 256):
        for N, K in shapes:
            sw = N in (28672, 57344)
            a = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            b = torch.randn(N, K, device=DEV, dtype=torch.bfloat16)
            res = {}
            for bn in (64, 128):
                per = bn // 2 if sw else bn
                if (N // 2 if sw else N) % per:
                    continue
                for S in (1, 2, 4, 8):
                    if K % (S * 64) or K // S < 256:
                        continue
                    res[(bn, S)] = timeit(lambda: L.ws_linear(a, b, sw, bn, S), iters=10, warmup=2)
            tb = timeit(lambda: (ops.silu_mul(torch.nn.functional.linear(a, b)) if sw
                                 else torch.nn.functional.linear(a, b)), iters=10, warmup=2)
            best = min(res, key=res.get)
            plan = tuple(L.ws_plan(M, N, K, sw))
            rows.append({"case": f"ws-sweep M{M} N{N} K{K}{' swiglu' if sw else ''}",
                         "us": res[best] * 1e6, "best": f"BN{best[0]} S{best[1]}",
                         "plan": f"BN{plan[0]} S{plan[1]} {res.get(plan, float('nan')) * 1e6:.1f}us",
                         "all": {f"{k[0]}/{k[1]}": round(v * 1e6, 1) for k, v in res.items()},
                         "hipblaslt_us": tb * 1e6, "speedup": tb / res[best]})
    return rows


LLAMA8B_SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]


CASES = {
    "decode": lambda: [case_decode(), case_decode(B=128, ctx=1000), case_decode(B=8, ctx=3000)],
    "decode_bs": lambda: [case_decode(B=128, ctx=1000, BS=bs) for bs in (16, 32, 64)] +
                         [case_decode(B=64, ctx=1000, BS=bs) for bs in (16, 32, 64)],
    "prefill": lambda: [case_prefill(), case_prefill(B=8, L=4096), case_prefill_chunk()],
    "prefill_chunk": lambda: [case_prefill_chunk()],
    "encoder": lambda: [case_encoder_attn()],
    "act": lambda: [case_gelu(), case_gelu(8192), case_gelu(65536)],
    "ln": lambda: [case_layernorm(), case_layernorm(8192), case_layernorm(32768, 384), case_layernorm(4096, 1024)],
    "norm": lambda: [case_rmsnorm(), case_silu(), case_silu(3584), case_silu(4096), case_silu(128), case_silu(4096, 1792),
                     case_silu_down(3584), case_silu_down(4096)],
    "knn": lambda: [case_knn(), case_knn(nq=8), case_knn(N=1_000_000, nq=8), case_knn(N=1_000_000, nq=128)],
    "gemm": lambda: [case_gemm(64, 6144, 4096), case_gemm(64, 28672, 4096), case_gemm(64, 4096, 14336),
                     case_gemm(32768, 6144, 4096), case_gemm(32768, 28672, 4096), case_gemm(32768, 4096, 14336)],
    "skinny": lambda: [case_skinny(M, N, K, N == 28672) for M in (1, 16, 32, 64, 128, 256)
                       for (N, K) in LLAMA8B_SHAPES + [(128256, 4096)]],
    "ws": lambda: [case_ws(M, N, K, N in (28672, 57344)) for M in (64, 128, 192, 256)
                   for (N, K) in LLAMA8B_SHAPES + [(128256, 4096), (10240, 8192), (8192, 8192), (57344, 8192),
                                                   (8192, 28672)]],
    "ws_sweep": lambda: case_ws_sweep(),
    "gemm_mid": lambda: [case_gemm(M, N, K) for M in (1024, 2048, 2560, 3072, 3328, 3584, 3840, 4096, 4352,
                                                      5120, 5376, 6144, 8192)
                         for (N, K) in LLAMA8B_SHAPES],
    "prefill_gemm": lambda: [case_prefill_gemm(M, N, K, N == 28672) for M in (1024, 2048, 3328, 3584, 3840, 4096, 8192)
                    for (N, K) in LLAMA8B_SHAPES],
    "gemm_sweep": lambda: [case_gemm(M, N, K, lay) for M in (128, 256, 1024, 4096, 8192, 16384)
                           for (N, K) in LLAMA8B_SHAPES for lay in ("NT", "NN")],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cases", nargs="*", default=list(CASES))
    ap.add_argument("--md", default=None)
    a = ap.parse_args()
    rows = []
    for c in a.cases:
        for r in CASES[c]():
            r = {k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}
            print(json.dumps(r), flush=True)
            rows.append(r)
    if a.md:
        with open(a.md, "w") as f:
            f.write("| case | us | GB/s | TFLOP/s | skinny us | hipBLASLt us | speedup vs hipBLASLt |\n"
                    "|---|---|---|---|---|---|---|\n")
            for r in rows:
                f.write(f"| {r['case']} | {r['us']} | {r.get('GB/s', '')} | {r.get('TFLOP/s', '')} "
                        f"| {r.get('skinny_us', '')} | {r.get('hipblaslt_us', '')} | {r.get('speedup', '')} |\n")


if __name__ == "__main__":
    main()
