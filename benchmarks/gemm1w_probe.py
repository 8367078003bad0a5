#!/usr/bin/env python3
"""One-wave-per-SIMD prefill GEMM (csrc/gemm1w.hip, loaded standalone through ctypes) vs the
serving GEMM (csrc/gemm.hip through ops.linear) vs hipBLASLt (F.linear), Llama-3-8B projections,
cold weights (rotated copies past the 256 MB MALL), interleaved rounds in one process, medians;
plus a numerics check of the new kernel against an fp32 torch matmul.

    python benchmarks/gemm1w_probe.py --build [--ms 4096,8192]

``--build`` compiles the probe library from the tracked ``csrc/gemm1w.hip`` (its ``extern "C"
lk_gemm1w_c`` entry) into ``benchmarks/probes/bin/libgemm1w.so`` with hipcc first -- the
library is a build product (git-ignored), the source is the serving kernel itself.  The
schedule-sweep arms of ``profiles/r5_gemm1w/`` (``libgemm1w_c7`` / ``_n2``...) were builds of
intermediate versions of that file; the kept schedule is the one in its history
(``git log -- csrc/gemm1w.hip``), so rebuilding a sweep arm means checking out that commit's
``csrc/gemm1w.hip`` and passing ``--build --so <name>``.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [("QKV", 6144, 4096, 0), ("O", 4096, 4096, 0), ("gate_up+SwiGLU", 28672, 4096, 1),
          ("down", 4096, 14336, 0), ("enc_ffn_up", 3072, 768, 0), ("enc_ffn_dn", 768, 3072, 0)]


def build_probe(out: str) -> str:
    """hipcc the serving kernel source into a standalone shared library (no torch, no bindings)."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-ffp-contract=fast",
           "-Wno-inline-asm", "-I", os.path.join(root, "csrc"), os.path.join(root, "csrc", "gemm1w.hip"), "-o", out]
    subprocess.run(cmd, check=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default="benchmarks/probes/bin/libgemm1w.so")
    ap.add_argument("--ms", default="4096,8192")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--group", type=int, default=4)
    ap.add_argument("--bm", type=int, default=256, help="row tile of the probed kernel (256 / 192 / 128)")
    ap.add_argument("--no-cur", action="store_true", help="skip the gemm.hip arm")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--extra", default="", help="extra shapes name:N:K[:swiglu],...")
    ap.add_argument("--build", action="store_true",
                    help="compile csrc/gemm1w.hip into the --so path (hipcc, gfx950) before probing")
    a = ap.parse_args()
    if a.build:
        build_probe(a.so.split(",")[0].partition(":")[0])
    fns = {}
    for spec in a.so.split(","):  # path[:group] -> one arm per entry
        path, _, grp = spec.partition(":")
        so = ctypes.CDLL(os.path.abspath(path))
        fn = so.lk_gemm1w_c
        fn.restype = ctypes.c_int
        fn.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                       ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                       ctypes.c_int]
        name = os.path.basename(path).replace("libgemm1w", "new").replace(".so", "") + (f"g{grp}" if grp else "")
        fns[name] = (fn, int(grp) if grp else a.group)
    ops = None
    if not a.no_cur:
        from llm_kubernetes_minikube_sharp4dev_amd import ops as _ops
        ops = _ops
    torch.manual_seed(0)
    stream = torch.cuda.current_stream().cuda_stream

    def new(x, w, out, epi, arm=None):
        fn, grp = fns[arm or next(iter(fns))]
        rc = fn(x.data_ptr(), x.stride(0), w.data_ptr(), None, x.shape[0], w.shape[0], x.shape[1], epi,
                out.data_ptr(), out.stride(0), stream, grp, a.bm)
        assert rc == 0, rc
        return out

    want = [s for s in a.shapes.split(",") if s]
    shapes = list(SHAPES)
    for e in [e for e in a.extra.split(",") if e]:
        f = e.split(":")
        shapes.append((f[0], int(f[1]), int(f[2]), int(f[3]) if len(f) > 3 else 0))
        want.append(f[0]) if want else None
    for name, N, K, sw in shapes:
        if want and name not in want:
            continue
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        n_cold = max(2, -(-(640 << 20) // (N * K * 2)))
        copies = [w] + [w.clone() for _ in range(n_cold - 1)]
        for M in [int(v) for v in a.ms.split(",")]:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            out = torch.empty(M, N // 2 if sw else N, device="cuda", dtype=torch.bfloat16)
            # numerics vs fp32
            errs = []
            for arm in fns:
                out.zero_()
                new(x, w, out, sw, arm)
                errs.append(out.float())
            ref = x.float() @ w.float().t()
            if sw:
                I = N // 2
                g, u = ref[:, :I].bfloat16().float(), ref[:, I:].bfloat16().float()
                ref = (F.silu(g).bfloat16().float() * u)
            err = max((o - ref).abs().max().item() for o in errs)
            scale = ref.abs().max().item()
            ok = err <= 0.02 * scale + 1e-2
            arms = {k: (lambda c, k=k: new(x, c, out, sw, k)) for k in fns}
            if ops is not None:
                arms["cur"] = (lambda c: ops.linear_swiglu(x, c)) if sw else (lambda c: ops.linear(x, c))
            arms["lib"] = (lambda c: F.silu(F.linear(x, c)[:, : N // 2])) if sw else (lambda c: F.linear(x, c))
            for f in arms.values():
                f(w)
            torch.cuda.synchronize()
            seq = copies[1:] + copies[:1]
            ts = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, f in arms.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for c in seq:
                        f(c)
                    e1.record()
                    e1.synchronize()
                    ts[k].append(e0.elapsed_time(e1) * 1e3 / len(seq))
            med = {k: statistics.median(v) for k, v in ts.items()}
            tf = {k: 2 * M * N * K / (v * 1e-6) / 1e12 for k, v in med.items()}
            parts = " ".join(f"{k} {med[k]:.1f}us/{tf[k]:.0f}TF" for k in arms)
            k0 = next(iter(fns))
            rel = " ".join(f"{k}/lib {med['lib'] / med[k]:.3f}x" for k in fns)
            print(f"{name:16s} M{M:5d} N{N:5d} K{K:5d} | {parts} | {rel}"
                  + (f" {k0}/cur {med['cur'] / med[k0]:.3f}x" if 'cur' in med else "")
                  + f" | maxerr {err:.3g} (scale {scale:.3g}) {'OK' if ok else 'BAD'}", flush=True)
        del copies


if __name__ == "__main__":
    main()
