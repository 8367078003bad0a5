#!/usr/bin/env python3
"""In-kernel s_memtime stamps of csrc/gemm1w.hip built with -DLK_G1W_STAMP=1 (diagnostic build:
stamps at the two barriers of K-tiles 8 and 9, lane 0 of every wave of the first 256 workgroups):
cycles per K-loop section against the MFMA-bound ideal (16 cycles per v_mfma_f32_16x16x32_bf16).

    python benchmarks/gemm1w_stamps.py --so benchmarks/probes/bin/libgemm1w_st.so [--N 4096 --K 4096]
"""
from __future__ import annotations

import argparse
import ctypes
import os
import statistics

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--so", default="benchmarks/probes/bin/libgemm1w_st.so")
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--N", type=int, default=4096)
    ap.add_argument("--K", type=int, default=4096)
    ap.add_argument("--b1", type=int, default=26)
    ap.add_argument("--b2", type=int, default=108)
    a = ap.parse_args()
    so = ctypes.CDLL(os.path.abspath(a.so))
    fn = so.lk_gemm1w_c
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                   ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_int,
                   ctypes.c_int]
    x = torch.randn(a.M, a.K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(a.N, a.K, device="cuda", dtype=torch.bfloat16) * 0.02
    out = torch.empty(a.M, a.N, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(400):  # ~2 s of back-to-back launches: clocks settle
        assert fn(x.data_ptr(), a.K, w.data_ptr(), None, a.M, a.N, a.K, 0, out.data_ptr(), a.N, st, 4, 256) == 0
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (256 * 4 * 8))()
    assert so.lk_gemm1w_stamps(buf) == 0
    v = list(buf)
    secs = {"B1 wait (lgkm0+barrier)": [], "DMA section": [], "B2 wait (vmcnt+barrier)": [],
            "read sections": [], "K-tile": []}
    for b in range(min(256, (a.M // 256) * (a.N // 256))):
        for wv in range(4):
            s = v[(b * 4 + wv) * 8:(b * 4 + wv) * 8 + 8]
            if not all(s):
                continue
            t8, t9 = s[:4], s[4:]
            secs["B1 wait (lgkm0+barrier)"].append(t8[1] - t8[0])
            secs["DMA section"].append(t8[2] - t8[1])
            secs["B2 wait (vmcnt+barrier)"].append(t8[3] - t8[2])
            secs["read sections"].append(t9[0] - t8[3])
            secs["K-tile"].append(t9[1] - t8[1])
    ideal = {"DMA section": 16 * (a.b2 - a.b1), "read sections": 16 * (128 - a.b2 + a.b1), "K-tile": 16 * 128}
    for k, xs in secs.items():
        if not xs:
            continue
        xs.sort()
        med = statistics.median(xs)
        line = f"{k:26s} median {med:7.0f}  p10 {xs[len(xs) // 10]:7.0f}  p90 {xs[9 * len(xs) // 10]:7.0f} cycles"
        if k in ideal:
            line += f"   ideal {ideal[k]} ({ideal[k] / med * 100:.0f} %)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
