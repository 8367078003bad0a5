#!/usr/bin/env python3
"""One flash-prefill shape, N launches (for rocprofv3 PMC passes): causal B8 L4096 or the
in-situ chunk shape.  LK_PREFILL_WAVES / LK_PREFILL_PIPE / LK_PREFILL_DEFER select the kernel variant."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from benchmarks.kernel_bench import paged_setup  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shape", choices=["long", "chunk"], default="long")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
B, q, ctx = (8, 4096, 4096) if a.shape == "long" else (6, 643, 930)
Hq, Hkv, D = 32, 8, 128
kc, vc, bt = paged_setup(B, ctx, Hkv, D)
qq = torch.randn(B * q, Hq * D, device="cuda", dtype=torch.bfloat16)
cu = torch.arange(0, B * q + 1, q, dtype=torch.int32, device="cuda")
cl = torch.full((B,), ctx, dtype=torch.int32, device="cuda")
ts, tq = ops.prefill_tiles([q] * B, [ctx] * B, Hq // Hkv, True)
tiles = (torch.from_numpy(ts).cuda(), torch.from_numpy(tq).cuda())
for _ in range(a.iters):
    ops.flash_prefill(qq, kc, vc, cu, Hq, Hkv, D, 1 / math.sqrt(D), True, block_tables=bt, ctx_lens=cl, tiles=tiles)
torch.cuda.synchronize()
print("ok")
