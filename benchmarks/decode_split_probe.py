#!/usr/bin/env python3
"""Paged decode attention: keys per workgroup (split) vs time at the engine's operating
points (B rows of ~ctx keys, Llama-3-8B heads), varied context lengths per row."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from benchmarks.kernel_bench import paged_setup, timeit  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

Hq, Hkv, D = 32, 8, 128
for B, ctx in ((120, 960), (120, 250), (64, 1000), (128, 2000)):
    kc, vc, bt = paged_setup(B, ctx, Hkv, D)
    q = torch.randn(B, Hq, D, device="cuda", dtype=torch.bfloat16)
    g = torch.Generator().manual_seed(B)
    cl = torch.randint(max(16, ctx // 2), ctx + 1, (B,), generator=g).int().cuda()
    bt_full = torch.zeros(B, 8192 // 16, dtype=torch.int32, device="cuda")
    bt_full[:, : bt.shape[1]] = bt
    res = {}
    ref = None
    for split in (256, 512, 1024, 2048):
        ms = ops.decode_splits(8192, split)
        po = torch.empty(B * Hq * ms * D, device="cuda")
        pm = torch.empty(B * Hq * ms * 2, device="cuda")
        f = lambda: ops.paged_decode(q, kc, vc, bt_full, cl, 1 / math.sqrt(D), ms, po.view(B, Hq, ms, D),  # noqa: E731
                                     pm.view(B, Hq, ms, 2), split=split)
        o = f()
        ref = o if ref is None else ref
        assert (o.float() - ref.float()).abs().max().item() < 2e-2
        res[f"split{split}"] = round(timeit(f) * 1e6, 1)
    print(json.dumps({"case": f"B{B} ctx<= {ctx}", "default_split": ops.decode_split_size(B, Hkv), **res}), flush=True)
