#!/usr/bin/env python3
"""One paged-decode shape (B sequences x ctx keys, Llama-3-8B heads), N launches -- for
rocprofv3 PMC passes."""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from benchmarks.kernel_bench import paged_setup  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--B", type=int, default=128)
ap.add_argument("--ctx", type=int, default=1000)
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()
Hq, Hkv, D = 32, 8, 128
kc, vc, bt = paged_setup(a.B, a.ctx, Hkv, D)
q = torch.randn(a.B, Hq, D, device="cuda", dtype=torch.bfloat16)
cl = torch.full((a.B,), a.ctx, dtype=torch.int32, device="cuda")
bt_full = torch.zeros(a.B, 512, dtype=torch.int32, device="cuda")
bt_full[:, : bt.shape[1]] = bt
for _ in range(a.iters):
    ops.paged_decode(q, kc, vc, bt_full, cl, 1 / math.sqrt(D))
torch.cuda.synchronize()
print("ok")
