#!/usr/bin/env python3
"""FETCH_SIZE calibration: kernels with known HBM read bytes (a 1 GiB bf16 reduction, a
1 GiB copy and the row-norm kernel over a 485,620 x 768 bf16 corpus), for
`rocprofv3 --pmc FETCH_SIZE TCC_EA0_RDREQ_sum` on gfx950.  Each buffer is 4x the 256 MB
MALL, so no pass is served from cache."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402

n = (1 << 30) // 2
x = torch.randn(n, device="cuda", dtype=torch.bfloat16)
y = torch.empty_like(x)
corpus = torch.randn(485620, 768, device="cuda", dtype=torch.bfloat16)
for _ in range(3):
    x.float().sum() if False else x.sum()
    y.copy_(x)
    ops.row_norms(corpus)
torch.cuda.synchronize()
print("logical read bytes: sum 1073741824, copy 1073741824 (+1 GiB written), row_norms", corpus.numel() * 2)
