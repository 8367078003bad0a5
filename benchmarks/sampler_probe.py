"""Probe: does the constrained sampler block the host while a long forward is queued?"""
import time

import numpy as np
import torch

dev = torch.device("cuda", 0)
V = 128256
a = torch.randn(8192, 8192, device=dev, dtype=torch.bfloat16)


def long_gpu():
    for _ in range(20):
        a @ a  # ~20 x 0.5 ms


def t():
    return time.perf_counter() * 1e3


for trial in [0, 1, 2, 0, 1, 2]:
    logits = torch.randn(120, V, device=dev)
    torch.cuda.synchronize()
    long_gpu()
    t0 = t()
    rows = np.repeat(np.arange(100), 50)
    toks = np.random.randint(0, V, rows.shape[0])
    r = torch.from_numpy(rows)
    tk = torch.from_numpy(toks)
    t1 = t()
    mask = torch.full((100, V), float("-inf"), device=dev)
    t2 = t()
    rd = r.to(dev, non_blocking=True)
    td = tk.to(dev, non_blocking=True)
    t3 = t()
    if trial == 0:
        mask[rd, td] = 0.0
    elif trial == 1:
        flat = torch.from_numpy(rows * V + toks).to(dev, non_blocking=True)
        mask.view(-1).index_fill_(0, flat, 0.0)
    else:
        mask.index_put_((rd, td), torch.zeros((), device=dev))
    t4 = t()
    sel = torch.as_tensor(list(range(100)), dtype=torch.long).to(dev, non_blocking=True)
    t5 = t()
    logits.index_add_(0, sel, mask)
    t6 = t()
    torch.cuda.synchronize()
    t7 = t()
    print(f"trial {trial}: from_numpy {t1-t0:.2f} full {t2-t1:.2f} h2d {t3-t2:.2f} setitem {t4-t3:.2f} "
          f"sel {t5-t4:.2f} index_add {t6-t5:.2f} | sync wait {t7-t6:.2f} ms")
print(torch.cuda.memory_stats().get("num_alloc_retries"), torch.cuda.memory_stats().get("num_device_alloc"))
