#!/usr/bin/env python3
"""Sampler step cost at the serving shape with Ollama's default parameters (temperature 0.8,
top-k 40, top-p 0.9, repeat penalty 1.1 / 64): GPU time per step (HIP events) and the host
time of Sampler.__call__."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import Sampler, SamplingParams  # noqa: E402

B, V = int(os.environ.get("B", "128")), 128256
lg = torch.randn(B, V, device="cuda") * 3
s = Sampler(V)
p = [SamplingParams() for _ in range(B)]
keys = list(range(B))
for _ in range(5):
    s(lg.clone(), p, [[]] * B, keys)
torch.cuda.synchronize()
x = lg.clone()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
t0 = time.perf_counter()
ev[0].record()
for _ in range(20):
    s(x, p, [[]] * B, keys)
ev[1].record()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"Sampler (Ollama defaults) B{B} V{V}: GPU {ev[0].elapsed_time(ev[1]) / 20 * 1e3:.1f} us/step, "
      f"host enqueue {(t1 - t0) / 20 * 1e6:.1f} us/step")
