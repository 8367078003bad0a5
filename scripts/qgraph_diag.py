"""Diagnose single-query encoder hipGraph replay against the eager encoder: capture the
encoder truncated at several depths (embedding LN only, 1 layer, all layers) for one
length and compare replay with eager output of the same truncated model."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd import ops  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models import build_encoder  # noqa: E402

DEV = torch.device("cuda:0")
enc = build_encoder("bge-base", device=DEV, dtype=torch.bfloat16)
cfg = enc.cfg
L = int(sys.argv[1]) if len(sys.argv) > 1 else 9


def run(ids, cu, pos, depth, tiles, stage):
    h = ops.embed_layernorm(ids, pos, None, enc.tok, enc.pos, enc.typ, enc.emb_ln_w, enc.emb_ln_b, cfg.norm_eps)
    H, nh, D = cfg.hidden, enc.nh, enc.D
    for Ly in enc.layers[:depth]:
        qkv = ops.linear(h, Ly.qkv, Ly.qkv_b)
        if stage == "qkv":
            return qkv
        a = ops.flash_prefill(qkv[:, :H], qkv[:, H:2 * H], qkv[:, 2 * H:], cu, nh, nh, D, enc.scale, False,
                              q_lens_cpu=[L], tiles=tiles)
        if stage == "attn":
            return a
        o = ops.linear(a, Ly.o, Ly.o_b)
        if stage == "o":
            return o
        h = ops.layernorm(o, Ly.ln1_w, Ly.ln1_b, cfg.norm_eps, residual=h)
        if stage == "ln1":
            return h
        f = ops.linear(h, Ly.fc1, Ly.fc1_b, act="gelu")
        if stage == "fc1":
            return f
        d = ops.linear(f, Ly.fc2, Ly.fc2_b)
        if stage == "fc2":
            return d
        h = ops.layernorm(d, Ly.ln2_w, Ly.ln2_b, cfg.norm_eps, residual=h)
    return h


with torch.inference_mode():
    cu = torch.tensor([0, L], dtype=torch.int32, device=DEV)
    pos = torch.arange(L, dtype=torch.int32, device=DEV)
    ts, tq = ops.prefill_tiles([L], [L], 1, False, enc.D)
    tiles = (torch.from_numpy(ts).to(DEV), torch.from_numpy(tq).to(DEV))
    real = torch.randint(1000, 20000, (L,), dtype=torch.int32, device=DEV)
    for depth, stage in [(0, None), (1, "qkv"), (1, "attn"), (1, "o"), (1, "ln1"), (1, "fc1"), (1, "fc2"),
                         (1, None), (12, None)]:
        ids = torch.full((L,), 101, dtype=torch.int32, device=DEV)
        side = torch.cuda.Stream(DEV)
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            run(ids, cu, pos, depth, tiles, stage)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            y = run(ids, cu, pos, depth, tiles, stage)
        ids.copy_(real)
        g.replay()
        torch.cuda.synchronize()
        want = run(real, cu, pos, depth, tiles, stage)
        warm = run(torch.full((L,), 101, dtype=torch.int32, device=DEV), cu, pos, depth, tiles, stage)
        torch.cuda.synchronize()
        print(f"L={L} depth={depth} stage={stage}: equal={torch.equal(y, want)} "
              f"maxdiff={(y.float() - want.float()).abs().max().item():.4g} "
              f"eq_warm={torch.equal(y, warm)}", flush=True)
