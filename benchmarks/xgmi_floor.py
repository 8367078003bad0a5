#!/usr/bin/env python3
"""Per-call floor of the TP tail collective (all-reduce + residual + RMSNorm, csrc/xgmi_allreduce.hip)
with W ranks as W processes on ONE MI355X, through the same start-up measurement the TP engine
runs (parallel.xgmi_ar.XgmiAllReduce.tune): one-shot and two-shot, per row bucket, at a model's
hidden size.  On one device every rank's bytes move through that device's HBM instead of xGMI
links, so this is the kernel + handshake floor, not the link-bandwidth term; ``bench.py --tp-sim``
adds it per call to the per-rank compute it measures.

    python benchmarks/xgmi_floor.py --world 8 --hidden 8192 --out profiles/r4_tp_collectives/floor_tp8_h8192.json
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, hidden, iters, out):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce

    tp = TPGroup(rank, world, dist.group.WORLD, ctrl=dist.group.WORLD, ranks=list(range(world)), ipc_only=True)
    x = XgmiAllReduce(tp, rccl=False)
    tim = x.tune(hidden, iters=iters)
    if rank == 0:
        res = {"world": world, "hidden": hidden, "ranks_per_device": world, "iters": iters,
               "blocks_cap": int(os.environ.get("LK_XGMI_AR_BLOCKS", "256")),
               "us_by_rows": {str(k): v for k, v in tim.items()},
               "route": {str(k): a for k, a in x.table.items()}, "error": x.error()}
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
        print(json.dumps(res))
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=16)
    ap.add_argument("--out", default="gpurun_out/xgmi_floor.json")
    a = ap.parse_args()
    os.environ.setdefault("LK_XGMI_AR_BLOCKS", "32")  # all ranks' workgroups co-resident on the one device
    import torch.multiprocessing as mp

    mp.spawn(_worker, args=(a.world, _port(), a.hidden, a.iters, a.out), nprocs=a.world, join=True)


if __name__ == "__main__":
    main()
