"""Process launch for tensor-parallel serving: one fresh process per TP rank, each joining a
process group of its own TP group (``serve --tp T``, ``all --tp T``, ``rag-app --tp T``).

Every rank is started with ``subprocess.Popen`` BEFORE any process touches the GPU (no
fork or exec of a HIP-initialised process), with the torchrun-style environment
``RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR / MASTER_PORT``; ``init_tp_rank`` then picks
the device and backend exactly as ``bench.py`` does under ``torch.distributed.run``:

  GPU            backend nccl (RCCL), rank r on local device LOCAL_RANK, IPC xGMI collectives
                 routed by the start-up self-check + tuning table (``LK_TP_COLLECTIVES=auto``)
  GPU one-device every rank on device 0 (a one-GPU box rehearsing TP=T): gloo for the host
                 collectives, the IPC kernels for every device collective, 2 hardware queues
                 per process, a capped all-reduce grid (bench.py ``--one-device``)
  CPU            gloo

The reference has no tensor parallelism (one Ollama process per model,
``Minimal_RAG/Program.cs:22-24``); this is the MI355X-side layout that serves a 70B TP=8
model behind the same :11434 seam."""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import Optional

MOD = "llm_kubernetes_minikube_sharp4dev_amd"


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_env(rank: int, world: int, local_rank: int, port: int, one_device: bool = False,
             base: Optional[dict] = None) -> dict:
    """Environment of one TP rank process."""
    env = dict(base if base is not None else os.environ)
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local_rank), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port))
    if one_device:
        env["LK_ONE_DEVICE"] = "1"
    return env


def spawn_ranks(argv_for_rank, world: int, port: int, first: int = 1, local_base: int = 0,
                one_device: bool = False) -> list:
    """Start ranks ``first .. world-1`` of one TP group as fresh processes running
    ``python -m <pkg> <argv_for_rank(rank)>``."""
    procs = []
    for r in range(first, world):
        env = rank_env(r, world, 0 if one_device else local_base + r, port, one_device)
        procs.append(subprocess.Popen([sys.executable, "-m", MOD] + list(argv_for_rank(r)), env=env))
    return procs


def init_tp_rank(tp_size: int, device: Optional[str] = None):
    """Join this process's TP group from the env written by :func:`rank_env`: set the device,
    initialise the process group, split it into the TP group (world == tp_size) and return
    ``(TPGroup, torch.device)``."""
    from datetime import timedelta

    one_device = os.environ.get("LK_ONE_DEVICE") == "1"
    on_cpu = device == "cpu"
    if one_device and not on_cpu:
        # read when HIP initialises: before the first device call of this process
        if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) > 2:
            os.environ["GPU_MAX_HW_QUEUES"] = "2"
        os.environ["LK_TP_COLLECTIVES"] = "ipc"
        os.environ.setdefault("LK_XGMI_AR_BLOCKS", "16")
    import torch
    import torch.distributed as dist

    from .tp import new_tp_groups

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != tp_size:
        raise SystemExit(f"TP rank started with WORLD_SIZE={world}, expected --tp {tp_size}")
    timeout = timedelta(seconds=float(os.environ.get("LK_DIST_TIMEOUT_S", "600")))
    if on_cpu or not torch.cuda.is_available():
        dev = torch.device("cpu")
        dist.init_process_group("gloo", timeout=timeout)
    else:
        local = 0 if one_device else int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        from .. import ops

        ops.lib()  # fail loudly if the HIP library is not built
        if one_device:  # RCCL refuses several ranks on one device
            dist.init_process_group("gloo", timeout=timeout)
        else:
            dist.init_process_group("nccl", device_id=dev, timeout=timeout)
    return new_tp_groups(tp_size), dev


def stop_group(procs, leader_first=True, wait_s: float = 30.0):
    """Terminate a TP group's processes: the leader first (it sends the workers "stop"),
    then whatever is still running after ``wait_s``."""
    import time

    if not procs:
        return
    order = procs if leader_first else procs[::-1]
    if order[0].poll() is None:
        order[0].terminate()
    t0 = time.time()
    while time.time() - t0 < wait_s and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=10)
        except subprocess.TimeoutExpired:
            p.kill()
