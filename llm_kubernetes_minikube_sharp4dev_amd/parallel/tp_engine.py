"""Tensor-parallel generation (Llama-3-70B TP=8 over xGMI, BASELINE.json config 4).

One process per GPU.  Rank 0 owns the scheduler, the block allocator and the
sampler; every step it broadcasts the host-side :class:`StepInputs` to the other
ranks over a small CPU (gloo) control group, then all ranks run the same forward
in lockstep — weights and KV heads sharded, two RCCL all-reduces per layer, vocab
all-gather for the logits.  Decode hipGraphs are captured on every rank for the
same batch buckets (RCCL calls inside the graph), so a TP decode step is one graph
replay per GPU.

    tp = init_distributed()                    # torchrun, backend nccl (RCCL)
    model = build_decoder("llama-3-70b", device=f"cuda:{rank}", tp=tp)
    if rank == 0:
        engine = make_tp_engine(model, tp, ...); engine.generate(...); shutdown(engine)
    else:
        run_tp_worker(model, tp, ...)
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from ..engine.model_runner import ModelRunner
from ..utils.logging import get_logger
from .tp import TPGroup

log = get_logger("tp")


class _Ctrl:
    def __init__(self, tp: TPGroup):
        self.tp = tp
        if tp.size > 1 and tp.ctrl is not None:
            self.group, self.src = tp.ctrl, tp.ranks[0]
        elif tp.size > 1:
            ranks = dist.get_process_group_ranks(tp.group) if tp.group is not None else list(range(tp.size))
            self.group = dist.new_group(ranks, backend="gloo")
            self.src = ranks[0]
        else:
            self.group, self.src = None, 0

    def bcast(self, obj=None):
        if self.tp.size == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=self.src, group=self.group)
        return box[0]


def _agree_num_blocks(model, tp: TPGroup, **kw) -> int:
    """Size the KV pool from this rank's free memory, then take the group minimum
    (rank 0's allocator hands out block ids that every rank must hold)."""
    keys = ("block_size", "max_model_len", "max_num_seqs", "kv_cache_gb", "gpu_memory_fraction")
    n = torch.tensor([ModelRunner.plan_num_blocks(model, **{k: kw[k] for k in keys if k in kw})], dtype=torch.int64)
    if tp.size > 1:
        if torch.cuda.is_available() and model.device.type == "cuda":
            n = n.to(model.device)
        dist.all_reduce(n, op=dist.ReduceOp.MIN, group=tp.group)
    return int(n.item())


def make_tp_runner(model, tp: TPGroup, **runner_kw) -> tuple[ModelRunner, _Ctrl]:
    ctrl = _Ctrl(tp)
    nb = runner_kw.pop("num_blocks", None)
    if nb is None:
        nb = _agree_num_blocks(model, tp, **runner_kw)
    runner = ModelRunner(model, num_blocks=nb, **runner_kw)
    return runner, ctrl


def make_tp_engine(model, tp: TPGroup, tokenizer=None, engine_kw: Optional[dict] = None, **runner_kw):
    """Rank 0: an LLMEngine whose runner broadcasts each step to the TP workers."""
    from ..engine.llm_engine import LLMEngine

    runner, ctrl = make_tp_runner(model, tp, **runner_kw)
    ekw = dict(engine_kw or {})
    eng = LLMEngine.__new__(LLMEngine)
    LLMEngine.__init__(eng, model, tokenizer, block_size=runner.bs, max_model_len=runner.max_model_len,
                       max_num_seqs=runner.max_num_seqs, num_blocks=runner.num_blocks, use_graphs=runner.use_graphs,
                       _runner=runner, **ekw)
    runner.step_hook = lambda si: ctrl.bcast(("step", si))
    eng.tp_ctrl = ctrl
    return eng


def tp_capture_all(engine, max_batch: Optional[int] = None, variants=(False, True)):
    """Capture decode graphs on every rank in lockstep."""
    r = engine.runner
    for B in r.graph_sizes:
        for v in variants:
            if (max_batch is None or B <= max_batch) and (B, v) not in r.graphs:
                engine.tp_ctrl.bcast(("capture", (B, v)))
                r.capture(B, v)


def shutdown_tp(engine):
    engine.tp_ctrl.bcast(("stop", None))


def tp_barrier(engine):
    """World barrier (after a device sync) from the TP driver while its workers sit in
    run_tp_worker: they receive a "barrier" command and join the same barrier."""
    ctrl = getattr(engine, "tp_ctrl", None)
    if ctrl is not None:
        ctrl.bcast(("barrier", None))
    if torch.cuda.is_available() and engine.model.device.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()


@torch.inference_mode()
def run_tp_worker(model, tp: TPGroup, **runner_kw):
    """Ranks > 0: execute whatever rank 0 schedules until it says stop."""
    from ..utils.watchdog import StepWatchdog

    stall_s = float(runner_kw.pop("stall_s", 600.0)) if "stall_s" in runner_kw else 600.0
    runner, ctrl = make_tp_runner(model, tp, **runner_kw)
    wd = StepWatchdog(f"tp-worker-{tp.rank}", stall_s=stall_s)
    n = 0
    pending: list = []
    while True:
        cmd, arg = ctrl.bcast(None)  # idle wait for the driver: not a stall
        wd.beat()
        if cmd == "stop":
            for ev in pending:
                ev.synchronize()
            break
        if cmd == "capture":
            runner.capture(*arg)
        elif cmd == "barrier":
            if torch.cuda.is_available() and model.device.type == "cuda":
                torch.cuda.synchronize()
            dist.barrier()
        elif cmd == "step":
            with wd.busy():  # a step that never returns (dead peer in an all-reduce) is a stall
                runner.execute(arg)
                if torch.cuda.is_available() and model.device.type == "cuda":
                    # keep <= 2 steps in flight (the driver pipelines: step N+1's inputs
                    # arrive before step N is done, so the device never idles waiting here)
                    ev = torch.cuda.Event()
                    ev.record()
                    pending.append(ev)
                    if len(pending) > 2:
                        pending.pop(0).synchronize()
            n += 1
    wd.stop()
    log.info("tp worker rank %d done after %d steps", tp.rank, n)
    return n
