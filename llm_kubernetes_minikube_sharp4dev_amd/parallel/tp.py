"""Tensor-parallel process group helpers (RCCL over xGMI through torch.distributed's
``nccl`` backend on ROCm; ``gloo`` for CPU tests).

Sharding scheme (Megatron-style, sized for 8xMI355X xGMI full mesh):
  * column-parallel: fused QKV (whole heads per rank), fused gate_up (I/tp per rank)
  * row-parallel:    o_proj, down_proj -> one all-reduce each per layer
  * vocab-parallel:  embedding (masked lookup + all-reduce) and LM head
                     (local logits; greedy = all-gather of per-rank (max, argmax))
  * sequence-parallel (prefill-sized steps, Megatron SP): the residual stream and
                     the RMSNorms run on T/tp rows; each row-parallel all-reduce
                     becomes a reduce-scatter, and an all-gather feeds the next
                     column-parallel GEMM (same bytes on the wire, 1/tp of the
                     norm / residual traffic and activation memory per rank)
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class TPGroup:
    rank: int = 0
    size: int = 1
    group: Optional[object] = None
    # CPU (gloo) control group of the same ranks + their global ranks; created on ALL
    # ranks by new_tp_groups (torch requires every rank to join every new_group call)
    ctrl: Optional[object] = None
    ranks: Optional[list] = None
    # xGMI collectives over IPC-mapped peer memory (parallel.xgmi_ar, K14): the fused
    # all-reduce + norm tails by the start-up-measured table, all-gathers / broadcasts
    xgmi: Optional[object] = None
    # the IPC self-check report of a group taken OFF the IPC path by it (xgmi is then None)
    xgmi_check: Optional[dict] = None
    # every device collective on the IPC path, never RCCL (several ranks on one device, where
    # RCCL refuses the communicator; LK_TP_COLLECTIVES=ipc)
    ipc_only: bool = False

    @property
    def enabled(self) -> bool:
        return self.size > 1

    def _ipc(self, t: torch.Tensor) -> bool:
        return self.xgmi is not None and t.is_cuda

    def _ipc_gather(self, t: torch.Tensor) -> bool:
        """IPC all-gather / broadcast: attached, verified against the reference at start-up
        (XgmiAllReduce.self_check), and the message fits the staging region."""
        return (self._ipc(t) and getattr(self.xgmi, "gather_ok", True)
                and t.numel() * t.element_size() <= self.xgmi.max_bytes)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self._ipc(t):
                if self.ipc_only:
                    return self.xgmi.all_reduce_(t)
                rows = t.shape[0] if t.dim() >= 2 else 1
                if self.xgmi.eligible(t) and self.xgmi.algo(rows, t.numel() * 2) != "rccl":
                    return self.xgmi.all_reduce_(t)
            dist.all_reduce(t, group=self.group)
        return t

    def all_reduce_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                           eps: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """RMSNorm(allreduce(x) + residual) * w, residual updated in place: the tail of every
        row-parallel projection.  On the IPC path ONE kernel (csrc/xgmi_allreduce.hip, one- or
        two-shot by the measured table); otherwise RCCL all-reduce + the fused add+norm kernel.
        ``out``: write the normed rows there (a row slice of a bigger buffer)."""
        from .. import ops

        if self.size > 1 and self._ipc(x) and self.xgmi.eligible_rows(x, residual):
            algo = self.xgmi.algo(x.shape[0], x.numel() * 2)
            if algo != "rccl":
                return self.xgmi.all_reduce_rmsnorm_(x, residual, w, eps, out=out, algo=algo)
        self.all_reduce_(x)
        return ops.rmsnorm(x, w, eps, residual=residual, out=out)

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Sum over ranks of t [size*n, ...], this rank's rows [rank*n, (rank+1)*n)."""
        if self.size == 1:
            return t
        n = t.shape[0] // self.size
        if self.ipc_only and self._ipc(t):
            self.all_reduce_(t)
            return t[self.rank * n:(self.rank + 1) * n].contiguous()
        if dist.get_backend(self.group) == "gloo":  # gloo has no reduce_scatter
            dist.all_reduce(t, group=self.group)
            return t[self.rank * n:(self.rank + 1) * n].contiguous()
        out = torch.empty((n,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.reduce_scatter_tensor(out, t.contiguous(), group=self.group)
        return out

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenation over ranks of t [n, ...] -> [size*n, ...]."""
        if self.size == 1:
            return t
        if self._ipc_gather(t):
            return self.xgmi.all_gather(t).reshape((t.shape[0] * self.size,) + tuple(t.shape[1:]))
        if dist.get_backend(self.group) == "gloo":
            return self.all_gather_cat(t, dim=0)
        out = torch.empty((t.shape[0] * self.size,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous(), group=self.group)
        return out

    def all_gather_cat(self, t: torch.Tensor, dim: int = -1) -> torch.Tensor:
        if self.size == 1:
            return t
        if self._ipc_gather(t):
            return torch.cat(list(self.xgmi.all_gather(t)), dim=dim)
        parts = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(parts, t.contiguous(), group=self.group)
        return torch.cat(parts, dim=dim)

    def greedy_ids(self, local_logits: torch.Tensor, vocab_lo: int = 0) -> torch.Tensor:
        """Greedy token ids from vocab-parallel logits [R, V/tp]: local (max, argmax),
        all-gather of R (value, id) pairs per rank instead of the [R, V] logits, pick the
        max (first rank on ties = lowest id, the single-GPU argmax order)."""
        from .. import ops

        if self.size == 1:
            ids = ops.select_tokens(local_logits)  # HIP argmax on the bf16 logits (first max), int32
            return ids if vocab_lo == 0 else ids + vocab_lo
        # ONE all-gather of packed (value, global id) pairs -- an order-preserving int64 key per
        # row (ops.argmax_key: the max's float bits high, ~id low, so the largest key is the
        # largest value and, on ties, the lowest id) -- then the max key over ranks
        key = ops.argmax_key(local_logits, vocab_lo)
        keys = self.all_gather_cat(key[None], dim=0)
        return ops.key_to_id(keys.max(dim=0).values)

    def broadcast_(self, t: torch.Tensor) -> torch.Tensor:
        """In place: the group leader's ``t`` on every rank."""
        if self.size > 1:
            if self._ipc_gather(t):
                return self.xgmi.broadcast_(t, root=0)
            dist.broadcast(t, src=self.ranks[0] if self.ranks else 0, group=self.group)
        return t

    def shard(self, n: int) -> tuple[int, int]:
        """[start, end) of this rank's slice of a dimension of size n (n % size == 0)."""
        if n % self.size:
            raise ValueError(f"dimension {n} not divisible by tp={self.size}")
        per = n // self.size
        return self.rank * per, (self.rank + 1) * per


SINGLE = TPGroup()


@dataclass
class SimulatedTPGroup(TPGroup):
    """Rank ``rank`` of a TP group of ``size`` ranks, simulated in ONE process on one device.

    The model instantiates exactly that rank's shard (its heads, its slice of the FFN, its
    vocab shard of the embedding / LM head), and every collective is a local stand-in with
    the real output shape: all-reduce = identity, reduce-scatter = this rank's rows,
    all-gathers = this rank's part replicated.  Values are one rank's partial sums, not the
    model's (random-init weights either way), but every kernel the rank runs runs at its
    serving shape -- so a single MI355X measures the per-rank compute of a 70B TP=8 step,
    and rocprof shows which kernels that rank would run (``bench.py --tp-sim 8``).  The
    collectives themselves are budgeted from their message sizes (bench.py reports the
    all-reduce bytes of the timed steps)."""

    simulated: bool = True

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        return t

    def reduce_scatter_rows(self, t: torch.Tensor) -> torch.Tensor:
        n = t.shape[0] // self.size
        return t[self.rank * n:(self.rank + 1) * n].contiguous()

    def all_gather_rows(self, t: torch.Tensor) -> torch.Tensor:
        return t.repeat(self.size, *([1] * (t.dim() - 1)))

    def all_gather_cat(self, t: torch.Tensor, dim: int = -1) -> torch.Tensor:
        return torch.cat([t] * self.size, dim=dim)

    def greedy_ids(self, local_logits: torch.Tensor, vocab_lo: int = 0) -> torch.Tensor:
        from .. import ops

        return (ops.select_tokens(local_logits).long() + vocab_lo).int()

    def broadcast_(self, t: torch.Tensor) -> torch.Tensor:
        return t


def init_distributed(backend: Optional[str] = None) -> TPGroup:
    """Initialise torch.distributed from RANK/WORLD_SIZE/MASTER_* env (torchrun) and return
    a TP group spanning the world.  No-op (single rank) when WORLD_SIZE is unset."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return SINGLE
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29500")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        # collectives on a dead / hung rank fail after this instead of blocking forever
        from datetime import timedelta

        dist.init_process_group(backend=backend,
                                timeout=timedelta(seconds=float(os.environ.get("LK_DIST_TIMEOUT_S", "600"))))
    return TPGroup(dist.get_rank(), dist.get_world_size(), dist.group.WORLD)


def new_tp_groups(tp_size: int, with_ctrl: bool = True) -> TPGroup:
    """Split the world into contiguous TP groups of ``tp_size`` (DP across groups).
    Every rank creates every group (device group on the default backend -- RCCL on the
    GPU -- and, with ``with_ctrl``, a gloo control group for the TP engine's step
    broadcasts) in the same order."""
    ws, rank = dist.get_world_size(), dist.get_rank()
    if ws % tp_size:
        raise ValueError("world size must be a multiple of tp size")
    mine = None
    for g in range(ws // tp_size):
        ranks = list(range(g * tp_size, (g + 1) * tp_size))
        grp = dist.new_group(ranks)
        ctrl = dist.new_group(ranks, backend="gloo") if with_ctrl and tp_size > 1 else None
        if rank in ranks:
            mine = TPGroup(ranks.index(rank), tp_size, grp, ctrl, ranks)
    if mine is not None and tp_size > 1:
        mode = collectives_mode()
        if mode == "ipc":
            mine.ipc_only = True
        if mode == "auto" and not _same_host(mine):
            mode = "rccl"  # IPC handles map only within one host: a group spanning nodes stays on RCCL
        if mode in ("ipc", "auto") and torch.cuda.is_available():
            from .xgmi_ar import attach  # xGMI IPC collectives (K14); the table is tuned with the model

            attach(mine, rccl=mode == "auto" and dist.get_backend(mine.group) == "nccl")
    return mine


def _same_host(tp: TPGroup) -> bool:
    """Every rank of the group on this rank's host (gathered over the control group)."""
    import socket

    group = tp.ctrl if tp.ctrl is not None else tp.group
    names = [None] * tp.size
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return len(set(names)) == 1


def collectives_mode() -> str:
    """LK_TP_COLLECTIVES: ``auto`` (default: IPC kernels attached, each all-reduce size routed by
    the start-up measurement, RCCL one of the candidates), ``rccl`` (RCCL only, round-3
    behaviour), ``ipc`` (IPC kernels only -- the mode for several ranks on one device)."""
    m = os.environ.get("LK_TP_COLLECTIVES", "auto")
    if os.environ.get("LK_XGMI_AR") == "0":
        m = "rccl"
    if m not in ("auto", "rccl", "ipc"):
        raise ValueError(f"LK_TP_COLLECTIVES must be auto / rccl / ipc, not {m!r}")
    return m
