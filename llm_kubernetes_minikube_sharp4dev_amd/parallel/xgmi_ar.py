"""One-shot xGMI all-reduce (K14, csrc/xgmi_allreduce.hip) for latency-bound TP decode.

Each rank exports an IPC staging + signal buffer; the handles are exchanged once over
the TP group's CPU (gloo) control group, every rank maps its peers' buffers, and
:meth:`XgmiAllReduce.all_reduce_` then runs one kernel: stage -> per-workgroup flag
handshake -> read and sum all ranks' slices -> handshake.  hipGraph-capturable (the
epochs live in device memory).  Messages larger than the staging buffer, non-bf16 or
non-contiguous tensors go to RCCL.

Opt-in (``LK_XGMI_AR=1``, or :func:`attach`): RCCL stays the default collective.  On a
full-mesh node each MI355X reads its 7 peers' slices over 7 links at once, so a
B x 8192 bf16 decode all-reduce is one kernel instead of RCCL's multi-hop ring.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops import lib


class XgmiAllReduce:
    def __init__(self, tp, max_bytes: int = 8 << 20):
        self.tp = tp
        self.max_bytes = max_bytes
        self.state = lib().XgmiAr(tp.rank, tp.size, max_bytes)
        mine = self.state.handles()
        blobs = [None] * tp.size
        group = tp.ctrl if tp.ctrl is not None else tp.group
        dist.all_gather_object(blobs, mine, group=group)
        self.state.open(blobs)

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
                and t.numel() * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        self.state.all_reduce(t, t)
        return t

    def eligible_rows(self, x: torch.Tensor, residual: torch.Tensor) -> bool:
        return (self.eligible(x) and x.dim() == 2 and residual.is_contiguous() and residual.shape == x.shape
                and residual.dtype == torch.bfloat16 and x.shape[1] % 8 == 0)

    def all_reduce_rmsnorm_(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                            out: torch.Tensor | None = None) -> torch.Tensor:
        """RMSNorm(allreduce(x) + residual) * w in ONE kernel (residual updated in place):
        the TP decode layer's "row-parallel GEMM -> all-reduce -> add -> norm" tail."""
        if out is None:
            out = torch.empty_like(x)
        self.state.all_reduce_rmsnorm(x, residual, w.contiguous(), float(eps), out)
        return out

    def error(self) -> int:
        """Non-zero if a handshake ever timed out (a peer missing a call)."""
        return self.state.error()


def attach(tp, max_bytes: int = 8 << 20) -> XgmiAllReduce:
    """Route this TP group's eligible all-reduces through the one-shot kernel."""
    tp.xgmi = XgmiAllReduce(tp, max_bytes)
    return tp.xgmi
