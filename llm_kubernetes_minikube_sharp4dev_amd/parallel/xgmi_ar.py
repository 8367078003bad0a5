"""xGMI all-reduce over IPC-mapped peer memory (K14, csrc/xgmi_allreduce.hip).

Each rank exports an IPC staging (two regions) + signal buffer; the handles are exchanged
once over the TP group's CPU (gloo) control group, every rank maps its peers' buffers, and
every call is ONE kernel with per-workgroup flag handshakes (hipGraph-capturable: the epochs
live in device memory):

* one-shot (decode-sized messages): stage -> handshake -> read and sum every rank's copy ->
  handshake.  Latency-optimal; each of the 7 links carries the whole message S.
* two-shot (prefill-sized messages, ``>= LK_XGMI_2SHOT_MIN_KB`` on >= 4 ranks): reduce-scatter
  + all-gather through the same mappings, 2S/world per link (S/4 on 8 ranks) for one more
  handshake.  Bit-identical to one-shot.

Both have a fused residual + RMSNorm form (:meth:`XgmiAllReduce.all_reduce_rmsnorm_`), the
tail of every row-parallel projection.  Messages larger than the staging region, non-bf16 or
non-contiguous tensors go to RCCL.

Opt-in (``LK_XGMI_AR=1``, or :func:`attach`): RCCL stays the default collective.  Staging
region size: ``LK_XGMI_AR_MB`` (default 64 MB = a 4096-token x 8192 bf16 prefill message; the
buffer holds two regions).  The one-/two-shot crossover is a link-model default that the
8-GPU run should re-tune.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from ..ops import lib


def _default_bytes() -> int:
    return int(float(os.environ.get("LK_XGMI_AR_MB", "64")) * (1 << 20)) // 16 * 16


class XgmiAllReduce:
    def __init__(self, tp, max_bytes: int | None = None, two_shot: bool | None = None):
        self.tp = tp
        self.max_bytes = max_bytes if max_bytes is not None else _default_bytes()
        # None: by size (>= two_shot_min bytes on >= 4 ranks); True / False: always / never
        self.two_shot = two_shot
        self.two_shot_min = int(float(os.environ.get("LK_XGMI_2SHOT_MIN_KB", "1024")) * 1024)
        self.state = lib().XgmiAr(tp.rank, tp.size, self.max_bytes)
        mine = self.state.handles()
        blobs = [None] * tp.size
        group = tp.ctrl if tp.ctrl is not None else tp.group
        dist.all_gather_object(blobs, mine, group=group)
        self.state.open(blobs)

    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
                and t.numel() * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def use_two_shot(self, t: torch.Tensor) -> bool:
        if self.two_shot is not None:
            return self.two_shot
        return self.tp.size >= 4 and t.numel() * 2 >= self.two_shot_min

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.use_two_shot(t):
            v = t.view(-1, t.shape[-1]) if t.dim() >= 2 and t.shape[-1] % 8 == 0 else t.view(-1, 8)
            self.state.all_reduce2(v, v)
        else:
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
        if self.use_two_shot(x):
            self.state.all_reduce2(x, out, residual, w.contiguous(), float(eps))
        else:
            self.state.all_reduce_rmsnorm(x, residual, w.contiguous(), float(eps), out)
        return out

    def error(self) -> int:
        """Non-zero if a handshake ever timed out (a peer missing a call)."""
        return self.state.error()


def attach(tp, max_bytes: int | None = None) -> XgmiAllReduce:
    """Route this TP group's eligible all-reduces through the xGMI kernels."""
    tp.xgmi = XgmiAllReduce(tp, max_bytes)
    return tp.xgmi
