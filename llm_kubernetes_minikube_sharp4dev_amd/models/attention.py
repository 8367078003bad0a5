"""Attention metadata + the paged attention dispatch shared by all decoders.

A batch is laid out as ``[prefill tokens of seq 0..P-1 | one decode token per seq]``.
Prefill rows go through the flash kernel reading K/V from the paged cache (so
chunked prefill and prefix-cache hits are the same code path), decode rows go
through the split-K paged decode kernel.  All index tensors are int32 and built
once per step by the model runner, then shared by every layer.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import ops


@dataclass
class AttnMeta:
    positions: torch.Tensor                  # [T] int32
    slots: torch.Tensor                      # [T] int32 (-1 = do not cache)
    num_prefill_tokens: int = 0              # Tp
    num_prefill_seqs: int = 0
    num_decode: int = 0                      # Bd
    # prefill part
    cu_q: Optional[torch.Tensor] = None      # [Bp+1]
    ctx_lens_p: Optional[torch.Tensor] = None
    block_tables_p: Optional[torch.Tensor] = None
    q_lens_cpu: list = field(default_factory=list)
    ctx_lens_cpu: list = field(default_factory=list)
    tiles: Optional[tuple] = None
    # decode part
    block_tables_d: Optional[torch.Tensor] = None
    ctx_lens_d: Optional[torch.Tensor] = None
    max_splits: Optional[int] = None
    decode_split: Optional[int] = None
    part_o: Optional[torch.Tensor] = None
    part_ml: Optional[torch.Tensor] = None
    # rows whose hidden state feeds the LM head (last token of each prefill + decode rows)
    logits_idx: Optional[torch.Tensor] = None

    @property
    def num_tokens(self) -> int:
        return self.num_prefill_tokens + self.num_decode

    def ensure_tiles(self, Hq: int, Hkv: int, device):
        """Build the flash-kernel tile list once per step (GPU only)."""
        if self.tiles is None and self.num_prefill_seqs and device.type == "cuda":
            ts, tq = ops.prefill_tiles(self.q_lens_cpu, self.ctx_lens_cpu, Hq // Hkv, True)
            self.tiles = (torch.from_numpy(ts).to(device, non_blocking=True),
                          torch.from_numpy(tq).to(device, non_blocking=True))


def paged_attention(qkv: torch.Tensor, k_cache, v_cache, meta: AttnMeta, Hq: int, Hkv: int, D: int,
                    scale: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """qkv: [T, (Hq+2Hkv)*D] after RoPE (K/V already written to the cache)."""
    T = qkv.shape[0]
    if out is None:
        out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    Tp = meta.num_prefill_tokens
    if Tp:
        meta.ensure_tiles(Hq, Hkv, qkv.device)
        ops.flash_prefill(qkv[:Tp, : Hq * D], k_cache, v_cache, meta.cu_q, Hq, Hkv, D, scale, True,
                          block_tables=meta.block_tables_p, ctx_lens=meta.ctx_lens_p,
                          q_lens_cpu=meta.q_lens_cpu, ctx_lens_cpu=meta.ctx_lens_cpu,
                          tiles=meta.tiles, out=out[:Tp])
    Bd = meta.num_decode
    if Bd:
        q = qkv[Tp:Tp + Bd, : Hq * D].view(Bd, Hq, D)
        o = out[Tp:Tp + Bd].view(Bd, Hq, D)
        ops.paged_decode(q, k_cache, v_cache, meta.block_tables_d, meta.ctx_lens_d, scale,
                         meta.max_splits, meta.part_o, meta.part_ml, out=o, split=meta.decode_split)
    return out
