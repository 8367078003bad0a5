"""Attention metadata + the paged attention dispatch shared by all decoders.

A batch is laid out as ``[prefill tokens of seq 0..P-1 | one decode token per seq]``.
Prefill rows go through the flash kernel reading K/V from the paged cache (so
chunked prefill and prefix-cache hits are the same code path), decode rows go
through the split-K paged decode kernel.  All index tensors are int32 and built
once per step by the model runner, then shared by every layer.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Optional

import torch

from .. import ops

# Mixed (chunked-prefill + decode) steps: run the memory-bound paged-decode kernel on a
# side HIP stream concurrently with the MFMA-bound flash prefill of the same layer.
OVERLAP_ATTN = os.environ.get("LK_OVERLAP_ATTN", "0") == "1"  # measured neutral on MI355X (off)
_side: dict = {}


def _side_stream(device):
    s = _side.get(device)
    if s is None:
        s = _side[device] = torch.cuda.Stream(device)
    return s


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
    # cascade decode: the first shared_len (device int32 [1]) keys of every decode row are
    # the same cache blocks (the batch's common system prompt): attended once for all rows
    # by the flash kernel (queries = the decode rows, keys = shared_tables' blocks) into
    # (pp_o, pp_ml), merged by the split-K reduce
    shared_len: Optional[torch.Tensor] = None
    shared_cu: Optional[torch.Tensor] = None
    shared_tables: Optional[torch.Tensor] = None
    shared_tiles: Optional[tuple] = None
    pp_o: Optional[torch.Tensor] = None
    pp_ml: Optional[torch.Tensor] = None
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
    Bd = meta.num_decode

    def decode():
        q = qkv[Tp:Tp + Bd, : Hq * D].view(Bd, Hq, D)
        o = out[Tp:Tp + Bd].view(Bd, Hq, D)
        prefix = None
        if meta.shared_len is not None:
            ops.flash_prefill(qkv[Tp:Tp + Bd, : Hq * D], k_cache, v_cache, meta.shared_cu, Hq, Hkv, D, scale,
                              False, block_tables=meta.shared_tables, ctx_lens=meta.shared_len,
                              tiles=meta.shared_tiles, part=(meta.pp_o, meta.pp_ml))
            prefix = (meta.pp_o, meta.pp_ml)
        ops.paged_decode(q, k_cache, v_cache, meta.block_tables_d, meta.ctx_lens_d, scale,
                         meta.max_splits, meta.part_o, meta.part_ml, out=o, split=meta.decode_split,
                         k_start=meta.shared_len, prefix=prefix)

    side = None
    if (Tp and Bd and OVERLAP_ATTN and qkv.is_cuda and not torch.cuda.is_current_stream_capturing()):
        cur = torch.cuda.current_stream(qkv.device)
        side = _side_stream(qkv.device)
        side.wait_stream(cur)  # Q and the freshly written K/V are ready
        with torch.cuda.stream(side):
            decode()
        qkv.record_stream(side)
        out.record_stream(side)
    if Tp:
        meta.ensure_tiles(Hq, Hkv, qkv.device)
        ops.flash_prefill(qkv[:Tp, : Hq * D], k_cache, v_cache, meta.cu_q, Hq, Hkv, D, scale, True,
                          block_tables=meta.block_tables_p, ctx_lens=meta.ctx_lens_p,
                          q_lens_cpu=meta.q_lens_cpu, ctx_lens_cpu=meta.ctx_lens_cpu,
                          tiles=meta.tiles, out=out[:Tp])
    if side is not None:
        torch.cuda.current_stream(qkv.device).wait_stream(side)
    elif Bd:
        decode()
    return out
