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
# Round 2 (8192-row steps) measured it neutral; with round 3's 4096-row steps (flash ~60 us,
# paged decode ~84 us per layer) it read 103.38 / 103.18 vs 102.97 / 102.81 q/s with identical
# schedules (mixed-step GPU time -0.45 %, profiles/r3_overlap/): on by default.
OVERLAP_ATTN = os.environ.get("LK_OVERLAP_ATTN", "1") == "1"
# Which kernel goes to the side stream.  The main stream's kernel starts right behind the QKV GEMM,
# the side stream's only after a cross-queue event, so the main one takes the CUs first
# (LK_ATTN_SIDE=decode: the flash kernel leads; =flash: the paged decode leads).
ATTN_SIDE = os.environ.get("LK_ATTN_SIDE", "decode")
# Unified mixed-step attention: ONE flash launch over [prompt rows | decode rows], each decode
# row a one-token sequence (causal, past = ctx - 1) in the same heaviest-first tile list, so the
# HBM-bound decode tiles and the MFMA-bound prompt tiles share every CU instead of two kernels
# waiting for each other's CUs (the model runner builds the combined cu / ctx / block table /
# tile list once per step: ModelRunner._meta).
UNIFIED_ATTN = os.environ.get("LK_UNIFIED_ATTN", "0") == "1"
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
    # unified mixed-step attention (UNIFIED_ATTN): sequences = the prefill chunks, then one
    # per decode row (q_len 1); block tables padded to one width; the flash tile list
    cu_u: Optional[torch.Tensor] = None
    ctx_lens_u: Optional[torch.Tensor] = None
    block_tables_u: Optional[torch.Tensor] = None
    tiles_u: Optional[tuple] = None
    # context parallelism (paged_attention's cp_group): the block tables / ctx_lens above
    # describe THIS rank's contiguous shard of every sequence's keys, whose first key sits
    # at global position cp_key_start_{p,d}[b] (host ints); queries are replicated
    cp_key_start_p: Optional[list] = None
    cp_key_start_d: Optional[list] = None

    @property
    def num_tokens(self) -> int:
        return self.num_prefill_tokens + self.num_decode

    def ensure_tiles(self, Hq: int, Hkv: int, device, D: int = 128):
        """Build the flash-kernel tile list once per step (GPU only)."""
        if self.tiles is None and self.num_prefill_seqs and device.type == "cuda":
            ts, tq = ops.prefill_tiles(self.q_lens_cpu, self.ctx_lens_cpu, Hq // Hkv, True, D)
            self.tiles = (torch.from_numpy(ts).to(device, non_blocking=True),
                          torch.from_numpy(tq).to(device, non_blocking=True))


def paged_attention(qkv: torch.Tensor, k_cache, v_cache, meta: AttnMeta, Hq: int, Hkv: int, D: int,
                    scale: float, out: Optional[torch.Tensor] = None, cp_group=None) -> torch.Tensor:
    """qkv: [T, (Hq+2Hkv)*D] after RoPE (K/V already written to the cache).

    ``cp_group``: a context-parallel process group (default None = no CP).  Each of its
    ranks holds a contiguous shard of every sequence's keys (``meta``'s tables and
    ``cp_key_start_*``) and the same queries; see :func:`cp_paged_attention`."""
    T = qkv.shape[0]
    if out is None:
        out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
    if cp_group is not None and torch.distributed.get_world_size(cp_group) > 1:
        return cp_paged_attention(qkv, k_cache, v_cache, meta, Hq, Hkv, D, scale, out, cp_group)
    Tp = meta.num_prefill_tokens
    Bd = meta.num_decode
    if meta.cu_u is not None and Tp and Bd:
        T = Tp + Bd
        ops.flash_prefill(qkv[:T, : Hq * D], k_cache, v_cache, meta.cu_u, Hq, Hkv, D, scale, True,
                          block_tables=meta.block_tables_u, ctx_lens=meta.ctx_lens_u, tiles=meta.tiles_u,
                          out=out[:T])
        return out

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

    def prefill():
        meta.ensure_tiles(Hq, Hkv, qkv.device, D)
        ops.flash_prefill(qkv[:Tp, : Hq * D], k_cache, v_cache, meta.cu_q, Hq, Hkv, D, scale, True,
                          block_tables=meta.block_tables_p, ctx_lens=meta.ctx_lens_p,
                          q_lens_cpu=meta.q_lens_cpu, ctx_lens_cpu=meta.ctx_lens_cpu,
                          tiles=meta.tiles, out=out[:Tp])

    if (Tp and Bd and OVERLAP_ATTN and qkv.is_cuda and not torch.cuda.is_current_stream_capturing()):
        cur = torch.cuda.current_stream(qkv.device)
        side = _side_stream(qkv.device)
        side.wait_stream(cur)  # Q and the freshly written K/V are ready
        on_side, on_main = (prefill, decode) if ATTN_SIDE == "flash" else (decode, prefill)
        with torch.cuda.stream(side):
            on_side()
        qkv.record_stream(side)
        out.record_stream(side)
        on_main()
        cur.wait_stream(side)
        return out
    if Tp:
        prefill()
    if Bd:
        decode()
    return out


# ---------------------------------------------------------------- context parallelism
def partial_attention(q, k, v, q_pos, k_pos0: int, scale: float, causal: bool = True):
    """Attention of q [S, Hq, D] over one key shard k/v [n, Hkv, D] whose key j sits at
    global position ``k_pos0 + j``; query i at ``q_pos[i]`` sees keys at positions <= its
    own when ``causal``.  Returns (o f32 [S, Hq, D] normalised over the shard, lse f32
    [S, Hq]); a query that sees no key of the shard gets o = 0, lse = -inf."""
    S, Hq, D = q.shape
    n, Hkv, _ = k.shape
    if n == 0:
        return (torch.zeros(S, Hq, D, dtype=torch.float32, device=q.device),
                torch.full((S, Hq), float("-inf"), dtype=torch.float32, device=q.device))
    g = Hq // Hkv
    kf = k.float().repeat_interleave(g, dim=1)
    vf = v.float().repeat_interleave(g, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal:
        kpos = k_pos0 + torch.arange(n, device=q.device)
        s = s.masked_fill((kpos[None, :] > q_pos.to(q.device).long()[:, None])[None], float("-inf"))
    lse = torch.logsumexp(s, dim=-1)                                 # [Hq, S]
    p = torch.exp(s - torch.where(torch.isfinite(lse), lse, torch.zeros_like(lse))[..., None])
    o = torch.einsum("hqk,khd->qhd", p, vf)
    return o, lse.transpose(0, 1).contiguous()


def merge_partials(o: torch.Tensor, lse: torch.Tensor) -> torch.Tensor:
    """LSE-weighted merge of per-shard partials: o [C, S, Hq, D], lse [C, S, Hq] ->
    [S, Hq, D] (exactly softmax attention over the union of the shards)."""
    m = lse.max(dim=0).values
    m = torch.where(torch.isfinite(m), m, torch.zeros_like(m))
    w = torch.exp(lse - m[None])                                     # -inf -> 0
    den = w.sum(dim=0).clamp_min(1e-30)
    return (w[..., None] * o).sum(dim=0) / den[..., None]


_LN2 = 0.6931471805599453


def cp_local_partials(qkv, k_cache, v_cache, meta: AttnMeta, Hq: int, Hkv: int, D: int, scale: float):
    """This rank's attention partials over its key shard: (o f32 [T, Hq, D] normalised over
    the shard, lse f32 [T, Hq], natural log; -inf where a query sees no key of the shard).

    On the GPU: two flash-kernel launches in partial mode and no host sync -- prefill rows
    causally with the mask shifted by the shard's first key position (``q_past`` = global
    position of the first query - ``cp_key_start_p``), decode rows as one-query sequences over
    all their local keys -- so the hook runs inside a captured step.  On the CPU: the fp32
    per-sequence reference (``partial_attention``)."""
    Tp, Bd = meta.num_prefill_tokens, meta.num_decode
    T = Tp + Bd
    if qkv.is_cuda and ops.use_hip(qkv):
        dev = qkv.device
        po = torch.empty(T, Hq, D, dtype=torch.float32, device=dev)
        pml = torch.empty(T, Hq, 2, dtype=torch.float32, device=dev)
        if Tp:
            B = meta.num_prefill_seqs or (meta.cu_q.numel() - 1)
            starts = meta.cp_key_start_p or [0] * B
            k0 = torch.tensor(starts, dtype=torch.int32).to(dev, non_blocking=True)
            q_past = (meta.positions.index_select(0, meta.cu_q[:-1].long()) - k0).to(torch.int32)
            ts, tq = ops.prefill_tiles(meta.q_lens_cpu, meta.ctx_lens_cpu, Hq // Hkv, True, D)
            tiles = (torch.from_numpy(ts).to(dev, non_blocking=True), torch.from_numpy(tq).to(dev, non_blocking=True))
            ops.flash_prefill(qkv[:Tp, : Hq * D], k_cache, v_cache, meta.cu_q, Hq, Hkv, D, scale, True,
                              block_tables=meta.block_tables_p, ctx_lens=meta.ctx_lens_p, tiles=tiles,
                              part=(po[:Tp], pml[:Tp]), q_past=q_past)
        if Bd:
            # decode rows: one-query "sequences" over all their local keys (no mask)
            cu = torch.arange(Bd + 1, dtype=torch.int32, device=dev)
            ts, tq = ops.prefill_tiles([1] * Bd, [1] * Bd, Hq // Hkv, False, D)
            tiles = (torch.from_numpy(ts).to(dev, non_blocking=True), torch.from_numpy(tq).to(dev, non_blocking=True))
            ops.flash_prefill(qkv[Tp:T, : Hq * D], k_cache, v_cache, cu, Hq, Hkv, D, scale, False,
                              block_tables=meta.block_tables_d, ctx_lens=meta.ctx_lens_d, tiles=tiles,
                              part=(po[Tp:], pml[Tp:]))
        m, l = pml[..., 0], pml[..., 1]
        seen = l > 0
        o = torch.where(seen[..., None], po / l.clamp_min(1e-30)[..., None], torch.zeros_like(po))
        lse = torch.where(seen, (m + torch.log2(l.clamp_min(1e-30))) * _LN2, torch.full_like(m, float("-inf")))
        return o, lse
    from ..ops import reference as ref

    q_all = qkv[:T, : Hq * D].reshape(T, Hq, D)
    o_loc = torch.zeros(T, Hq, D, dtype=torch.float32, device=qkv.device)
    l_loc = torch.full((T, Hq), float("-inf"), dtype=torch.float32, device=qkv.device)
    pos = meta.positions[:T].long()
    if Tp:
        cu = [int(x) for x in meta.cu_q.tolist()]
        starts = meta.cp_key_start_p or [0] * (len(cu) - 1)
        for b in range(len(cu) - 1):
            s0, e0 = cu[b], cu[b + 1]
            n = int(meta.ctx_lens_p[b])
            kb = ref.gather_paged(k_cache, meta.block_tables_p[b], n)
            vb = ref.gather_paged(v_cache, meta.block_tables_p[b], n)
            o_loc[s0:e0], l_loc[s0:e0] = partial_attention(q_all[s0:e0], kb, vb, pos[s0:e0], starts[b], scale)
    if Bd:
        starts = meta.cp_key_start_d or [0] * Bd
        for i in range(Bd):
            n = int(meta.ctx_lens_d[i])
            kb = ref.gather_paged(k_cache, meta.block_tables_d[i], n)
            vb = ref.gather_paged(v_cache, meta.block_tables_d[i], n)
            r = Tp + i
            o_loc[r:r + 1], l_loc[r:r + 1] = partial_attention(q_all[r:r + 1], kb, vb, pos[r:r + 1], starts[i],
                                                               scale)
    return o_loc, l_loc


def cp_paged_attention(qkv, k_cache, v_cache, meta: AttnMeta, Hq: int, Hkv: int, D: int, scale: float,
                       out: torch.Tensor, cp_group) -> torch.Tensor:
    """Context-parallel attention: every rank attends the (replicated) queries over its
    local key shard (:func:`cp_local_partials`) -- prefill rows causally by global position,
    decode rows over all their keys -- then ONE all-gather of (o, lse) over ``cp_group`` and
    an LSE merge give each rank the full result.  Collective volume per layer:
    T x Hq x (D + 1) f32 per rank, independent of the context length (the KV shards never
    move)."""
    import torch.distributed as dist

    T = meta.num_prefill_tokens + meta.num_decode
    o_loc, l_loc = cp_local_partials(qkv, k_cache, v_cache, meta, Hq, Hkv, D, scale)
    C = dist.get_world_size(cp_group)
    packed = torch.cat([o_loc.reshape(T, -1), l_loc], dim=1)         # one collective
    allp = [torch.empty_like(packed) for _ in range(C)]
    dist.all_gather(allp, packed, group=cp_group)
    allp = torch.stack(allp)
    o = allp[..., : Hq * D].reshape(C, T, Hq, D)
    lse = allp[..., Hq * D:]
    out[:T] = merge_partials(o, lse).reshape(T, Hq * D).to(out.dtype)
    return out
