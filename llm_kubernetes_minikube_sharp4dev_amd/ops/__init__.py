"""Kernel entry points.  GPU tensors -> hand-written gfx950 HIP kernels (``_C``);
CPU tensors -> fp32 torch references (``reference``).  See ``_ext`` for the policy.

Layouts are documented in :mod:`.reference`.
"""
from __future__ import annotations

import logging
import math
import os
from typing import Optional, Sequence

import numpy as np
import torch

from . import reference as ref
from ._ext import available, force_reference, lib, use_hip  # noqa: F401

__all__ = [
    "rmsnorm", "layernorm", "embed_layernorm", "silu_mul", "gelu_", "relu_", "rope_kv_",
    "kv_write", "paged_decode", "flash_prefill", "prefill_tiles", "knn_topk", "knn_merge",
    "pool_normalize", "row_norms", "select_tokens", "repeat_penalty_", "sample", "linear", "linear_swiglu",
    "decode_splits", "rope_cos_sin", "argmax_key", "key_to_id", "tune_gemm", "tune_decode", "gemm", "linear_add_rmsnorm", "linear_rope_kv",
    "prefill_chain_ok", "linear_resid", "linear_qkv_fused", "linear_swiglu_scaled", "embed_rows", "scatter_ids",
    "gather_rows",
]

rope_cos_sin = ref.rope_cos_sin
DECODE_MAX_SPLIT = 2048  # csrc/attn_decode.hip kMaxSplit


def rmsnorm(x, w, eps: float, residual: Optional[torch.Tensor] = None, out=None):
    """out = RMSNorm(x [+ residual]) * w; if ``residual`` is given it is updated in
    place to ``x + residual`` (fused add+norm of the pre-norm decoder block)."""
    if use_hip(x):
        return lib().rmsnorm(x, w, eps, residual, out)
    y = ref.rmsnorm(x, w, eps, residual)
    if out is not None:
        out.copy_(y)
        return out
    return y


def layernorm(x, w, b, eps: float, residual=None, write_residual: bool = False):
    if use_hip(x):
        return lib().layernorm(x, w, b, eps, residual, write_residual)
    return ref.layernorm(x, w, b, eps, residual, write_residual)


def embed_layernorm(ids, pos_ids, type_ids, tok, pos, typ, w, b, eps: float):
    if use_hip(tok):
        return lib().embed_layernorm(ids, pos_ids, type_ids, tok, pos, typ, w, b, eps)
    return ref.embed_layernorm(ids, pos_ids, type_ids, tok, pos, typ, w, b, eps)


def silu_mul(x, out=None):
    if use_hip(x):
        return lib().silu_mul(x, out)
    y = ref.silu_mul(x)
    if out is not None:
        out.copy_(y)
        return out
    return y


def gelu_(x, bias=None, approximate: str = "none"):
    kind = 1 if approximate == "tanh" else 0
    if use_hip(x):
        lib().activation_(x, bias, kind)
        return x
    return ref.activation_(x, bias, kind)


def relu_(x, bias=None):
    if use_hip(x):
        lib().activation_(x, bias, 2)
        return x
    return ref.activation_(x, bias, 2)


def rope_kv_(qkv, positions, cos_sin, Hq: int, Hkv: int, D: int, k_cache=None, v_cache=None,
             slots=None, neox: bool = True, write_k_inplace: bool = False):
    if use_hip(qkv):
        lib().rope_kv_(qkv, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox,
                       write_k_inplace)
        return qkv
    return ref.rope_kv_(qkv, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox,
                        write_k_inplace)


def kv_write(k, v, k_cache, v_cache, slots):
    if use_hip(k):
        return lib().kv_write(k, v, k_cache, v_cache, slots)
    return ref.kv_write(k, v, k_cache, v_cache, slots)


# keys per decode workgroup once the batch alone fills the CUs (B * Hkv >= 512); LK_DECODE_SPLIT
# overrides it (A/B knob: three 256-thread workgroups per CU make 768 slots, so ~1.1-1.5 rounds
# of unsplit workgroups at the serving batch leave part of the last round idle).  2048: the RAG
# bench's ~1k-key rows stay in one split, so no step launches the split-merge kernel (same box,
# interleaved: mixed-step GPU time 9.21 / 9.18 vs 9.25 / 9.25 s, 108.2 / 108.3 vs 108.2 / 107.8 q/s)
DECODE_SPLIT_LARGE = int(os.environ.get("LK_DECODE_SPLIT", "2048"))
# keys per decode workgroup below 32 (sequence, kv head) pairs (batch 1: 8 kv heads)
DECODE_SPLIT_SMALL = int(os.environ.get("LK_DECODE_SPLIT_SMALL", "128"))


def decode_split_size(B: int, Hkv: int) -> int:
    """Keys per decode workgroup (mirrors lk_decode_split_size): small batches split the
    context finer so 256 CUs stay busy; static per (B, Hkv) for hipGraph capture."""
    bh = B * Hkv
    return DECODE_SPLIT_LARGE if bh >= 512 else 512 if bh >= 128 else 256 if bh >= 32 else DECODE_SPLIT_SMALL


def decode_splits(max_context: int, split: int) -> int:
    return max(1, (int(max_context) + split - 1) // split)


# Split decode: the last split workgroup of each (sequence, kv head) merges the partials
# itself (csrc/attn_decode.hip merge_splits) instead of a decode_reduce launch after the kernel.
# Needs one zero-initialised int32 ticket per (sequence, kv head), reset by its last taker: a
# per-device buffer made before any graph capture.  Used where the batch fills the CUs unsplit
# (B x Hkv >= 512, 2048-key workgroups): rows of <= 2048 keys write their output directly and the
# reduce launch (which round 5 made on every layer of every step, to find nothing to merge) is
# gone.  At small batches, where every row splits, the separate reduce kernel measured faster
# (batch 1, same box, twice each: decode step 3.74 / 3.73 ms fused vs 3.65 / 3.61 ms,
# profiles/r6_fused_merge/): the split workgroups' write-through partials and ticket sit on the
# critical path.  LK_DECODE_FUSED_REDUCE=0: never, =2: always.
DECODE_FUSED_REDUCE = int(os.environ.get("LK_DECODE_FUSED_REDUCE", "1") or 0)
_DECODE_TICKETS: dict = {}


def decode_tickets(device, n: int):
    device = torch.device(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = _DECODE_TICKETS.get(key)
    if t is None or t.numel() < n:
        t = _DECODE_TICKETS[key] = torch.zeros(max(n, 1 << 16), dtype=torch.int32, device=device)
    return t


def paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale: float, max_splits: Optional[int] = None,
                 part_o=None, part_ml=None, out=None, split: Optional[int] = None, k_start=None, prefix=None,
                 reduce: bool = True):
    """q [B, Hq, D] -> [B, Hq, D].  ``split`` keys per workgroup (default from
    :func:`decode_split_size`), ``max_splits`` = splits covering the block-table width —
    both static, so the launch is hipGraph-capturable.

    Cascade: ``k_start`` (device int32 [1]) keys are a prefix shared by every row whose
    attention was computed once for the batch by :func:`flash_prefill` in partial mode
    into ``prefix`` = (o [B, Hq, D], ml [B, Hq, 2]); this call attends the rest and
    merges (the CPU reference attends everything directly).  ``reduce=False`` (GPU, no
    tickets): rows with more than one split keep their partials in ``part_o`` / ``part_ml`` for
    the consumer to merge (:func:`ws_pro` kind 2)."""
    if use_hip(q):
        BS = k_cache.shape[2]
        if split is None:
            split = max(decode_split_size(q.shape[0], k_cache.shape[1]), BS)
        if max_splits is None:
            max_splits = decode_splits(block_tables.shape[1] * BS, split)
        pp_o, pp_ml = prefix if prefix is not None else (None, None)
        bh = q.shape[0] * k_cache.shape[1]
        fused = reduce and (DECODE_FUSED_REDUCE == 2 or (DECODE_FUSED_REDUCE == 1 and bh >= 512))
        tickets = decode_tickets(q.device, bh) if fused else None
        return lib().paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, max_splits, split, scale,
                                  part_o, part_ml, out, k_start, pp_o, pp_ml, tickets, reduce)
    y = ref.paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, scale)
    if out is not None:
        out.copy_(y)
        return out
    return y


def prefill_rows_per_tile(G: int, D: int = 128) -> int:
    """Query rows per flash-prefill tile: the HIP library's choice for (GQA group, head dim)
    (8-wave 64-row workgroups for G >= 4, D >= 64 under LK_PREFILL_WAVES=8), else 32 / 4-wave."""
    try:
        return int(lib().prefill_rows_per_tile(G, D))
    except Exception:  # no extension (CPU): the tiles only matter to the HIP kernel
        return 32 if G >= 4 else 32 * (4 // G)


def prefill_tiles(q_lens: Sequence[int], ctx_lens: Sequence[int], G: int, causal: bool, D: int = 128):
    """Query tiles (seq, q0) for the flash kernel, heaviest first (LPT scheduling:
    with causal masking a tile's cost grows with the keys it sees)."""
    qb = prefill_rows_per_tile(G, D)
    seqs, q0s, cost = [], [], []
    for b, (ql, cl) in enumerate(zip(q_lens, ctx_lens)):
        past = cl - ql
        for q0 in range(0, ql, qb):
            seqs.append(b)
            q0s.append(q0)
            cost.append(min(cl, past + q0 + qb) if causal else cl)
    order = np.argsort(-np.asarray(cost, dtype=np.int64), kind="stable")
    return (np.asarray(seqs, dtype=np.int32)[order], np.asarray(q0s, dtype=np.int32)[order])


def flash_prefill(q, k, v, cu_q, Hq: int, Hkv: int, D: int, scale: float, causal: bool,
                  block_tables=None, ctx_lens=None, q_lens_cpu=None, ctx_lens_cpu=None,
                  tiles=None, out=None, part=None, q_past=None):
    """Varlen flash attention.  Paged when ``block_tables`` is given (K/V caches
    ``[NB, Hkv, BS, D]``), else dense K/V rows ``[T, >=Hkv*D]`` (encoder).
    ``part`` = (o f32 [T, Hq, D], ml f32 [T, Hq, 2]): write unnormalised partials for a
    cascade / context-parallel merge instead of ``out`` (GPU only; ml = (running max, sum) in
    the log2 domain).  ``q_past`` (int32 [B], GPU only): position of each sequence's first
    query relative to its first key for the causal mask (a context-parallel key shard), instead
    of ctx_len - q_len.

    ``q_lens_cpu`` / ``ctx_lens_cpu``: host copies of the lengths (the scheduler has
    them), used to build the tile list without a device sync."""
    if use_hip(q):
        if tiles is None:
            if q_lens_cpu is None:
                cu = cu_q.cpu().tolist()
                q_lens_cpu = [cu[i + 1] - cu[i] for i in range(len(cu) - 1)]
            if ctx_lens_cpu is None:
                ctx_lens_cpu = ctx_lens.cpu().tolist() if ctx_lens is not None else list(q_lens_cpu)
            if block_tables is not None:
                BS = k.shape[2]
                need = max((int(c) + BS - 1) // BS for c in ctx_lens_cpu) if ctx_lens_cpu else 0
                if need > block_tables.shape[1]:
                    raise ValueError("block table too narrow for the context lengths")
            ts, tq = prefill_tiles(q_lens_cpu, ctx_lens_cpu, Hq // Hkv, causal, D)
            tiles = (torch.from_numpy(ts).to(q.device, non_blocking=True),
                     torch.from_numpy(tq).to(q.device, non_blocking=True))
        pp_o, pp_ml = part if part is not None else (None, None)
        if out is not None and part is None and (out.data_ptr() % 16 or out.stride(0) % 8):
            # the kernel's output rows leave as 16-byte stores: stage a misaligned view
            y = lib().flash_prefill(q, k, v, block_tables, cu_q, ctx_lens, tiles[0], tiles[1], Hq,
                                    Hkv, D, scale, causal, None, None, None, q_past)
            out[:, : Hq * D].copy_(y)
            return out
        return lib().flash_prefill(q, k, v, block_tables, cu_q, ctx_lens, tiles[0], tiles[1], Hq,
                                   Hkv, D, scale, causal, out, pp_o, pp_ml, q_past)
    if q_past is not None:
        raise NotImplementedError("q_past: GPU kernel only")
    y = ref.flash_prefill(q, k, v, block_tables, cu_q, ctx_lens, Hq, Hkv, D, scale, causal)
    if out is not None:
        out[:, : Hq * D].copy_(y)
        return out
    return y


def knn_topk(corpus, cnorm, queries, qnorm, K: int):
    """Cosine top-K (scores f32 [nq,K], indices int32 [nq,K]; -1 pads)."""
    if use_hip(corpus):
        s, i = lib().knn_topk(corpus, cnorm, queries, qnorm, K)
        return s, i
    return ref.knn_topk(corpus, cnorm, queries, qnorm, K)


def knn_merge(cand_s, cand_i, K: int):
    if use_hip(cand_s):
        return tuple(lib().knn_merge(cand_s.contiguous(), cand_i.contiguous(), K))
    nq = cand_s.shape[0]
    out_s = torch.full((nq, K), float("-inf"))
    out_i = torch.full((nq, K), -1, dtype=torch.int32)
    for r in range(nq):
        pairs = [(float(s), int(i)) for s, i in zip(cand_s[r].tolist(), cand_i[r].tolist()) if int(i) >= 0]
        pairs.sort(key=lambda p: (-p[0], p[1]))
        for j, (s, i) in enumerate(pairs[:K]):
            out_s[r, j] = s
            out_i[r, j] = i
    return out_s, out_i


def pool_normalize(hidden, cu, mode: int, normalize: bool = True, out=None):
    """Pooled (mean / CLS), L2-normalised sentence vectors; ``out``: destination rows [B, H]
    (f32 or bf16; the kernel writes them directly), default a new f32 [B, H]."""
    if use_hip(hidden):
        return lib().pool_normalize(hidden, cu, mode, normalize, out)
    y = ref.pool_normalize(hidden, cu, mode, normalize)
    if out is not None:
        out.copy_(y)
        return out
    return y


def row_norms(x):
    if use_hip(x):
        return lib().row_norms(x.contiguous())
    return ref.row_norms(x)


def select_tokens(logits, temps=None, seed: int = 0, step: int = 0, out=None):
    if use_hip(logits):
        return lib().select_tokens(logits, temps, int(seed) & ((1 << 63) - 1), int(step), out)
    return ref.select_tokens(logits, temps, seed, step)


def argmax_key(logits, vocab_lo: int = 0):
    """Per row an order-preserving int64 key of (max value, vocab_lo + first argmax): the larger
    key is the larger value, then the LOWER id (torch.argmax's tie order), so the max of the
    keys gathered from the vocab shards picks the global greedy token (parallel/tp.py)."""
    if use_hip(logits):
        return lib().argmax_key(logits, int(vocab_lo))
    return ref.argmax_key(logits, vocab_lo)


def key_to_id(keys):
    """Global ids from [W, R] gathered argmax keys (max over W), int32 [R]; a [R] key row
    decodes directly."""
    if keys.dim() == 1:
        keys = keys[None]
    if use_hip(keys):
        return lib().keys_to_ids(keys.contiguous())
    return ref.keys_to_ids(keys)


def sample(logits, prm, hist, hist_len, seed: int = 0, out=None):
    """Ollama-default sampling of every row (repeat penalty from the device history ring,
    top-k, top-p, temperature; greedy rows = argmax); appends the tokens to the ring."""
    if use_hip(logits):
        return lib().sample(logits, prm, hist, hist_len, int(seed) & ((1 << 63) - 1), out)
    return ref.sample(logits, prm, hist, hist_len, seed)


def repeat_penalty_(logits, window, penalty):
    if use_hip(logits):
        lib().repeat_penalty_(logits, window, penalty)
        return logits
    return ref.repeat_penalty_(logits, window, penalty)


# Decode-regime GEMMs (csrc/skinny_gemm.hip) vs the library GEMM, from the MI355X
# sweeps in profiles/r1_skinny_gemm.md and profiles/r1_ws_sweep.md:
#  * M <= 256: the LDS-DMA weight-streaming kernel: 1.2-2.3x hipBLASLt on every
#    Llama projection (QKV / O / down; gate_up+SwiGLU fused up to M = 160), and its
#    split-K reduction fused into the consumer (RMSNorm+residual, RoPE+KV write);
#  * the LM head (N >= 65536) at M <= 16: the fragment-load kernel (weights straight to
#    VGPRs, split-K); larger M: the prefill GEMM.
# The fragment-load kernel also served every projection at M <= 16 until round 2; the
# fused weight-streaming path beat it end to end at every small batch (bench.py --batch
# 1/2/4/8 on MI355X: p50 227 -> 201, 235 -> 207, 252 -> 224, 292 -> 259 ms), so
# LK_SKINNY_MAX_M now defaults to 0.
SKINNY_MAX_M = int(os.environ.get("LK_SKINNY_MAX_M", "0"))
LM_HEAD_SKINNY_MAX_M = 16
# LM head (N >= 65536) at 16 < M <= 256: weight-streaming kernel (1) or the prefill GEMM (0)
WS_LM_HEAD = os.environ.get("LK_WS_LM_HEAD", "0") == "1"
WS_MAX_M = int(os.environ.get("LK_WS_MAX_M", "256"))
WS_SWIGLU_MAX_M = 160


# Measured per-shape choice between the weight-streaming kernel and the prefill GEMM for
# decode batches (``tune_decode``, cold weights, at engine start): the static rule below is
# wrong in both directions on some shapes (benchmarks/decode_route.py on MI355X,
# profiles/r3_decode_route/: the 70B TP=8 gate_up shard at M 192-256 ran the prefill GEMM at
# 0.35x of the ws kernel; the 70B QKV at M 160-256 ran ws at 0.79-0.90x of the GEMM).
# {(M bucket, N, K, swiglu): "ws" | "gemm"}; buckets are the tuned M values, a batch uses the
# smallest bucket >= M.
_DECODE_TABLE: dict = {}
DECODE_TUNE_MS = (32, 64, 96, 128, 160, 192, 224, 256)


def _decode_bucket(M: int) -> Optional[int]:
    for b in DECODE_TUNE_MS:
        if M <= b:
            return b
    return None


def _decode_gemm_kind(x, w, swiglu: bool) -> Optional[str]:
    if not (use_hip(x) and x.dim() == 2 and w.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16):
        return None
    M = x.shape[0]
    N, K = w.shape
    if M < 1 or K % 256 or x.stride(1) != 1 or x.stride(0) % 8 or not w.is_contiguous():
        return None
    if swiglu:
        if N % 2 or (N // 2) % 64:
            return None
    elif N % 128:
        return None
    if M <= SKINNY_MAX_M:
        return "skinny"
    if _DECODE_TABLE and M > LM_HEAD_SKINNY_MAX_M:
        b = _decode_bucket(M)
        choice = _DECODE_TABLE.get((b, N, K, bool(swiglu))) if b is not None else None
        if choice is not None:
            return "ws" if choice == "ws" else None
    if N >= 65536 and not swiglu:
        if M <= LM_HEAD_SKINNY_MAX_M:
            return "skinny"
        return "ws" if WS_LM_HEAD and M <= WS_MAX_M else None
    if M <= (WS_SWIGLU_MAX_M if swiglu else WS_MAX_M):
        return "ws"
    return None


# Prefill / encoder-regime GEMMs (M > WS_MAX_M, and every GEMM with a bias / activation
# epilogue): the hand-written 256 x {256, 192} MFMA kernel of csrc/gemm.hip with the SwiGLU /
# bias / GELU / ReLU epilogue fused.  Two tunables per call: the column tile (192 turns
# N = 6144 into whole waves of 256 CUs) and the K-loop schedule (4 or 2 phases per K-tile).
# ``tune_gemm`` measures them per (M bucket, N, K, epilogue) at engine start-up; untuned
# shapes use the wave-quantisation heuristic of ``_gemm_default``.  The vendor library is
# only reached for shapes the kernel does not support (K % 64, N % 192) -- counted in
# ``LIBRARY_FALLBACKS`` so a test can assert the serving path never takes it.
EPI = {None: 0, "swiglu": 1, "bias": 2, "gelu": 3, "relu": 4}
# measurement knob only: LK_GEMM_LIBRARY=1 sends the prefill-regime GEMMs to hipBLASLt (+ the
# separate activation kernels) for in-situ A/B against the hand-written kernel; =2 only the plain
# ones (no bias / activation / SwiGLU epilogue: QKV, O, down), the fused ones stay hand-written.
# Either turns the fused prefill chain off (its epilogues exist only in gemm.hip).
GEMM_LIBRARY = int(os.environ.get("LK_GEMM_LIBRARY", "0") or 0)
# K-loop schedule of untuned shapes (0: 4 phases per K-tile with per-cluster priority flips,
# 1: 2 phases, 2: 4 phases with a static priority for the lagging half of the waves).  Default:
# 2 for the decoder's K >= 4096 projections (1-5 % faster cold on every Llama-3-8B shape at
# M 4096 / 8192), 0 for the encoder's K 768 / 3072 (neutral there, and 2 lost 8 % on the
# bge QKV at M 65536): profiles/r2_gemm_prio.md.  LK_GEMM_SCHED forces one for every shape.
GEMM_SCHED = int(os.environ["LK_GEMM_SCHED"]) if os.environ.get("LK_GEMM_SCHED") else None


def _gemm_sched(K: int) -> int:
    if GEMM_SCHED is not None:
        return GEMM_SCHED
    return 2 if K >= 4096 else 0
_GEMM_TABLE: dict = {}
LIBRARY_FALLBACKS: dict = {}
# measured (variant, bn, splits) per (M bucket, N, K, epilogue) for the shipped models' projections
# (benchmarks/gemm_table.py on an MI355X; LK_GEMM_STATIC=0 ignores it)
GEMM_TABLE_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_table_mi355x.json")
_STATIC: Optional[dict] = None
_STATIC_TOP: dict = {}  # (N, K, epi) -> largest measured M bucket


_CUS: Optional[int] = None


def device_cus() -> int:
    """Compute units of the current device (256 on a whole MI355X; fewer on a partitioned one,
    e.g. CPX mode): the wave size every tile-count policy below quantises against.  256 without a
    GPU (CPU runs never dispatch GPU kernels)."""
    global _CUS
    if _CUS is None:
        _CUS = 256
        if torch.cuda.is_available():
            _CUS = int(torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count) or 256
    return _CUS


def _table_matches_device(doc: dict) -> bool:
    """The shipped table was measured on one device configuration: use it only on the same arch
    and CU count (a partitioned MI355X has different waves, so its measured picks do not apply)."""
    if not torch.cuda.is_available():
        return True
    arch = getattr(torch.cuda.get_device_properties(torch.cuda.current_device()), "gcnArchName", "") or ""
    return arch.split(":")[0] == doc.get("arch", "gfx950") and int(doc.get("cus", 256)) == device_cus()


def _static_table() -> dict:
    global _STATIC
    if _STATIC is None:
        _STATIC = {}
        if os.environ.get("LK_GEMM_STATIC", "1") != "0" and os.path.exists(GEMM_TABLE_FILE):
            import json

            with open(GEMM_TABLE_FILE) as f:
                doc = json.load(f)
            if not _table_matches_device(doc):
                logging.getLogger("lk.ops").warning("gemm table %s was measured on %s / %s CUs; this device differs: not used",
                            GEMM_TABLE_FILE, doc.get("arch"), doc.get("cus", 256))
                return _STATIC
            for mb, n, k, epi, v, bn, ks in doc["entries"]:
                _STATIC[(mb, n, k, epi)] = (v, bn, ks)
                _STATIC_TOP[(n, k, epi)] = max(mb, _STATIC_TOP.get((n, k, epi), 0))
    return _STATIC


def _static_cfg(key):
    """The measured entry of an M bucket; past the largest measured bucket of the shape (the
    encoder's 100k-row batches: many whole waves, where the choice no longer moves with M) the
    largest one's."""
    t = _static_table()
    cfg = t.get(key)
    if cfg is None:
        top = _STATIC_TOP.get(key[1:])
        if top is not None and key[0] > top:
            cfg = t.get((top,) + key[1:])
    return cfg


def _gemm_key(M: int, N: int, K: int, epi: int):
    return ((M + 255) // 256, N, K, epi)


# Variants 3 / 4 / 5 = csrc/gemm1w.hip, the one-wave-per-SIMD kernel on hipBLASLt's gfx950 K-loop
# schedule, 256-wide column tiles and 256 / 192 / 128-row tiles: 1.04-1.09x gemm.hip and
# 0.95-1.10x hipBLASLt on the Llama-3-8B projections at 256 rows (profiles/r5_gemm1w/).  The
# smaller row tiles fill the 256 CUs where 256-row tiles leave most of a wave idle: at the
# serving bench's mixed-step sizes (prefill chunk + ~105 decode rows) they are 1.2-1.4x the
# round-4 dispatch (M 2664: QKV on 128-row tiles 109.5 vs 151.6 us, O / down on 192-row tiles
# 66.7 / 220.8 vs 82.3 / 295.5 us; benchmarks/gemm_tiles.py, profiles/r5_gemm_tiles/).
# Which tile wins depends on M through the wave quantisation AND the chip's clocks (a partly
# filled wave runs at a higher clock), so the choice is MEASURED: ``tune_gemm`` times every
# candidate per 256-row M bucket, and a table of those measurements for the shipped models
# (gemm_table_mi355x.json, written by benchmarks/gemm_table.py on an MI355X) is the default;
# ``_gemm_default`` below is the fallback for shapes the table does not hold.
# LK_GEMM1W=0 restores round 4's gemm.hip-only choice.
GEMM1W = os.environ.get("LK_GEMM1W", "1") != "0"
GEMM1W_MIN_TILES = 256
GEMM1W_BM = {3: 256, 4: 192, 5: 128, 6: 256, 7: 256}
# Variants 6 / 7: column split (csrc/gemm1w.hip launch1w_tiles) -- the column tiles that fill whole
# waves of the CUs on 256-row tiles, the rest (under a wave) on 128 / 192-row tiles, two launches.
# QKV at M 4096 = 16 x 24 256-row tiles = 1.5 waves: 16 x 16 tiles, then 32 x 8 128-row tiles.
GEMM1W_SPLIT = {6: 128, 7: 192}
SPLIT_ON = os.environ.get("LK_GEMM_SPLIT", "1") != "0"  # 0: measured 6 / 7 entries run as variant 3 (A/B)


def gemm1w_split_cols(M: int, N: int, epi: int, cus: Optional[int] = None) -> int:
    """Column tiles a variant 6 / 7 launch runs on 256-row tiles (mirrors lk_gemm1w_split_cols,
    which uses the device's CU count too); 0 or all of them: no split (the launch is variant 3's)."""
    cus = cus or device_cus()
    tn = N // 256
    tm = (M + 255) // 256
    return min(tn, (tm * tn // cus) * cus // tm)


def _split_applies(M: int, N: int, epi: int) -> bool:
    return 0 < gemm1w_split_cols(M, N, epi) < N // 256


def _gemm_configs(N: int, epi: int):
    """(schedule / variant, column tile) candidates the kernels support for this N / epilogue."""
    bns = [256] if epi == 1 else [bn for bn in (256, 192) if N % bn == 0]
    cfgs = [(sched, bn) for bn in bns for sched in (0, 1, 2)]
    if 256 in bns and GEMM1W:
        cfgs += [(v, 256) for v in GEMM1W_BM]
    return cfgs


def _gemm_default(M: int, N: int, K: int, epi: int):
    """Fallback policy for shapes without a measured entry.  gemm.hip: fewest tile-columns x
    waves, cost(bn) = ceil(tiles / 256 CUs) * bn (ties -> 256), 4-phase schedule (fastest of its
    schedules with weights streamed from HBM: profiles/r2_gemm.md).  gemm1w.hip (256-row tiles)
    instead once its tiles fill a wave, and its 192-row tiles where 256-row tiles would leave
    over a third of a single wave idle while 192-row ones still fit in one."""
    tm = (M + 255) // 256
    cus = device_cus()
    best = None
    for _, bn in _gemm_configs(N, epi):
        n_cols = N // 2 // 128 if epi == 1 else N // bn
        cost = -(-tm * n_cols // cus) * (256 if epi == 1 else bn)
        if best is None or cost < best[0]:
            best = (cost, bn)
    if best is None:
        return None
    bn = best[1]
    ks = _gemm_splits(M, N, K, epi, bn)
    tiles = tm * (N // 2 // 128 if epi == 1 else N // bn)
    if GEMM1W and bn == 256 and ks == 1 and K // 64 >= 3:
        if tiles >= GEMM1W_MIN_TILES:
            return (3, 256, 1)
        tiles192 = -(-M // 192) * (N // 2 // 128 if epi == 1 else N // 256)
        if tiles < 0.7 * cus and tiles192 <= cus:
            return (4, 256, 1)
    return (_gemm_sched(K), bn, ks)


# split-K for shapes with at most half as many tiles as CUs (M <= 2048 O / down projections,
# the 70B TP=8 QKV shard at N 1280), and 3 K-ranges for long-K shapes of 129-160 tiles:
# fp32 partials of up to 4 K-ranges, each of >= 8 K-tiles,
# summed by a reduce kernel that applies the epilogue (profiles/r2_gemm_splitk.md); LK_GEMM_SPLITK=0
# turns it off
GEMM_SPLITK = os.environ.get("LK_GEMM_SPLITK", "1") != "0"


def _gemm_splits(M: int, N: int, K: int, epi: int, bn: int) -> int:
    if not GEMM_SPLITK or epi == 1:
        return 1
    tiles = ((M + 255) // 256) * (N // bn)
    if tiles > 128:
        # long K just past half a wave: three K-ranges give ~1.7-1.9 waves of tiles
        # (M 2304 / 2560 down projection: 295 -> 278, 277 -> 255 us; from 176 tiles on, worse)
        return 3 if tiles <= 160 and K >= 8192 else 1
    return max(1, min(4, device_cus() // tiles, K // 64 // 8))


def _gemm_ok(x, w) -> bool:
    return (use_hip(x) and x.dim() == 2 and w.dim() == 2 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.stride(1) == 1 and x.stride(0) % 8 == 0
            and w.is_contiguous() and x.data_ptr() % 16 == 0)


def gemm(x, w, b=None, epi: int = 0, out=None):
    """epi(x w^T (+ b)) on the hand-written kernel; None if the shape is unsupported."""
    M, K = x.shape
    N = w.shape[0]
    # the epilogue stores / bias loads are 16-byte vectors
    if b is not None and (b.data_ptr() % 16 or not b.is_contiguous()):
        return None
    if out is not None and (out.data_ptr() % 16 or out.stride(0) % 8 or out.stride(1) != 1):
        return None
    cfg = _cfg_of(M, N, K, epi)
    if cfg is None or not lib().gemm_supported(M, N, K, epi, cfg[1], cfg[2], cfg[0]):
        return None
    return lib().gemm(x, w, b, epi, cfg[1], out, cfg[0], cfg[2])


def _library(x, w, b, act, key):
    LIBRARY_FALLBACKS[key] = LIBRARY_FALLBACKS.get(key, 0) + 1
    y = torch.nn.functional.linear(x, w, b)
    if act == "gelu":
        gelu_(y)
    elif act == "relu":
        relu_(y)
    return y


def tune_gemm(weights, max_m: int, min_m: int = 512, iters: int = 6, cold_bytes: int = 600 << 20,
              ms: Optional[list] = None) -> dict:
    """Time every (schedule / variant, column tile) of the prefill kernels for each 256-row M
    bucket in [min_m, max_m] (or the row counts ``ms``) and each (weight, epilogue) pair; keep
    the fastest.  gemm.hip candidates run with the split-K the policy gives them, gemm1w.hip
    unsplit.  As in serving, the weights arrive from HBM: each launch reads the next of enough
    weight copies to overflow the 256 MB MALL (a warm-weight tuning picks the 2-phase schedule for
    the SwiGLU projection, which is 3 % slower in situ).  Candidates are timed round-robin so
    clock drift hits all alike.  ``weights``: [(w [N, K] bf16 CUDA tensor, epi)].  Returns
    {key: {cfg: us}} and fills the tuned table."""
    import statistics

    L = lib()
    out = {}

    def once(fn):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        return a.elapsed_time(b) * 1e3

    rows = ms if ms is not None else [mb * 256 for mb in range(max(min_m, 256) // 256, max_m // 256 + 1)]
    for w, epi in weights:
        N, K = w.shape
        copies = [w] + [w.clone() for _ in range(max(0, -(-cold_bytes // (N * K * 2)) - 1))]
        rot = [0]

        def wn():
            rot[0] = (rot[0] + 1) % len(copies)
            return copies[rot[0]]

        bias = torch.zeros(N, device=w.device, dtype=torch.bfloat16) if epi >= 2 else None
        xmax = torch.randn(max(rows), K, device=w.device, dtype=torch.bfloat16)
        for M in rows:
            x = xmax[:M]
            cfgs = []
            for v, bn in _gemm_configs(N, epi):
                if v in GEMM1W_SPLIT and not _split_applies(M, N, epi):
                    continue  # the same launch as variant 3
                ks = 1 if v in GEMM1W_BM else _gemm_splits(M, N, K, epi, bn)
                if not L.gemm_supported(M, N, K, epi, bn, ks, v):
                    ks = 1
                if L.gemm_supported(M, N, K, epi, bn, ks, v):
                    cfgs.append((v, bn, ks))
            if not cfgs:
                continue
            fns = {c: (lambda c=c: L.gemm(x, wn(), bias, epi, c[1], None, c[0], c[2])) for c in cfgs}
            for f in fns.values():
                f()
            ts = {c: [] for c in cfgs}
            for _ in range(iters):
                for c, f in fns.items():
                    ts[c].append(once(f))
            med = {c: statistics.median(v) for c, v in ts.items()}
            key = _gemm_key(M, N, K, epi)
            _GEMM_TABLE[key] = min(med, key=med.get)
            out[key] = {f"v{c[0]}/{c[1]}/k{c[2]}": round(t, 1) for c, t in med.items()}
        del copies
    return out


# decode tuner: also pick the weight-streaming kernel variant per row tile (LK_WS_VARIANT_TUNE=0:
# keep LK_WS_LOADER's default everywhere)
WS_VARIANT_TUNE = os.environ.get("LK_WS_VARIANT_TUNE", "1") != "0"
_WS_VARIANTS: dict = {}  # (row-tile top M, N, K, swiglu) -> 0 ring / 1 loader waves (also set in _C)


def apply_ws_variants(table: dict):
    """Install measured weight-streaming kernel variants (a TP worker applies its leader's)."""
    _WS_VARIANTS.clear()
    _WS_VARIANTS.update(table)
    if table and available():
        L = lib()
        for (M, N, K, sw), v in table.items():
            L.ws_set_variant(M, N, K, sw, v)


def tune_decode(weights, ms: Sequence[int] = DECODE_TUNE_MS, iters: int = 5, cold_bytes: int = 640 << 20) -> dict:
    """For each decode-sized M bucket and each (weight, swiglu) pair, time the weight-streaming
    kernel against the prefill GEMM with the weights arriving from HBM (each launch reads the
    next of enough copies to overflow the 256 MB MALL, back-to-back launches as in a decode
    graph) and record the faster in the dispatch table.  Returns {(M, N, K, swiglu): {arm: us}}
    plus, per measured row tile, {(M, N, K, swiglu, "ws_variant"): {"ring" / "loader": us}}."""
    import statistics

    L = lib()
    out = {}
    for w, swiglu in weights:
        N, K = w.shape
        swiglu = bool(swiglu)
        copies = [w] + [w.clone() for _ in range(max(1, -(-cold_bytes // (N * K * 2)) - 1))]

        def timed(fns):
            ts = {k: [] for k in fns}
            for fn in fns.values():  # warm-up (and first-launch attributes)
                fn(copies[0])
            torch.cuda.synchronize()
            for _ in range(iters):
                for k, fn in fns.items():
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for c in copies[1:] + copies[:1]:
                        fn(c)
                    b.record()
                    b.synchronize()
                    ts[k].append(a.elapsed_time(b) * 1e3 / len(copies))
            return {k: statistics.median(v) for k, v in ts.items()}

        # the weight-streaming kernel's variant per row tile (64 / 128 / 192 / 256 rows): one LDS
        # ring vs loader waves (csrc/skinny_gemm.hip wsgemm_lw_kernel), measured at the tile's
        # largest M, before the routing below times the ws arm with it
        if WS_VARIANT_TUNE and _decode_static_ok(N, K, swiglu):
            for M in [m for m in (64, 128, 192, 256) if m in ms]:
                x = torch.randn(M, K, device=w.device, dtype=torch.bfloat16)
                fns = {}
                for v in (0, 1):
                    fns[v] = (lambda c, v=v: (L.ws_set_variant(M, N, K, swiglu, v), L.ws_linear(x, c, swiglu)))
                med = timed(fns)
                best = min(med, key=med.get)
                L.ws_set_variant(M, N, K, swiglu, best)
                _WS_VARIANTS[(M, N, K, swiglu)] = best
                out[(M, N, K, swiglu, "ws_variant")] = {("ring", "loader")[v]: round(t, 1) for v, t in med.items()}
        for M in ms:
            x = torch.randn(M, K, device=w.device, dtype=torch.bfloat16)
            arms = {}
            if M <= 256 and _decode_static_ok(N, K, swiglu):
                arms["ws"] = lambda c, x=x: L.ws_linear(x, c, swiglu)
            epi = 1 if swiglu else 0
            cfg = _gemm_default(M, N, K, epi)
            if cfg is not None and L.gemm_supported(M, N, K, epi, cfg[1], cfg[2], cfg[0]):
                arms["gemm"] = lambda c, x=x, cfg=cfg: L.gemm(x, c, None, epi, cfg[1], None, cfg[0], cfg[2])
            if len(arms) < 2:
                continue
            med = timed(arms)
            _DECODE_TABLE[(M, N, K, swiglu)] = min(med, key=med.get)
            out[(M, N, K, swiglu)] = {k: round(v, 1) for k, v in med.items()}
        del copies
    return out


def _decode_static_ok(N: int, K: int, swiglu: bool) -> bool:
    if K % 256:
        return False
    return (N % 2 == 0 and (N // 2) % 64 == 0) if swiglu else N % 128 == 0


def linear(x, w, b=None, act: Optional[str] = None):
    """Projection GEMM (+ bias, + GELU / ReLU): decode-sized batches without an epilogue on
    the weight-streaming MFMA kernels (skinny / ws), everything else on the prefill kernel
    with the epilogue fused."""
    if not use_hip(x):
        y = torch.nn.functional.linear(x, w, b)
        if act is not None:
            y = ref.activation_(y, None, 0 if act == "gelu" else 2)
        return y
    if b is None and act is None:
        if _gemv_ok(x, w, 0):
            return lib().gemv_decode(0, x, w)
        kind = _decode_gemm_kind(x, w, False)
        if kind == "skinny":
            return lib().skinny_linear(x, w)
        if kind == "ws":
            return lib().ws_linear(x, w)
    epi = EPI["bias" if act is None else act] if b is not None else 0
    if act is not None and b is None:
        b = torch.zeros(w.shape[0], device=x.device, dtype=x.dtype)
        epi = EPI[act]
    lib_arm = GEMM_LIBRARY == 1 or (GEMM_LIBRARY == 2 and epi == 0 and x.shape[0] > WS_MAX_M)
    y = gemm(x, w, b, epi) if _gemm_ok(x, w) and not lib_arm else None
    if y is None:
        y = _library(x, w, b, act, (x.shape[0] > WS_MAX_M, w.shape[0], w.shape[1], epi))
    return y


def linear_swiglu(x, w_gate_up):
    """silu(x Wg^T) * (x Wu^T) for a fused [Wg; Wu] weight: one kernel (GEMM with the
    SwiGLU epilogue) in every regime."""
    if not use_hip(x):
        return silu_mul(linear(x, w_gate_up))
    if _gemv_ok(x, w_gate_up, 2):
        return lib().gemv_decode(2, x, w_gate_up)
    kind = _decode_gemm_kind(x, w_gate_up, True)
    if kind == "skinny":
        return lib().skinny_linear(x, w_gate_up, True)
    if kind == "ws":
        return lib().ws_linear(x, w_gate_up, True)
    y = gemm(x, w_gate_up, None, 1) if _gemm_ok(x, w_gate_up) and GEMM_LIBRARY != 1 else None
    if y is None:
        y = silu_mul(_library(x, w_gate_up, None, None, (True, w_gate_up.shape[0], w_gate_up.shape[1], 1)))
    return y


# Decode-step fusions: when the weight-streaming GEMM splits K (S >= 2 partial slabs),
# the consumer kernel does the split-K reduction itself -- RMSNorm(+residual) after the
# o / down projections, RoPE + paged-KV write after QKV -- so each of those projections
# costs one launch fewer (three per layer; bit-identical to the unfused ops).
DECODE_FUSION = os.environ.get("LK_DECODE_FUSION", "1") != "0"
_WS_PLANS: dict = {}


def _ws_split_plan(x, w):
    """(BN, S) of the weight-streaming GEMM when it runs split-K for this shape, else None."""
    if not DECODE_FUSION or _decode_gemm_kind(x, w, False) != "ws":
        return None
    key = (x.shape[0], w.shape[0], w.shape[1])
    plan = _WS_PLANS.get(key)
    if plan is None:
        plan = _WS_PLANS[key] = tuple(lib().ws_plan(*key, False))
    return plan if plan[1] in (2, 4, 8) else None


# Split-K decode GEMMs whose reduction runs in their own last workgroup(s) (csrc/skinny_gemm.hip
# WsTail): the QKV projection's RoPE + paged-KV write (one ticket per head), and for <= 4 rows the
# o / down projections' residual + RMSNorm -- no reduce launch after them.  Measured OFF: at batch 1
# (same box, twice each, profiles/r6_ws_tail/) a decode step took 4.34 / 4.32 ms with the tails vs
# 3.685 / 3.672 ms with the three ~5 us reduce launches per layer (p50 161.8 vs 139.4 ms): the
# write-through partials and the one-workgroup reductions cost more than the launches they save.
# LK_WS_FUSED_TAIL=1 turns them on (numerics: tests/test_kernels_gpu.py *fused_tail*).
WS_FUSED_TAIL = os.environ.get("LK_WS_FUSED_TAIL", "0") == "1"
_WS_TICKETS: dict = {}


def ws_tickets(device):
    """Zeroed int32 tickets of the fused split-K tails (one buffer per device, made before any
    graph capture by the model runner; every ticket is reset by its last taker)."""
    device = torch.device(device)
    key = device.index if device.index is not None else torch.cuda.current_device()
    t = _WS_TICKETS.get(key)
    if t is None:
        t = _WS_TICKETS[key] = torch.zeros(4096, dtype=torch.int32, device=device)
    return t


# Consumer-side prologues in the decode step (csrc/skinny_gemm.hip WsPro, rows <= XPRO_MAX_M, one
# GPU without TP): the O projection merges the paged-decode split partials itself (no
# decode_reduce launch) and gate_up / the next layer's QKV compute residual add + RMSNorm of the
# previous projection's split-K slabs themselves (no rmsnorm launch) -- three launches fewer per
# layer, bit-identical values (models/llama.py _forward_decode_xpro).  Measured slower at batch 1
# (decode step 4.23 vs 3.58 ms: every workgroup re-reads and re-normalises the producer's fp32 slabs,
# and the O projection's merge prologue costs 17 us; profiles/r6_xpro/): off unless LK_DECODE_XPRO=1.
XPRO = os.environ.get("LK_DECODE_XPRO", "0") == "1"
XPRO_MAX_M = int(os.environ.get("LK_DECODE_XPRO_MAX_M", "16"))
_PLAN_CACHE: dict = {}


def ws_plan(M: int, N: int, K: int, swiglu: bool = False) -> tuple:
    """(BN, S) of the weight-streaming GEMM for this shape (lk_wsgemm_plan)."""
    key = (M, N, K, swiglu)
    p = _PLAN_CACHE.get(key)
    if p is None:
        p = _PLAN_CACHE[key] = tuple(lib().ws_plan(M, N, K, swiglu))
    return p


def ws_pro(x, w, plan, kind: int, swiglu: bool = False, reduce: bool = False, **kw):
    """Weight-streaming GEMM with a consumer-side X prologue (``kind`` 1: x = RMSNorm(bf16(sum of
    ``pp``) + ``res_in``) * ``gamma``, ``res_out`` = the summed residual; 2: x = the paged-decode
    output with its split partials ``po`` / ``pml`` merged; 0: plain x).  Returns the f32 partial
    slabs [S, M, N] (S > 1 and not ``reduce``) or the bf16 / SwiGLU output."""
    return lib().ws_pro(x, w, swiglu, plan[0], plan[1], kind, reduce, **kw)


# Decode GEMV for one or two rows (csrc/gemv_decode.hip): no split-K slabs, the RMSNorm in the
# consumer's prologue, residual add / SwiGLU / RoPE + paged-KV write in the epilogue -- a Llama
# block's batch-1 decode step is QKV -> paged decode -> O -> gate_up -> down, with no reduce, norm
# or RoPE launch (models/llama.py _forward_decode_gemv).  LK_DECODE_GEMV=0: the weight-streaming path.
GEMV = os.environ.get("LK_DECODE_GEMV", "1") != "0"
GEMV_MAX_M = 2
# LK_GEMV_MERGE=1: the O projection's GEMV merges the paged-decode split partials itself (no
# decode_reduce launch).  Measured slightly slower at batch 1 (decode step 3.129 / 3.133 vs 3.104 /
# 3.110 ms: every workgroup re-reads all split partials), so the reduce kernel stays the default
GEMV_MERGE = os.environ.get("LK_GEMV_MERGE", "0") == "1"
_GEMV_OK: dict = {}


# The long-K projections (K split into an even number >= 2 of streaming blocks: down at K 14,336,
# the 70B QKV / gate_up at K 8,192) take two waves per pair of W rows, a K half each, their sums
# joined in LDS (LK_GEMV_KSPLIT=0: one wave per pair).  Tried and removed: the first W block
# prefetched before the X prologue, in registers (batch-1 decode step 3.199 vs 3.17 ms) and by
# LDS-DMA (3.31 vs 3.10; profiles/r6_gemv/).  Workgroup target (LK_GEMV_WGS, 0: 512)
GEMV_KSPLIT = os.environ.get("LK_GEMV_KSPLIT", "1") != "0"
GEMV_WGS = int(os.environ.get("LK_GEMV_WGS", "0") or 0)


# Batch-1 decode: while the latency-bound paged-decode kernels leave HBM idle, a side stream reads
# the O projection's weights (and the first LK_GEMV_L3_PREFETCH_MB of gate_up's gate / up rows)
# through the 256 MiB Infinity Cache so the GEMVs behind the attention read them from L3.
# -1: off; 0: O only.
GEMV_L3_MB = int(os.environ.get("LK_GEMV_L3_PREFETCH_MB", "-1") or -1)
GEMV_L3_WGS = int(os.environ.get("LK_GEMV_L3_WGS", "128") or 128)
_L3_SINK: dict = {}


def l3_prefetch(t, r0: int, r1: int):
    """Read rows [r0, r1) of a contiguous 2-D GPU tensor (values unused) on the current stream."""
    s = _L3_SINK.get(t.device)
    if s is None:
        s = _L3_SINK[t.device] = torch.zeros(1, dtype=torch.int32, device=t.device)
    lib().l3_prefetch(t, r0, r1, GEMV_L3_WGS, s)


def gemv_supported(M: int, N: int, K: int, mode: int) -> bool:
    key = (M, N, K, mode)
    ok = _GEMV_OK.get(key)
    if ok is None:
        if not _GEMV_OK:  # first use: the launch knobs
            lib().gemv_set_ksplit(GEMV_KSPLIT)
            lib().gemv_set_wgs(GEMV_WGS)
        ok = _GEMV_OK[key] = bool(lib().gemv_supported(M, N, K, mode))
    return ok


def _gemv_ok(x, w, mode: int) -> bool:
    """A plain / SwiGLU projection of <= 2 rows goes to the decode GEMV (faster than the weight-
    streaming kernels at every decode shape measured: benchmarks/gemv_bench.py, profiles/r6_gemv/)."""
    M = x.shape[0]
    return (GEMV and M <= GEMV_MAX_M and x.dim() == 2 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
            and w.is_contiguous() and x.stride(-1) == 1
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and gemv_supported(M, w.shape[0], w.shape[1], mode))


def gemv_decode(mode: int, x, w, gamma=None, eps: float = 1e-5, res=None, positions=None, cos_sin=None,
                Hq: int = 0, Hkv: int = 0, D: int = 0, k_cache=None, v_cache=None, slots=None, neox: bool = True,
                po=None, pml=None, ctx=None, max_splits: int = 0, split: int = 0):
    """mode 0: x W^T; 1: ``res`` += x W^T in place (returned); 2: SwiGLU(x [Wg; Wu]^T) [M, N/2];
    3: packed QKV with RoPE applied to q (and to k in the paged cache, k kept unrotated in the
    row), K/V written at ``slots``.  ``gamma``: the GEMV's input is RMSNorm(x) * gamma.  ``po`` /
    ``pml`` (mode 1, GPU): x's rows that :func:`paged_decode` (``reduce=False``) left as split
    partials are merged in the GEMV's prologue (no decode_reduce launch)."""
    if use_hip(x):
        return lib().gemv_decode(mode, x, w, gamma, eps, res, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache,
                                 slots, neox, po, pml, ctx, max_splits, split)
    if po is not None:
        raise NotImplementedError("gemv_decode: the split-merge prologue is a GPU kernel")
    xin = ref.rmsnorm(x, gamma, eps) if gamma is not None else x
    y = xin.float() @ w.float().t()
    if mode == 0:
        return y.to(x.dtype)
    if mode == 1:
        res.copy_((y.to(res.dtype).float() + res.float()).to(res.dtype))
        return res
    if mode == 2:
        I = w.shape[0] // 2
        g, u = y[:, :I].to(x.dtype).float(), y[:, I:].to(x.dtype).float()
        return (torch.nn.functional.silu(g).to(x.dtype).float() * u).to(x.dtype)
    qkv = y.to(x.dtype)
    rope_kv_(qkv, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox, False)
    return qkv


def splitk_rope_kv(part, positions, cos_sin, Hq: int, Hkv: int, D: int, k_cache, v_cache, slots, neox: bool,
                   write_k_inplace: bool = False):
    return lib().splitk_rope_kv(part, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox, write_k_inplace)


def splitk_rmsnorm(part, residual, w, eps: float):
    """RMSNorm(bf16(sum of part's slabs) + residual) * w; residual updated in place."""
    return lib().splitk_rmsnorm(part, residual, w, eps)


def linear_add_rmsnorm(x, w, residual, norm_w, eps: float):
    """RMSNorm(x W^T + residual) * norm_w, with ``residual`` updated in place to
    x W^T + residual (the pre-norm block's "o / down projection -> add -> norm")."""
    plan = _ws_split_plan(x, w)
    if plan is not None and residual.is_contiguous():
        tk = ws_tickets(x.device) if WS_FUSED_TAIL and x.shape[0] <= 4 else None
        return lib().ws_linear_rmsnorm(x, w, residual, norm_w, eps, plan[0], plan[1], tk)
    return rmsnorm(linear(x, w), norm_w, eps, residual=residual)


def linear_rope_kv(x, w, positions, cos_sin, Hq: int, Hkv: int, D: int, k_cache=None, v_cache=None,
                   slots=None, neox: bool = True, write_k_inplace: bool = False):
    """qkv = x W^T, then :func:`rope_kv_` on it (one launch fewer on split-K decode shapes; on
    prefill-sized steps of a folded model -- interleaved RoPE, e.g. the tensor-parallel block,
    where the whole fused chain does not apply -- the QKV GEMM's epilogue does the RoPE and the
    paged-KV write).  Rows <= 2 (the tensor-parallel decode step at batch 1-2): the decode GEMV
    with its RoPE + paged-KV epilogue."""
    if (not write_k_inplace and k_cache is not None and slots is not None and _gemv_ok(x, w, 3)
            and w.shape[0] == (Hq + 2 * Hkv) * D):
        return lib().gemv_decode(3, x, w, None, 1e-5, None, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache,
                                 slots, neox)
    plan = _ws_split_plan(x, w)
    if plan is not None:
        # (rows <= 64: past that the last workgroup of a head reduces >= 128 KB of partials alone,
        # as long as the reduce kernel's whole launch)
        tk = ws_tickets(x.device) if WS_FUSED_TAIL and plan[0] == D == 128 and x.shape[0] <= 64 else None
        return lib().ws_linear_rope_kv(x, w, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox,
                                       write_k_inplace, plan[0], plan[1], tk)
    if _qkv_epilogue_ok(x, w, neox, write_k_inplace, k_cache, slots):
        return linear_qkv_fused(x, w, None, 1e-5, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots)
    qkv = linear(x, w)
    rope_kv_(qkv, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots, neox, write_k_inplace)
    return qkv


def _qkv_epilogue_ok(x, w, neox: bool, write_k_inplace: bool, k_cache, slots) -> bool:
    if neox or write_k_inplace or not PREFILL_CHAIN or GEMM_LIBRARY or not _gemm_ok(x, w):
        return False
    if x.shape[0] <= WS_MAX_M or (k_cache is not None and slots is None):
        return False
    M, K = x.shape
    N = w.shape[0]
    c = _cfg_of(M, N, K, 0)
    return c is not None and c[2] == 1 and lib().gemm_supported(M, N, K, EPI_QKV, c[1], 1, c[0])


# ---------------------------------------------------------------- fused prefill chain
# Prefill-sized steps (M > WS_MAX_M rows) of a decoder whose norm weights are folded into its
# projections (LlamaModel.fold_norms) run the pre-norm block as four GEMMs and nothing else:
#   QKV     x_or_r W_qkv'^T  * s_in(row)  -> interleaved RoPE, K / V into the paged cache  (epi QKV)
#   O       r += attn W_o^T, partial sums of squares of r per 256 columns               (epi RESID)
#   gate_up silu / mul of r W_gu'^T * s_post(row)                                       (epi SWIGLU)
#   down    r += a W_down^T, partial sums of squares                                    (epi RESID)
# s(row) = rsqrt(sum of the partials / H + eps) is recomputed by each consumer tile from the
# producer's partials (no norm pass, no normalised activation in HBM, no RoPE / KV pass).
# LK_PREFILL_CHAIN=0 keeps the round-3 path (GEMM -> rmsnorm / rope_kv kernels).
PREFILL_CHAIN = os.environ.get("LK_PREFILL_CHAIN", "1") != "0"
EPI_RESID, EPI_QKV = 6, 7


def _cfg_of(M: int, N: int, K: int, epi: int):
    """(schedule / variant, bn, splits) of the prefill GEMM for this shape: the start-up tuned
    table (LK_GEMM_TUNE=1), else the shipped measurements (gemm_table_mi355x.json), else the
    fallback policy."""
    key = _gemm_key(M, N, K, epi)
    cfg = _GEMM_TABLE.get(key)
    if cfg is None:
        cfg = _static_cfg(key)
        if cfg is not None and (not GEMM1W and cfg[0] in GEMM1W_BM):
            cfg = None
        elif cfg is not None and not SPLIT_ON and cfg[0] in GEMM1W_SPLIT:
            cfg = (3, 256, 1)
    return cfg if cfg is not None else _gemm_default(M, N, K, epi)


def _resid_cfg(M: int, N: int, K: int):
    c = _cfg_of(M, N, K, 0)
    if c is not None and c[0] in GEMM1W_BM:
        return c  # (variant, 256, 1)
    sched = c[0] if c is not None else _gemm_sched(K)
    return sched, 256, _gemm_splits(M, N, K, 0, 256)


def prefill_chain_ok(x, w_qkv, w_o, w_gate_up, w_down) -> bool:
    """Whether a step of x.shape[0] rows can run the fused chain on the HIP kernels: prefill-sized,
    every projection on the hand-written GEMM, the QKV GEMM unsplit (its epilogue is in-kernel)."""
    if not (PREFILL_CHAIN and use_hip(x) and not GEMM_LIBRARY and x.dtype == torch.bfloat16):
        return False
    M = x.shape[0]
    if M <= WS_MAX_M:
        return False
    L = lib()
    N, K = w_qkv.shape
    c = _cfg_of(M, N, K, 0)
    if c is None or c[2] != 1 or not L.gemm_supported(M, N, K, EPI_QKV, c[1], 1, c[0]):
        return False
    N, K = w_gate_up.shape
    c = _cfg_of(M, N, K, 1)
    if c is None or c[2] != 1 or not L.gemm_supported(M, N, K, 1, c[1], 1, c[0]):
        return False
    for w in (w_o, w_down):
        N, K = w.shape
        sched, bn, ks = _resid_cfg(M, N, K)
        if not L.gemm_supported(M, N, K, EPI_RESID, bn, ks, sched):
            return False
    return True


def ss_buffer(M: int, N: int, device) -> torch.Tensor:
    """Partial sums of squares of a [M, N] residual: [N / 256, M] f32."""
    return torch.empty((N // 256, M), dtype=torch.float32, device=device)


def linear_resid(x, w, residual, ss_out):
    """residual += x W^T (bf16 rounding as the unfused linear -> add), and the partial sums of
    squares of the new residual per 256 columns into ss_out [N / 256, >= M] (one GEMM)."""
    if not use_hip(x):
        return ref.linear_resid(x, w, residual, ss_out)
    M, K = x.shape
    N = w.shape[0]
    sched, bn, ks = _resid_cfg(M, N, K)
    return lib().gemm_fused(x, w, EPI_RESID, bn, None, sched, ks, resid=residual, ss_out=ss_out)


def linear_swiglu_scaled(x, w_gate_up, ss, eps: float):
    """silu(s * x Wg^T) * (s * x Wu^T), s = the folded norm's per-row rsqrt from ``ss``."""
    if not use_hip(x):
        return ref.gemm_scaled(x, w_gate_up, ss, x.shape[1], eps, swiglu=True)
    M, K = x.shape
    N = w_gate_up.shape[0]
    sched, bn, _ = _cfg_of(M, N, K, 1)
    return lib().gemm_fused(x, w_gate_up, 1, bn, None, sched, 1, ss_in=ss, eps=eps)


def linear_qkv_fused(x, w, ss, eps: float, positions, cos_sin, Hq: int, Hkv: int, D: int,
                     k_cache=None, v_cache=None, slots=None):
    """qkv = s * x W^T (ss None: unscaled), interleaved-pair RoPE on q / k, K / V into the paged
    cache: the QKV projection, the input norm's scale and rope_kv_ in one GEMM."""
    if not use_hip(x):
        return ref.qkv_fused(x, w, ss, x.shape[1], eps, positions, cos_sin, Hq, Hkv, D, k_cache, v_cache, slots)
    M, K = x.shape
    N = w.shape[0]
    sched, bn, _ = _cfg_of(M, N, K, 0)
    return lib().gemm_fused(x, w, EPI_QKV, bn, None, sched, 1, ss_in=ss, eps=eps, positions=positions,
                            cos_sin=cos_sin, slots=slots, k_cache=k_cache, v_cache=v_cache, hq=Hq, hkv=Hkv, hd=D)


# ---------------------------------------------------------------- per-step gathers (csrc/step_ops.hip)
def embed_rows(table, ids, lo: int = 0, n_local: Optional[int] = None):
    """Rows of ``table`` for int32 ``ids``; with ``lo`` / ``n_local`` a vocab-parallel shard:
    ids outside [lo, lo + n_local) give zero rows (summed over the TP group afterwards)."""
    whole = lo == 0 and n_local is None
    n_local = table.shape[0] if n_local is None else n_local
    if use_hip(table) and ids.dtype == torch.int32:
        # the whole table: an out-of-range id is counted on the device (lib().embed_errors(),
        # polled by the engine's health check) instead of becoming a silent zero row
        return lib().embed_rows(table, ids.contiguous(), lo, -1 if whole else n_local)
    if whole:
        return table[ids.long()]  # raises on a bad id, like an nn.Embedding lookup
    local = ids.long() - lo
    mask = (local < 0) | (local >= n_local)
    return table[local.clamp(0, max(0, n_local - 1))].masked_fill(mask[:, None], 0)


def scatter_ids(ids, dst, prev, src):
    """ids[dst] = prev[src] (the in-flight decode inputs of a pipelined step), one launch."""
    if use_hip(ids) and ids.dtype == torch.int32 and prev.dtype == torch.int32:
        lib().scatter_ids(ids, dst.contiguous(), prev.contiguous(), src.contiguous())
        return ids
    ids.index_copy_(0, dst, prev.index_select(0, src).to(ids.dtype))
    return ids


def gather_rows(x, idx):
    """x[idx] (rows), one launch on the GPU."""
    if (use_hip(x) and x.dtype == torch.bfloat16 and idx.dtype == torch.int64 and x.dim() == 2
            and x.stride(-1) == 1 and x.shape[1] % 8 == 0 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0):
        return lib().gather_rows(x, idx.contiguous())
    return x.index_select(0, idx)


def softmax_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)
