"""Model runner: paged KV cache ownership, per-step input/metadata construction, and
hipGraph-captured decode.

* KV cache: one allocation ``[L, 2, num_blocks, Hkv, BS, D]`` sized from free HBM
  (288 GB on MI355X: millions of tokens of Llama-3-8B KV at 128 KiB/token).
* Mixed steps: ``[prefill chunk tokens | decode tokens]`` in one forward; metadata
  (slots, cu_seqlens, block tables, flash tile list) is built once per step.
* Pure-decode steps replay a ``torch.cuda.CUDAGraph`` (= hipGraph on ROCm)
  captured per batch-size bucket with static input buffers: the whole 32/80-layer
  step (GEMMs, fused norms, RoPE+KV write, split-K paged attention, LM head) is one
  graph launch instead of ~10 launches per layer from Python.
"""
from __future__ import annotations

import bisect
import os
from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

try:  # native step-input builder (csrc/runtime/step_builder.cpp)
    from ..native import runtime as _nrt

    _native_rt = _nrt.load() if _nrt.available() and hasattr(_nrt.load(), "decode_rows") else None
except Exception:  # pragma: no cover
    _native_rt = None

from .. import ops
from ..models import attention as _attn
from ..models.attention import AttnMeta
from ..utils.logging import get_logger

log = get_logger("engine.runner")

# extend chunks of generated tokens up to this many tokens run as decode rows (0: as prefill)
EXTEND_AS_DECODE = int(os.environ.get("LK_EXTEND_AS_DECODE", "16"))


class _PinnedStager:
    """One host->device copy per step: the step's small host arrays (token ids, positions,
    slots, block tables, ...) are packed into a pinned staging buffer (16-B aligned slots)
    and land with ONE async copy in a device buffer whose slices become the step's input
    tensors -- instead of ~10 pageable copies, each a host-staged blit on the GPU queue.
    A ring of staging buffers, each reused only after the copy that read it has run
    (event), keeps this safe while the host runs ahead of the device (pipelined steps)."""

    def __init__(self, device, ring: int = 4):
        self.dev = device
        self.ring = [[None, None] for _ in range(ring)]  # [pinned uint8 buffer, event]
        self.k = 0

    @staticmethod
    def layout(arrays):
        offs, n = [], 0
        for a in arrays:
            n = (n + 15) & ~15
            offs.append(n)
            n += a.nbytes
        return offs, n

    def upload(self, arrays, dst: Optional[torch.Tensor] = None):
        """arrays: C-contiguous numpy arrays -> device tensors (views of ``dst``, a uint8
        device buffer large enough for the packed layout, or a fresh one)."""
        offs, n = self.layout(arrays)
        self.k = (self.k + 1) % len(self.ring)
        slot = self.ring[self.k]
        if slot[1] is not None:
            slot[1].synchronize()  # the copy that last read this buffer has run
        if slot[0] is None or slot[0].numel() < n:
            slot[0] = torch.empty(max(2 * n, 1 << 16), dtype=torch.uint8, pin_memory=True)
            slot[1] = None
        host = slot[0].numpy()
        for a, o in zip(arrays, offs):
            host[o:o + a.nbytes] = a.reshape(-1).view(np.uint8)
        if dst is None:
            dst = torch.empty(max(n, 16), dtype=torch.uint8, device=self.dev)
        dst[:n].copy_(slot[0][:n], non_blocking=True)
        if slot[1] is None:
            slot[1] = torch.cuda.Event()
        slot[1].record()
        return [dst[o:o + a.nbytes].view(torch.from_numpy(a[:0].reshape(-1)).dtype).view(a.shape)
                for a, o in zip(arrays, offs)]


class ModelRunner:
    def __init__(self, model, block_size: int = 16, max_model_len: int = 8192, max_num_seqs: int = 256,
                 num_blocks: Optional[int] = None, kv_cache_gb: Optional[float] = None,
                 gpu_memory_fraction: float = 0.85, use_graphs: bool = True,
                 graph_batch_sizes=(1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256)):
        self.model = model
        self.device = model.device
        self.bs = block_size
        self.max_model_len = max_model_len
        self.max_blocks = (max_model_len + block_size - 1) // block_size
        self.max_num_seqs = max_num_seqs
        cfg = model.cfg
        self.L = cfg.num_layers
        self.hq, self.hkv, self.D = model.hq, model.hkv, model.D
        dt = model.dtype
        block_bytes = self.block_bytes(model, block_size)
        if num_blocks is None:
            num_blocks = self.plan_num_blocks(model, block_size, max_model_len, max_num_seqs, kv_cache_gb,
                                              gpu_memory_fraction)
        self.num_blocks = num_blocks
        self.kv = torch.empty((self.L, 2, num_blocks, self.hkv, block_size, self.D), dtype=dt, device=self.device)
        self.kv_caches = [(self.kv[l, 0], self.kv[l, 1]) for l in range(self.L)]
        log.info("kv cache: %d blocks x %d tokens (%.1f GB)", num_blocks, block_size,
                 num_blocks * block_bytes / 2**30)
        self.use_graphs = use_graphs and self.device.type == "cuda"
        if self.device.type == "cuda":  # the fused split-decode / split-K tail tickets exist before any capture
            ops.decode_tickets(self.device, 2 * max_num_seqs * self.hkv)
            ops.ws_tickets(self.device)
        # cascade decode attention over the batch's shared prompt prefix (GPU kernels; opt-in
        # LK_CASCADE=1).  Measured on MI355X at the RAG operating point (B=120, 288 of ~950
        # keys shared): 8.06 ms per decode step with vs 7.71 without -- the shared blocks
        # are already served from the 256 MB Infinity Cache, so the extra flash pass and
        # the unconditional merge cost more than the HBM bytes they save.
        self.cascade = self.device.type == "cuda" and os.environ.get("LK_CASCADE", "0") == "1"
        # sampled-logits steps return the LM head's bf16 output as is on the GPU: the HIP select /
        # select_allowed kernels read bf16 and the fused sampler converts what it needs, so no
        # [rows, vocab] fp32 copy is written per step (LK_LOWP_LOGITS=0: fp32 logits)
        self.logits_dtype = (None if self.device.type == "cuda" and os.environ.get("LK_LOWP_LOGITS", "1") != "0"
                             else torch.float32)
        # buckets up to twice the sequence cap: jump-forward extend chunks add decode rows
        self.graph_sizes = sorted(b for b in graph_batch_sizes if b <= 2 * max_num_seqs)
        self.graphs: dict = {}
        self._graph_pool = None
        self._ws = None
        self.step_hook = None
        self.prev_ids: Optional[torch.Tensor] = None  # previous step's sampled ids (device)
        self.prev_sampled_rows = 0  # rows of prev_ids sampled on the driver only (non-greedy step)
        self._stager = (_PinnedStager(self.device) if self.device.type == "cuda"
                        and os.environ.get("LK_PINNED_STAGE", "1") != "0" else None)
        self.gemm_tuning = {}
        self.decode_kv_keys = 0  # sum over steps of the decode rows' context lengths (prepare())
        if self.device.type == "cuda" and hasattr(model, "gemm_shapes") and self._gemm_tune_on(model):
            # opt-in (LK_GEMM_TUNE=1): pick the prefill GEMM's column tile / K-loop schedule per
            # 256-row M bucket by a cold-weight micro-benchmark at load (< 1 s for Llama-3-8B).
            # Off by default: in situ it is within the run-to-run spread of the static policy
            # (round 2, profiles/r2_gemm.md; round 4, profiles/r4_gemm_tune/: -1.1 .. +2.7 % per pair)
            self.gemm_tuning = self._tune_gemm(model)
            log.info("prefill GEMM tuned for %d (M bucket, N, K, epilogue) shapes", len(self.gemm_tuning))
        self.decode_tuning = {}
        if (self.device.type == "cuda" and os.environ.get("LK_DECODE_TUNE", "1") == "1"
                and hasattr(model, "decode_gemm_shapes")):
            self.decode_tuning = self._tune_decode(model)

    @staticmethod
    def _gemm_tune_on(model) -> bool:
        return os.environ.get("LK_GEMM_TUNE", "0") == "1"

    @staticmethod
    def _tune_gemm(model) -> dict:
        """ops.tune_gemm over the model's projections; under TP the leader's table is used by
        every rank (the ranks of a group run the same kernels)."""
        tp = getattr(model, "tp", None)
        lead = tp is None or not tp.enabled or getattr(tp, "simulated", False) or tp.rank == 0
        res = ops.tune_gemm(model.gemm_shapes(), int(os.environ.get("LK_GEMM_TUNE_MAX_M", "4096"))) if lead else {}
        if tp is not None and tp.enabled and not getattr(tp, "simulated", False):
            import torch.distributed as dist

            box = [dict(ops._GEMM_TABLE) if lead else None]
            dist.broadcast_object_list(box, src=tp.ranks[0] if tp.ranks else 0, group=tp.ctrl or tp.group)
            ops._GEMM_TABLE.clear()
            ops._GEMM_TABLE.update(box[0])
        return res

    @staticmethod
    def _tune_decode(model) -> dict:
        """Weight-streaming kernel vs prefill GEMM per decode M bucket and projection
        (ops.tune_decode, ~1 s).  Under TP the leader's measurements are used by every rank, so
        the ranks of a group run the same kernels."""
        tp = getattr(model, "tp", None)
        lead = tp is None or not tp.enabled or getattr(tp, "simulated", False) or tp.rank == 0
        res = ops.tune_decode(model.decode_gemm_shapes()) if lead else {}
        if tp is not None and tp.enabled and not getattr(tp, "simulated", False):
            import torch.distributed as dist

            box = [(dict(ops._DECODE_TABLE), dict(ops._WS_VARIANTS)) if lead else None]
            dist.broadcast_object_list(box, src=tp.ranks[0] if tp.ranks else 0, group=tp.ctrl or tp.group)
            ops._DECODE_TABLE.clear()
            ops._DECODE_TABLE.update(box[0][0])
            if not lead:
                ops.apply_ws_variants(box[0][1])
        picks = {}
        for (m, n, k, sw), arm in sorted(ops._DECODE_TABLE.items()):
            picks.setdefault(f"N{n} K{k}{' swiglu' if sw else ''}", []).append(f"{m}:{arm}")
        log.info("decode GEMM routing (M bucket: kernel): %s", "; ".join(f"{k} {' '.join(v)}" for k, v in picks.items()))
        if ops._WS_VARIANTS:
            log.info("weight-streaming kernel per row tile (1 = loader waves): %s",
                     "; ".join(f"M{m} N{n} K{k}{' swiglu' if sw else ''}: {v}"
                               for (m, n, k, sw), v in sorted(ops._WS_VARIANTS.items())))
        return res

    @staticmethod
    def block_bytes(model, block_size: int) -> int:
        esz = torch.tensor([], dtype=model.dtype).element_size()
        return model.cfg.num_layers * 2 * model.hkv * block_size * model.D * esz

    @staticmethod
    def plan_num_blocks(model, block_size=16, max_model_len=8192, max_num_seqs=256, kv_cache_gb=None,
                        gpu_memory_fraction=0.85) -> int:
        """KV blocks this rank can hold: an explicit GB budget, else the free HBM left
        after weights minus the reserved fraction, capped at what max_num_seqs x
        max_model_len could ever use."""
        bb = ModelRunner.block_bytes(model, block_size)
        if kv_cache_gb is not None:
            n = int(kv_cache_gb * (1 << 30) // bb)
        elif model.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(model.device)
            n = int(max(free - (1 - gpu_memory_fraction) * total, 0) // bb)
        else:
            n = 512
        cap = max_num_seqs * ((max_model_len + block_size - 1) // block_size) + 64
        return max(16, min(n, cap))

    # ----------------------------------------------------------- workspaces
    def decode_split(self, B: int):
        split = max(ops.decode_split_size(B, self.hkv), self.bs)
        return split, ops.decode_splits(self.max_blocks * self.bs, split)

    def _decode_ws(self, B: int):
        split, ms = self.decode_split(B)
        n = B * self.hq * ms
        if self._ws is None or self._ws[0].numel() < n * self.D:
            self._ws = (torch.empty(max(n, 1) * self.D, dtype=torch.float32, device=self.device),
                        torch.empty(max(n, 1) * 2, dtype=torch.float32, device=self.device))
        po = self._ws[0][: n * self.D].view(B, self.hq, ms, self.D)
        pm = self._ws[1][: n * 2].view(B, self.hq, ms, 2)
        return po, pm

    def _slots(self, table, start, n):
        pos = np.arange(start, start + n, dtype=np.int64)
        blk = np.asarray(table, dtype=np.int64)[pos // self.bs]
        return (blk * self.bs + pos % self.bs).astype(np.int32), pos.astype(np.int32)

    def _decode_rows(self, dec, width, pad_to=0):
        """(ids, positions, slots, ctx, block tables) of the decode rows; native
        (csrc/runtime/step_builder.cpp) when the runtime is built.  An item of n > 1 tokens
        (a short extend chunk: jump-forward tokens) becomes n rows with causal contexts."""
        if all(n == 1 for _, _, n in dec):
            tables = [s.block_table for s, _, _ in dec]
            starts = [st for _, st, _ in dec]
            # an in-flight input token (pipelined stepping) is not on the host yet: 0 here,
            # gathered on the device from the previous step's ids (StepInputs.gather)
            toks = [s.token_at(st) if st < s.length else 0 for s, st, _ in dec]
            lens = [s.length + s.num_inflight for s, _, _ in dec]
        else:
            tables, starts, toks, lens = [], [], [], []
            for s, st, n in dec:
                if n == 1:
                    tables.append(s.block_table)
                    starts.append(st)
                    toks.append(s.token_at(st) if st < s.length else 0)
                    lens.append(s.length + s.num_inflight)
                    continue
                for i in range(st, st + n):  # extend tokens are host-known (never in flight)
                    tables.append(s.block_table)
                    starts.append(i)
                    toks.append(s.token_at(i))
                    lens.append(i + 1)
        if _native_rt is not None:
            return _native_rt.decode_rows(tables, starts, toks, lens, self.bs, width, pad_to)
        P = max(len(tables), pad_to)
        ids = np.zeros(P, dtype=np.int32)
        pos = np.zeros(P, dtype=np.int32)
        slots = np.full(P, -1, dtype=np.int32)
        ctx = np.ones(P, dtype=np.int32)
        bt = np.zeros((P, width), dtype=np.int32)
        for i, t in enumerate(tables):
            bt[i, : len(t)] = t
            ids[i], pos[i], ctx[i] = toks[i], starts[i], lens[i]
            slots[i] = t[starts[i] // self.bs] * self.bs + starts[i] % self.bs
        return ids, pos, slots, ctx, bt

    def _shared_len(self, bt: np.ndarray, ctx: np.ndarray, n: int) -> int:
        """Tokens of the longest run of leading cache blocks that ALL n decode rows share
        (prefix-cache hits on a common system prompt), each row keeping >= 1 own key."""
        if not self.cascade or n < 2:
            return 0
        eq = (bt[:n] == bt[0]).all(axis=0)
        S = int(eq.argmin()) if not eq.all() else bt.shape[1]
        S = min(S, (int(ctx[:n].min()) - 1) // self.bs)
        return S * self.bs if S >= 2 else 0

    def _bt(self, tables, width):
        bt = np.zeros((len(tables), width), dtype=np.int32)
        for i, t in enumerate(tables):
            bt[i, : len(t)] = t
        return bt

    # ----------------------------------------------------------- step inputs (host)
    def prepare(self, items, greedy: bool = False):
        """items [(seq, start, n)] -> (StepInputs of host arrays, rows [(seq, row)]).
        Everything a rank needs to run the step; a TP driver broadcasts it.  ``greedy``:
        the step returns token ids (distributed argmax under TP) instead of logits."""
        si, rows = self._prepare(items)
        si.greedy = bool(greedy)
        if si.num_decode:  # keys the decode attention reads this step (in-situ bandwidth accounting)
            self.decode_kv_keys += int(np.asarray(si.ctx_d[: si.num_decode], dtype=np.int64).sum())
        return si, rows

    @staticmethod
    def _gather(dec, offset: int):
        """(dst rows, src rows in the previous step's ids) of decode rows whose input
        token is still in flight, or None."""
        g, r = [], offset
        for s, st, n in dec:
            if n == 1 and st >= s.length:
                g.append((r, s.inflight_row))
            r += n
        if not g:
            return None
        a = np.asarray(g, dtype=np.int64)
        return a[:, 0].copy(), a[:, 1].copy()

    def _as_decode(self, seq, start: int, n: int) -> bool:
        """Decode rows: one-token steps, and short extend chunks of generated tokens
        (jump-forward): n causal decode rows over the paged KV beat a flash-prefill tile
        whose few query rows each walk the whole context in one workgroup."""
        if seq.is_decode:
            return True
        return 1 < n <= EXTEND_AS_DECODE and start >= len(seq.prompt_ids) and seq.num_inflight == 0

    def _prepare(self, items):
        if (self.use_graphs and items and all(self._as_decode(*it) for it in items)
                and sum(n for _, _, n in items) <= self.graph_sizes[-1]):
            return self._prepare_graph(items)
        pre = [it for it in items if not self._as_decode(*it)]
        dec = [it for it in items if self._as_decode(*it)]
        ids, pos, slots = [], [], []
        q_lens, ctx, tables = [], [], []
        rows = []
        r = 0
        for seq, start, n in pre:
            ids.extend(seq.tokens(start, start + n))
            s, p = self._slots(seq.block_table, start, n)
            slots.append(s)
            pos.append(p)
            q_lens.append(n)
            ctx.append(start + n)
            tables.append(seq.block_table)
            r += n
            if start + n == seq.length + seq.num_inflight:
                rows.append((seq, r - 1))
        ctx_d = tables_d = None
        if dec:
            d_ids, d_pos, d_slots, ctx_d, tables_d = self._decode_rows(
                dec, max(len(s.block_table) for s, _, _ in dec))
            ids.extend(d_ids.tolist())
            pos.append(d_pos)
            slots.append(d_slots)
            for seq, start, n in dec:
                r += n
                if start + n == seq.length + seq.num_inflight:
                    rows.append((seq, r - 1))
        nd = len(ctx_d) if dec else 0
        shared = self._shared_len(tables_d, ctx_d, nd) if dec else 0
        si = StepInputs(decode_graph=0, ids=np.asarray(ids, dtype=np.int32), positions=np.concatenate(pos),
                        slots=np.concatenate(slots), q_lens=q_lens, ctx_lens=ctx,
                        tables_p=self._bt(tables, max(len(t) for t in tables)) if pre else None,
                        ctx_d=ctx_d, tables_d=tables_d,
                        num_decode=nd, logits_rows=np.asarray([row for _, row in rows], dtype=np.int64),
                        gather=self._gather(dec, r - nd) if dec else None, shared_len=shared)
        return si, rows

    def _prepare_graph(self, items):
        """Decode rows (one-token steps and short extend chunks, expanded to causal rows)
        for the hipGraph of the smallest bucket that holds them; the graph computes every
        row's logits, the step keeps the rows that end a sequence's new tokens."""
        B = sum(n for _, _, n in items)
        Bg = self._graph_bucket(B)
        ids, pos, slots, ctx, bt = self._decode_rows(items, self.max_blocks, Bg)
        rows, r = [], 0
        for seq, start, n in items:
            r += n
            if start + n == seq.length + seq.num_inflight:
                rows.append((seq, r - 1))
        si = StepInputs(decode_graph=Bg, ids=ids, positions=pos, slots=slots, ctx_d=ctx, tables_d=bt,
                        num_decode=B, logits_rows=np.asarray([row for _, row in rows], dtype=np.int64),
                        gather=self._gather(items, 0), shared_len=self._shared_len(bt, ctx, B))
        return si, rows

    # ----------------------------------------------------------- execution (device)
    def _upload(self, named: dict) -> dict:
        """{name: host array} -> {name: device tensor}: one pinned copy on the GPU, plain
        tensors on the CPU."""
        arrays = {k: np.ascontiguousarray(v) for k, v in named.items() if v is not None}
        if self._stager is None:
            return {k: torch.from_numpy(v).to(self.device, non_blocking=True) for k, v in arrays.items()}
        return dict(zip(arrays, self._stager.upload(list(arrays.values()))))

    def _meta(self, si: "StepInputs"):
        Tp = int(sum(si.q_lens))
        host = {"ids": si.ids, "pos": si.positions, "slots": si.slots}
        if si.q_lens:
            cu = np.zeros(len(si.q_lens) + 1, dtype=np.int32)
            cu[1:] = np.cumsum(si.q_lens)
            host.update(cu=cu, ctx_p=np.asarray(si.ctx_lens, dtype=np.int32), bt_p=si.tables_p)
        if si.num_decode:
            host.update(bt_d=si.tables_d, ctx_d=si.ctx_d)
            if si.shared_len:
                host["shared"] = np.asarray([si.shared_len], dtype=np.int32)
        uni = _attn.UNIFIED_ATTN and bool(si.q_lens) and si.num_decode > 0 and not si.shared_len
        if uni:  # one attention launch for the whole step (models/attention.py UNIFIED_ATTN)
            self.unified_attn_steps = getattr(self, "unified_attn_steps", 0) + 1
            nd, P = si.num_decode, len(si.q_lens)
            ql = list(si.q_lens) + [1] * nd
            cl = list(si.ctx_lens) + np.asarray(si.ctx_d[:nd]).tolist()
            cu_u = np.zeros(len(ql) + 1, dtype=np.int32)
            cu_u[1:] = np.cumsum(ql)
            wp, wd = si.tables_p.shape[1], si.tables_d.shape[1]
            bt_u = np.zeros((len(ql), max(wp, wd)), dtype=np.int32)
            bt_u[:P, :wp] = si.tables_p
            bt_u[P:, :wd] = si.tables_d[:nd]
            host.update(cu_u=cu_u, ctx_u=np.asarray(cl, dtype=np.int32), bt_u=bt_u)
            if self.device.type == "cuda":
                host["ts_u"], host["tq_u"] = ops.prefill_tiles(ql, cl, self.hq // self.hkv, True, self.D)
        if len(si.logits_rows):
            host["logits"] = si.logits_rows
        if si.gather is not None:
            host.update(g_dst=si.gather[0], g_src=si.gather[1])
        d = self._upload(host)
        meta = AttnMeta(positions=d["pos"], slots=d["slots"], num_prefill_tokens=Tp,
                        num_prefill_seqs=len(si.q_lens), num_decode=si.num_decode)
        if si.q_lens:
            meta.cu_q, meta.ctx_lens_p, meta.block_tables_p = d["cu"], d["ctx_p"], d["bt_p"]
            meta.q_lens_cpu, meta.ctx_lens_cpu = list(si.q_lens), list(si.ctx_lens)
        if si.num_decode:
            meta.block_tables_d, meta.ctx_lens_d = d["bt_d"], d["ctx_d"]
            meta.decode_split = max(ops.decode_split_size(si.num_decode, self.hkv), self.bs)
            meta.max_splits = ops.decode_splits(si.tables_d.shape[1] * self.bs, meta.decode_split)
            if si.shared_len:
                self._cascade_meta(meta, si.num_decode, d["shared"])
        if uni:
            meta.cu_u, meta.ctx_lens_u, meta.block_tables_u = d["cu_u"], d["ctx_u"], d["bt_u"]
            if "ts_u" in d:
                meta.tiles_u = (d["ts_u"], d["tq_u"])
        meta.logits_idx = d.get("logits")
        ids = d["ids"]
        if si.gather is not None:
            self._apply_gather(ids, d["g_dst"], d["g_src"])
        return ids, meta

    def _apply_gather(self, ids: torch.Tensor, dst: torch.Tensor, src: torch.Tensor):
        """Fill in-flight input tokens (rows ``dst``) from the previous step's device ids
        (rows ``src``): no host sync."""
        if self.prev_ids is None:
            raise RuntimeError("step has in-flight input tokens but no previous step ids")
        ops.scatter_ids(ids, dst, self.prev_ids, src)

    def _cascade_meta(self, meta, B: int, shared_len: torch.Tensor):
        """Cascade fields of ``meta`` for B decode rows (static shapes per B: graph-safe)."""
        dev = self.device
        rpt = ops.prefill_rows_per_tile(self.hq // self.hkv, self.D)
        nt = (B + rpt - 1) // rpt
        meta.shared_len = shared_len
        meta.shared_cu = torch.tensor([0, B], dtype=torch.int32, device=dev)
        meta.shared_tables = meta.block_tables_d[0:1]
        meta.shared_tiles = (torch.zeros(nt, dtype=torch.int32, device=dev),
                             torch.arange(0, nt * rpt, rpt, dtype=torch.int32, device=dev))
        meta.pp_o = torch.empty(B, self.hq, self.D, dtype=torch.float32, device=dev)
        meta.pp_ml = torch.empty(B, self.hq, 2, dtype=torch.float32, device=dev)

    @torch.inference_mode()
    def execute(self, si: "StepInputs"):
        """Run one step on this rank; returns logits [R, V] f32, or int32 token ids [R]
        for a greedy step (None if no rows)."""
        self._sync_prev(si)
        if si.decode_graph:
            out = self._graph_execute(si)
        else:
            ids, meta = self._meta(si)
            if meta.logits_idx is None:
                self.model(ids, meta, self.kv_caches)  # partial prefill chunks only: KV write, no logits
                return None
            h = self.model(ids, meta, self.kv_caches)
            out = self.model.greedy(h) if si.greedy else self.model.logits(h, dtype=self.logits_dtype)
        if si.greedy:
            self.prev_ids = out  # every TP rank holds the same greedy ids (distributed argmax)
        return out

    def _sync_prev(self, si: "StepInputs"):
        """Pipelined TP steps: ids sampled by the driver (non-greedy previous step) exist on
        rank 0 only; broadcast them over the TP device group (RCCL, no host round trip)
        before this step gathers its in-flight decode inputs from them."""
        tp = getattr(self.model, "tp", None)
        if not si.prev_bcast or tp is None or not tp.enabled:
            return
        if tp.rank == 0:
            buf = self.prev_ids[: si.prev_bcast].to(torch.int32).contiguous()
        else:
            buf = torch.empty(si.prev_bcast, dtype=torch.int32, device=self.device)
        self.prev_ids = tp.broadcast_(buf)

    def forward_logits(self, items, greedy: bool = False):
        """Run one step; returns (rows [(seq,row)], logits [R, V] f32 -- or int32 token
        ids [R] when ``greedy``)."""
        if not items:
            return [], None
        si, rows = self.prepare(items, greedy)
        if si.gather is not None:
            si.prev_bcast = self.prev_sampled_rows
        if self.step_hook is not None:
            self.step_hook(si)  # e.g. TP driver broadcast to worker ranks
        lg = self.execute(si)
        return rows, (lg if rows else None)

    # ----------------------------------------------------------- hipGraph decode
    def _graph_bucket(self, B):
        i = bisect.bisect_left(self.graph_sizes, B)
        return self.graph_sizes[i]

    def _static(self, B):
        dev = self.device
        po, pm = self._decode_ws(B)
        # the graph's inputs are slices of ONE device buffer, refilled by one pinned copy per
        # replay: int32 [ids | pos | slots | ctx | block table | shared_len], then room for
        # the int64 in-flight gather rows (dst, src) and sampled rows of up to B rows
        nb = self.max_blocks
        n32 = 4 * B + B * nb + 1
        _, nbytes = _PinnedStager.layout([np.zeros(n32, np.int32)] + [np.zeros(B, np.int64)] * 3)
        raw = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
        i32 = raw[: 4 * n32].view(torch.int32)
        st = {
            "raw": raw,
            "ids": i32[0:B],
            "pos": i32[B:2 * B],
            "slots": i32[2 * B:3 * B].fill_(-1),
            "ctx": i32[3 * B:4 * B].fill_(1),
            "bt": i32[4 * B:4 * B + B * nb].view(B, nb),
            "shared": i32[4 * B + B * nb:],
        }
        split, ms = self.decode_split(B)
        st["meta"] = AttnMeta(positions=st["pos"], slots=st["slots"], num_decode=B,
                              block_tables_d=st["bt"], ctx_lens_d=st["ctx"], max_splits=ms,
                              decode_split=split, part_o=po, part_ml=pm)
        if self.cascade and B >= 2:
            st["shared_len"] = st["shared"]
            self._cascade_meta(st["meta"], B, st["shared_len"])
        return st

    def capture(self, B, greedy: bool = False):
        st = self._static(B)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm-up (allocator + lazy library init) outside capture
                h = self.model(st["ids"], st["meta"], self.kv_caches)
                self.model.greedy(h) if greedy else self.model.logits(h, dtype=self.logits_dtype)
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        g = torch.cuda.CUDAGraph()
        # thread-local capture: a serving process's other threads (HTTP handlers, the
        # embedding engine's own stream) may touch the device while a bucket is captured
        with torch.cuda.graph(g, pool=self._graph_pool, capture_error_mode="thread_local"):
            h = self.model(st["ids"], st["meta"], self.kv_caches)
            st["logits"] = self.model.greedy(h) if greedy else self.model.logits(h, dtype=self.logits_dtype)
        st["graph"] = g
        self.graphs[(B, greedy)] = st
        return st

    @torch.inference_mode()
    def capture_all(self, max_batch: Optional[int] = None, variants=(False, True)):
        """Capture the decode graphs of every batch bucket (<= max_batch), for the
        sampled-logits and/or the greedy-ids output variant."""
        for B in self.graph_sizes:
            if max_batch is None or B <= max_batch:
                for v in variants:
                    if (B, v) not in self.graphs:
                        self.capture(B, v)

    def _graph_execute(self, si):
        Bg = si.decode_graph
        st = self.graphs.get((Bg, si.greedy)) or self.capture(Bg, si.greedy)
        static = np.concatenate([si.ids, si.positions, si.slots, si.ctx_d, si.tables_d.reshape(-1),
                                 np.asarray([si.shared_len], dtype=np.int32)]).astype(np.int32, copy=False)
        if static.size != 4 * Bg + st["bt"].numel() + 1:
            raise ValueError("decode graph inputs do not match the captured bucket's layout")
        arrays = [static]
        if si.gather is not None:
            arrays += [si.gather[0], si.gather[1]]
        # extend rows: only the last row of each chunk is sampled
        subset = len(si.logits_rows) != si.num_decode
        if subset:
            arrays.append(np.ascontiguousarray(si.logits_rows, dtype=np.int64))
        if self._stager is not None:
            views = self._stager.upload(arrays, dst=st["raw"])
        else:  # pageable copies (LK_PINNED_STAGE=0)
            n32 = static.size
            st["raw"][: 4 * n32].view(torch.int32).copy_(torch.from_numpy(static), non_blocking=True)
            views = [None] + [torch.from_numpy(a).to(self.device, non_blocking=True) for a in arrays[1:]]
        if si.gather is not None:
            self._apply_gather(st["ids"], views[1], views[2])
        st["graph"].replay()
        if subset:
            return ops.gather_rows(st["logits"], views[-1])
        return st["logits"][: si.num_decode]


@dataclass
class StepInputs:
    """Host-side description of one engine step (broadcast to TP worker ranks)."""

    ids: np.ndarray
    positions: np.ndarray
    slots: np.ndarray
    num_decode: int = 0
    decode_graph: int = 0                 # >0: replay the decode hipGraph of this bucket
    q_lens: list = field(default_factory=list)
    ctx_lens: list = field(default_factory=list)
    tables_p: Optional[np.ndarray] = None
    ctx_d: Optional[np.ndarray] = None
    tables_d: Optional[np.ndarray] = None
    logits_rows: np.ndarray = field(default_factory=lambda: np.zeros(0, dtype=np.int64))
    greedy: bool = False                  # return token ids (argmax) instead of logits
    gather: Optional[tuple] = None        # (dst rows, src rows): in-flight ids from the previous step
    shared_len: int = 0                   # cascade: leading keys shared by every decode row
    prev_bcast: int = 0                   # TP: rows of driver-sampled previous ids to broadcast
