"""Batched embedding inference (the ``/api/embeddings`` compute).

Texts are tokenized ([CLS] .. [SEP], truncated to the encoder's max length), packed
varlen into token-budgeted micro-batches (no padding FLOPs) and run through the
encoder; the pooled + L2-normalised vectors come back as one [n, D] f32 tensor.
Index builds embed hundreds of thousands of chunks this way in seconds instead of
one HTTP round-trip per chunk (``RagIndex.cs:47``).
"""
from __future__ import annotations

import itertools
import os
import threading
import time
from typing import Optional

import numpy as np
import torch

from ..utils import metrics as M


def _nullctx():
    import contextlib

    return contextlib.nullcontext()

# high-priority HIP streams for concurrent serving embeddings (one per in-flight micro-batch)
EMBED_STREAMS = int(os.environ.get("LK_EMBED_STREAMS", "2"))
# bulk embedding (index build): consecutive micro-batches alternate over this many HIP streams,
# so one batch's memory-bound kernels (attention, LayerNorm, pooling) and its GEMMs' partial last
# waves overlap the next batch's work instead of draining the device between kernels
BUILD_STREAMS = int(os.environ.get("LK_EMBED_BUILD_STREAMS", "2"))
# The LK_GEMM_LIBRARY=1 measurement arm sends the encoder's GEMMs to hipBLASLt, whose gfx950
# stream-K kernels (..._SK3_...) keep workgroups waiting on other workgroups' partial tiles: two
# such persistent grids on two streams can fill the CUs with waiters whose producers cannot be
# dispatched (round 4 recorded a 485k-chunk index build that stalled 180 s under that arm).  Our
# own kernels never wait across workgroups outside gemm.hip's guarded stream-K path, so only that
# arm drops to ONE stream for builds and serving embeddings.
if os.environ.get("LK_GEMM_LIBRARY", "0") == "1":
    BUILD_STREAMS = EMBED_STREAMS = 1


# One query of at most QUERY_GRAPH_MAX_LEN tokens (the batch-1 serving path: a request's
# retrieval is on its own critical path) replays a hipGraph of the whole encoder captured for its
# length by :meth:`EmbeddingEngine.capture_queries`, instead of ~85 eager launches (~1 ms of host
# time the device waits through).  LK_EMBED_GRAPHS=0: always eager.
QUERY_GRAPHS = os.environ.get("LK_EMBED_GRAPHS", "1") != "0"
QUERY_GRAPH_MAX_LEN = 64


class EmbeddingEngine:
    def __init__(self, model, tokenizer, name: str = "encoder", max_tokens_per_batch: int = 65536,
                 max_len: Optional[int] = None):
        self.model = model
        self.tok = tokenizer
        self.name = name
        self.budget = max_tokens_per_batch
        self.max_len = min(max_len or model.cfg.max_position, model.cfg.max_position)
        self.device = model.device
        self.lock = threading.Lock()

    @property
    def dim(self) -> int:
        return self.model.cfg.hidden

    def tokenize(self, texts: list[str]) -> list[list[int]]:
        ids = self.tok.encode_for_embedding(texts, self.max_len)
        V = self.model.cfg.vocab_size
        return [[t % V for t in s] for s in ids]

    def _flat(self, seqs) -> tuple[np.ndarray, np.ndarray]:
        """(flat int32 ids folded into the encoder vocabulary, lengths) -- C-level loops."""
        lens = np.fromiter(map(len, seqs), dtype=np.int64, count=len(seqs))
        flat = np.fromiter(itertools.chain.from_iterable(seqs), dtype=np.int64, count=int(lens.sum()))
        V = self.model.cfg.vocab_size
        if flat.size and flat.max() >= V:
            np.remainder(flat, V, out=flat)
        return flat.astype(np.int32), lens

    @torch.inference_mode()
    def _run(self, flat: np.ndarray, lens: np.ndarray, out: torch.Tensor, row0: int, streams=None):
        """Embed packed sequences into out[row0:]: token-budgeted varlen micro-batches,
        launched asynchronously (the caller tokenises the next texts meanwhile).  With
        ``streams`` the micro-batches alternate over them (the caller joins them afterwards)."""
        d = self.device
        starts = np.zeros(len(lens) + 1, dtype=np.int64)
        starts[1:] = np.cumsum(lens)
        i, k = 0, 0
        while i < len(lens):
            j = i + 1
            while j < len(lens) and starts[j + 1] - starts[i] <= self.budget:
                j += 1
            a, b = int(starts[i]), int(starts[j])
            ln = lens[i:j]
            pos = (np.arange(b - a, dtype=np.int64) - np.repeat(starts[i:j] - a, ln)).astype(np.int32)
            cu = (starts[i:j + 1] - a).astype(np.int32)
            st = streams[k % len(streams)] if streams else None
            if j - i == 1 and st is None and self._replay_query(flat[a:b], out[row0 + i:row0 + j]):
                i, k = j, k + 1
                continue
            with torch.cuda.stream(st) if st is not None else _nullctx():
                dst = out[row0 + i:row0 + j]
                # on the GPU the pooling kernel writes the rows of ``out`` (f32 or bf16) itself
                emb = self.model(torch.from_numpy(flat[a:b]).to(d, non_blocking=True),
                                 torch.from_numpy(cu).to(d, non_blocking=True),
                                 torch.from_numpy(pos).to(d, non_blocking=True), ln.tolist(),
                                 out=dst if d.type == "cuda" else None)
                if emb.data_ptr() != dst.data_ptr():
                    dst.copy_(emb)
            i, k = j, k + 1

    # ------------------------------------------------------------------ query hipGraphs
    @torch.inference_mode()
    def capture_queries(self, max_len: int = QUERY_GRAPH_MAX_LEN, dtypes=(torch.bfloat16, torch.float32),
                        priority: int = 0) -> int:
        """Capture one hipGraph of the encoder per single-query length 1..max_len (and output
        dtype), sharing one memory pool; returns the number captured.  Call once at start-up,
        while nothing else runs on the device (capture is thread-local: other threads' launches
        stay legal).  ``priority``: of the stream the replays run on (-1: a serving process's
        query embeddings go ahead of the LLM engine's queued kernels, as embed_cpu's do)."""
        if self.device.type != "cuda" or not QUERY_GRAPHS:
            return 0
        from .. import ops

        d = self.device
        self._qgraphs = getattr(self, "_qgraphs", {})
        self._qpool = getattr(self, "_qpool", None) or torch.cuda.graph_pool_handle()
        n = 0
        with self.lock:
            for dt in dtypes:
                for L in range(1, max_len + 1):
                    if (L, dt) in self._qgraphs:
                        continue
                    ids = torch.full((L,), 101 % self.model.cfg.vocab_size, dtype=torch.int32, device=d)
                    cu = torch.tensor([0, L], dtype=torch.int32, device=d)
                    pos = torch.arange(L, dtype=torch.int32, device=d)
                    out = torch.empty((1, self.dim), dtype=dt, device=d)
                    G = self.model.nh // self.model.nh  # (encoder attention: one kv head per head)
                    ts, tq = ops.prefill_tiles([L], [L], G, False, self.model.D)
                    tiles = (torch.from_numpy(ts).to(d), torch.from_numpy(tq).to(d))
                    side = torch.cuda.Stream(d)
                    side.wait_stream(torch.cuda.current_stream(d))
                    with torch.cuda.stream(side):  # warm-up launch (lazy kernel attributes, allocator)
                        self.model(ids, cu, pos, [L], out=out, tiles=tiles)
                    torch.cuda.current_stream(d).wait_stream(side)
                    g = torch.cuda.CUDAGraph()
                    try:
                        with torch.cuda.graph(g, pool=self._qpool, capture_error_mode="thread_local"):
                            self.model(ids, cu, pos, [L], out=out, tiles=tiles)
                    except Exception as e:  # an op that cannot be captured: stay eager (loudly)
                        import logging

                        logging.getLogger("lk.embed").warning("query encoder graph capture failed at "
                                                              "length %d (%r): eager launches", L, e)
                        self._qgraphs.clear()
                        return 0
                    # every tensor the graph reads stays referenced here: a freed ``cu`` / ``pos``
                    # goes back to the caching allocator, and a replay would read whatever
                    # reuses it (garbage segment bounds / positions)
                    self._qgraphs[(L, dt)] = (g, ids, out, tiles, cu, pos)
                    n += 1
            self._gstream = torch.cuda.Stream(d, priority=priority)
        return n

    def _replay_query(self, seq: np.ndarray, dst: torch.Tensor) -> bool:
        """One query's encoder pass by graph replay into ``dst`` [1, D] (False: no graph).
        Called under ``self.lock``; input copy, replay and output copy all go on one stream of
        this engine, so concurrent callers (the server's embedding threads) never overwrite a
        graph's buffers under a replay still in flight."""
        graphs = getattr(self, "_qgraphs", None)
        if not graphs or torch.cuda.is_current_stream_capturing():
            return False
        ent = graphs.get((len(seq), dst.dtype))
        if ent is None:
            return False
        g, ids, out = ent[:3]
        host = torch.from_numpy(np.ascontiguousarray(seq, dtype=np.int32)).pin_memory()
        cur = torch.cuda.current_stream(self.device)
        gs = self._gstream
        gs.wait_stream(cur)  # dst exists (and whatever the caller queued before it)
        with torch.cuda.stream(gs):
            ids.copy_(host, non_blocking=True)
            g.replay()
            dst.copy_(out)
        dst.record_stream(gs)
        cur.wait_stream(gs)
        return True

    @torch.inference_mode()
    def embed_ids(self, seqs: list[list[int]]) -> torch.Tensor:
        out = torch.empty((len(seqs), self.dim), dtype=torch.float32, device=self.device)
        if seqs:
            flat, lens = self._flat(seqs)
            self._run(flat, lens, out, 0)
        return out

    @torch.inference_mode()
    def _embed_texts(self, texts: list[str], group: int = 4096, bulk: bool = False,
                     dtype=torch.float32) -> torch.Tensor:
        """Tokenise group by group: group g+1 is tokenised on the CPU (native encoder,
        GIL released) while the device runs group g's encoder batches.  ``bulk`` (index
        builds): the micro-batches alternate over BUILD_STREAMS streams, joined at the end.
        ``dtype``: of the returned rows (bf16: the kNN query operand, written by the pooling
        kernel)."""
        out = torch.empty((len(texts), self.dim), dtype=dtype, device=self.device)
        streams = None
        if bulk and self.device.type == "cuda" and BUILD_STREAMS > 1 and len(texts) > group:
            if getattr(self, "_build_streams", None) is None:
                self._build_streams = [torch.cuda.Stream(self.device) for _ in range(BUILD_STREAMS)]
            streams = self._build_streams
            cur = torch.cuda.current_stream(self.device)
            for st in streams:  # out (and anything before it) exists before the side streams write
                st.wait_stream(cur)
                out.record_stream(st)
        for g0 in range(0, len(texts), group):
            ids = self.tok.encode_for_embedding(texts[g0:g0 + group], self.max_len)
            flat, lens = self._flat(ids)
            self._run(flat, lens, out, g0, streams)
        if streams:
            cur = torch.cuda.current_stream(self.device)
            for st in streams:
                cur.wait_stream(st)
        return out

    def embed_cpu(self, texts: list[str]) -> torch.Tensor:
        """Host f32 [n, D] embeddings computed on one of this engine's high-priority HIP
        streams and copied back on it: a serving process's query embeddings do not queue
        behind the LLM engine's pipelined steps.  The lock covers only the launches; the wait
        for the copy happens outside it, so concurrent callers (the server's micro-batcher
        runs up to two batches at once) overlap their device waits."""
        if self.device.type != "cuda":
            return self.embed(texts).float()
        t0 = time.perf_counter()
        with self.lock:
            if getattr(self, "_streams", None) is None:
                # high priority: a query embedding (a few ms of small kernels) is dispatched
                # ahead of the queued kernels of the LLM engine's step instead of behind them
                self._streams = [torch.cuda.Stream(self.device, priority=-1) for _ in range(EMBED_STREAMS)]
                self._next = 0
            st = self._streams[self._next]
            self._next = (self._next + 1) % len(self._streams)
            with torch.cuda.stream(st):
                r = self._embed_texts(list(texts)) if texts else torch.zeros((0, self.dim), device=self.device)
                host = torch.empty(r.shape, dtype=torch.float32, pin_memory=True)
                host.copy_(r, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st)
        ev.synchronize()
        M.EMBED_LAT.observe(time.perf_counter() - t0)
        return host

    def embed(self, texts: list[str], dtype=torch.float32) -> torch.Tensor:
        t0 = time.perf_counter()
        with self.lock:
            r = (self._embed_texts(list(texts), bulk=True, dtype=dtype) if texts
                 else torch.zeros((0, self.dim), dtype=dtype))
        M.EMBED_LAT.observe(time.perf_counter() - t0)
        return r
