"""In-memory vector store — the MI355X counterpart of ``Helpers/RagIndex.cs``.

Ingestion (``RagIndex.cs:14-56``): recursive enumeration of ``.md/.txt/.yaml/.yml``
(case-insensitive), UTF-8 read, header split / sliding window, sanitize, skip blank
chunks, chunk id ``"{filename}#{i}"`` (``i`` counts kept chunks), source = path,
``[RAG]`` log lines; a missing folder logs a warning and leaves the index empty.
Unlike the reference (one HTTP embedding round-trip per chunk, serially) chunks
are embedded in large GPU batches.

Query (``RagIndex.cs:59-67``): embed the query, cosine against EVERY chunk, stable
descending sort, take ``max(1, topK)``.  Backends:

* ``exact`` — the reference's arithmetic: f32 products accumulated in f64,
  ``dot / (sqrt(na)*sqrt(nb) + 1e-9)``; dimension mismatch scores -1.
* ``gpu``   — corpus matrix resident in HBM (bf16 + f32 norms); the fused HIP
  cosine + top-k kernel (``csrc/knn.hip``) with the same tie order.

Checkpoint/resume: :meth:`save` / :meth:`load` persist embeddings +
metadata (safetensors + JSON) keyed by file content hash, so a restart re-embeds
only changed files.
"""
from __future__ import annotations

import hashlib
import json
import os
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Optional, Sequence

import numpy as np
import torch

from .. import ops
from ..utils import metrics as M
from ..utils.logging import get_logger
from .chunking import chunk_document, chunk_sliding, is_blank, sanitize, split_by_markdown_headers

log = get_logger("rag")

EXTENSIONS = (".md", ".txt", ".yaml", ".yml")


@dataclass
class RagChunk:                      # record RagChunk(Id, Source, Text, Embedding) — Program.cs:326
    id: str
    source: str
    text: str


@dataclass
class RagHit:                        # record RagHit(Id, Source, Text, double Score) — Program.cs:327
    id: str
    source: str
    text: str
    score: float


def cosine_exact(a: np.ndarray, b: np.ndarray) -> float:
    """``RagIndex.Cosine``: f32 element products, f64 accumulation, +1e-9."""
    if a.shape[-1] != b.shape[-1]:
        return -1.0
    a = a.astype(np.float32)
    b = b.astype(np.float32)
    dot = float(np.sum((a * b).astype(np.float64)))
    na = float(np.sum((a * a).astype(np.float64)))
    nb = float(np.sum((b * b).astype(np.float64)))
    return dot / (np.sqrt(na) * np.sqrt(nb) + 1e-9)


def enumerate_files(folder: str) -> list[str]:
    out = []
    for root, _dirs, files in os.walk(folder):
        for f in files:
            if f.lower().endswith(EXTENSIONS):
                out.append(os.path.join(root, f))
    return sorted(out)


class RagIndex:
    def __init__(self, embedder, backend: str = "auto", device: Optional[str] = None,
                 gpu_threshold: int = 20000):
        self.embedder = embedder
        self.backend = backend
        self.device = torch.device(device) if device else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self.gpu_threshold = gpu_threshold
        self.chunks: list[RagChunk] = []
        self._emb: list[np.ndarray] = []       # host f32 rows (exact backend / persistence)
        self._mat: Optional[np.ndarray] = None
        self._gpu = None                       # (corpus bf16, norms f32) on device
        self.file_hashes: dict[str, str] = {}

    # ------------------------------------------------------------ ingestion
    def __len__(self):
        return len(self.chunks)

    def add(self, ids: Sequence[str], sources: Sequence[str], texts: Sequence[str], emb: np.ndarray):
        for i, s, t, e in zip(ids, sources, texts, emb):
            self.chunks.append(RagChunk(i, s, t))
            self._emb.append(np.asarray(e, dtype=np.float32))
        self._mat = None
        self._gpu = None

    def build_from_folder(self, folder: str, chunk_size: int = 800, overlap: int = 120,
                          batch_chunks: int = 4096) -> int:
        if not os.path.isdir(folder):
            log.warning("[RAG] Cartella non trovata: %s", folder)
            return 0
        files = enumerate_files(folder)
        log.info("[RAG] File trovati in %s: %d", folder, len(files))
        pend_ids, pend_src, pend_txt = [], [], []

        def flush():
            if pend_txt:
                self.add(pend_ids, pend_src, pend_txt, self.embedder.embed(pend_txt))
                pend_ids.clear(), pend_src.clear(), pend_txt.clear()

        for path in files:
            log.info("[RAG] Indicizzo file: %s", path)
            with open(path, "rb") as fh:
                raw = fh.read()
            self.file_hashes[path] = hashlib.sha256(raw).hexdigest()
            text = raw.decode("utf-8", errors="replace")
            if text.startswith("﻿"):
                text = text[1:]  # File.ReadAllTextAsync(UTF8) drops the BOM
            chunks = chunk_document(text, chunk_size, overlap)
            name = os.path.basename(path)
            for i, c in enumerate(chunks):
                pend_ids.append(f"{name}#{i}")
                pend_src.append(path)
                pend_txt.append(c)
            log.info("[RAG] Chunks dal file %s: %d", path, len(chunks))
            if len(pend_txt) >= batch_chunks:
                flush()
        flush()
        log.info("[RAG] Totale chunks indicizzati: %d", len(self.chunks))
        return len(self.chunks)

    # ------------------------------------------------------------ query
    def matrix(self) -> np.ndarray:
        if self._mat is None:
            self._mat = np.stack(self._emb) if self._emb else np.zeros((0, 0), np.float32)
        return self._mat

    def _use_gpu(self) -> bool:
        if self.backend == "gpu":
            local = True
        elif self.backend == "exact":
            local = False
        else:
            local = self.device.type == "cuda" and len(self.chunks) >= self.gpu_threshold
        if getattr(self, "_sharded", None) is not None:
            # the sharded scan ranks exactly like the single-GPU bf16 scan; where this process
            # would score on the host instead (backend 'exact', or 'auto' below the threshold) and
            # still holds the fp32 matrix, it does -- so a TP server ranks near-ties like TP=1
            return local or not self._emb
        return local

    def gpu_tensors(self):
        if self._gpu is None:
            corpus = torch.from_numpy(self.matrix()).to(self.device, torch.bfloat16).contiguous()
            self._gpu = (corpus, ops.row_norms(corpus))
        return self._gpu

    def set_gpu_corpus(self, corpus_bf16: torch.Tensor, norms: Optional[torch.Tensor] = None):
        """Attach a corpus matrix produced directly on the GPU (bulk index builds)."""
        self._gpu = (corpus_bf16.contiguous(), norms if norms is not None else ops.row_norms(corpus_bf16))

    def set_sharded(self, search_fn, dim: Optional[int] = None):
        """Route searches through a corpus-sharded kNN: ``search_fn(queries [nq, D] bf16, k) ->
        (scores f32 [nq, k], ids int32 [nq, k])`` (parallel.tp_engine.tp_knn_search: every TP
        rank scans its shard, merged in the single-scan order).  None restores the local scan.
        With a sharded search this process keeps no device copy of the corpus; ``dim`` (the
        corpus width) lets a mismatched query fail here rather than inside the sharded kNN."""
        self._sharded = search_fn
        self._sharded_dim = dim
        if search_fn is not None:
            self._gpu = None

    def search_vectors_async(self, q: np.ndarray | torch.Tensor, top_k: int) -> "PendingSearch":
        """Launch a batched search without blocking the host: on the GPU the kNN kernel and
        one non-blocking copy of its (scores, ids) into pinned memory are enqueued on the
        current stream behind an event; :meth:`PendingSearch.result` waits for that event
        only (an engine thread collects it after its next step, when it has long completed).
        Elsewhere the search runs synchronously."""
        k = max(1, top_k)
        n = len(self.chunks)
        if n == 0 or not self._use_gpu():
            return PendingSearch(done=self.search_vectors(q, top_k) if n else [[] for _ in range(len(q))])
        qt = torch.as_tensor(q)
        sharded = getattr(self, "_sharded", None)
        if sharded is not None:
            # the shard's dtype (bf16 on the GPU, f32 on the CPU) is applied by the search
            dim = getattr(self, "_sharded_dim", None)
            if dim is not None and qt.shape[-1] != dim:
                raise ValueError(f"query width {qt.shape[-1]} != corpus width {dim}")
            s, i = sharded(qt.reshape(-1, qt.shape[-1]), min(k, 64))
        else:
            corpus, norms = self.gpu_tensors()
            # host queries are cast on the host (a few KB) and copied once: no device cast kernel
            qt = (qt.to(torch.bfloat16).to(self.device) if qt.device.type == "cpu"
                  else qt.to(self.device, torch.bfloat16)).reshape(-1, corpus.shape[1]).contiguous()
            qn = ops.row_norms(qt) if qt.is_cuda else qt.float().norm(dim=-1)
            s, i = ops.knn_topk(corpus, norms, qt, qn, min(k, 64))
        if not s.is_cuda:
            return PendingSearch(done=_rows(s.tolist(), i.tolist(), min(k, n)))
        hs = torch.empty(s.shape, dtype=s.dtype, pin_memory=True)
        hi = torch.empty(i.shape, dtype=i.dtype, pin_memory=True)
        hs.copy_(s, non_blocking=True)
        hi.copy_(i, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        return PendingSearch(host=(hs, hi, min(k, n)), event=ev)

    def search_vectors(self, q: np.ndarray | torch.Tensor, top_k: int) -> list[list[tuple[int, float]]]:
        """Batched: q [nq, D] -> per query [(chunk_index, score)] (stable order)."""
        k = max(1, top_k)
        n = len(self.chunks)
        if n == 0:
            return [[] for _ in range(len(q))]
        if self._use_gpu():
            return self.search_vectors_async(q, top_k).result()
        mat = self.matrix()
        qa = np.asarray(q.float().cpu().numpy() if isinstance(q, torch.Tensor) else q, dtype=np.float32)
        if qa.ndim == 1:
            qa = qa[None]
        out = []
        for qv in qa:
            if qv.shape[-1] != mat.shape[1]:
                scores = np.full(n, -1.0)
            else:
                prod = (mat * qv[None, :]).astype(np.float64).sum(1)
                na = float(np.sum((qv * qv).astype(np.float64)))
                nb = (mat * mat).astype(np.float64).sum(1)
                scores = prod / (np.sqrt(na) * np.sqrt(nb) + 1e-9)
            order = np.argsort(-scores, kind="stable")[: min(k, n)]
            out.append([(int(j), float(scores[j])) for j in order])
        return out

    def query(self, query: str, top_k: int = 5) -> list[RagHit]:
        qv = self.embedder.embed([query])
        return self.hits(self.search_vectors(qv, top_k)[0])

    def query_batch(self, queries: Sequence[str], top_k: int = 5) -> list[list[RagHit]]:
        qv = self.embedder.embed(list(queries))
        return [self.hits(r) for r in self.search_vectors(qv, top_k)]

    def hits(self, res) -> list[RagHit]:
        return [RagHit(self.chunks[j].id, self.chunks[j].source, self.chunks[j].text, s) for j, s in res]

    # ------------------------------------------------------------ persistence
    def save(self, path: str):
        from safetensors.numpy import save_file

        p = Path(path)
        p.mkdir(parents=True, exist_ok=True)
        save_file({"embeddings": self.matrix().astype(np.float32)}, str(p / "embeddings.safetensors"))
        meta = {"chunks": [c.__dict__ for c in self.chunks], "file_hashes": self.file_hashes,
                "model": getattr(self.embedder, "model", None), "saved_at": time.time()}
        (p / "index.json").write_text(json.dumps(meta, ensure_ascii=False), encoding="utf-8")

    def load(self, path: str) -> bool:
        from safetensors.numpy import load_file

        p = Path(path)
        if not (p / "index.json").exists():
            return False
        meta = json.loads((p / "index.json").read_text(encoding="utf-8"))
        if meta.get("model") != getattr(self.embedder, "model", None):
            log.warning("[RAG] cached index built with %s, embedder is %s: ignoring cache",
                        meta.get("model"), getattr(self.embedder, "model", None))
            return False
        emb = load_file(str(p / "embeddings.safetensors"))["embeddings"]
        self.chunks = [RagChunk(**c) for c in meta["chunks"]]
        self._emb = list(emb)
        self._mat = emb if len(emb) else None
        self._gpu = None
        self.file_hashes = meta.get("file_hashes", {})
        return True

    def build_incremental(self, folder: str, cache_dir: str, chunk_size: int = 800, overlap: int = 120) -> dict:
        """Load the cached index, re-embed only files whose content hash changed."""
        old = RagIndex(self.embedder, self.backend, str(self.device))
        have = old.load(cache_dir)
        files = enumerate_files(folder) if os.path.isdir(folder) else []
        reused = embedded = 0
        self.chunks, self._emb, self.file_hashes = [], [], {}
        by_src: dict[str, list[int]] = {}
        if have:
            for j, c in enumerate(old.chunks):
                by_src.setdefault(c.source, []).append(j)
        for path in files:
            raw = open(path, "rb").read()
            h = hashlib.sha256(raw).hexdigest()
            self.file_hashes[path] = h
            if have and old.file_hashes.get(path) == h and path in by_src:
                for j in by_src[path]:
                    self.chunks.append(old.chunks[j])
                    self._emb.append(old._emb[j])
                reused += len(by_src[path])
                continue
            text = raw.decode("utf-8", errors="replace").lstrip("﻿")
            chunks = chunk_document(text, chunk_size, overlap)
            name = os.path.basename(path)
            if chunks:
                self.add([f"{name}#{i}" for i in range(len(chunks))], [path] * len(chunks), chunks,
                         self.embedder.embed(chunks))
            embedded += len(chunks)
        self._mat = None
        self._gpu = None
        self.save(cache_dir)
        return {"reused": reused, "embedded": embedded, "total": len(self.chunks)}


__all__ = ["RagIndex", "RagChunk", "RagHit", "cosine_exact", "enumerate_files", "split_by_markdown_headers",
           "chunk_sliding", "sanitize", "is_blank"]


def _rows(s, i, k):
    return [[(ii, ss) for ss, ii in zip(sr, ir) if ii >= 0][:k] for sr, ir in zip(s, i)]


class PendingSearch:
    """A launched :meth:`RagIndex.search_vectors_async`: ``ready()`` polls its event,
    ``result()`` waits for it (not for the device) and decodes the rows once."""

    def __init__(self, host=None, event=None, done=None):
        self._host, self._event, self._done = host, event, done
        self.wait_s = 0.0  # host time spent blocked in result()

    def ready(self) -> bool:
        return self._done is not None or self._event is None or self._event.query()

    def result(self) -> list:
        if self._done is None:
            t0 = time.perf_counter()
            if self._event is not None:
                self._event.synchronize()
            self.wait_s = time.perf_counter() - t0
            hs, hi, k = self._host
            self._done = _rows(hs.tolist(), hi.tolist(), k)
            M.KNN_LAT.observe(self.wait_s)
        return self._done
