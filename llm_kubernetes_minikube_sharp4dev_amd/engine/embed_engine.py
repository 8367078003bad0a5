"""Batched embedding inference (the ``/api/embeddings`` compute).

Texts are tokenized ([CLS] .. [SEP], truncated to the encoder's max length), packed
varlen into token-budgeted micro-batches (no padding FLOPs) and run through the
encoder; the pooled + L2-normalised vectors come back as one [n, D] f32 tensor.
Index builds embed hundreds of thousands of chunks this way in seconds instead of
one HTTP round-trip per chunk (``RagIndex.cs:47``).
"""
from __future__ import annotations

import threading
import time
from typing import Optional

import numpy as np
import torch

from ..utils import metrics as M


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
        return [[t if t < V else t % V for t in s] for s in ids]

    @torch.inference_mode()
    def embed_ids(self, seqs: list[list[int]]) -> torch.Tensor:
        out = torch.empty((len(seqs), self.dim), dtype=torch.float32, device=self.device)
        i = 0
        while i < len(seqs):
            j, tot = i, 0
            while j < len(seqs) and (tot + len(seqs[j]) <= self.budget or j == i):
                tot += len(seqs[j])
                j += 1
            chunk = seqs[i:j]
            lens = [len(s) for s in chunk]
            flat = np.fromiter((t for s in chunk for t in s), dtype=np.int32, count=tot)
            pos = np.concatenate([np.arange(n, dtype=np.int32) for n in lens])
            cu = np.zeros(len(chunk) + 1, dtype=np.int32)
            cu[1:] = np.cumsum(lens)
            d = self.device
            emb = self.model(torch.from_numpy(flat).to(d, non_blocking=True),
                             torch.from_numpy(cu).to(d, non_blocking=True),
                             torch.from_numpy(pos).to(d, non_blocking=True), lens)
            out[i:j] = emb
            i = j
        return out

    def embed(self, texts: list[str]) -> torch.Tensor:
        t0 = time.perf_counter()
        with self.lock:
            r = self.embed_ids(self.tokenize(texts)) if texts else torch.zeros((0, self.dim))
        M.EMBED_LAT.observe(time.perf_counter() - t0)
        return r
