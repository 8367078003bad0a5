"""Synthetic knowledge-base construction at benchmark scale (100k-1M documents).

Documents (``rag.synthetic``) go through the reference ingestion rules
(``chunking.chunk_document``) in a process pool; chunk ids follow
``"{filename}#{i}"``.  Multi-GPU runs shard the *embedding* work across ranks and
all-gather the corpus matrix over RCCL, so index build time drops with N.
"""
from __future__ import annotations

import multiprocessing as mp
import os
from typing import Optional

from .chunking import chunk_document
from .synthetic import make_document


def _work(args):
    lo, hi, seed, min_c, max_c, sec = args
    import random

    out = []
    rng = random.Random(seed * 7 + lo)
    for i in range(lo, hi):
        name = f"runbook_{i:07d}.md"
        doc = make_document(i, seed, rng.randint(min_c, max_c), sec)
        for j, c in enumerate(chunk_document(doc)):
            out.append((f"{name}#{j}", f"./knowledge/{name}", c))
    return out


def build_chunks(n_docs: int, seed: int = 0, workers: Optional[int] = None, min_chars: int = 400,
                 max_chars: int = 2400, section_chars: int = 0) -> list[tuple[str, str, str]]:
    """All chunks (id, source, text) of ``n_docs`` synthetic runbooks, in document order
    (``section_chars``: the long-evidence corpus, :func:`.synthetic.make_document`)."""
    workers = workers or max(1, min(16, (os.cpu_count() or 2)))
    step = max(1, (n_docs + workers * 4 - 1) // (workers * 4))
    tasks = [(lo, min(n_docs, lo + step), seed, min_chars, max_chars, section_chars)
             for lo in range(0, n_docs, step)]
    if workers == 1 or n_docs < 2000:
        parts = [_work(t) for t in tasks]
    else:
        with mp.get_context("fork").Pool(workers) as pool:
            parts = pool.map(_work, tasks)
    return [c for p in parts for c in p]
