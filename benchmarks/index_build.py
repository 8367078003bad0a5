#!/usr/bin/env python3
"""Corpus ingest alone (the index build of bench.py, one GPU): synthetic runbook docs ->
chunks -> bge-base embeddings in HBM.  Prints wall time, tokens, and the host time spent
tokenising vs the device time of the encoder, so a rocprofv3 --stats run of this script shows
whether the build is device- or host-bound.

    python benchmarks/index_build.py [--docs 100000] [--embedder bge-base]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=100000)
    ap.add_argument("--embedder", default="bge-base")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--budget", type=int, default=262144, help="tokens per encoder micro-batch")
    a = ap.parse_args()
    from llm_kubernetes_minikube_sharp4dev_amd.rag.corpus import build_chunks

    t = time.perf_counter()
    chunks = build_chunks(a.docs, a.seed, workers=8)
    t_chunks = time.perf_counter() - t
    import torch

    from llm_kubernetes_minikube_sharp4dev_amd.engine.embed_engine import EmbeddingEngine
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_encoder
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer

    dev = torch.device("cuda", 0)
    tok = builtin_tokenizer()
    enc = build_encoder(a.embedder, device=dev, seed=a.seed, dtype=torch.bfloat16)
    eng = EmbeddingEngine(enc, tok, name=a.embedder, max_tokens_per_batch=a.budget)
    texts = [c[2] for c in chunks]
    eng.embed(texts[:2048])  # warm-up (kernel attributes, allocator)
    torch.cuda.synchronize()
    t = time.perf_counter()
    ids = eng.tok.encode_for_embedding(texts, eng.max_len)
    t_tok = time.perf_counter() - t
    ntok = sum(map(len, ids))
    torch.cuda.synchronize()
    t = time.perf_counter()
    out = eng.embed_ids(ids)
    torch.cuda.synchronize()
    t_dev = time.perf_counter() - t
    t = time.perf_counter()
    out2 = eng.embed(texts)
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t
    assert out2.shape == out.shape
    print(json.dumps({"docs": a.docs, "chunks": len(texts), "tokens": ntok, "chunk_build_s": round(t_chunks, 2),
                      "tokenize_s": round(t_tok, 2), "encoder_from_ids_s": round(t_dev, 2),
                      "embed_texts_s": round(t_all, 2), "tokens_per_s": round(ntok / t_all),
                      "mean_len": round(ntok / len(texts), 1)}), flush=True)


if __name__ == "__main__":
    main()
