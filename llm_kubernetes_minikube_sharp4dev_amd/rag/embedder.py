"""Embedders.

* :class:`OllamaEmbedder` — port of ``Helpers/Embedder.cs``: POSTs
  ``/api/embeddings`` with up to three payload shapes in order
  (``{model, input: str}``, ``{model, input: [str]}``, ``{model, prompt: str}``,
  ``Embedder.cs:14,19,24``), accepts three response shapes (``{"embedding"}``,
  ``{"embeddings": [[..]]}`` first row, OpenAI ``{"data": [{"embedding"}]}``,
  ``Embedder.cs:43-60``); a non-2xx or empty vector moves on; all failing raises
  (``Embedder.cs:28``).
* :class:`LocalEmbedder` — the MI355X path: in-process batched encoder
  (:class:`~..engine.embed_engine.EmbeddingEngine`), no HTTP hop.
* :class:`HashEmbedder` — deterministic bag-of-words vectors for CPU tests.
"""
from __future__ import annotations

import hashlib
import json
import re
from typing import Optional, Sequence

import numpy as np
import torch


class EmbeddingError(RuntimeError):
    pass


def parse_embedding_response(body: dict | list) -> Optional[list]:
    if isinstance(body, dict):
        e = body.get("embedding")
        if isinstance(e, list):
            return [float(x) for x in e]
        m = body.get("embeddings")
        if isinstance(m, list) and m:
            first = m[0]
            if isinstance(first, list):
                return [float(x) for x in first]
        d = body.get("data")
        if isinstance(d, list) and d:
            first = d[0]
            if isinstance(first, dict) and isinstance(first.get("embedding"), list):
                return [float(x) for x in first["embedding"]]
    return None


class OllamaEmbedder:
    MESSAGE = "Impossibile ottenere embeddings da Ollama. Verifica il modello/endpoint."

    def __init__(self, base_url: str = "http://localhost:11434", model: str = "nomic-embed-text",
                 client=None, timeout: float = 120.0):
        import httpx

        self.model = model
        self.base_url, self.timeout = base_url, timeout
        self.client = client or httpx.Client(base_url=base_url, timeout=timeout)
        self._aclient = None
        self.attempts = 0

    async def aembed_one(self, text: str) -> np.ndarray:
        """Async twin of :meth:`embed_one` for an event-loop front-end (same payload order,
        one pooled aiohttp connection per concurrent request, no worker thread)."""
        from ..serving.backends import AioSession

        if self._aclient is None:
            self._aclient = AioSession(self.base_url, self.timeout)
        sess = self._aclient.get()
        for payload in ({"model": self.model, "input": text},
                        {"model": self.model, "input": [text]},
                        {"model": self.model, "prompt": text}):
            self.attempts += 1
            async with sess.post(self._aclient.url("/api/embeddings"),
                                 data=json.dumps(payload, ensure_ascii=False).encode("utf-8"),
                                 headers={"Content-Type": "application/json; charset=utf-8"}) as r:
                if 200 <= r.status < 300:
                    try:
                        e = parse_embedding_response(json.loads(await r.read()))
                    except ValueError:
                        e = None
                    if e:
                        return np.asarray(e, dtype=np.float32)
        raise EmbeddingError(self.MESSAGE)

    def _try(self, payload: dict) -> Optional[list]:
        self.attempts += 1
        r = self.client.post("/api/embeddings", content=json.dumps(payload, ensure_ascii=False).encode("utf-8"),
                             headers={"Content-Type": "application/json; charset=utf-8"})
        if not (200 <= r.status_code < 300):
            return None
        try:
            return parse_embedding_response(r.json())
        except ValueError:
            return None

    def embed_one(self, text: str) -> np.ndarray:
        for payload in ({"model": self.model, "input": text},
                        {"model": self.model, "input": [text]},
                        {"model": self.model, "prompt": text}):
            e = self._try(payload)
            if e:
                return np.asarray(e, dtype=np.float32)
        raise EmbeddingError(self.MESSAGE)

    def embed(self, texts: Sequence[str]) -> np.ndarray:
        # the reference embeds serially, one request per chunk (RagIndex.cs:47)
        return np.stack([self.embed_one(t) for t in texts]) if texts else np.zeros((0, 0), np.float32)


class LocalEmbedder:
    def __init__(self, engine):
        self.engine = engine
        self.model = engine.name

    @property
    def dim(self) -> int:
        return self.engine.dim

    def embed(self, texts: Sequence[str]) -> np.ndarray:
        return self.engine.embed(list(texts)).float().cpu().numpy()

    def embed_tensor(self, texts: Sequence[str]):
        """Device query vectors for the kNN kernels: bf16 rows written by the pooling kernel on
        the GPU (the corpus operand's dtype), f32 on the CPU."""
        dt = torch.bfloat16 if self.engine.device.type == "cuda" else torch.float32
        return self.engine.embed(list(texts), dtype=dt)


_TOKEN = re.compile(r"\w+", re.UNICODE)


class HashEmbedder:
    """Feature-hashed bag of words (+ character trigrams): texts sharing words get high
    cosine, unrelated texts low — enough to exercise gating/threshold logic on CPU."""

    def __init__(self, dim: int = 384, model: str = "hash"):
        self.dim = dim
        self.model = model

    def _vec(self, text: str) -> np.ndarray:
        v = np.zeros(self.dim, np.float32)
        for w in _TOKEN.findall(text.lower()):
            for feat in (w,) + tuple(w[i:i + 3] for i in range(max(1, len(w) - 2))):
                h = int.from_bytes(hashlib.blake2b(feat.encode(), digest_size=8).digest(), "little")
                v[h % self.dim] += 1.0 if (h >> 63) == 0 else -1.0
        return v

    def embed(self, texts: Sequence[str]) -> np.ndarray:
        return np.stack([self._vec(t) for t in texts]) if texts else np.zeros((0, self.dim), np.float32)
