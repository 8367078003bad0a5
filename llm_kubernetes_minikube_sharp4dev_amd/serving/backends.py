"""Generation backends used by the agent apps.

* :class:`OllamaHTTPGenerate` — what OllamaSharp 5.4.7's ``GenerateAsync(prompt)`` does
  for the reference (C8): ``POST /api/generate {"model", "prompt", "stream": true}``,
  NDJSON chunks concatenated by ``response``; no options, so the server's defaults
  apply.  Works against this repo's server or a real Ollama.
* :class:`LocalGenerate` — in-process call into the MI355X engine (no HTTP hop),
  same template and sampling defaults as the server.
* :class:`ScriptedGenerate` — fake LLM for tests: scripted outputs, latency and fault
  injection.
"""
from __future__ import annotations

import asyncio
import itertools
import json
import random
from typing import Optional


class GenerateError(RuntimeError):
    pass


class AioSession:
    """One aiohttp session per event loop for a front-end's calls to the model server.

    httpx/httpcore rescans its whole pool for every request (``_assign_requests_to_
    connections``): at 128 concurrent sessions -- 128 streaming generates plus 128 embeds
    in flight -- that scan was the RAG app's largest CPU cost (24 M ``is_idle`` calls in
    16 s, measured with LK_PYPROFILE).  aiohttp's connector keeps idle connections in a
    per-host deque.  No connection cap (every concurrent session holds one stream)."""

    def __init__(self, base_url: str, timeout: float):
        self.base_url = base_url.rstrip("/")
        self.timeout = timeout
        self._loop = self._session = None

    def get(self):
        import aiohttp

        loop = asyncio.get_running_loop()
        if self._session is None or self._loop is not loop or self._session.closed:
            self._loop = loop
            self._session = aiohttp.ClientSession(
                connector=aiohttp.TCPConnector(limit=0, keepalive_timeout=60.0),
                timeout=aiohttp.ClientTimeout(total=self.timeout))
        return self._session

    def url(self, path: str) -> str:
        return self.base_url + path


class OllamaHTTPGenerate:
    def __init__(self, base_url: str = "http://127.0.0.1:11434", model: str = "llama3.1:8b", client=None,
                 timeout: float = 300.0, options: Optional[dict] = None):
        self.model = model
        self.options = options
        # ``client``: an httpx.AsyncClient (tests drive the ASGI app in-process through one);
        # otherwise aiohttp to the server
        self.client = client
        self.aio = AioSession(base_url, timeout) if client is None else None

    def _done_chunk(self, msg: dict):
        if msg.get("done") and "total_duration" in msg:
            # the server's own timing of this request (Ollama's done-chunk fields)
            from ..utils import tracing

            pe, ev, tot = (msg.get(k, 0) / 1e9 for k in ("prompt_eval_duration", "eval_duration", "total_duration"))
            tracing.record("ollama", "prompt_eval", pe)
            tracing.record("ollama", "eval", ev)
            tracing.record("ollama", "server_total", tot)

    def _line(self, line, parts: list):
        if not line.strip():
            return
        msg = json.loads(line)
        if msg.get("error"):
            raise GenerateError(msg["error"])
        parts.append(msg.get("response") or "")
        self._done_chunk(msg)

    async def generate(self, prompt: str) -> str:
        body = {"model": self.model, "prompt": prompt, "stream": True}
        if self.options:
            body["options"] = self.options
        parts: list = []
        if self.aio is not None:
            async with self.aio.get().post(self.aio.url("/api/generate"), json=body) as r:
                if r.status >= 300:
                    text = (await r.read()).decode("utf-8", "replace")
                    raise GenerateError(f"Ollama /api/generate returned {r.status}: {text}")
                async for line in r.content:  # NDJSON: one chunk per line
                    self._line(line, parts)
            return "".join(parts)
        async with self.client.stream("POST", "/api/generate", json=body) as r:
            if r.status_code >= 300:
                text = (await r.aread()).decode("utf-8", "replace")
                raise GenerateError(f"Ollama /api/generate returned {r.status_code}: {text}")
            async for line in r.aiter_lines():
                self._line(line, parts)
        return "".join(parts)


class LocalGenerate:
    def __init__(self, manager, model: str = "llama3.1:8b", params=None, processor_factory=None):
        self.manager = manager
        self.model = model
        self.params = params
        self.processor_factory = processor_factory

    async def generate(self, prompt: str) -> str:
        from ..engine.sampling import SamplingParams

        h = await asyncio.to_thread(self.manager.generator, self.model)
        e = self.manager.cfg.engine
        sp = self.params or SamplingParams.from_ollama(None, e, e.default_max_new_tokens)
        sp = SamplingParams(**{**sp.__dict__})
        if self.processor_factory is not None:
            sp.logits_processor = self.processor_factory(h.tokenizer)
        ids = h.tokenizer.chat_prompt(prompt, style=h.chat_style) if h.chat_style != "raw" else \
            h.tokenizer.encode(prompt, add_bos=True)
        seq = await h.async_engine.generate(ids, sp)
        return h.tokenizer.decode([t for t in seq.output_ids if t not in h.engine.eos_ids])


class ScriptedGenerate:
    def __init__(self, outputs, latency_s: float = 0.0, fault_rate: float = 0.0, seed: int = 0):
        self.outputs = itertools.cycle([outputs] if isinstance(outputs, str) else list(outputs))
        self.latency_s = latency_s
        self.fault_rate = fault_rate
        self.rng = random.Random(seed)
        self.prompts: list[str] = []

    async def generate(self, prompt: str) -> str:
        self.prompts.append(prompt)
        if self.latency_s:
            await asyncio.sleep(self.latency_s)
        if self.fault_rate and self.rng.random() < self.fault_rate:
            raise GenerateError("injected LLM fault")
        out = next(self.outputs)
        return out(prompt) if callable(out) else out
