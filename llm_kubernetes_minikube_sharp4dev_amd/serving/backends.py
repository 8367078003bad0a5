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


class OllamaHTTPGenerate:
    def __init__(self, base_url: str = "http://127.0.0.1:11434", model: str = "llama3.1:8b", client=None,
                 timeout: float = 300.0, options: Optional[dict] = None):
        import httpx

        self.model = model
        self.options = options
        # no pool cap: every concurrent /agent_rag session holds one streaming /api/generate
        # (httpx's default of 100 connections queued the 101st..128th sessions behind others)
        self.client = client or httpx.AsyncClient(base_url=base_url, timeout=timeout,
                                                  limits=httpx.Limits(max_connections=None,
                                                                      max_keepalive_connections=512))

    async def generate(self, prompt: str) -> str:
        body = {"model": self.model, "prompt": prompt, "stream": True}
        if self.options:
            body["options"] = self.options
        parts = []
        async with self.client.stream("POST", "/api/generate", json=body) as r:
            if r.status_code >= 300:
                text = (await r.aread()).decode("utf-8", "replace")
                raise GenerateError(f"Ollama /api/generate returned {r.status_code}: {text}")
            async for line in r.aiter_lines():
                if not line.strip():
                    continue
                msg = json.loads(line)
                if msg.get("error"):
                    raise GenerateError(msg["error"])
                parts.append(msg.get("response") or "")
                if msg.get("done") and "total_duration" in msg:
                    # the server's own timing of this request (Ollama's done-chunk fields)
                    from ..utils import tracing

                    pe, ev, tot = (msg.get(k, 0) / 1e9 for k in ("prompt_eval_duration", "eval_duration",
                                                                  "total_duration"))
                    tracing.record("ollama", "prompt_eval", pe)
                    tracing.record("ollama", "eval", ev)
                    tracing.record("ollama", "server_total", tot)
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
