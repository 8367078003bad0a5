"""Model registry of the serving process: maps the model names the .NET clients send
(``llama3.1:8b``, ``nomic-embed-text`` — ``Minimal_RAG/Program.cs:18,24``) to
architecture presets, loads them lazily (random-init or a safetensors directory)
onto this process's GPU, and owns one engine per model.

Tensor-parallel cores (``serve --tp T``, ``ModelManager(tp=group)``): the manager of rank 0 builds
its generator as the TP leader (``parallel.tp_engine.make_tp_engine``: the scheduler, sampler and
block allocator live here, every step is broadcast to the T-1 follower ranks), and each follower
rank's manager runs :meth:`ModelManager.run_tp_worker` for the same model -- built from the same
preset / checkpoint / seed and the same engine sizes, so both sides join the start-up
collectives (IPC self-check and tuning, KV-pool agreement, decode-graph capture) in one order.
A TP core serves exactly one generator (its followers hold that model's shards); embedders stay
on the leader's GPU."""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Optional

import torch

from ..config import Config
from ..engine.embed_engine import EmbeddingEngine
from ..engine.llm_engine import AsyncLLMEngine, LLMEngine
from ..models import build_decoder, build_encoder
from ..models.configs import DECODERS, ENCODERS, param_count
from ..models.tokenizer import load_tokenizer
from ..utils.logging import get_logger

log = get_logger("serving.models")


@dataclass
class GeneratorHandle:
    name: str
    preset: str
    engine: LLMEngine
    async_engine: AsyncLLMEngine
    tokenizer: object
    chat_style: str
    loaded_at: float = field(default_factory=time.time)
    load_s: float = 0.0


@dataclass
class EmbedderHandle:
    name: str
    preset: str
    engine: EmbeddingEngine
    loaded_at: float = field(default_factory=time.time)
    load_s: float = 0.0


class ModelManager:
    def __init__(self, cfg: Optional[Config] = None, device: Optional[str] = None,
                 aliases: Optional[dict] = None, checkpoints: Optional[dict] = None,
                 engine_overrides: Optional[dict] = None, tp=None):
        self.cfg = cfg or Config()
        self.tp = tp if tp is not None and tp.size > 1 else None
        self.device = torch.device(device) if device else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self.aliases = dict(aliases or {})
        self.checkpoints = dict(checkpoints or {})
        self.engine_overrides = dict(engine_overrides or {})
        self.generators: dict[str, GeneratorHandle] = {}
        self.embedders: dict[str, EmbedderHandle] = {}
        self.lock = threading.RLock()

    # ------------------------------------------------------------ resolution
    def resolve(self, name: str) -> tuple[str, str]:
        """-> (kind, preset) for a client-side model name."""
        n = self.aliases.get(name, name)
        base = n.split(":latest")[0]
        gens, embs = self.cfg.models.generators, self.cfg.models.embedders
        for cand in (n, base):
            if cand in gens:
                return "generate", gens[cand]
            if cand in embs:
                return "embed", embs[cand]
            if cand in DECODERS:
                return "generate", cand
            if cand in ENCODERS:
                return "embed", cand
        raise KeyError(f"model '{name}' not found")

    def known_models(self) -> list[tuple[str, str, str]]:
        out = []
        for n, p in self.cfg.models.generators.items():
            out.append((n, "generate", self.aliases.get(n, p) if n in self.aliases else p))
        for n, p in self.cfg.models.embedders.items():
            out.append((n, "embed", p))
        return out

    # ------------------------------------------------------------ loading
    def generator(self, name: str) -> GeneratorHandle:
        with self.lock:
            if name in self.generators:
                return self.generators[name]
            kind, preset = self.resolve(name)
            if kind != "generate":
                raise KeyError(f"model '{name}' does not support generate")
            for h in self.generators.values():  # same preset under another name
                if h.preset == preset:
                    self.generators[name] = h
                    return h
            if self.tp is not None and self.generators:
                other = next(iter(self.generators.values()))
                raise KeyError(f"model '{name}': this TP={self.tp.size} core serves '{other.name}' only")
            t0 = time.perf_counter()
            e = self.cfg.engine
            model, tok = self._build_generator(name, preset)
            runner_kw, engine_kw = self._engine_kwargs(model)
            if self.tp is not None:
                from ..parallel.tp_engine import make_tp_engine, tp_capture_all

                eng = make_tp_engine(model, self.tp, tok, engine_kw=engine_kw, **runner_kw)
                if eng.runner.use_graphs and e.capture_graphs_at_load:
                    tp_capture_all(eng, max_batch=e.max_num_seqs)
            else:
                eng = LLMEngine(model, tok, **runner_kw, **engine_kw)
                if eng.runner.use_graphs and e.capture_graphs_at_load:
                    # every decode bucket (sampled-logits and greedy-ids variants) before the first
                    # request: no capture ever runs concurrently with serving traffic
                    eng.runner.capture_all(max_batch=e.max_num_seqs)
            style = "llama3" if model.cfg.arch == "llama" else "raw"
            h = GeneratorHandle(name, preset, eng, AsyncLLMEngine(eng, request_timeout_s=self.cfg.agent.request_timeout_s),
                                tok, style,
                                load_s=time.perf_counter() - t0)
            self.generators[name] = h
            log.info("loaded generator %s (%s) in %.1fs", name, preset, h.load_s)
            return h

    def _dtype(self) -> torch.dtype:
        """Weight / activation dtype of the served models (``engine.dtype``; bf16 by default,
        float32 for exact CPU comparisons)."""
        dt = getattr(torch, self.cfg.engine.dtype, None)
        if not isinstance(dt, torch.dtype):
            raise ValueError(f"engine.dtype {self.cfg.engine.dtype!r} is not a torch dtype")
        return dt

    def _build_generator(self, name: str, preset: str):
        ck = self.checkpoints.get(name) or self.checkpoints.get(preset)
        model = build_decoder(preset, device=self.device, seed=self.cfg.engine.seed, checkpoint=ck, dtype=self._dtype(),
                              **({"tp": self.tp} if self.tp is not None else {}))
        return model, load_tokenizer(ck)

    # runner-side sizes (every TP rank builds a runner with these) vs leader-only engine settings
    _RUNNER_KEYS = ("block_size", "max_model_len", "max_num_seqs", "use_graphs", "gpu_memory_fraction",
                    "kv_cache_gb", "num_blocks")

    def _engine_kwargs(self, model) -> tuple[dict, dict]:
        e = self.cfg.engine
        kw = dict(block_size=e.kv_block_size, max_model_len=min(e.max_model_len, model.cfg.max_position),
                  max_num_seqs=e.max_num_seqs, max_num_batched_tokens=e.max_num_batched_tokens,
                  enable_prefix_caching=e.enable_prefix_caching, use_graphs=e.use_hip_graphs,
                  gpu_memory_fraction=e.gpu_memory_fraction, kv_cache_gb=e.kv_cache_gb, seed=e.seed)
        if self.device.type == "cpu":
            kw["num_blocks"] = 2048
        if "LK_PREFILL_HOLD" not in os.environ:
            kw["prefill_hold"] = e.prefill_hold
        kw.update(self.engine_overrides)
        runner = {k: v for k, v in kw.items() if k in self._RUNNER_KEYS}
        return runner, {k: v for k, v in kw.items() if k not in self._RUNNER_KEYS}

    def tp_generator_name(self, preload=None) -> str:
        """The one generator a TP core serves: the first ``--preload`` that is a generator,
        else the agent's configured model (``cfg.agent.gen_model``)."""
        for m in preload or []:
            if self.resolve(m)[0] == "generate":
                return m
        return self.cfg.agent.gen_model

    def run_tp_worker(self, name: str):
        """Follower rank of a TP core: build this rank's shard of ``name`` and execute the
        leader's steps (and sharded kNN searches) until it stops the group."""
        from ..parallel.tp_engine import run_tp_worker

        if self.tp is None:
            raise RuntimeError("run_tp_worker needs a ModelManager(tp=group) with tp.size > 1")
        kind, preset = self.resolve(name)
        if kind != "generate":
            raise KeyError(f"model '{name}' does not support generate")
        model, _ = self._build_generator(name, preset)
        runner_kw, _ = self._engine_kwargs(model)
        return run_tp_worker(model, self.tp, **runner_kw)

    def embedder(self, name: str) -> EmbedderHandle:
        with self.lock:
            if name in self.embedders:
                return self.embedders[name]
            kind, preset = self.resolve(name)
            if kind != "embed":
                raise KeyError(f"model '{name}' does not support embeddings")
            t0 = time.perf_counter()
            ck = self.checkpoints.get(name) or self.checkpoints.get(preset)
            enc = build_encoder(preset, device=self.device, seed=self.cfg.engine.seed, checkpoint=ck, dtype=self._dtype())
            eng = EmbeddingEngine(enc, load_tokenizer(ck), name=name)
            if self.device.type == "cuda":  # one-query /api/embeddings calls replay hipGraphs
                eng.capture_queries(dtypes=(torch.float32,), priority=-1)
            h = EmbedderHandle(name, preset, eng, load_s=time.perf_counter() - t0)
            self.embedders[name] = h
            log.info("loaded embedder %s (%s) in %.1fs", name, preset, h.load_s)
            return h

    def details(self, name: str) -> dict:
        kind, preset = self.resolve(name)
        if kind == "generate":
            c = DECODERS[preset]
            n = param_count(c)
            fam = c.arch
        else:
            c = ENCODERS[preset]
            n = c.num_layers * 12 * c.hidden * c.hidden + c.vocab_size * c.hidden
            fam = "nomic-bert" if c.arch == "nomic_bert" else "bert"
        size = f"{n / 1e9:.1f}B" if n >= 1e9 else f"{n / 1e6:.0f}M"
        return {"format": "safetensors" if (self.checkpoints.get(name) or self.checkpoints.get(preset)) else "random-init",
                "family": fam, "families": [fam], "parameter_size": size, "quantization_level": "BF16",
                "params": n, "preset": preset, "kind": kind}

    def shutdown(self):
        for h in {id(h): h for h in self.generators.values()}.values():
            h.async_engine.shutdown()
            if getattr(h.engine, "tp_ctrl", None) is not None:
                from ..parallel.tp_engine import shutdown_tp

                with h.engine.lock:
                    shutdown_tp(h.engine)  # the followers leave run_tp_worker
