"""Typed configuration whose defaults equal every constant the reference hard-codes.

Reference constants (``Minimal_RAG/Program.cs:11-18,22-31,50,72,78,96,116,126,159,
230,243``; ``Minimal_Agent_RAG/Program.cs:11-19``; ``Helpers/RagIndex.cs:22-26,80,
92-95,118-121``; ``Helpers/Embedder.cs:9``; ``Properties/launchSettings.json:8,17``).
The region header at ``Minimal_RAG/Program.cs:1`` says they "could be moved to
appsettings.json" — here they are: every field can be overridden from a YAML/JSON
file, ``LK_*`` environment variables, or CLI flags (see :func:`load_config`).
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field, fields
from pathlib import Path
from typing import Any, Optional


@dataclass
class RagConfig:
    """Retrieval constants (reference RAG service)."""

    knowledge_dir: str = "./knowledge"                 # Program.cs:50
    chunk_size: int = 800                              # Program.cs:50 (effectively unused, quirk A.7.1)
    chunk_overlap: int = 120                           # Program.cs:50
    extensions: tuple = (".md", ".txt", ".yaml", ".yml")  # RagIndex.cs:22-26
    header_regex: str = r"^\s*#{1,6}\s+"                # RagIndex.cs:80
    section_max_chars: int = 1200                      # RagIndex.cs:92
    resplit_size: int = 800                            # RagIndex.cs:95
    resplit_overlap: int = 120                         # RagIndex.cs:95
    sanitize_max_chars: int = 2000                     # RagIndex.cs:121
    redact_regex: str = r"(?i)(ignore previous instructions|disregard all prior rules|system prompt)"
    cosine_eps: float = 1e-9                           # RagIndex.cs:134
    search_default_topk: int = 5                       # Program.cs:72
    search_topk_min: int = 1
    search_topk_max: int = 10
    search_min_score: float = 0.20                     # Program.cs:78
    preview_chars: int = 260                           # Program.cs:96
    agent_topk: int = 6                                # Program.cs:116
    evidence_min_score: float = 0.35                   # Program.cs:15
    citation_best_ratio: float = 0.6                   # Program.cs:126
    evidence_text_chars: int = 1500                    # Program.cs:159
    embed_model: str = "nomic-embed-text"              # Program.cs:18
    index_backend: str = "auto"                        # auto | exact (cpu f64) | gpu (HIP kNN)
    cache_dir: str = ""                                # persisted embeddings (checkpoint/resume)


@dataclass
class AgentConfig:
    """Agent / gating constants."""

    allowed_namespaces: tuple = ("dev", "staging", "sharp4dev", "test-ns-giovanni")  # Program.cs:11-12
    gen_model: str = "llama3.1:8b"                     # Program.cs:24, Agent Program.cs:12
    log_tail_lines: int = 200                          # Program.cs:230
    log_max_chars: int = 4000                          # Program.cs:243
    log_truncation_suffix: str = "\n...[truncated]"    # Program.cs:244
    default_namespace: str = "default"                 # Program.cs:198, Agent Program.cs:85
    ollama_url: str = "http://127.0.0.1:11434"         # Program.cs:22 / Agent Program.cs:11
    embedder_url: str = "http://localhost:11434"       # Embedder.cs:9
    kubeconfig: str = r"C:\Users\ACADEMY\.kube\config"  # Program.cs:29 (overridable: $KUBECONFIG)
    fake_cluster: bool = True                          # no kube-apiserver in this environment
    # quirk switches; defaults reproduce the reference behaviour
    agent_strip_fences: bool = False                   # /agent has no fence stripping (A.7.4)
    enforce_runbook_limits: bool = False               # "+2 / <=10 replicas" is prose only (A.7.8)
    request_timeout_s: float = 300.0


@dataclass
class ServerConfig:
    host: str = "127.0.0.1"
    rag_port: int = 5103                               # Minimal_RAG launchSettings.json:8
    rag_https_port: int = 7172                         # Minimal_RAG launchSettings.json:17
    agent_port: int = 5217                             # Minimal_Agent launchSettings.json:8
    agent_https_port: int = 7198                       # Minimal_Agent launchSettings.json:17
    ollama_port: int = 11434
    https_redirection: bool = False                    # reference enables it (A.7.10); no certs here


@dataclass
class EngineConfig:
    """MI355X engine knobs (no reference counterpart: Ollama's internals)."""

    device: str = "auto"                               # auto | cuda | cpu
    dtype: str = "bfloat16"
    kv_block_size: int = 16
    gpu_memory_fraction: float = 0.85                  # of the 288 GB HBM3E
    kv_cache_gb: Optional[float] = None                # explicit KV budget (overrides the fraction)
    max_num_seqs: int = 256
    # per step: whole waves of 256x256 GEMM tiles (profiles/r2_sched_sweep.md).  The .NET-facing
    # server path samples with Ollama's defaults (no grammar, so no jump-forward): round 2's
    # 8192 stays; the grammar-constrained bench runs 4096 (profiles/r3_mbt/)
    max_num_batched_tokens: int = 8192
    # prefill hold-back steps (engine/scheduler.py): the in-process engine default is 4; requests
    # that reach the server one by one through the front-ends lose more to the wait than the
    # fuller steps gain (-1.6 % q/s at 128 sessions, profiles/r5_http/final/), so 0 here
    # (LK_PREFILL_HOLD, when set, overrides both)
    prefill_hold: int = 0
    max_model_len: int = 8192
    enable_prefix_caching: bool = True
    use_hip_graphs: bool = True
    capture_graphs_at_load: bool = True                # serve: capture every decode bucket up front
    graph_batch_sizes: tuple = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256)
    tp_size: int = 1
    seed: int = 0
    # Ollama server-side sampling defaults (applied when a request sets no options)
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.9
    repeat_penalty: float = 1.1
    repeat_last_n: int = 64
    num_ctx: int = 4096
    num_predict: int = -1
    default_max_new_tokens: int = 256


@dataclass
class ModelPresets:
    """Model name (as the .NET clients send it) -> architecture preset."""

    generators: dict = field(default_factory=lambda: {
        "llama3.1:8b": "llama-3-8b",
        "llama3:8b": "llama-3-8b",
        "llama3.1:70b": "llama-3-70b",
        "llama3:70b": "llama-3-70b",
        "opt-125m": "opt-125m",
        "llama-tiny": "llama-tiny",
    })
    embedders: dict = field(default_factory=lambda: {
        "nomic-embed-text": "nomic-embed-text",
        "bge-base": "bge-base",
        "bge-base-en-v1.5": "bge-base",
        "all-minilm": "minilm-l6",
        "minilm": "minilm-l6",
        "bert-tiny": "bert-tiny",
    })


@dataclass
class Config:
    rag: RagConfig = field(default_factory=RagConfig)
    agent: AgentConfig = field(default_factory=AgentConfig)
    server: ServerConfig = field(default_factory=ServerConfig)
    engine: EngineConfig = field(default_factory=EngineConfig)
    models: ModelPresets = field(default_factory=ModelPresets)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


def _coerce(cur: Any, val: Any) -> Any:
    if cur is None and isinstance(val, str):  # Optional numeric knobs (e.g. engine.kv_cache_gb)
        for t in (int, float):
            try:
                return t(val)
            except ValueError:
                pass
        return None if val.lower() in ("", "none", "null") else val
    if isinstance(cur, bool):
        if isinstance(val, str):
            return val.strip().lower() in ("1", "true", "yes", "on")
        return bool(val)
    if isinstance(cur, int) and not isinstance(cur, bool):
        return int(val)
    if isinstance(cur, float):
        return float(val)
    if isinstance(cur, tuple):
        if isinstance(val, str):
            val = [v.strip() for v in val.split(",") if v.strip()]
        items = list(val)
        if cur and isinstance(cur[0], int):
            items = [int(v) for v in items]
        return tuple(items)
    return val


def apply_overrides(cfg: Config, overrides: dict) -> Config:
    """Apply nested ``{"rag": {"agent_topk": 8}}`` or dotted ``{"rag.agent_topk": 8}``."""
    for key, val in overrides.items():
        if isinstance(val, dict) and hasattr(cfg, key):
            sub = getattr(cfg, key)
            for k2, v2 in val.items():
                if not hasattr(sub, k2):
                    raise KeyError(f"unknown config key {key}.{k2}")
                setattr(sub, k2, _coerce(getattr(sub, k2), v2))
        elif "." in key:
            sec, name = key.split(".", 1)
            sub = getattr(cfg, sec)
            if not hasattr(sub, name):
                raise KeyError(f"unknown config key {key}")
            setattr(sub, name, _coerce(getattr(sub, name), val))
        else:
            raise KeyError(f"unknown config key {key}")
    return cfg


def load_config(path: str | os.PathLike | None = None, env: dict | None = None,
                cli: dict | None = None) -> Config:
    """Defaults <- file (YAML/JSON) <- ``LK_<SECTION>__<KEY>`` env vars <- CLI dict."""
    cfg = Config()
    path = path or os.environ.get("LK_CONFIG")
    if path:
        text = Path(path).read_text(encoding="utf-8")
        if str(path).endswith((".yaml", ".yml")):
            import yaml

            data = yaml.safe_load(text) or {}
        else:
            data = json.loads(text)
        apply_overrides(cfg, data)
    env = os.environ if env is None else env
    for k, v in env.items():
        if k.startswith("LK_") and "__" in k:
            sec, name = k[3:].lower().split("__", 1)
            if hasattr(cfg, sec) and hasattr(getattr(cfg, sec), name):
                apply_overrides(cfg, {f"{sec}.{name}": v})
    if os.environ.get("KUBECONFIG") and env is os.environ:
        cfg.agent.kubeconfig = os.environ["KUBECONFIG"]
    if cli:
        apply_overrides(cfg, cli)
    return cfg


def section_fields(section) -> list[str]:
    return [f.name for f in fields(section)]
