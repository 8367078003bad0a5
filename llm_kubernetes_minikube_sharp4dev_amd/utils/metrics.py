"""Prometheus metrics (the reference has logging only; SURVEY §5 asks for QPS,
latency percentiles, TTFT/TPOT, batch size, KV utilisation and kNN latency)."""
from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest

REGISTRY = CollectorRegistry(auto_describe=True)

_LAT = (0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60)

REQUESTS = Counter("lk_requests_total", "generation requests admitted", registry=REGISTRY)
GEN_TOKENS = Counter("lk_generated_tokens_total", "tokens generated", registry=REGISTRY)
STEP_TOKENS = Histogram("lk_step_tokens", "tokens per engine step", registry=REGISTRY,
                        buckets=(1, 8, 32, 64, 128, 256, 1024, 4096, 16384, 65536))
STEP_TIME = Histogram("lk_step_seconds", "engine step wall time", registry=REGISTRY, buckets=_LAT)
KV_USAGE = Gauge("lk_kv_cache_usage", "fraction of KV blocks in use", registry=REGISTRY)
RUNNING = Gauge("lk_running_seqs", "sequences in the running batch", registry=REGISTRY)
HTTP_LAT = Histogram("lk_http_request_seconds", "HTTP request latency", ["route"], registry=REGISTRY,
                     buckets=_LAT)
KNN_LAT = Histogram("lk_knn_seconds", "kNN query latency", registry=REGISTRY, buckets=_LAT)
EMBED_LAT = Histogram("lk_embed_seconds", "embedding batch latency", registry=REGISTRY, buckets=_LAT)
TTFT = Histogram("lk_ttft_seconds", "time to first token", registry=REGISTRY, buckets=_LAT)


def render() -> bytes:
    return generate_latest(REGISTRY)
