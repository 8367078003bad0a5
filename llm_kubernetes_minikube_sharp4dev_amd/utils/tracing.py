"""Per-request tracing spans (embed, kNN, prefill, decode, k8s).

Spans are recorded in a bounded ring buffer, exported as JSON lines to a file when
``LK_TRACE_FILE`` is set, and fed to the Prometheus latency histograms.  GPU work
inside a span can optionally be bracketed with ``torch.cuda.synchronize`` for
accurate device timings (``LK_TRACE_SYNC=1``) and annotated for rocprofv3 via
roctx ranges (``torch.cuda.nvtx`` maps to roctx on ROCm).
"""
from __future__ import annotations

import contextlib
import json
import os
import threading
import time
from collections import deque

_lock = threading.Lock()
_buffer: deque = deque(maxlen=10000)
_file = None


def _export(rec: dict):
    global _file
    path = os.environ.get("LK_TRACE_FILE")
    if not path:
        return
    with _lock:
        if _file is None:
            _file = open(path, "a", encoding="utf-8")
        _file.write(json.dumps(rec) + "\n")
        _file.flush()


class Tracer:
    def __init__(self, component: str):
        self.component = component
        self.sync = os.environ.get("LK_TRACE_SYNC", "0") == "1"
        self.roctx = os.environ.get("LK_TRACE_ROCTX", "0") == "1"

    @contextlib.contextmanager
    def span(self, name: str, **attrs):
        rng = None
        if self.sync or self.roctx:
            try:
                import torch

                if self.sync and torch.cuda.is_available():
                    torch.cuda.synchronize()
                if self.roctx and torch.cuda.is_available():
                    torch.cuda.nvtx.range_push(f"{self.component}.{name}")
                    rng = True
            except Exception:
                pass
        t0 = time.perf_counter()
        err = None
        try:
            yield
        except Exception as e:
            err = repr(e)
            raise
        finally:
            if self.sync:
                try:
                    import torch

                    if torch.cuda.is_available():
                        torch.cuda.synchronize()
                except Exception:
                    pass
            dur = time.perf_counter() - t0
            if rng:
                import torch

                torch.cuda.nvtx.range_pop()
            rec = {"ts": time.time(), "component": self.component, "span": name, "dur_s": dur, **attrs}
            if err:
                rec["error"] = err
            with _lock:
                _buffer.append(rec)
            _export(rec)


def record(component: str, span: str, dur_s: float, **attrs):
    """Add an externally timed span (e.g. durations an upstream server reported)."""
    rec = {"ts": time.time(), "component": component, "span": span, "dur_s": dur_s, **attrs}
    with _lock:
        _buffer.append(rec)
    _export(rec)


def count(component: str, name: str, value: float, **attrs):
    """Add a per-request count (tokens, preemptions, engine steps): summarised as n / mean /
    sum instead of a latency."""
    rec = {"ts": time.time(), "component": component, "span": name, "value": float(value), **attrs}
    with _lock:
        _buffer.append(rec)
    _export(rec)


def recent(n: int = 100) -> list:
    with _lock:
        return list(_buffer)[-n:]


def summary(since: float = 0.0) -> dict:
    """Per-span count / mean / p50 / p99 over the buffer (spans that ended after ``since``,
    a ``time.time()`` stamp)."""
    by: dict = {}
    counts: dict = {}
    for r in recent(len(_buffer)):
        if r["ts"] >= since:
            if "value" in r:
                counts.setdefault(f"{r['component']}.{r['span']}", []).append(r["value"])
            else:
                by.setdefault(f"{r['component']}.{r['span']}", []).append(r["dur_s"])
    out = {}
    for k, v in by.items():
        v = sorted(v)
        out[k] = {"n": len(v), "mean_s": sum(v) / len(v), "p50_s": v[len(v) // 2], "p99_s": v[min(len(v) - 1, int(0.99 * len(v)))]}
    for k, v in counts.items():
        out[k] = {"n": len(v), "mean": sum(v) / len(v), "sum": sum(v)}
    return out
