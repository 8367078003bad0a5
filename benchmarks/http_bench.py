#!/usr/bin/env python3
"""The .NET-facing serving path, measured end to end over HTTP (``bench.py --via-http``).

Two server processes on this GPU, wired exactly as the unchanged C# solution is:

  A  ``python -m llm_kubernetes_minikube_sharp4dev_amd serve`` -- the Ollama-compatible
     server on :P1 (Llama-3-8B bf16 as ``llama3.1:8b``, bge-base as ``nomic-embed-text``).
     Requests carry no ``options`` (OllamaSharp 5.4.7 ``GenerateAsync(prompt)``,
     ``Minimal_Agent_RAG/Program.cs:52``, ``Helpers.cs:116``), so the server's Ollama
     defaults apply: temperature 0.8, top-k 40, top-p 0.9, repeat penalty 1.1 -- the fused
     device sampler.  ``num_predict`` default = ``--max-new-tokens``.
  B  ``... rag-app --synthetic-docs N`` -- the Minimal_RAG port on :P2: index of bench.py's
     synthetic corpus (bulk-embedded once at start-up on the GPU), and per request: query
     embedding via ``POST /api/embeddings {"model", "input"}`` to A (``Embedder.cs:14,34``),
     GPU kNN, the evidence prompt, ``POST /api/generate`` (NDJSON stream) to A, JSON
     extraction, gating, the (fake) Kubernetes action.

This process (no GPU) drives ``POST /agent_rag`` at each concurrency level with closed-loop
clients and reports requests/s and latency percentiles per level as one JSON line.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import signal
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait(url, proc, timeout):
    import httpx

    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise SystemExit(f"server process exited with {proc.returncode} before {url} came up")
        try:
            if httpx.get(url, timeout=2.0).status_code < 500:
                return time.time() - t0
        except Exception:
            pass
        time.sleep(1.0)
    raise SystemExit(f"{url} not up after {timeout}s")


async def _drive(url, queries, concurrency, n):
    """Closed-loop clients over aiohttp (httpx's pool rescans every connection per request:
    at 128 clients the driver itself became the bottleneck)."""
    import aiohttp

    lat, status = [], {}
    it = iter(range(n))
    conn = aiohttp.TCPConnector(limit=concurrency + 4, keepalive_timeout=60.0)
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=600.0)) as c:
        async def worker():
            for i in it:
                t0 = time.perf_counter()
                async with c.post(url + "/agent_rag", json={"prompt": queries[i % len(queries)]}) as r:
                    await r.read()
                lat.append(time.perf_counter() - t0)
                status[r.status] = status.get(r.status, 0) + 1

        t0 = time.perf_counter()
        await asyncio.gather(*(worker() for _ in range(concurrency)))
        wall = time.perf_counter() - t0
    lat.sort()
    return {"requests": n, "wall_s": round(wall, 2), "value": round(n / wall, 3),
            "p50_latency_ms": round(statistics.median(lat) * 1000, 1),
            "p90_latency_ms": round(lat[int(0.9 * (len(lat) - 1))] * 1000, 1),
            "p99_latency_ms": round(lat[int(0.99 * (len(lat) - 1))] * 1000, 1),
            "http_status_counts": {str(k): v for k, v in sorted(status.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=100_000)
    ap.add_argument("--concurrency", default="1,8,128")
    ap.add_argument("--requests", default="16,64,768", help="requests timed per concurrency level")
    ap.add_argument("--max-new-tokens", type=int, default=48)
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--embedder", default="bge-base")
    ap.add_argument("--kv-gb", type=float, default=48.0)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--frontends", type=int, default=0,
                    help="split server: HTTP front-end processes in front of the GPU engine core (serve --frontends)")
    a = ap.parse_args()
    levels = [int(x) for x in a.concurrency.split(",")]
    counts = [int(x) for x in a.requests.split(",")]
    p1, p2 = _port(), _port()
    env = dict(os.environ, LK_ENGINE__DEFAULT_MAX_NEW_TOKENS=str(a.max_new_tokens),
               LK_ENGINE__KV_CACHE_GB=str(a.kv_gb), LK_ENGINE__MAX_NUM_BATCHED_TOKENS=os.environ.get("LK_ENGINE__MAX_NUM_BATCHED_TOKENS", "8192"),
               LK_ENGINE__MAX_NUM_SEQS="256", PYTHONUNBUFFERED="1")
    mod = "llm_kubernetes_minikube_sharp4dev_amd"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    logs = [open(os.path.join(ROOT, "gpurun_out", f"http_{n}.log"), "w") for n in ("server", "rag_app")]
    srv = subprocess.Popen([sys.executable, "-m", mod, "serve", "--port", str(p1),
                            "--alias", f"llama3.1:8b={a.model}", "--alias", f"nomic-embed-text={a.embedder}",
                            "--preload", "llama3.1:8b", "--preload", "nomic-embed-text"]
                           + (["--frontends", str(a.frontends)] if a.frontends else []),
                           cwd=ROOT, env=env, stdout=logs[0], stderr=subprocess.STDOUT, start_new_session=True)
    app = None
    try:
        t_srv = _wait(f"http://127.0.0.1:{p1}/api/tags", srv, 900)
        app = subprocess.Popen([sys.executable, "-m", mod, "rag-app", "--port", str(p2),
                                "--ollama-url", f"http://127.0.0.1:{p1}", "--synthetic-docs", str(a.docs),
                                "--bulk-embed", a.embedder],
                               cwd=ROOT, env=env, stdout=logs[1], stderr=subprocess.STDOUT, start_new_session=True)
        t_app = _wait(f"http://127.0.0.1:{p2}/health", app, 900)
        print(f"[http_bench] server up in {t_srv:.0f}s, rag-app up in {t_app:.0f}s", file=sys.stderr, flush=True)
        from llm_kubernetes_minikube_sharp4dev_amd.rag.synthetic import make_queries

        queries = make_queries(max(counts) + 64, seed=11)
        url = f"http://127.0.0.1:{p2}"
        asyncio.run(_drive(url, queries, 16, 32))  # warm-up: graphs, prefix cache, connections
        import httpx

        import psutil

        res = {}
        procs = {"server": psutil.Process(srv.pid), "rag_app": psutil.Process(app.pid)}
        for c, n in zip(levels, counts):
            since = time.time()
            cpu0 = {k: sum(p.cpu_times()[:2]) for k, p in procs.items()}
            try:
                res[str(c)] = asyncio.run(_drive(url, queries, c, n))
            except Exception:
                # name which process went away (a negative code is the signal that ended it)
                print(f"[http_bench] concurrency {c} failed: server exit={srv.poll()} "
                      f"rag-app exit={app.poll()}", file=sys.stderr, flush=True)
                raise
            wall = res[str(c)]["wall_s"]
            res[str(c)]["process_cpu_frac"] = {k: round((sum(p.cpu_times()[:2]) - cpu0[k]) / wall, 2)
                                               for k, p in procs.items()}
            spans = httpx.get(f"{url}/debug/spans", params={"since": since}, timeout=30).json()
            spans.update(httpx.get(f"http://127.0.0.1:{p1}/debug/spans", params={"since": since}, timeout=30).json())
            res[str(c)]["app_spans_ms"] = {k.split(".", 1)[1]: {"mean": round(v["mean_s"] * 1e3, 1),
                                                                  "p50": round(v["p50_s"] * 1e3, 1)}
                                           for k, v in spans.items() if "mean_s" in v}
            # the served engine's per-request accounting (prompt / cached-prefix / uncached tokens,
            # preemptions, engine steps queued and run): compare with bench.py's in-process JSON
            # (split server: the engine core's own counters, "core.*"; else the server's)
            src = "core." if any(k.startswith("core.req_") for k in spans) else "server."
            res[str(c)]["server_accounting"] = {k.split(".", 1)[1]: round(v["mean"], 2)
                                                for k, v in spans.items() if "mean" in v and k.startswith(src)}
            print(f"[http_bench] concurrency {c}: {res[str(c)]}", file=sys.stderr, flush=True)
        top = res[str(levels[-1])]
        out = {"metric": f"RAG queries/sec via HTTP (/agent_rag -> /api/embeddings + /api/generate), "
                         f"{'Llama-3-8B' if a.model == 'llama-3-8b' else a.model}",
               "value": top["value"], "unit": "queries/s", "n_gpus": 1, "higher_is_better": True,
               "dtype": "bf16", "data": f"synthetic ({a.docs} runbook docs; random-init weights)",
               "p50_latency_ms": top["p50_latency_ms"], "p90_latency_ms": top["p90_latency_ms"],
               "p99_latency_ms": top["p99_latency_ms"],
               "config": {"model": f"{a.model} (bf16) as llama3.1:8b + {a.embedder} as nomic-embed-text",
                          "server": (f"split: GPU engine core + {a.frontends} HTTP front-end processes"
                                     if a.frontends else "one process (HTTP + engine)"),
                          "sampling": "Ollama server defaults (no options sent): temperature 0.8, top-k 40, "
                                      "top-p 0.9, repeat penalty 1.1 / 64",
                          "num_predict": a.max_new_tokens, "levels": res}}
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    finally:
        for p in (app, srv):
            if p is not None and p.poll() is None:
                os.killpg(p.pid, signal.SIGTERM)
        for p in (app, srv):
            if p is not None:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    os.killpg(p.pid, signal.SIGKILL)


if __name__ == "__main__":
    main()
