#!/usr/bin/env python3
"""Load test of the .NET-facing serving path without GPUs: F HTTP front-end processes
(``serve-frontend``, SO_REUSEPORT on one port) route over R fake engine cores
(:mod:`llm_kubernetes_minikube_sharp4dev_amd.serving.fake_core`: 48 tokens per request, one
per 2 ms "step", frames batched per step as the real core sends them), driven by G client
processes of closed-loop OllamaSharp-style streaming ``POST /api/generate`` requests.  Every
response is checked: 48 NDJSON chunks + a final ``done`` chunk, or it counts as lost.

    python benchmarks/frontend_load.py --replicas 8 --frontends 3 --clients 2 --concurrency 128 --requests 4000
"""
from __future__ import annotations

import argparse
import asyncio
import json
import multiprocessing as mp
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOD = "llm_kubernetes_minikube_sharp4dev_amd"


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _client(url, conc, n, tokens, out_q):
    import aiohttp

    ok = bad = chunks = 0
    it = iter(range(n))
    body = {"model": "llama3.1:8b", "prompt": "Sei un agente DevOps. Elenca i pod nel namespace dev."}
    conn = aiohttp.TCPConnector(limit=conc + 4, keepalive_timeout=60.0)
    async with aiohttp.ClientSession(connector=conn, timeout=aiohttp.ClientTimeout(total=120.0)) as c:
        async def worker():
            nonlocal ok, bad, chunks
            for _ in it:
                try:
                    async with c.post(url + "/api/generate", json=body) as r:
                        lines = [ln for ln in (await r.read()).split(b"\n") if ln.strip()]
                    last = json.loads(lines[-1]) if lines else {}
                    chunks += len(lines)
                    if r.status == 200 and last.get("done") and last.get("eval_count") == tokens:
                        ok += 1
                    else:
                        bad += 1
                except Exception:  # noqa: BLE001 - a lost request
                    bad += 1

        await asyncio.gather(*(worker() for _ in range(conc)))
    out_q.put((ok, bad, chunks))


def _client_proc(url, conc, n, tokens, out_q):
    asyncio.run(_client(url, conc, n, tokens, out_q))


def _wait_http(url, timeout=120):
    import httpx

    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if httpx.get(url + "/api/version", timeout=2).status_code == 200:
                return
        except Exception:  # noqa: BLE001
            pass
        time.sleep(0.3)
    raise SystemExit("front-ends not up")


def run(replicas=8, frontends=3, clients=2, concurrency=128, requests=4000, tokens=48, step_s=0.002) -> dict:
    d = tempfile.mkdtemp(prefix="lk-fe-")
    paths = [os.path.join(d, f"core{i}.sock") for i in range(replicas)]
    port = _port()
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, "-m", f"{MOD}.serving.fake_core", ",".join(paths), str(tokens),
                               str(step_s)], cwd=ROOT, env=env, start_new_session=True)]
    try:
        while not all(os.path.exists(p) for p in paths):
            time.sleep(0.1)
        for _ in range(frontends):
            procs.append(subprocess.Popen([sys.executable, "-m", MOD, "serve-frontend", "--port", str(port),
                                           "--cores", ",".join(paths), "--preload", "llama3.1:8b"],
                                          cwd=ROOT, env=env, start_new_session=True))
        url = f"http://127.0.0.1:{port}"
        _wait_http(url)
        q = mp.get_context("spawn").Queue()
        # warm-up (connections, tokenizer)
        w = mp.get_context("spawn").Process(target=_client_proc, args=(url, 16, 64, tokens, q))
        w.start()
        w.join()
        q.get()
        per = requests // clients
        ps = [mp.get_context("spawn").Process(target=_client_proc, args=(url, concurrency // clients, per, tokens, q))
              for _ in range(clients)]
        t0 = time.perf_counter()
        for p in ps:
            p.start()
        res = [q.get() for _ in ps]
        wall = time.perf_counter() - t0
        for p in ps:
            p.join()
        ok, bad, chunks = (sum(r[i] for r in res) for i in range(3))
        return {"replicas": replicas, "frontends": frontends, "concurrency": concurrency, "requests": per * clients,
                "ok": ok, "lost": bad, "wall_s": round(wall, 2), "req_per_s": round(ok / wall, 1),
                "chunks_per_s": round(chunks / wall, 0), "tokens_per_request": tokens}
    finally:
        for p in procs:
            if p.poll() is None:
                os.killpg(p.pid, signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=8)
    ap.add_argument("--frontends", type=int, default=3)
    ap.add_argument("--clients", type=int, default=2)
    ap.add_argument("--concurrency", type=int, default=128)
    ap.add_argument("--requests", type=int, default=4000)
    ap.add_argument("--tokens", type=int, default=48)
    ap.add_argument("--step-ms", type=float, default=2.0)
    a = ap.parse_args()
    print(json.dumps(run(a.replicas, a.frontends, a.clients, a.concurrency, a.requests, a.tokens, a.step_ms / 1e3)),
          flush=True)


if __name__ == "__main__":
    main()
