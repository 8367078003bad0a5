"""Data-parallel replica router: one Ollama-compatible endpoint in front of N engine
replicas (one process per MI355X, or per TP group).

Policy: least outstanding requests, ties broken round-robin; streaming responses
are passed through chunk by chunk (NDJSON keeps flowing to the .NET client); a
replica that fails a health probe or a request is taken out of rotation and
re-probed in the background.  Model-admin routes (/api/tags, /api/version, ...)
are answered by the first healthy replica.
"""
from __future__ import annotations

import asyncio
import itertools
import time
from dataclasses import dataclass, field
from typing import Optional

from fastapi import Request

from ..utils.logging import get_logger

log = get_logger("router")


@dataclass
class Replica:
    url: str
    inflight: int = 0
    healthy: bool = True
    served: int = 0
    failures: int = 0
    last_probe: float = field(default_factory=time.time)


class ReplicaPool:
    def __init__(self, urls: list[str]):
        self.replicas = [Replica(u.rstrip("/")) for u in urls]
        self._rr = itertools.count()

    def pick(self) -> Replica:
        live = [r for r in self.replicas if r.healthy] or self.replicas
        m = min(r.inflight for r in live)
        cands = [r for r in live if r.inflight == m]
        return cands[next(self._rr) % len(cands)]

    def mark_failed(self, r: Replica):
        r.failures += 1
        r.healthy = False
        log.warning("replica %s marked unhealthy", r.url)


def create_router_app(urls: list[str], probe_interval_s: float = 5.0, timeout_s: float = 600.0):
    """The router ASGI app.  Upstream calls go through one aiohttp session per event loop
    (an unbounded keep-alive pool): httpx's pool scans grow with the connections in flight
    and took a whole core at 128 concurrent streams in the RAG app (profiles/r2_http_bench.md)."""
    import aiohttp
    from fastapi import FastAPI
    from fastapi.responses import JSONResponse, Response, StreamingResponse

    pool = ReplicaPool(urls)
    app = FastAPI(title="MI355X DP router")
    app.state.pool = pool
    sessions: dict = {}

    def session() -> "aiohttp.ClientSession":
        loop = asyncio.get_running_loop()
        s = sessions.get(loop)
        if s is None or s.closed:
            s = sessions[loop] = aiohttp.ClientSession(
                timeout=aiohttp.ClientTimeout(total=timeout_s),
                connector=aiohttp.TCPConnector(limit=0, keepalive_timeout=60))
        return s

    async def probe_loop():
        while True:
            await asyncio.sleep(probe_interval_s)
            for r in pool.replicas:
                try:
                    async with session().get(r.url + "/api/version", timeout=aiohttp.ClientTimeout(total=2.0)) as resp:
                        ok = resp.status == 200
                except Exception:
                    ok = False
                if ok and not r.healthy:
                    log.info("replica %s back in rotation", r.url)
                r.healthy = ok
                r.last_probe = time.time()

    @app.on_event("startup")
    async def _start():
        app.state.probe = asyncio.create_task(probe_loop())

    @app.on_event("shutdown")
    async def _stop():
        app.state.probe.cancel()
        for s in list(sessions.values()):
            await s.close()
        sessions.clear()

    @app.get("/router/status")
    async def status():
        return {"replicas": [vars(r) for r in pool.replicas]}

    @app.api_route("/{path:path}", methods=["GET", "POST", "DELETE", "HEAD"])
    async def proxy(path: str, request: Request):
        body = await request.body()
        headers = {k: v for k, v in request.headers.items() if k.lower() in ("content-type", "accept", "authorization")}
        tried = set()
        while True:
            r = pool.pick()
            if r.url in tried:
                return JSONResponse({"error": "no healthy replica"}, status_code=503)
            tried.add(r.url)
            r.inflight += 1
            try:
                resp = await session().request(request.method, f"{r.url}/{path}", data=body or None, headers=headers,
                                               params=list(request.query_params.multi_items()))
            except Exception:
                r.inflight -= 1
                pool.mark_failed(r)
                continue

            async def relay(resp=resp, rep=r):
                try:
                    async for chunk in resp.content.iter_any():
                        yield chunk
                finally:
                    resp.release()
                    rep.inflight -= 1
                    rep.served += 1

            media = resp.headers.get("content-type")
            if media and "ndjson" in media:
                return StreamingResponse(relay(), status_code=resp.status, media_type=media)
            data = b"".join([c async for c in relay()])
            return Response(data, status_code=resp.status, media_type=media)

    return app
