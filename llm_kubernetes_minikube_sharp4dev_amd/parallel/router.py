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
    import httpx
    from fastapi import FastAPI
    from fastapi.responses import JSONResponse, Response, StreamingResponse

    pool = ReplicaPool(urls)
    app = FastAPI(title="MI355X DP router")
    app.state.pool = pool
    client = httpx.AsyncClient(timeout=timeout_s)

    async def probe_loop():
        while True:
            await asyncio.sleep(probe_interval_s)
            for r in pool.replicas:
                try:
                    ok = (await client.get(r.url + "/api/version", timeout=2.0)).status_code == 200
                except Exception:
                    ok = False
                if ok and not r.healthy:
                    log.info("replica %s back in rotation", r.url)
                r.healthy = ok
                r.last_probe = time.time()

    @app.on_event("startup")
    async def _start():
        app.state.probe = asyncio.create_task(probe_loop())

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
                req = client.build_request(request.method, f"{r.url}/{path}", content=body, headers=headers,
                                           params=dict(request.query_params))
                resp = await client.send(req, stream=True)
            except Exception:
                r.inflight -= 1
                pool.mark_failed(r)
                continue

            async def relay(resp=resp, rep=r):
                try:
                    async for chunk in resp.aiter_raw():
                        yield chunk
                finally:
                    await resp.aclose()
                    rep.inflight -= 1
                    rep.served += 1

            media = resp.headers.get("content-type")
            if media and "ndjson" in media:
                return StreamingResponse(relay(), status_code=resp.status_code, media_type=media)
            data = b"".join([c async for c in relay()])
            return Response(data, status_code=resp.status_code, media_type=media)

    return app
