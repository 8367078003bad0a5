"""Port of the ``Minimal_Agent`` service (``Minimal_Agent_RAG/Program.cs``):

  GET  /health  -> {"status":"OK"}   (upper-case, unlike the RAG service: quirk A.7.9)
  POST /agent   JSON-prompted tool call -> list_pods / get_logs / scale_deployment
                (no namespace allow-list, no fence stripping, k8s errors unhandled
                -> the framework's default 500, exactly like the reference)
"""
from __future__ import annotations

from fastapi import Request  # module level: FastAPI resolves string annotations here

import time
from typing import Optional

from ..agent.prompts import agent_prompt
from ..agent.tools import UnhandledK8sError, dispatch_agent_tool
from ..config import Config
from ..utils import metrics as M
from ..utils.tracing import Tracer
from .common import BindError, NetJSONResponse, add_https_redirection, bind_body, member, respond


def create_agent_app(cfg: Optional[Config] = None, llm=None, k8s=None):
    import asyncio

    from fastapi import FastAPI, Request
    from starlette.responses import PlainTextResponse, Response

    cfg = cfg or Config()
    app = FastAPI(title="Minimal_Agent (MI355X)")
    app.state.cfg, app.state.llm, app.state.k8s = cfg, llm, k8s
    tracer = Tracer("agent_app")
    if cfg.server.https_redirection:
        add_https_redirection(app, cfg.server.agent_https_port)

    @app.get("/health")
    async def health():
        return NetJSONResponse({"status": "OK"})

    @app.post("/agent")
    async def agent(request: Request):
        t0 = time.perf_counter()
        try:
            body = await bind_body(request)
            prompt = member(body, "prompt")
        except BindError:
            return Response(status_code=400)
        full = agent_prompt(prompt or "")
        with tracer.span("llm.generate"):
            raw = await app.state.llm.generate(full)
        try:
            status, out = await asyncio.to_thread(dispatch_agent_tool, app.state.k8s, raw, cfg)
        except UnhandledK8sError as e:
            return PlainTextResponse(f"An unhandled exception has occurred: {e}", status_code=500)
        M.HTTP_LAT.labels("/agent").observe(time.perf_counter() - t0)
        return respond(status, out)

    return app
