"""Port of the ``Minimal_RAG`` service (``Minimal_RAG/Program.cs``) with identical routes
and JSON contracts:

  GET  /health       -> {"status":"ok"}                                  (C2, :55)
  POST /rag/search   pure retrieval, topK default 5 clamp [1,10], best-score
                     0.20 floor, 260-char previews                        (C3, :62-100)
  POST /agent_rag    retrieve top-6 -> citations -> LLM tool call -> gated k8s
                     action -> {result, citations, note}                  (C4, :106-316)

Bootstrap (C1): the index is built from ``knowledge_dir`` BEFORE serving
(``Program.cs:50``), constants come from :class:`~..config.Config`.  The LLM and the
embedder are pluggable: HTTP to an Ollama-compatible server (as the reference), or
in-process MI355X engines.
"""
from __future__ import annotations

from fastapi import Request  # module level: FastAPI resolves string annotations here

import asyncio
import time
from typing import Optional

from ..agent.dotnet_json import _num as net_num
from ..agent.json_extract import extract_json_object
from ..agent.policy import select_citations
from ..agent.prompts import RAG_AGENT_SYSTEM, json_prompt, rag_agent_input
from ..agent.tools import dispatch_rag_tool
from ..config import Config
from ..rag.chunking import is_blank, u16len, u16slice
from ..utils import metrics as M
from ..utils.logging import get_logger
from ..utils.tracing import Tracer
from .common import BindError, NetJSONResponse, add_https_redirection, bind_body, member, respond

log = get_logger("RAG.Search")


def create_rag_app(cfg: Optional[Config] = None, index=None, llm=None, k8s=None, build_index: bool = True):
    from fastapi import FastAPI, Request
    from starlette.responses import Response

    cfg = cfg or Config()
    r = cfg.rag
    app = FastAPI(title="Minimal_RAG (MI355X)")
    app.state.cfg, app.state.index, app.state.llm, app.state.k8s = cfg, index, llm, k8s
    tracer = Tracer("rag_app")
    app.state.tracer = tracer
    if build_index and index is not None and len(index) == 0:
        if r.cache_dir:
            index.build_incremental(r.knowledge_dir, r.cache_dir, r.chunk_size, r.chunk_overlap)
        else:
            index.build_from_folder(r.knowledge_dir, r.chunk_size, r.chunk_overlap)
    if cfg.server.https_redirection:
        add_https_redirection(app, cfg.server.rag_https_port)

    import numpy as np

    from ..serving.batcher import MicroBatcher

    # the app's kNN shares the GPU with the model server's engine: its few small kernels go on a
    # high-priority stream so they are dispatched ahead of the engine's queued step kernels
    knn_stream = None
    if getattr(getattr(index, "device", None), "type", "cpu") == "cuda":
        import torch

        knn_stream = torch.cuda.Stream(index.device, priority=-1)

    def knn_batch(qs):
        qa = np.stack([np.asarray(q, dtype=np.float32) for q in qs])
        if knn_stream is None:
            return index.search_vectors(qa, r.agent_topk)
        import torch

        with torch.cuda.stream(knn_stream):
            return index.search_vectors(qa, r.agent_topk)

    knn_batcher = MicroBatcher(knn_batch, max_items=64)

    @app.get("/health")
    async def health():
        return NetJSONResponse({"status": "ok"})

    @app.post("/rag/search")
    async def rag_search(request: Request):
        t0 = time.perf_counter()
        try:
            body = await bind_body(request)
            query = member(body, "query")
            top_k = member(body, "topK", "int")
        except BindError:
            return Response(status_code=400)
        if is_blank(query):
            return NetJSONResponse({"error": "Query vuota"}, status_code=400)
        k = r.search_default_topk if top_k is None else min(max(top_k, r.search_topk_min), r.search_topk_max)
        with tracer.span("rag.search", k=k):
            hits = await asyncio.to_thread(index.query, query, k)
        if not hits:
            return NetJSONResponse({"info": "Nessun risultato. L'indice potrebbe essere vuoto.", "results": []})
        best = max(h.score for h in hits)
        log.info("[RAG] Best score = %s", best)
        M.HTTP_LAT.labels("/rag/search").observe(time.perf_counter() - t0)
        if best < r.search_min_score:
            return NetJSONResponse({
                "info": f"Best score basso ({net_num(best)}). Aggiungi runbook più pertinenti o verifica l'indice.",
                "results": [{"id": h.id, "source": h.source, "score": h.score} for h in hits]})
        out = []
        for h in hits:
            prev = u16slice(h.text, 0, r.preview_chars) + "..." if u16len(h.text) > r.preview_chars else h.text
            out.append({"id": h.id, "source": h.source, "score": h.score, "preview": prev})
        return NetJSONResponse(out)

    @app.post("/agent_rag")
    async def agent_rag(request: Request):
        t0 = time.perf_counter()
        try:
            body = await bind_body(request)
            prompt = member(body, "prompt")
        except BindError:
            return Response(status_code=400)
        if is_blank(prompt):
            return NetJSONResponse({"error": "Prompt mancante"}, status_code=400)
        with tracer.span("rag.retrieve"):
            if hasattr(index, "search_vectors") and hasattr(index, "embedder"):
                with tracer.span("rag.embed"):
                    if hasattr(index.embedder, "aembed_one"):  # HTTP embedder: no worker thread
                        qv = (await index.embedder.aembed_one(prompt))[None]
                    else:
                        qv = await asyncio.to_thread(index.embedder.embed, [prompt])
                with tracer.span("rag.knn"):
                    # concurrent requests' queries share one kNN launch (one corpus pass)
                    res = await knn_batcher.submit([qv[0]])
                hits = index.hits(res[0])
            else:
                hits = await asyncio.to_thread(index.query, prompt, r.agent_topk)
        if not hits:
            return NetJSONResponse({"result": None, "citations": [], "note": "Nessuna evidenza trovata nei runbook."})
        citations, evidence = select_citations(hits, r.evidence_min_score, r.citation_best_ratio)
        full = json_prompt(RAG_AGENT_SYSTEM, rag_agent_input(prompt, evidence, r.evidence_text_chars))
        with tracer.span("llm.generate", prompt_chars=len(full)):
            raw = await app.state.llm.generate(full)
        tool_json = extract_json_object(raw)
        with tracer.span("agent.dispatch"):
            status, out = await asyncio.to_thread(dispatch_rag_tool, app.state.k8s, tool_json, citations, evidence, cfg)
        M.HTTP_LAT.labels("/agent_rag").observe(time.perf_counter() - t0)
        return respond(status, out)

    @app.get("/debug/spans")
    async def spans(since: float = 0.0):
        """Per-span latency summary (count / mean / p50 / p99) since a time.time() stamp."""
        from ..utils import tracing

        return NetJSONResponse(tracing.summary(since))

    @app.get("/metrics")
    async def metrics():
        return Response(M.render(), media_type="text/plain; version=0.0.4")

    return app
