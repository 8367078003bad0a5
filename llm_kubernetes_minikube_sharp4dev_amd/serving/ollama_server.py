"""Ollama-compatible HTTP server (default ``:11434``) backed by the MI355X engines.

This is the seam both .NET services hard-code (``Minimal_RAG/Program.cs:22``,
``Minimal_Agent_RAG/Program.cs:11``, ``Helpers/Embedder.cs:9``), so the unchanged
C# solution drives MI355X by pointing at this process.

Routes (Ollama REST API):
  POST /api/generate   streamed NDJSON (default) or one JSON; chat template applied
                       unless ``raw``; ``system``, ``options``, ``format`` ("json" or a
                       JSON schema -> grammar-constrained decoding), final chunk with
                       done_reason / context / *_duration / *_count fields
  POST /api/chat       messages -> message chunks
  POST /api/embeddings legacy single embedding; accepts ``prompt`` AND ``input`` (str or
                       [str]) so the first payload of ``Embedder.cs:14`` succeeds
  POST /api/embed      batched ``input`` -> ``embeddings``
  GET  /api/tags, POST /api/show, GET /api/ps, GET /api/version, GET|HEAD /
  POST /api/pull (presets are local: reports success), DELETE /api/delete
  OpenAI compatibility: POST /v1/chat/completions, /v1/completions, /v1/embeddings,
                        GET /v1/models
  GET  /metrics        Prometheus
"""
from __future__ import annotations

from fastapi import Request  # module level: FastAPI resolves string annotations here

import asyncio
import json
import os
import time
import uuid
from datetime import datetime, timezone
from typing import Any, Optional

from ..engine.sampling import SamplingParams
from ..utils import tracing
from ..models.tokenizer import IncrementalDetokenizer
from ..utils import metrics as M
from ..utils.logging import get_logger
from .model_manager import ModelManager

log = get_logger("serving.ollama")
OLLAMA_VERSION = "0.6.8"


_now_cache = [0.0, ""]


def _now() -> str:
    """RFC 3339 timestamp of the chunk (cached for 1 ms: hundreds of streams emit a chunk per
    engine step)."""
    t = time.time()
    if t - _now_cache[0] >= 1e-3:
        _now_cache[0] = t
        _now_cache[1] = datetime.fromtimestamp(t, timezone.utc).isoformat().replace("+00:00", "Z")
    return _now_cache[1]


def _chat_to_prompt(messages: list) -> tuple[Optional[str], str]:
    sys_parts = [m.get("content", "") for m in messages if m.get("role") == "system"]
    turns = [m for m in messages if m.get("role") != "system"]
    prompt = "\n".join(f"{m.get('role', 'user')}: {m.get('content', '')}" if len(turns) > 1 else m.get("content", "")
                       for m in turns)
    return ("\n".join(sys_parts) if sys_parts else None), prompt


def _tp_of(h) -> int:
    """Tensor-parallel ranks behind a generator handle (local engine or remote core)."""
    if hasattr(h, "tp"):
        return int(h.tp)
    ctrl = getattr(getattr(h, "engine", None), "tp_ctrl", None)
    return int(ctrl.tp.size) if ctrl is not None else 1


def create_app(manager: Optional[ModelManager] = None, cfg=None):
    from .batcher import MicroBatcher

    from fastapi import FastAPI, Request
    from fastapi.responses import JSONResponse, PlainTextResponse, Response, StreamingResponse

    mgr = manager or ModelManager(cfg)
    app = FastAPI(title="Ollama-compatible MI355X server")
    app.state.manager = mgr

    def err(status: int, msg: str):
        return JSONResponse({"error": msg}, status_code=status)

    # loaded models are looked up on the event loop (a dict read); only a first request that
    # has to LOAD a model hops to a worker thread.  (A thread hop per request queued 128
    # concurrent lookups in the default executor in front of the embedding batches.)
    async def _gen_handle(model: str):
        h = mgr.generators.get(model)
        return h if h is not None else await asyncio.to_thread(mgr.generator, model)

    async def _emb_handle(model: str):
        h = mgr.embedders.get(model)
        return h if h is not None else await asyncio.to_thread(mgr.embedder, model)

    async def body_of(request: Request) -> dict:
        raw = await request.body()
        if not raw:
            return {}
        try:
            b = json.loads(raw)
        except ValueError:
            raise ValueError("invalid JSON body")
        if not isinstance(b, dict):
            raise ValueError("request body must be a JSON object")
        return b

    def params_for(b: dict, h) -> SamplingParams:
        sp = SamplingParams.from_ollama(b.get("options"), mgr.cfg.engine, mgr.cfg.engine.default_max_new_tokens)
        fmt = b.get("format")
        if fmt:
            from ..engine.constrained import json_logits_processor

            sp.format = fmt  # a remote engine core rebuilds the processor from the spec
            sp.logits_processor = json_logits_processor(h.tokenizer, fmt if isinstance(fmt, dict) else None)
        return sp

    def prompt_ids(h, prompt: str, system: Optional[str], raw: bool) -> list:
        tok = h.tokenizer
        if raw or h.chat_style == "raw":
            return tok.encode(prompt, add_bos=True)
        return tok.chat_prompt(prompt, system=system, style=h.chat_style)

    async def run_stream(h, ids, sp, mk_chunk, mk_final, stream: bool):
        """Drive the async engine; stream NDJSON chunks or accumulate one JSON."""
        t0 = time.perf_counter_ns()
        detok = IncrementalDetokenizer(h.tokenizer)
        stop_strs = [s for s in sp.stop if s]

        async def gen():
            text = ""
            seq = None
            first_ns = None
            emitted = 0
            try:
                async for tid, fin, s in h.async_engine.stream(ids, sp):
                    seq = s
                    if tid < 0 and getattr(s, "error", None):  # engine failure / watchdog stall
                        yield json.dumps({"error": f"generation failed: {s.error}"}) + ("\n" if stream else "")
                        return
                    if first_ns is None:
                        first_ns = time.perf_counter_ns()
                    piece = detok.push(tid) if tid >= 0 and not (fin and tid in h.engine.eos_ids) else ""
                    text += piece
                    if stop_strs:
                        cut = min((text.find(st) for st in stop_strs if st in text), default=-1)
                        if cut >= 0:
                            piece = piece[: max(0, len(piece) - (len(text) - cut))]
                            text = text[:cut]
                    if piece and stream:
                        yield json.dumps(mk_chunk(piece), ensure_ascii=False) + "\n"
                    emitted += 1
            except asyncio.TimeoutError:
                yield json.dumps({"error": "request timed out"}) + ("\n" if stream else "")
                return
            end = time.perf_counter_ns()
            first_ns = first_ns or end
            stats = {
                "total_duration": end - t0,
                "load_duration": 0,
                "prompt_eval_count": len(ids) - (seq.num_cached_prefix if seq else 0),
                "prompt_eval_duration": first_ns - t0,
                "eval_count": len(seq.output_ids) if seq else 0,
                "eval_duration": end - first_ns,
            }
            reason = (seq.finish_reason if seq else "stop") or "stop"
            if reason not in ("stop", "length"):
                reason = "stop"
            if seq and seq.first_token_at:
                M.TTFT.observe(seq.first_token_at - seq.arrival)
            if seq is not None:  # per-request engine accounting (/debug/spans counters)
                from ..utils import tracing

                cached = seq.num_cached_prefix
                q = getattr(seq, "steps_queued", None)
                if q is None and getattr(seq, "step_first", None) is not None:
                    q = seq.step_first - seq.step_arrival
                for name, v in (("req_prompt_tokens", len(ids)), ("req_cached_prefix_tokens", cached),
                                ("req_uncached_prompt_tokens", len(ids) - cached),
                                ("req_output_tokens", len(seq.output_ids)),
                                ("req_preemptions", getattr(seq, "num_preemptions", 0)),
                                ("req_steps_queued", q), ("req_steps_run", getattr(seq, "steps_run", None))):
                    if v is not None:
                        tracing.count("server", name, v)
            final = mk_final(text, reason, stats, ids + (seq.output_ids if seq else []))
            yield json.dumps(final, ensure_ascii=False) + ("\n" if stream else "")

        if stream:
            return StreamingResponse(gen(), media_type="application/x-ndjson")
        out = ""
        async for part in gen():
            out = part
        status = 500 if out.startswith('{"error"') else 200
        return Response(out, status_code=status, media_type="application/json; charset=utf-8")

    # ------------------------------------------------------------------ generate
    @app.post("/api/generate")
    async def generate(request: Request):
        t_req = time.perf_counter()
        try:
            b = await body_of(request)
        except ValueError as e:
            return err(400, str(e))
        model = b.get("model")
        if not model:
            return err(400, "model is required")
        try:
            h = await _gen_handle(model)
        except KeyError as e:
            return err(404, str(e).strip("'\""))
        prompt = b.get("prompt") or ""
        if not prompt and not b.get("system"):
            return JSONResponse({"model": model, "created_at": _now(), "response": "", "done": True,
                                 "done_reason": "load"})
        ids = prompt_ids(h, prompt, b.get("system"), bool(b.get("raw")))
        if len(ids) >= h.engine.max_model_len:
            ids = ids[-(h.engine.max_model_len - 1):]  # Ollama truncates to num_ctx
        sp = params_for(b, h)
        stream = b.get("stream", True) is not False

        def chunk(piece):
            return {"model": model, "created_at": _now(), "response": piece, "done": False}

        def final(text, reason, stats, ctx):
            d = {"model": model, "created_at": _now(), "response": "" if stream else text, "done": True,
                 "done_reason": reason, "context": ctx if not b.get("raw") else []}
            d.update(stats)
            return d

        from ..utils import tracing

        tracing.record("server", "generate_admit", time.perf_counter() - t_req)
        r = await run_stream(h, ids, sp, chunk, final, stream)
        M.HTTP_LAT.labels("/api/generate").observe(time.perf_counter() - t_req)
        return r

    @app.post("/api/chat")
    async def chat(request: Request):
        try:
            b = await body_of(request)
        except ValueError as e:
            return err(400, str(e))
        model = b.get("model")
        if not model:
            return err(400, "model is required")
        try:
            h = await _gen_handle(model)
        except KeyError as e:
            return err(404, str(e).strip("'\""))
        msgs = b.get("messages") or []
        if not msgs:
            return JSONResponse({"model": model, "created_at": _now(), "message": {"role": "assistant", "content": ""},
                                 "done": True, "done_reason": "load"})
        system, prompt = _chat_to_prompt(msgs)
        ids = prompt_ids(h, prompt, system, False)
        sp = params_for(b, h)
        stream = b.get("stream", True) is not False

        def chunk(piece):
            return {"model": model, "created_at": _now(), "message": {"role": "assistant", "content": piece},
                    "done": False}

        def final(text, reason, stats, ctx):
            d = {"model": model, "created_at": _now(),
                 "message": {"role": "assistant", "content": "" if stream else text}, "done": True,
                 "done_reason": reason}
            d.update(stats)
            return d

        return await run_stream(h, ids, sp, chunk, final, stream)

    # ------------------------------------------------------------------ embeddings
    batchers: dict = {}

    async def _embed(model: str, texts: list[str]):
        """Concurrent requests for one model share packed encoder passes (MicroBatcher)."""
        t0 = time.perf_counter()
        h = await _emb_handle(model)
        b = batchers.get(h.name)
        if b is None:
            from ..engine.embed_engine import EMBED_STREAMS

            eng = h.engine

            def run(texts, eng=eng):  # the batch's own time, apart from its queueing
                t = time.perf_counter()
                out = eng.embed_cpu(texts)
                tracing.record("server", "embed_batch", time.perf_counter() - t, n=len(texts))
                return out

            b = batchers[h.name] = MicroBatcher(run, max_inflight=EMBED_STREAMS,
                                                max_wait_s=float(os.environ.get("LK_EMBED_WAIT_MS", "2")) / 1e3)
        vec = await b.submit(texts) if texts else h.engine.embed_cpu(texts)
        tracing.record("server", "embed_request", time.perf_counter() - t0)
        return h, vec.tolist()

    @app.post("/api/embeddings")
    async def embeddings(request: Request):
        try:
            b = await body_of(request)
        except ValueError as e:
            return err(400, str(e))
        model = b.get("model")
        text = b.get("prompt")
        if text is None:
            inp = b.get("input")
            text = inp[0] if isinstance(inp, list) and inp else inp
        if not model:
            return err(400, "model is required")
        if text is None:
            return JSONResponse({"embedding": []})
        if not isinstance(text, str):
            return err(400, "prompt must be a string")
        try:
            _, v = await _embed(model, [text])
        except KeyError as e:
            return err(404, str(e).strip("'\""))
        return JSONResponse({"embedding": v[0]})

    @app.post("/api/embed")
    async def embed(request: Request):
        t0 = time.perf_counter_ns()
        try:
            b = await body_of(request)
        except ValueError as e:
            return err(400, str(e))
        model, inp = b.get("model"), b.get("input")
        if not model:
            return err(400, "model is required")
        texts = [inp] if isinstance(inp, str) else list(inp or [])
        if not all(isinstance(t, str) for t in texts):
            return err(400, "input must be a string or a list of strings")
        try:
            h, v = await _embed(model, texts)
        except KeyError as e:
            return err(404, str(e).strip("'\""))
        n_tok = sum(len(x) for x in h.engine.tokenize(texts)) if texts else 0
        return JSONResponse({"model": model, "embeddings": v, "total_duration": time.perf_counter_ns() - t0,
                             "load_duration": 0, "prompt_eval_count": n_tok})

    # ------------------------------------------------------------------ model admin
    def _tag(name, kind, preset):
        d = mgr.details(name)
        return {"name": name if ":" in name else name + ":latest", "model": name if ":" in name else name + ":latest",
                "modified_at": _now(), "size": int(d["params"] * 2),
                "digest": uuid.uuid5(uuid.NAMESPACE_URL, f"lk/{preset}").hex * 2,
                "details": {k: d[k] for k in ("format", "family", "families", "parameter_size", "quantization_level")}}

    @app.get("/api/tags")
    async def tags():
        return {"models": [_tag(n, k, p) for n, k, p in mgr.known_models()]}

    @app.post("/api/show")
    async def show(request: Request):
        b = await body_of(request)
        name = b.get("model") or b.get("name")
        try:
            d = mgr.details(name)
        except (KeyError, TypeError):
            return err(404, f"model '{name}' not found")
        caps = ["completion"] if d["kind"] == "generate" else ["embedding"]
        return {"modelfile": f"FROM {d['preset']}\n", "parameters": "", "template": "{{ .Prompt }}",
                "details": {k: d[k] for k in ("format", "family", "families", "parameter_size", "quantization_level")},
                "model_info": {"general.architecture": d["family"], "general.parameter_count": d["params"]},
                "capabilities": caps}

    @app.get("/debug/spans")
    async def spans(since: float = 0.0):
        from ..utils import tracing

        out = tracing.summary(since)
        pool = getattr(mgr, "pool", None)
        if pool is not None:  # split server: the engine cores' spans and request counters too
            for c in pool.clients:
                try:
                    core = (await asyncio.wait_for(c.request("spans", since), 10.0))[2]
                except Exception:  # noqa: BLE001 - a core that does not answer is left out
                    continue
                for k, v in core.items():
                    if k in out and "sum" in v and "sum" in out[k]:
                        n = out[k]["n"] + v["n"]
                        tot = out[k]["sum"] + v["sum"]
                        out[k] = {"n": n, "mean": tot / n, "sum": tot}
                    else:
                        out.setdefault(k, v)
        return JSONResponse(out)

    @app.get("/health")
    async def health():
        """Engine health (watchdog): 503 while a loaded generator's step loop is stalled."""
        eng = {n: {"healthy": h.async_engine.healthy, "steps": h.async_engine.watchdog.steps,
                   "stalls": h.async_engine.watchdog.stalls, "tp": _tp_of(h)} for n, h in list(mgr.generators.items())}
        ok = all(v["healthy"] for v in eng.values())
        return JSONResponse({"status": "ok" if ok else "degraded", "generators": eng}, status_code=200 if ok else 503)

    @app.get("/api/ps")
    async def ps():
        out = []
        for n, h in list(mgr.generators.items()) + list(mgr.embedders.items()):
            out.append({"name": n, "model": n, "size": 0, "digest": "", "details": {}, "expires_at": "0001-01-01T00:00:00Z",
                        "size_vram": 0})
        return {"models": out}

    @app.post("/api/pull")
    async def pull(request: Request):
        b = await body_of(request)
        name = b.get("model") or b.get("name")
        try:
            mgr.resolve(name)
        except (KeyError, TypeError):
            return err(404, "pull model manifest: file does not exist")
        return {"status": "success"}

    @app.delete("/api/delete")
    async def delete(request: Request):
        b = await body_of(request)
        name = b.get("model") or b.get("name")
        mgr.generators.pop(name, None)
        mgr.embedders.pop(name, None)
        return Response(status_code=200)

    @app.get("/api/version")
    async def version():
        return {"version": OLLAMA_VERSION}

    @app.get("/")
    async def root():
        return PlainTextResponse("Ollama is running")

    @app.head("/")
    async def root_head():
        return Response(status_code=200)

    @app.get("/metrics")
    async def metrics():
        return Response(M.render(), media_type="text/plain; version=0.0.4")

    # ------------------------------------------------------------------ OpenAI compatibility
    @app.post("/v1/chat/completions")
    async def oa_chat(request: Request):
        b = await body_of(request)
        model = b.get("model")
        try:
            h = await _gen_handle(model)
        except KeyError as e:
            return JSONResponse({"error": {"message": str(e), "type": "invalid_request_error"}}, status_code=404)
        system, prompt = _chat_to_prompt(b.get("messages") or [])
        ids = prompt_ids(h, prompt, system, False)
        opts = {"temperature": b.get("temperature", 1.0), "top_p": b.get("top_p", 1.0), "seed": b.get("seed"),
                "stop": b.get("stop"), "num_predict": b.get("max_tokens") or -1}
        sp = SamplingParams.from_ollama({k: v for k, v in opts.items() if v is not None}, mgr.cfg.engine,
                                        mgr.cfg.engine.default_max_new_tokens)
        seq = await h.async_engine.generate(ids, sp)
        text = h.tokenizer.decode(seq.output_ids)
        cid = "chatcmpl-" + uuid.uuid4().hex[:12]
        return {"id": cid, "object": "chat.completion", "created": int(time.time()), "model": model,
                "choices": [{"index": 0, "message": {"role": "assistant", "content": text},
                             "finish_reason": seq.finish_reason}],
                "usage": {"prompt_tokens": len(ids), "completion_tokens": len(seq.output_ids),
                          "total_tokens": len(ids) + len(seq.output_ids)}}

    @app.post("/v1/completions")
    async def oa_comp(request: Request):
        b = await body_of(request)
        model = b.get("model")
        try:
            h = await _gen_handle(model)
        except KeyError as e:
            return JSONResponse({"error": {"message": str(e)}}, status_code=404)
        ids = h.tokenizer.encode(b.get("prompt") or "", add_bos=True)
        sp = SamplingParams.from_ollama({"temperature": b.get("temperature", 1.0),
                                         "num_predict": b.get("max_tokens") or 16}, mgr.cfg.engine)
        seq = await h.async_engine.generate(ids, sp)
        return {"id": "cmpl-" + uuid.uuid4().hex[:12], "object": "text_completion", "created": int(time.time()),
                "model": model, "choices": [{"index": 0, "text": h.tokenizer.decode(seq.output_ids),
                                             "finish_reason": seq.finish_reason}]}

    @app.post("/v1/embeddings")
    async def oa_emb(request: Request):
        b = await body_of(request)
        inp = b.get("input")
        texts = [inp] if isinstance(inp, str) else list(inp or [])
        try:
            _, v = await _embed(b.get("model"), texts)
        except KeyError as e:
            return JSONResponse({"error": {"message": str(e)}}, status_code=404)
        return {"object": "list", "data": [{"object": "embedding", "index": i, "embedding": e} for i, e in enumerate(v)],
                "model": b.get("model")}

    @app.get("/v1/models")
    async def oa_models():
        return {"object": "list", "data": [{"id": n, "object": "model", "owned_by": "library"}
                                           for n, _, _ in mgr.known_models()]}

    @app.on_event("shutdown")
    def _shutdown():
        mgr.shutdown()

    return app
