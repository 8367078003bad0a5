"""Split server (engine core process + HTTP front-ends): the front-end
app over a Unix-socket engine core answers exactly like the in-process server (greedy text,
NDJSON framing, embeddings, grammar-constrained JSON), aborts on client disconnect, and a
front-end spreads requests over several cores by their load."""
import asyncio
import json
import os
import tempfile
import time

import pytest
from fastapi.testclient import TestClient

from llm_kubernetes_minikube_sharp4dev_amd.config import Config
from llm_kubernetes_minikube_sharp4dev_amd.serving.engine_core import EngineCore
from llm_kubernetes_minikube_sharp4dev_amd.serving.model_manager import ModelManager
from llm_kubernetes_minikube_sharp4dev_amd.serving.ollama_server import create_app
from llm_kubernetes_minikube_sharp4dev_amd.serving.remote import CorePool, create_frontend_app

ALIASES = {"llama3.1:8b": "llama-tiny", "nomic-embed-text": "bert-tiny"}


def _cfg():
    cfg = Config()
    cfg.engine.max_model_len = 2048
    cfg.engine.default_max_new_tokens = 8
    return cfg


@pytest.fixture(scope="module")
def split():
    d = tempfile.mkdtemp()
    mgrs, cores = [], []
    for i in range(2):  # two "GPU replicas" (CPU engines here)
        m = ModelManager(_cfg(), device="cpu", aliases=ALIASES)
        mgrs.append(m)
        cores.append(EngineCore(m, os.path.join(d, f"core{i}.sock")))
    local = ModelManager(_cfg(), device="cpu", aliases=ALIASES)
    fe = create_frontend_app([c.path for c in cores], _cfg(), ALIASES, preload=["llama3.1:8b", "nomic-embed-text"])
    with TestClient(fe) as c_fe, TestClient(create_app(local)) as c_local:
        yield c_fe, c_local, fe, cores, mgrs
    for c in cores:
        c.close()
    for m in mgrs + [local]:
        m.shutdown()


def test_generate_matches_in_process_server(split):
    c_fe, c_local, *_ = split
    body = {"model": "llama3.1:8b", "prompt": "ciao", "stream": False, "options": {"num_predict": 6, "temperature": 0}}
    a, b = c_fe.post("/api/generate", json=body).json(), c_local.post("/api/generate", json=body).json()
    assert a["response"] == b["response"] and a["eval_count"] == b["eval_count"] == 6
    assert a["context"] == b["context"] and a["done_reason"] == b["done_reason"]
    with c_fe.stream("POST", "/api/generate", json={**body, "stream": True}) as r:
        lines = [json.loads(l) for l in r.iter_lines() if l.strip()]
    assert all(not l["done"] for l in lines[:-1]) and lines[-1]["done"]
    assert "".join(l["response"] for l in lines) == b["response"]


def test_embeddings_and_json_format_and_chat(split):
    c_fe, c_local, *_ = split
    for payload in ({"model": "nomic-embed-text", "input": "hello"}, {"model": "nomic-embed-text", "prompt": "hello"}):
        va = c_fe.post("/api/embeddings", json=payload).json()["embedding"]
        vb = c_local.post("/api/embeddings", json=payload).json()["embedding"]
        assert len(va) == 128 and max(abs(x - y) for x, y in zip(va, vb)) < 1e-5
    r = c_fe.post("/api/generate", json={"model": "llama3.1:8b", "prompt": "dammi json", "stream": False,
                                         "format": "json", "options": {"num_predict": 12, "temperature": 0}}).json()
    from llm_kubernetes_minikube_sharp4dev_amd.engine.constrained import JSON_START, json_feed_text

    assert json_feed_text(JSON_START, r["response"]) is not None
    body = {"model": "llama3.1:8b", "messages": [{"role": "user", "content": "hi"}], "stream": False,
            "options": {"num_predict": 4, "temperature": 0}}
    assert c_fe.post("/api/chat", json=body).json()["message"] == c_local.post("/api/chat", json=body).json()["message"]
    assert c_fe.post("/api/generate", json={"model": "nope", "prompt": "x"}).status_code == 404
    assert any(t["name"] == "llama3.1:8b" for t in c_fe.get("/api/tags").json()["models"])


def test_requests_spread_over_cores_and_finish(split):
    c_fe, _, fe, cores, mgrs = split
    pool: CorePool = fe.state.manager.pool

    async def many():
        import httpx

        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=fe), base_url="http://t", timeout=120) as c:
            rs = await asyncio.gather(*(c.post("/api/generate", json={
                "model": "llama3.1:8b", "prompt": f"q{i}", "stream": False,
                "options": {"num_predict": 4, "temperature": 0}}) for i in range(16)))
        return [r.json() for r in rs]

    # ASGITransport runs in this loop: reconnect the pool's clients here
    async def run():
        p2 = CorePool([c.path for c in cores])
        await p2.connect()
        fe.state.manager.pool = p2
        for h in fe.state.manager.generators.values():
            h.async_engine.pool = p2
        for h in fe.state.manager.embedders.values():
            h.engine.pool = p2
        out = await many()
        return out, p2

    out, p2 = asyncio.run(run())
    assert all(o["done"] and o["eval_count"] == 4 for o in out)
    assert all(c.outstanding == 0 for c in p2.clients)
    assert all(c.served >= 4 for c in p2.clients), [c.served for c in p2.clients]  # both cores took work
    fe.state.manager.pool = pool
    for h in fe.state.manager.generators.values():
        h.async_engine.pool = pool
    for h in fe.state.manager.embedders.values():
        h.engine.pool = pool


def test_empty_embed_input_and_health(split):
    """an empty /api/embed input must answer (it used to block the front-end's
    event loop on a round trip that loop had to run), and /health must work over remote
    cores (the remote handle had no watchdog: 500)."""
    c_fe, c_local, *_ = split
    for body in ({"model": "nomic-embed-text", "input": []}, {"model": "nomic-embed-text", "input": ""}):
        r = c_fe.post("/api/embed", json=body, timeout=30)
        assert r.status_code == c_local.post("/api/embed", json=body).status_code
    h = c_fe.get("/health")
    assert h.status_code == 200, h.text
    js = h.json()
    assert js["status"] == "ok" and js["generators"]["llama3.1:8b"]["healthy"] is True
    assert js["generators"]["llama3.1:8b"]["stalls"] == 0
    # the front-end still serves after the empty request
    assert len(c_fe.post("/api/embeddings", json={"model": "nomic-embed-text", "input": "x"}).json()["embedding"]) == 128


def test_api_embed_nonempty_matches_local(split):
    """/api/embed over remote cores (it used to call a tokenizer the remote handle lacked)."""
    c_fe, c_local, *_ = split
    body = {"model": "nomic-embed-text", "input": ["alpha beta", "gamma"]}
    a, b = c_fe.post("/api/embed", json=body).json(), c_local.post("/api/embed", json=body).json()
    assert a["prompt_eval_count"] == b["prompt_eval_count"] > 0
    assert len(a["embeddings"]) == 2 and max(abs(x - y) for x, y in zip(a["embeddings"][1], b["embeddings"][1])) < 1e-5
