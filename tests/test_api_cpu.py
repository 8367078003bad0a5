"""HTTP contracts: Minimal_RAG / Minimal_Agent ports (scripted fake LLM + fake
cluster) and the Ollama-compatible server (tiny random-init models on CPU), plus
the reference's clients (Embedder 3-payload fallback, OllamaSharp-style streaming,
kube REST client) talking to them."""
import asyncio
import json
import os

import httpx
import pytest
from fastapi.testclient import TestClient

from llm_kubernetes_minikube_sharp4dev_amd.apps.agent_app import create_agent_app
from llm_kubernetes_minikube_sharp4dev_amd.apps.rag_app import create_rag_app
from llm_kubernetes_minikube_sharp4dev_amd.config import Config
from llm_kubernetes_minikube_sharp4dev_amd.k8s.client import K8sApiError, RestK8sClient
from llm_kubernetes_minikube_sharp4dev_amd.k8s.fake import FakeCluster, make_apiserver_app
from llm_kubernetes_minikube_sharp4dev_amd.rag.embedder import HashEmbedder, OllamaEmbedder
from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagIndex
from llm_kubernetes_minikube_sharp4dev_amd.serving.backends import OllamaHTTPGenerate, ScriptedGenerate
from llm_kubernetes_minikube_sharp4dev_amd.serving.model_manager import ModelManager
from llm_kubernetes_minikube_sharp4dev_amd.serving.ollama_server import create_app

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rag_client(outputs, k8s=None, knowledge=None):
    cfg = Config()
    cfg.rag.knowledge_dir = knowledge or os.path.join(ROOT, "knowledge")
    idx = RagIndex(HashEmbedder(256), backend="exact", device="cpu")
    llm = ScriptedGenerate(outputs)
    app = create_rag_app(cfg, idx, llm, k8s or FakeCluster.default())
    return TestClient(app), llm, idx


def test_rag_health_and_index_built_before_serving():
    c, _, idx = _rag_client("{}")
    assert len(idx) > 0 and idx.chunks[0].id.endswith("#0")
    r = c.get("/health")
    assert r.status_code == 200 and r.json() == {"status": "ok"}


def test_rag_search_contract():
    c, _, _ = _rag_client("{}")
    assert c.post("/rag/search", json={"query": "  "}).json() == {"error": "Query vuota"}
    assert c.post("/rag/search", json={"query": "  "}).status_code == 400
    r = c.post("/rag/search", json={"Query": "scalare repliche deployment", "topK": "50"})
    body = r.json()
    assert r.status_code == 200 and isinstance(body, list) and len(body) <= 10
    assert set(body[0]) == {"id", "source", "score", "preview"}
    assert all(len(h["preview"]) <= 263 for h in body)
    assert len(c.post("/rag/search", json={"query": "scalare", "topK": 0}).json()) == 1
    # low best score branch
    low = c.post("/rag/search", json={"query": "zzzz qqqq"}).json()
    assert isinstance(low, dict) and low["info"].startswith("Best score basso (")
    assert set(low["results"][0]) == {"id", "source", "score"}
    assert "\\u00F9" in c.post("/rag/search", json={"query": "zzzz qqqq"}).text  # .NET escaping of "più"
    assert c.post("/rag/search", content=b"{bad").status_code == 400


def test_rag_search_empty_index(tmp_path):
    c, _, _ = _rag_client("{}", knowledge=str(tmp_path / "none"))
    assert c.post("/rag/search", json={"query": "x"}).json() == {
        "info": "Nessun risultato. L'indice potrebbe essere vuoto.", "results": []}
    r = c.post("/agent_rag", json={"prompt": "x"})
    assert r.json() == {"result": None, "citations": [], "note": "Nessuna evidenza trovata nei runbook."}


def test_agent_rag_flow_and_prompt():
    k8s = FakeCluster.default()
    c, llm, _ = _rag_client('```json\n{"action":"scale_deployment","namespace":"dev","name":"api","replicas":4}\n```',
                            k8s=k8s)
    assert c.post("/agent_rag", json={"prompt": ""}).json() == {"error": "Prompt mancante"}
    r = c.post("/agent_rag", json={"prompt": "scala il deployment api a 4 repliche nel namespace dev scaling"})
    body = r.json()
    assert r.status_code == 200, body
    assert body["result"] == {"namespace": "dev", "name": "api", "replicas_prev": 2, "replicas_now": 4}
    assert body["note"].startswith("scale_deployment eseguito perch")
    p = llm.prompts[-1]
    assert p.startswith("Sei un agente DevOps RAG-only.") and p.endswith("\nRispondi SOLO con JSON valido:")
    user = p.split("\nUtente:\n", 1)[1].rsplit("\nRispondi SOLO", 1)[0]
    payload = json.loads(user)
    assert list(payload) == ["user", "evidence"] and set(payload["evidence"][0]) == {"Id", "Source", "Score", "text"}


def test_agent_rag_problem_on_k8s_error():
    k8s = FakeCluster.default()
    c, _, _ = _rag_client('{"action":"scale_deployment","namespace":"dev","name":"missing","replicas":1}', k8s=k8s)
    r = c.post("/agent_rag", json={"prompt": "scalare deployment repliche scaling"})
    assert r.status_code == 500 and r.headers["content-type"].startswith("application/problem+json")
    assert r.json()["title"] == "Operazione fallita"


def test_agent_app_contract():
    k8s = FakeCluster.default()
    llm = ScriptedGenerate(['{"action":"list_pods","namespace":"default"}', "not json",
                            '{"action":"get_logs","namespace":"dev","pod":"nope"}'])
    c = TestClient(create_agent_app(Config(), llm, k8s))
    assert c.get("/health").json() == {"status": "OK"}
    r = c.post("/agent", json={"prompt": "mostrami i pod"})
    assert r.status_code == 200 and r.json()["ns"] == "default" and len(r.json()["pods"]) == 2
    assert "Utente: mostrami i pod\nRisposta JSON:" in llm.prompts[0]
    r = c.post("/agent", json={"prompt": "x"})
    assert r.status_code == 400 and r.json()["error"] == "JSON Parse error" and r.json()["data"] == "not json"
    r = c.post("/agent", json={"prompt": "x"})
    assert r.status_code == 500  # unhandled k8s error, as in the reference


def test_fault_injection_llm():
    llm = ScriptedGenerate("{}", fault_rate=1.0)
    c = TestClient(create_agent_app(Config(), llm, FakeCluster.default()), raise_server_exceptions=False)
    assert c.post("/agent", json={"prompt": "x"}).status_code == 500


# --------------------------------------------------------------------------- Ollama server
@pytest.fixture(scope="module")
def ollama():
    cfg = Config()
    cfg.engine.max_model_len = 2048
    cfg.engine.default_max_new_tokens = 8
    mgr = ModelManager(cfg, device="cpu", aliases={"llama3.1:8b": "llama-tiny", "nomic-embed-text": "bert-tiny"})
    app = create_app(mgr)
    with TestClient(app) as c:
        yield c, app
    mgr.shutdown()


def test_ollama_generate_stream_and_final_chunk(ollama):
    c, _ = ollama
    with c.stream("POST", "/api/generate", json={"model": "llama3.1:8b", "prompt": "ciao",
                                                 "options": {"num_predict": 5, "temperature": 0}}) as r:
        lines = [json.loads(l) for l in r.iter_lines() if l.strip()]
    assert r.headers["content-type"].startswith("application/x-ndjson")
    assert all(not l["done"] for l in lines[:-1]) and lines[-1]["done"]
    fin = lines[-1]
    for k in ("total_duration", "load_duration", "prompt_eval_count", "prompt_eval_duration", "eval_count",
              "eval_duration", "context", "done_reason"):
        assert k in fin
    assert fin["eval_count"] == 5 and fin["done_reason"] in ("length", "stop")


def test_ollama_generate_nonstream_json_format(ollama):
    c, _ = ollama
    r = c.post("/api/generate", json={"model": "llama3.1:8b", "prompt": "dammi json", "stream": False,
                                      "format": "json", "options": {"num_predict": 12, "temperature": 0}})
    d = r.json()
    assert d["done"] and isinstance(d["response"], str)
    from llm_kubernetes_minikube_sharp4dev_amd.engine.constrained import JSON_START, json_feed_text

    assert json_feed_text(JSON_START, d["response"]) is not None  # valid JSON prefix
    assert c.post("/api/generate", json={"model": "nope", "prompt": "x"}).status_code == 404
    assert c.post("/api/generate", json={"model": "llama3.1:8b"}).json()["done_reason"] == "load"


def test_ollama_embeddings_variants_and_reference_client(ollama):
    c, _ = ollama
    for payload in ({"model": "nomic-embed-text", "input": "hello"},
                    {"model": "nomic-embed-text", "input": ["hello"]},
                    {"model": "nomic-embed-text", "prompt": "hello"}):
        v = c.post("/api/embeddings", json=payload).json()["embedding"]
        assert len(v) == 128
    emb = c.post("/api/embed", json={"model": "nomic-embed-text", "input": ["a", "b c"]}).json()
    assert len(emb["embeddings"]) == 2 and emb["prompt_eval_count"] > 0
    # the reference Embedder client: first payload ({model, input: str}) succeeds -> 1 round trip
    e = OllamaEmbedder(model="nomic-embed-text", client=c)
    assert e.embed(["uno", "due"]).shape == (2, 128) and e.attempts == 2


def test_ollama_admin_and_openai_routes(ollama):
    c, _ = ollama
    tags = c.get("/api/tags").json()["models"]
    assert any(t["name"] == "llama3.1:8b" for t in tags)
    assert c.post("/api/show", json={"model": "llama3.1:8b"}).json()["capabilities"] == ["completion"]
    assert c.get("/api/version").json()["version"]
    assert c.get("/").text == "Ollama is running"
    r = c.post("/v1/chat/completions", json={"model": "llama3.1:8b", "messages": [{"role": "user", "content": "hi"}],
                                             "max_tokens": 3, "temperature": 0}).json()
    assert r["object"] == "chat.completion" and r["usage"]["completion_tokens"] == 3
    assert len(c.post("/v1/embeddings", json={"model": "nomic-embed-text", "input": "x"}).json()["data"]) == 1
    assert b"lk_requests_total" in c.get("/metrics").content


def test_ollamasharp_style_streaming_client(ollama):
    _, app = ollama

    async def go():
        client = httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://test")
        g = OllamaHTTPGenerate(model="llama3.1:8b", client=client, options={"num_predict": 4, "temperature": 0})
        return await g.generate("Sei un agente\nUtente: ciao\nRisposta JSON:")

    out = asyncio.run(go())
    assert isinstance(out, str)


def test_rest_k8s_client_against_fake_apiserver():
    cluster = FakeCluster.default()
    client = RestK8sClient("http://fake")
    client.http = TestClient(make_apiserver_app(cluster), base_url="http://fake")
    assert len(client.list_namespaced_pod("default")["items"]) == 2
    pod = client.list_namespaced_pod("dev")["items"][0]["metadata"]["name"]
    assert len(client.read_namespaced_pod_log(pod, "dev", tail_lines=200).splitlines()) == 200
    sc = client.read_namespaced_deployment_scale("echoserver", "default")
    sc["spec"]["replicas"] = 5
    assert client.replace_namespaced_deployment_scale("echoserver", "default", sc)["spec"]["replicas"] == 5
    assert len(client.list_pod_for_all_namespaces()["items"]) == cluster.list_pod_for_all_namespaces()["items"].__len__()
    assert client.list_node()["items"][0]["metadata"]["name"] == "minikube"
    with pytest.raises(K8sApiError) as e:
        client.read_namespaced_deployment_scale("nope", "default")
    assert "NotFound" in str(e.value)


def test_ollama_concurrent_clients_share_one_engine(ollama):
    """16 simultaneous streaming clients on one continuous-batching engine (the engine
    loop is the single writer of scheduler state; requests interleave per step)."""
    _, app = ollama

    async def one(client, i):
        async with client.stream("POST", "/api/generate", json={
                "model": "llama3.1:8b", "prompt": f"richiesta {i} " * (1 + i % 5),
                "options": {"num_predict": 4 + i % 3, "temperature": 0}}) as r:
            lines = [json.loads(l) async for l in r.aiter_lines() if l.strip()]
        return i, lines

    async def main():
        transport = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=transport, base_url="http://t") as client:
            return await asyncio.gather(*(one(client, i) for i in range(16)))

    res = asyncio.run(main())
    assert len(res) == 16
    for i, lines in res:
        assert lines[-1]["done"] and lines[-1]["eval_count"] == 4 + i % 3
    r = TestClient(app).get("/health")
    assert r.status_code == 200 and r.json()["status"] == "ok"


def test_request_timeout_aborts_and_watchdog_flags_stall():
    import time as _t

    import torch

    from llm_kubernetes_minikube_sharp4dev_amd.engine.llm_engine import AsyncLLMEngine, LLMEngine
    from llm_kubernetes_minikube_sharp4dev_amd.engine.sampling import SamplingParams
    from llm_kubernetes_minikube_sharp4dev_amd.models import build_decoder
    from llm_kubernetes_minikube_sharp4dev_amd.utils.watchdog import StepWatchdog

    stalls = []
    wd = StepWatchdog("t", stall_s=0.2, on_stall=stalls.append, poll_s=0.02)
    with wd.busy():
        _t.sleep(0.5)
    assert stalls and not wd.healthy
    wd.beat()
    assert wd.healthy
    wd.stop()

    m = build_decoder("llama-tiny", dtype=torch.float32)
    eng = LLMEngine(m, None, max_model_len=512, max_num_seqs=4, num_blocks=64, use_graphs=False, eos_ids=set())
    aeng = AsyncLLMEngine(eng, request_timeout_s=1e-4)

    async def go():
        with pytest.raises(asyncio.TimeoutError):
            await aeng.generate(list(range(5, 60)), SamplingParams.greedy(10_000))

    asyncio.run(go())
    for _ in range(100):
        if not eng.has_work():
            break
        _t.sleep(0.01)
    assert not eng.has_work()  # the timed-out request was aborted
    aeng.shutdown()
