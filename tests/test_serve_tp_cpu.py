"""Tensor-parallel serving on the CPU (gloo, world 2): ``serve --tp 2`` (split server: the TP
leader is the engine core the front-end talks to, one follower process) answers /api/generate
with exactly the tokens of the single-process server on the same checkpoint; ``all --tp 2``
shards the RAG corpus over the group and its /rag/search and /agent_rag answers equal those of
the one-process app (single scan, TP=1 generator); ``rag-app --tp 2`` (kNN-only followers)
returns the single-scan hits.  The processes are real CLI launches (fresh process per rank)."""
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile
import time

import pytest
import torch

transformers = pytest.importorskip("transformers")
httpx = pytest.importorskip("httpx")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MOD = "llm_kubernetes_minikube_sharp4dev_amd"
ALIASES = ["llama3.1:8b=llama-tiny", "nomic-embed-text=bert-tiny"]
PROMPTS = ["ciao, come stai?", "kubectl get pods -n demo", "scale the echoserver deployment"]
DOCS = {
    "echoserver.md": "# Echoserver\n\nThe echoserver deployment in namespace demo answers HTTP on port 8080.\n\n"
                     "## Scaling\n\nScale it with kubectl scale deployment echoserver --replicas=3.\n",
    "pods.md": "# Pods\n\nPods in CrashLoopBackOff: read the logs of the previous container first.\n\n"
               "## Logs\n\nkubectl logs <pod> -n demo --previous shows the last crash.\n",
    "dns.md": "# DNS\n\nCoreDNS resolves services as <svc>.<ns>.svc.cluster.local.\n",
}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def ckpt():
    """A llama-tiny-shaped HF checkpoint (safetensors): TP ranks slice the same weights."""
    d = tempfile.mkdtemp()
    cfg = transformers.LlamaConfig(vocab_size=32768, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                   num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=4096,
                                   rope_theta=10000.0, rms_norm_eps=1e-5, tie_word_embeddings=False)
    torch.manual_seed(5)
    m = transformers.LlamaForCausalLM(cfg).eval()
    with torch.no_grad():  # non-unit norms, as a real checkpoint has
        for n, p in m.named_parameters():
            if n.endswith("norm.weight"):
                p.uniform_(0.5, 1.5)
    m.save_pretrained(d, safe_serialization=True)
    return d


def _config(tmp, **server):
    c = {"engine": {"max_model_len": 1024, "default_max_new_tokens": 8, "max_num_seqs": 16, "dtype": "float32"},
         "server": server}
    path = os.path.join(tmp, "cfg.json")
    with open(path, "w") as f:
        json.dump(c, f)
    return path


def _model_flags(ckpt, cfg_path):
    return sum([["--alias", a] for a in ALIASES], []) + ["--checkpoint", f"llama-tiny={ckpt}", "--config", cfg_path]


def _launch(argv, tmp):
    env = dict(os.environ, LK_CORE_DIR=tmp, PYTHONPATH=ROOT, OMP_NUM_THREADS="2", LK_TP_CTRL_TIMEOUT_S="120")
    log = open(os.path.join(tmp, f"{argv[0]}.log"), "w")
    return subprocess.Popen([sys.executable, "-m", MOD] + argv, env=env, cwd=ROOT, stdout=log, stderr=subprocess.STDOUT,
                            start_new_session=True), log


def _wait_ready(proc, url, body, tmp, name, timeout=300):
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise AssertionError(f"{name} exited rc={proc.returncode}:\n" + open(os.path.join(tmp, f"{name}.log")).read()[-4000:])
        try:
            r = httpx.post(url, json=body, timeout=60) if body is not None else httpx.get(url, timeout=10)
            if r.status_code == 200:
                return r
        except httpx.HTTPError:
            pass
        time.sleep(1.0)
    raise AssertionError(f"{name} not ready after {timeout}s:\n" + open(os.path.join(tmp, f"{name}.log")).read()[-4000:])


def _stop(proc, log):
    """SIGTERM the launcher and wait: its whole session (leader, followers, front-ends) must end."""
    try:
        proc.send_signal(signal.SIGTERM)
        proc.wait(timeout=90)
    finally:
        if proc.poll() is None:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(timeout=30)
        log.close()
    t0 = time.time()
    while time.time() - t0 < 60:  # every rank of the group left with it
        try:
            os.killpg(proc.pid, 0)
        except ProcessLookupError:
            return
        time.sleep(0.5)
    os.killpg(proc.pid, signal.SIGKILL)
    raise AssertionError("processes of the TP group outlived their launcher")


def _gen_body(prompt):
    return {"model": "llama3.1:8b", "prompt": prompt, "stream": False, "options": {"num_predict": 8, "temperature": 0}}


def _local_manager(ckpt, cfg_path):
    from llm_kubernetes_minikube_sharp4dev_amd.config import load_config
    from llm_kubernetes_minikube_sharp4dev_amd.serving.model_manager import ModelManager

    cfg = load_config(cfg_path)
    return cfg, ModelManager(cfg, device="cpu", aliases=dict(a.split("=") for a in ALIASES),
                             checkpoints={"llama-tiny": ckpt})


def test_serve_tp2_generate_matches_tp1(ckpt):
    from fastapi.testclient import TestClient

    from llm_kubernetes_minikube_sharp4dev_amd.serving.ollama_server import create_app

    with tempfile.TemporaryDirectory() as tmp:
        cfg_path = _config(tmp)
        port = _free_port()
        proc, log = _launch(["serve", "--tp", "2", "--device", "cpu", "--frontends", "1", "--port", str(port),
                             "--preload", "llama3.1:8b"] + _model_flags(ckpt, cfg_path), tmp)
        try:
            url = f"http://127.0.0.1:{port}/api/generate"
            _wait_ready(proc, url, _gen_body("warm up"), tmp, "serve")
            got = [httpx.post(url, json=_gen_body(p), timeout=120).json() for p in PROMPTS]
            health = httpx.get(f"http://127.0.0.1:{port}/health", timeout=30).json()
        finally:
            _stop(proc, log)
        _, mgr = _local_manager(ckpt, cfg_path)
    try:
        with TestClient(create_app(mgr)) as c:
            ref = [c.post("/api/generate", json=_gen_body(p)).json() for p in PROMPTS]
    finally:
        mgr.shutdown()
    assert health["generators"]["llama3.1:8b"]["tp"] == 2, health  # the front-end routed to a TP=2 core
    for g, r in zip(got, ref):
        assert g["eval_count"] == r["eval_count"] == 8
        assert g["context"] == r["context"], (g["response"], r["response"])
        assert g["response"] == r["response"]


def _rag_reference(ckpt, cfg_path, kdir):
    """The one-process RAG app: TP=1 generator, single-scan index of the same folder."""
    from fastapi.testclient import TestClient

    from llm_kubernetes_minikube_sharp4dev_amd.__main__ import _backends
    from llm_kubernetes_minikube_sharp4dev_amd.apps.rag_app import create_rag_app
    from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagIndex

    cfg, mgr = _local_manager(ckpt, cfg_path)
    cfg.rag.knowledge_dir = kdir

    class _A:
        pass

    emb, llm, k8s = _backends(_A(), cfg, mgr)
    idx = RagIndex(emb, backend="exact")
    app = create_rag_app(cfg, idx, llm, k8s)
    return mgr, TestClient(app)


def _knowledge(tmp):
    kdir = os.path.join(tmp, "knowledge")
    os.makedirs(kdir)
    for n, t in DOCS.items():
        with open(os.path.join(kdir, n), "w") as f:
            f.write(t)
    return kdir


def _same_hits(a, b):
    assert [h["id"] for h in a] == [h["id"] for h in b]
    assert all(abs(x["score"] - y["score"]) < 1e-4 for x, y in zip(a, b))


def test_all_tp2_sharded_index_matches_single_scan(ckpt):
    queries = ["how do I scale the echoserver", "pod crash logs", "service dns name"]
    with tempfile.TemporaryDirectory() as tmp:
        kdir = _knowledge(tmp)
        ports = dict(ollama_port=_free_port(), rag_port=_free_port(), agent_port=_free_port())
        cfg_path = _config(tmp, **ports)
        proc, log = _launch(["all", "--tp", "2", "--device", "cpu", "--knowledge", kdir]
                            + _model_flags(ckpt, cfg_path), tmp)
        try:
            base = f"http://127.0.0.1:{ports['rag_port']}"
            _wait_ready(proc, base + "/health", None, tmp, "all")
            got_s = [httpx.post(base + "/rag/search", json={"query": q, "topK": 3}, timeout=60).json() for q in queries]
            got_a = [httpx.post(base + "/agent_rag", json={"prompt": q}, timeout=120) for q in queries]
            gen = httpx.post(f"http://127.0.0.1:{ports['ollama_port']}/api/generate", json=_gen_body("ciao"),
                             timeout=120).json()
            health = httpx.get(f"http://127.0.0.1:{ports['ollama_port']}/health", timeout=30).json()
        finally:
            _stop(proc, log)
        assert "chunks sharded over tp2" in open(os.path.join(tmp, "all.log")).read()
        mgr, c = _rag_reference(ckpt, cfg_path, kdir)
        try:
            with c:
                ref_s = [c.post("/rag/search", json={"query": q, "topK": 3}).json() for q in queries]
                ref_a = [c.post("/agent_rag", json={"prompt": q}) for q in queries]
            from fastapi.testclient import TestClient

            from llm_kubernetes_minikube_sharp4dev_amd.serving.ollama_server import create_app

            with TestClient(create_app(mgr)) as co:
                ref_gen = co.post("/api/generate", json=_gen_body("ciao")).json()
        finally:
            mgr.shutdown()
    for g, r in zip(got_s, ref_s):
        g, r = (g if isinstance(g, list) else g["results"]), (r if isinstance(r, list) else r["results"])
        assert g, "the sharded index returned no hits"
        _same_hits(g, r)
    for g, r in zip(got_a, ref_a):
        assert g.status_code == r.status_code
        gj, rj = g.json(), r.json()
        for j in (gj, rj):
            j.pop("raw", None) if isinstance(j, dict) else None
        assert gj == rj
    assert gen["context"] == ref_gen["context"]
    assert health["generators"]["llama3.1:8b"]["tp"] == 2, health


def test_rag_app_tp2_knn_only_group_matches_single_scan():
    """``rag-app --tp 2 --synthetic-docs N``: the bulk-built corpus scattered over a kNN-only
    follower; /rag/search hits == the one-process app's single scan of the same corpus."""
    import numpy as np

    from llm_kubernetes_minikube_sharp4dev_amd.__main__ import _synthetic_index

    queries = ["deployment scaling runbook", "ingress certificate expired", "node pressure eviction"]
    with tempfile.TemporaryDirectory() as tmp:
        cfg_path = _config(tmp)
        emb_port, rag_port = _free_port(), _free_port()
        # the query embedder: an in-process Ollama server on its own port (HTTP, as the reference)
        srv, srv_log = _launch(["serve", "--device", "cpu", "--frontends", "0", "--port", str(emb_port),
                                "--preload", "nomic-embed-text", "--alias", ALIASES[1], "--config", cfg_path], tmp)
        try:
            _wait_ready(srv, f"http://127.0.0.1:{emb_port}/api/tags", None, tmp, "serve")
            proc, log = _launch(["rag-app", "--tp", "2", "--device", "cpu", "--port", str(rag_port), "--synthetic-docs",
                                 "60", "--bulk-embed", "bert-tiny", "--ollama-url", f"http://127.0.0.1:{emb_port}",
                                 "--config", cfg_path], tmp)
            try:
                base = f"http://127.0.0.1:{rag_port}"
                _wait_ready(proc, base + "/health", None, tmp, "rag-app", timeout=400)
                got = [httpx.post(base + "/rag/search", json={"query": q, "topK": 5}, timeout=60).json() for q in queries]
            finally:
                _stop(proc, log)
            assert "sharded over tp2" in open(os.path.join(tmp, "rag-app.log")).read()

            class _A:
                synthetic_docs, bulk_embed, device = 60, "bert-tiny", "cpu"

            from llm_kubernetes_minikube_sharp4dev_amd.rag.embedder import OllamaEmbedder

            idx = _synthetic_index(_A(), OllamaEmbedder(f"http://127.0.0.1:{emb_port}", "nomic-embed-text"))
            ref = [idx.query(q, 5) for q in queries]
        finally:
            _stop(srv, srv_log)
    for g, r in zip(got, ref):
        g = g if isinstance(g, list) else g["results"]
        assert [h["id"] for h in g] == [h.id for h in r]
        assert np.allclose([h["score"] for h in g], [h.score for h in r], atol=1e-4)
