"""``serve --tp 2 --one-device`` on the MI355X: the split server's engine core is the leader of a
TP=2 group whose two ranks share the box's one GPU (gloo host collectives, every device
collective on the IPC kernels, decode hipGraphs capturing them, as tests/test_tp_ipc_gpu.py),
driven over HTTP by /api/generate.  Greedy tokens == the TP=1 engine on the same checkpoint, up
to near-ties (bf16 partial sums summed in a different order); /health reports the TP size."""
import os
import tempfile

import pytest
import torch

from test_serve_tp_cpu import _config, _free_port, _gen_body, _launch, _model_flags, _stop, _wait_ready

transformers = pytest.importorskip("transformers")
httpx = pytest.importorskip("httpx")

pytestmark = pytest.mark.gpu
PROMPTS = ["ciao, come stai?", "kubectl get pods -n demo", "scale the echoserver deployment to three replicas",
           "why is my pod in CrashLoopBackOff"]


def _gpu_config(tmp):
    path = _config(tmp)
    import json

    c = json.load(open(path))
    c["engine"]["dtype"] = "bfloat16"
    c["engine"]["kv_cache_gb"] = 2.0  # two ranks and the test process share the one device
    json.dump(c, open(path, "w"))
    return path


@pytest.mark.timeout(900)
def test_serve_tp2_one_device_http_matches_tp1():
    from test_serve_tp_cpu import ALIASES

    from llm_kubernetes_minikube_sharp4dev_amd.config import load_config
    from llm_kubernetes_minikube_sharp4dev_amd.serving.model_manager import ModelManager

    with tempfile.TemporaryDirectory() as tmp:
        ck = os.path.join(tmp, "ckpt")
        cfg = transformers.LlamaConfig(vocab_size=32768, hidden_size=256, intermediate_size=512, num_hidden_layers=2,
                                       num_attention_heads=4, num_key_value_heads=2, max_position_embeddings=4096,
                                       rope_theta=10000.0, rms_norm_eps=1e-5, tie_word_embeddings=False)
        torch.manual_seed(5)
        hf = transformers.LlamaForCausalLM(cfg).eval()
        with torch.no_grad():
            for n, p in hf.named_parameters():
                if n.endswith("norm.weight"):
                    p.uniform_(0.5, 1.5)
        hf.save_pretrained(ck, safe_serialization=True)
        cfg_path = _gpu_config(tmp)
        port = _free_port()
        proc, log = _launch(["serve", "--tp", "2", "--one-device", "--frontends", "1", "--port", str(port),
                             "--preload", "llama3.1:8b"] + _model_flags(ck, cfg_path), tmp)
        try:
            url = f"http://127.0.0.1:{port}/api/generate"
            _wait_ready(proc, url, _gen_body("warm up"), tmp, "serve", timeout=600)
            got = [httpx.post(url, json=_gen_body(p), timeout=120).json() for p in PROMPTS]
            health = httpx.get(f"http://127.0.0.1:{port}/health", timeout=30).json()
        finally:
            _stop(proc, log)
        text = open(os.path.join(tmp, "serve.log")).read()
        mgr = ModelManager(load_config(cfg_path), aliases=dict(a.split("=") for a in ALIASES),
                           checkpoints={"llama-tiny": ck})
        try:
            from fastapi.testclient import TestClient

            from llm_kubernetes_minikube_sharp4dev_amd.serving.ollama_server import create_app

            with TestClient(create_app(mgr)) as c:
                ref = [c.post("/api/generate", json=_gen_body(p)).json() for p in PROMPTS]
        finally:
            mgr.shutdown()
    assert health["generators"]["llama3.1:8b"]["tp"] == 2, health
    assert "Traceback" not in text, text[-3000:]
    for g, r in zip(got, ref):
        assert g["eval_count"] == r["eval_count"] == 8
        gc, rc = g["context"], r["context"]
        if gc == rc:
            continue
        k = next(i for i, (a, b) in enumerate(zip(gc, rc)) if a != b)
        with torch.no_grad():
            want = hf(torch.tensor([rc[:k]])).logits[0, -1]
        gap = abs(want[gc[k]] - want[rc[k]]).item()
        assert gap < 0.05 * want.abs().max().item() + 0.05, (k, gc[k], rc[k], gap)
