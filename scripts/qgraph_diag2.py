"""Single-query encoder graphs through EmbeddingEngine: which arrangement breaks equality
with the eager engine -- shared capture pool or not, one dtype or two, replay on the
current stream or on the engine's graph stream."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd.engine import embed_engine as ee  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models import build_encoder  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer  # noqa: E402

DEV = torch.device("cuda:0")
enc = build_encoder("bge-base", device=DEV, dtype=torch.bfloat16)
tok = builtin_tokenizer()
eager = ee.EmbeddingEngine(enc, tok, name="e")
texts = ["scale the api deployment in staging", "logs of pod web-1", "x", "how do I restart the worker"]
want = {(t, dt): eager.embed([t], dtype=dt) for t in texts for dt in (torch.float32, torch.bfloat16)}
print("lengths", [len(s) for s in eager.tokenize(texts)], flush=True)


def check(name, eng):
    bad = []
    for t in texts:
        for dt in (torch.float32, torch.bfloat16):
            got = eng.embed([t], dtype=dt)
            if not torch.equal(got, want[(t, dt)]):
                bad.append((texts.index(t), str(dt)[6:], round((got.float() - want[(t, dt)].float()).abs().max().item(), 4)))
    print(f"{name}: {'OK' if not bad else bad}", flush=True)


for name, max_len, dtypes, shared in [("f32 only, L<=12, shared pool", 12, (torch.float32,), True),
                                      ("both, L<=12, shared pool", 12, (torch.bfloat16, torch.float32), True),
                                      ("both, L<=24, shared pool", 24, (torch.bfloat16, torch.float32), True),
                                      ("both, L<=24, own pools", 24, (torch.bfloat16, torch.float32), False)]:
    g = ee.EmbeddingEngine(enc, tok, name="g")
    if not shared:
        real = torch.cuda.graph_pool_handle

        class _P:
            def __bool__(self):
                return False

        orig = g.capture_queries

        def cap(max_len, dtypes):
            n = 0
            for dt in dtypes:
                for L in range(1, max_len + 1):
                    g._qpool = real()
                    n += orig(max_len=L, dtypes=(dt,))
            return n
        n = cap(max_len, dtypes)
    else:
        n = g.capture_queries(max_len=max_len, dtypes=dtypes)
    print(name, "captured", n, flush=True)
    check(name, g)
    del g
    torch.cuda.synchronize()
