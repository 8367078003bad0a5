"""Grammar-constrained decoding: every sampled continuation stays inside the grammar."""
import json
import random

import pytest

from llm_kubernetes_minikube_sharp4dev_amd.agent.dotnet_json import RAG_TOOL_CALL, parse_record
from llm_kubernetes_minikube_sharp4dev_amd.engine.constrained import (JSON_START, JsonGrammar, ToolCallGrammar,
                                                                      json_feed_text)
from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer


@pytest.mark.parametrize("text,ok", [('{"a": [1, -2.5e3, true, null, "x\\u00e8"]}', True), ('{"a" 1}', False),
                                      ('[01]', False), ('"unterminated', True), ('{"a":1,}', False)])
def test_json_pda(text, ok):
    assert (json_feed_text(JSON_START, text) is not None) == ok


def _walk(proc, tok, steps, seed):
    rng = random.Random(seed)
    ids = []
    for _ in range(steps):
        allowed = proc(ids)
        assert allowed
        t = rng.choice(allowed)
        if t in tok.eos_ids:
            return ids, True
        ids.append(t)
    return ids, False


def test_tool_call_grammar_random_walks():
    tok = builtin_tokenizer()
    g = ToolCallGrammar(tok)
    done = 0
    for seed in range(30):
        ids, fin = _walk(g, tok, 200, seed)
        text = tok.decode(ids)
        if fin:
            done += 1
            call = parse_record(text, RAG_TOOL_CALL)
            assert call["action"] in ("list_pods", "get_logs", "scale_deployment", "cluster_context", "final_answer")
            if call["action"] == "scale_deployment":
                assert isinstance(call["replicas"], int) and call["name"] and call["namespace"]
    assert done >= 25


def test_json_grammar_random_walk_prefix_valid():
    tok = builtin_tokenizer()
    g = JsonGrammar(tok)
    for seed in range(3):
        ids, fin = _walk(g, tok, 40, seed)
        assert json_feed_text(JSON_START, tok.decode(ids)) is not None
        if fin:
            json.loads(tok.decode(ids))


def test_tool_call_grammar_enums_and_fast_forward():
    """Enum-valued fields (namespace allowlist / deployment names) and forced literals
    emitted as the longest vocabulary token; random walks always produce parseable,
    strictly typed tool calls with allowlisted namespaces."""
    import json
    import random

    from llm_kubernetes_minikube_sharp4dev_amd.engine.constrained import tool_call_processor
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer

    tok = builtin_tokenizer()
    ns = ["dev", "staging", "sharp4dev", "test-ns-giovanni", "default"]
    proc = tool_call_processor(tok, max_str=16, enums={"namespace": ns, "name": ["echoserver", "api"]})
    rng = random.Random(3)
    eos = set(tok.eos_ids)
    for _ in range(60):
        ids = []
        for _ in range(64):
            allowed = proc(ids)
            if set(allowed) <= eos:
                break
            ids.append(rng.choice(list(allowed)))
        obj = json.loads(tok.decode(ids))
        assert obj["action"] in ("list_pods", "get_logs", "scale_deployment", "cluster_context", "final_answer")
        if "namespace" in obj:
            assert obj["namespace"] in ns
        if "replicas" in obj:
            assert isinstance(obj["replicas"], int) and (obj["replicas"] == 0 or not str(obj["replicas"]).startswith("0"))
        assert len(ids) <= 40


def test_tool_call_grammar_incremental_text_matches_full_decode():
    """The grammar extends a running history's decoded text token by token (printable-ASCII
    pieces, EOS dropped) instead of re-decoding it every step; the text and the allowed sets
    must equal the full-decode ones along random constrained generations."""
    import random

    from llm_kubernetes_minikube_sharp4dev_amd.config import Config
    from llm_kubernetes_minikube_sharp4dev_amd.engine.constrained import tool_call_processor
    from llm_kubernetes_minikube_sharp4dev_amd.models.tokenizer import builtin_tokenizer

    tok = builtin_tokenizer()
    cfg = Config()
    enums = {"namespace": list(cfg.agent.allowed_namespaces) + ["default"], "name": ["echoserver", "api"]}
    inc = tool_call_processor(tok, max_str=16, enums=enums)
    ref = tool_call_processor(tok, max_str=16, enums=enums)
    rng = random.Random(1)
    for _ in range(25):
        ids: list = []
        for _ in range(40):
            allowed = inc(ids)
            assert inc._text(ids) == (tok.decode(ids) if ids else "")
            ref._texts = {}  # no text cache: the full-decode path
            assert list(allowed) == list(ref(list(ids)))
            ids.append(rng.choice(list(allowed)))


def test_tool_call_grammar_enum_keyed_by_earlier_field():
    """An enum given as {"__by__": field, value: [...]} allows only the values listed for the
    value the object already chose for that field (pods of the chosen namespace); random
    walks always end in an existing (namespace, pod) / (namespace, deployment) pair."""
    tok = builtin_tokenizer()
    pods = {"dev": ["api-1", "api-2"], "staging": ["web-7"]}
    deps = {"dev": ["api"], "staging": ["web"]}
    g = ToolCallGrammar(tok, max_str=16, enums={"namespace": ["dev", "staging"],
                                                 "pod": {"__by__": "namespace", **pods},
                                                 "name": {"__by__": "namespace", **deps}})
    rng = random.Random(3)
    seen = set()
    for _ in range(150):
        ids = []
        for _ in range(48):
            a = g(ids)
            ids.append(rng.choice(a))
        obj = json.loads(tok.decode([i for i in ids if i not in tok.eos_ids]))
        if obj["action"] == "get_logs":
            assert obj["pod"] in pods[obj["namespace"]], obj
            seen.add("get_logs")
        if obj["action"] == "scale_deployment":
            assert obj["name"] in deps[obj["namespace"]], obj
            seen.add("scale")
    assert seen == {"get_logs", "scale"}
