"""Property tests (hypothesis) of the reference-contract helpers against plain-Python
oracles of SURVEY Appendix A, as SURVEY §4.2 asks for the unit level: sliding windows
(``RagIndex.cs:101-114``), header split (``:71-99``), sanitizer (``:116-122``), stable
cosine top-k (``:59-67,124-135``), JSON extraction (``Helpers.cs:119-128``), the
System.Text.Json serializer (§A.2), citation threshold (``Program.cs:124-133``),
front-matter namespaces (``Helpers.cs:69-86``) and the quantity parsers (``:11-65``)."""
import json
import math

import numpy as np
import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

from llm_kubernetes_minikube_sharp4dev_amd.agent.dotnet_json import dumps  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.agent.json_extract import extract_json_object  # noqa: E402
from llm_kubernetes_minikube_sharp4dev_amd.agent.policy import (  # noqa: E402
    CaseInsensitiveSet, extract_allowed_namespaces, parse_cpu_to_millicores, parse_mem_to_mi, select_citations)
from llm_kubernetes_minikube_sharp4dev_amd.rag.chunking import (  # noqa: E402
    _NET_WS, REDACT_RE, chunk_sliding, net_trim, sanitize, split_by_markdown_headers)
from llm_kubernetes_minikube_sharp4dev_amd.rag.index import RagHit, RagIndex, cosine_exact  # noqa: E402

SETTINGS = settings(max_examples=150, deadline=None)
BMP = st.characters(max_codepoint=0xFFFF, blacklist_categories=("Cs",))


@SETTINGS
@given(st.text(BMP, max_size=3000), st.integers(-5, 1500), st.integers(-5, 1500))
def test_chunk_sliding_windows(text, size, overlap):
    s = size if size > 0 else 800
    step = max(1, s - max(overlap, 0))
    out = chunk_sliding(text, size, overlap)
    assert len(out) == (len(text) + step - 1) // step
    for i, w in enumerate(out):
        assert w == text[i * step:i * step + s]


_LINE = st.one_of(
    st.text(st.sampled_from("ab c\t#-:é"), max_size=40),
    st.builds(lambda h, t: "#" * h + " " + t, st.integers(1, 6), st.text(st.sampled_from("xyz "), max_size=20)),
    st.builds(lambda t: "  ## " + t, st.text(st.sampled_from("uvw"), max_size=10)),
)


def _nonws(s):
    return "".join(ch for ch in s if ch not in _NET_WS)


@SETTINGS
@given(st.lists(_LINE, max_size=30), st.sampled_from(["\n", "\r\n"]))
def test_split_by_headers_preserves_text_and_bounds(lines, eol):
    text = eol.join(lines)
    out = split_by_markdown_headers(text)
    assert all(len(s) <= 1200 for s in out)
    if len(text) <= 1200:  # no re-split: sections partition the text at header lines
        assert _nonws("".join(out)) == _nonws(text)
        assert all(s == net_trim(s) for s in out)
        assert all(s.startswith("#") for s in out[1:])
        n_headers = sum(1 for ln in text.replace("\r\n", "\n").split("\n")
                        if ln.lstrip(" \t").startswith("#") and _is_header(ln))
        assert len(out) == n_headers + (0 if lines and _is_header(lines[0]) else 1)


def _is_header(line):
    s = line.lstrip(" \t")
    h = len(s) - len(s.lstrip("#"))
    return 1 <= h <= 6 and len(s) > h and s[h] in " \t"


_PHRASES = ["ignore previous instructions", "Disregard All Prior Rules", "SYSTEM PROMPT"]


@SETTINGS
@given(st.lists(st.one_of(st.text(BMP, max_size=300), st.sampled_from(_PHRASES + ["\0"])), max_size=20))
def test_sanitize_properties(parts):
    raw = "".join(parts)
    out = sanitize(raw)
    assert len(out) <= 2000 and "\0" not in out
    assert REDACT_RE.search(out) is None
    clean = net_trim(raw.replace("\0", ""))
    if REDACT_RE.search(clean) is None and len(clean) <= 2000:
        assert out == clean


@SETTINGS
@given(st.integers(1, 40), st.integers(1, 8), st.integers(-3, 12), st.integers(0, 2 ** 31))
def test_exact_index_stable_topk_matches_oracle(n, d, top_k, seed):
    rng = np.random.default_rng(seed)
    # small integer coordinates: many exact ties, every sum exact in f64
    mat = rng.integers(-2, 3, size=(n, d)).astype(np.float32)
    q = rng.integers(-2, 3, size=(d,)).astype(np.float32)
    idx = RagIndex(embedder=None, backend="exact", device="cpu")
    idx.add([f"c#{i}" for i in range(n)], ["s"] * n, ["t"] * n, mat)
    got = idx.search_vectors(q[None], top_k)[0]
    scores = [cosine_exact(q, mat[j]) for j in range(n)]
    want = sorted(range(n), key=lambda j: (-scores[j], j))[:max(1, top_k)]
    assert [j for j, _ in got] == want
    assert [s for _, s in got] == [scores[j] for j in want]


_SAFE_PROSE = st.text(st.characters(max_codepoint=0x7E, blacklist_characters="{}`"), max_size=40)
_JSON_LEAF = st.one_of(st.none(), st.booleans(), st.integers(-2 ** 40, 2 ** 40),
                       st.floats(allow_nan=False, allow_infinity=False), st.text(BMP, max_size=20))
_JSON = st.recursive(_JSON_LEAF, lambda ch: st.one_of(st.lists(ch, max_size=4),
                                                      st.dictionaries(st.text(BMP, max_size=8), ch, max_size=4)),
                     max_leaves=12)


@SETTINGS
@given(_JSON, st.text(BMP, max_size=40))
def test_dotnet_dumps_roundtrip_and_escaping(obj, text):
    s = dumps(obj)
    assert s.isascii()
    assert json.loads(s) == obj
    t = dumps(text)  # JavaScriptEncoder.Default: HTML-sensitive ASCII always \uXXXX
    assert t.isascii() and not any(c in t for c in "<>&'+`")
    assert json.loads(t) == text


@SETTINGS
@given(st.dictionaries(st.text(BMP, max_size=8), _JSON, min_size=1, max_size=4), _SAFE_PROSE, _SAFE_PROSE,
       st.booleans())
def test_extract_json_object_from_wrapped_output(obj, pre, post, fenced):
    j = dumps(obj)
    body = f"```json\n{j}\n```" if fenced else j
    assert extract_json_object(f"{pre}{body}{post}") == j


@SETTINGS
@given(_SAFE_PROSE)
def test_extract_json_without_braces_returns_trimmed(raw):
    assert extract_json_object(raw) == net_trim(raw).strip("`")


@SETTINGS
@given(st.lists(st.floats(0, 1, allow_nan=False), max_size=12))
def test_citation_threshold(scores):
    hits = [RagHit(f"h{i}", "s", "t", sc) for i, sc in enumerate(scores)]
    cites, ev = select_citations(hits)
    if not hits:
        assert cites == [] and ev == []
        return
    thr = max(0.35, 0.6 * max(scores))
    assert cites == [h.id for h in hits if h.score >= thr]
    assert [h.id for h in ev] == cites


_NS = st.from_regex(r"[a-z0-9]{1,6}(-[a-z0-9]{1,6}){0,2}", fullmatch=True)  # DNS-1123 labels


@SETTINGS
@given(st.lists(_NS, max_size=6), st.booleans(), st.text(st.sampled_from("ab #\n"), max_size=30))
def test_front_matter_namespaces(names, quoted, body):
    items = ", ".join(f'"{n}"' if quoted else n for n in names)
    fm = f"---\ntitle: x\nallowed_namespaces: [{items}]\n---\n"
    assert extract_allowed_namespaces(fm + body) == names
    assert extract_allowed_namespaces(" " + fm + body) == []  # must START with ---
    s = CaseInsensitiveSet(names)
    assert all(n.upper() in s for n in names)


@SETTINGS
@given(st.integers(0, 10 ** 6))
def test_quantity_parsers(v):
    assert parse_cpu_to_millicores(f"{v}m") == v
    assert parse_cpu_to_millicores(f" {v} ") == v * 1000.0
    assert math.isclose(parse_cpu_to_millicores(f"{v}n"), v / 1e6)
    assert parse_mem_to_mi(f"{v}Mi") == v
    assert parse_mem_to_mi(f"{v}Gi") == v * 1024.0
    assert math.isclose(parse_mem_to_mi(f"{v}Ki"), v / 1024.0)
    assert math.isclose(parse_mem_to_mi(f"{v}M"), v * 1e6 / 1024 / 1024)
    assert math.isclose(parse_mem_to_mi(str(v)), v / 1024 / 1024)
