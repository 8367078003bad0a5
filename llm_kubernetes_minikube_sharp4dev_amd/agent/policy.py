"""Gating / policy helpers of the RAG agent.

* :func:`select_citations` — ``Minimal_RAG/Program.cs:124-133``: citations are the hits
  with ``score >= max(0.35, 0.6 * best)``; evidence is those hits.
* :func:`extract_allowed_namespaces` — ``Helpers.cs:69-86`` (C12): only a chunk that
  STARTS with ``---`` counts as front-matter; regex
  ``allowed_namespaces:\\s*\\[(.*?)\\]`` (case-insensitive) inside it.
* :func:`has_scaling_evidence` — ``Program.cs:266-270``.
* :func:`build_cluster_context` — ``Helpers.cs:89-105`` (C13).
* :func:`parse_cpu_to_millicores` / :func:`parse_mem_to_mi` — ``Helpers.cs:11-65``
  (C14; dead code in the reference, kept as library functions for metrics features).
"""
from __future__ import annotations

import re
from typing import Iterable, Optional

from .dotnet_json import dumps as net_dumps

_FM_NS = re.compile(r"allowed_namespaces:\s*\[(.*?)\]", re.IGNORECASE)


def select_citations(hits: list, evidence_min: float = 0.35, ratio: float = 0.6):
    if not hits:
        return [], []
    best = max(h.score for h in hits)
    thr = max(evidence_min, best * ratio)
    citations = [h.id for h in hits if h.score >= thr]
    cset = set(citations)
    evidence = [h for h in hits if h.id in cset]
    return citations, evidence


def extract_allowed_namespaces(chunk_text: str) -> list[str]:
    if chunk_text.find("---") != 0:
        return []
    end = chunk_text.find("---", 3)
    if end <= 0:
        return []
    fm = chunk_text[: end + 3]
    m = _FM_NS.search(fm)
    if not m:
        return []
    out = []
    for s in m.group(1).split(","):
        s = s.replace('"', "").strip()
        if s:
            out.append(s)
    return out


class CaseInsensitiveSet:
    """HashSet<string>(StringComparer.OrdinalIgnoreCase) keeping first-seen casing/order."""

    def __init__(self, items: Iterable[str] = ()):
        self._d: dict[str, str] = {}
        for i in items:
            self.add(i)

    def add(self, s: str):
        self._d.setdefault(s.lower(), s)

    def __contains__(self, s) -> bool:
        return s is not None and s.lower() in self._d

    def __len__(self):
        return len(self._d)

    def __iter__(self):
        return iter(self._d.values())


def has_scaling_evidence(evidence: list, min_score: float = 0.35) -> bool:
    for e in evidence:
        if e.score >= min_score and ("scaling" in e.id.lower() or "scaling" in e.source.lower()
                                     or "scale_deployment" in e.text.lower()):
            return True
    return False


def build_cluster_context(k8s) -> str:
    nodes = k8s.list_node()["items"]
    pods = k8s.list_pod_for_all_namespaces()["items"]
    deps = k8s.list_deployment_for_all_namespaces()["items"]
    by_ns: dict[str, int] = {}
    for p in pods:
        ns = (p.get("metadata") or {}).get("namespace") or "default"
        by_ns[ns] = by_ns.get(ns, 0) + 1
    summary = {
        "nodes": [{"Name": n["metadata"]["name"], "KubeletVersion": n["status"]["nodeInfo"]["kubeletVersion"]}
                  for n in nodes],
        "totals": {"pods": len(pods), "deployments": len(deps)},
        "podsByNs": by_ns,
    }
    return net_dumps(summary)


def _num(s: str) -> Optional[float]:
    try:
        return float(s)
    except ValueError:
        return None


def parse_cpu_to_millicores(cpu: Optional[str]) -> float:
    if cpu is None or not cpu.strip():
        return 0.0
    c = cpu.strip().lower()
    for suf, f in (("n", 1 / 1_000_000.0), ("u", 1 / 1000.0), ("m", 1.0)):
        if c.endswith(suf):
            v = _num(c[:-1])
            if v is not None:
                return v * f
    v = _num(c)
    return v * 1000.0 if v is not None else 0.0


def parse_mem_to_mi(mem: Optional[str]) -> float:
    if mem is None or not mem.strip():
        return 0.0
    u = mem.strip().upper()
    for suf, f in (("KI", 1 / 1024.0), ("MI", 1.0), ("GI", 1024.0), ("TI", 1024.0 * 1024.0)):
        if u.endswith(suf):
            v = _num(u[:-2])
            if v is not None:
                return v * f
    for suf, f in (("K", 1000.0), ("M", 1_000_000.0), ("G", 1_000_000_000.0)):
        if u.endswith(suf):
            v = _num(u[:-1])
            if v is not None:
                return v * f / (1024.0 * 1024.0)
    v = _num(u)
    return v / 1024.0 / 1024.0 if v is not None else 0.0
