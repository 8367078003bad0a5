"""Tool dispatch of both agents, returning ``(status, body)`` with the reference's
exact response shapes.

* :func:`dispatch_rag_tool`   — ``Minimal_RAG/Program.cs:165-315`` (C4a–C4e).
* :func:`dispatch_agent_tool` — ``Minimal_Agent_RAG/Program.cs:60-149`` (C17a–C17d).
"""
from __future__ import annotations

from typing import Any, Optional

from ..rag.chunking import is_blank
from .dotnet_json import AGENT_CALL_ACTION, RAG_TOOL_CALL, NetJsonError, loads_strict, parse_record
from .policy import CaseInsensitiveSet, build_cluster_context, extract_allowed_namespaces, has_scaling_evidence
from .prompts import FINAL_ANSWER_MESSAGE


class Problem:
    """``Results.Problem(title, detail, statusCode)`` -> application/problem+json."""

    def __init__(self, title: str, detail: str, status: int = 500):
        self.body = {"type": "https://tools.ietf.org/html/rfc9110#section-15.6.1", "title": title,
                     "status": status, "detail": detail}
        self.status = status


def _rag_response(result: Any, citations: list, note: Optional[str]) -> dict:
    return {"result": result, "citations": citations, "note": note}


def dispatch_rag_tool(k8s, tool_json: str, citations: list, evidence: list, cfg) -> tuple[int, Any]:
    """Deserialize the LLM's tool call and execute it under the RAG gating rules."""
    a = cfg.agent
    allowed = CaseInsensitiveSet(a.allowed_namespaces)
    try:
        call = parse_record(tool_json, RAG_TOOL_CALL)
    except NetJsonError:
        return 400, {"error": "Output del modello non valido", "raw": tool_json}
    if call is None or is_blank(call["action"]):
        return 400, {"error": "Nessuna azione proposta", "raw": tool_json}
    action = call["action"].lower()
    try:
        if action == "cluster_context":
            ctx = build_cluster_context(k8s)
            return 200, _rag_response(loads_strict(ctx), citations, "cluster_context eseguito sulla base dei runbook.")
        if action == "list_pods":
            ns = a.default_namespace if is_blank(call["namespace"]) else call["namespace"]
            if ns not in allowed:
                return 400, {"error": f"Namespace '{ns}' non ammesso", "citations": citations}
            pods = k8s.list_namespaced_pod(ns)["items"]
            lst = [{"ns": (p.get("metadata") or {}).get("namespace"), "name": (p.get("metadata") or {}).get("name"),
                    "phase": (p.get("status") or {}).get("phase")} for p in pods]
            return 200, _rag_response(lst, citations, "list_pods eseguito (RAG-only)")
        if action == "get_logs":
            ns = a.default_namespace if is_blank(call["namespace"]) else call["namespace"]
            if is_blank(call["pod"]):
                return 400, {"error": "Manca 'pod' per get_logs", "citations": citations}
            if ns not in allowed:
                return 400, {"error": f"Namespace '{ns}' non ammesso", "citations": citations}
            logs = k8s.read_namespaced_pod_log(call["pod"], ns, call["container"], a.log_tail_lines) or ""
            if len(logs) > a.log_max_chars:
                logs = logs[: a.log_max_chars] + a.log_truncation_suffix
            return 200, _rag_response({"ns": ns, "pod": call["pod"], "container": call["container"], "logs": logs},
                                      citations, "get_logs eseguito (RAG-only)")
        if action == "scale_deployment":
            ns = None if is_blank(call["namespace"]) else call["namespace"]
            name = None if is_blank(call["name"]) else call["name"]
            replicas = call["replicas"]
            if ns is None or name is None or replicas is None:
                return 400, {"error": "Servono 'namespace', 'name' e 'replicas' per scale_deployment",
                             "citations": citations}
            if ns not in allowed:
                return 400, {"error": f"Namespace '{ns}' non ammesso dalla policy locale", "citations": citations}
            if not has_scaling_evidence(evidence, cfg.rag.evidence_min_score):
                return 400, {"error": "Manca evidenza di runbook di scaling: azione bloccata (RAG-only).",
                             "citations": citations}
            fm = CaseInsensitiveSet(n for e in evidence for n in extract_allowed_namespaces(e.text))
            if len(fm) > 0 and ns not in fm:
                return 400, {"error": f"Namespace '{ns}' non consentito dal runbook (allowed: {','.join(fm)})",
                             "citations": citations}
            if a.enforce_runbook_limits:  # opt-in fix of quirk A.7.8 (prose-only limits)
                cur = (k8s.read_namespaced_deployment_scale(name, ns).get("spec") or {}).get("replicas") or 0
                if replicas > 10 or replicas - cur > 2:
                    return 400, {"error": "Limiti del runbook superati (max +2 repliche, replicas <= 10)",
                                 "citations": citations}
            scale = k8s.read_namespaced_deployment_scale(name, ns)
            prev = (scale.get("spec") or {}).get("replicas") or 0
            scale.setdefault("spec", {})["replicas"] = replicas
            updated = k8s.replace_namespaced_deployment_scale(name, ns, scale)
            return 200, _rag_response({"namespace": ns, "name": name, "replicas_prev": prev,
                                       "replicas_now": (updated.get("spec") or {}).get("replicas")},
                                      citations, "scale_deployment eseguito perché supportato da runbook (RAG-only).")
        summary = {"message": FINAL_ANSWER_MESSAGE, "evidence": [{"id": e.id, "score": e.score} for e in evidence]}
        return 200, _rag_response(summary, citations, "final_answer (RAG-only)")
    except Exception as ex:  # Program.cs:312-315
        p = Problem("Operazione fallita", str(ex), 500)
        return p.status, p


class UnhandledK8sError(RuntimeError):
    """/agent has no try/catch around the cluster calls (AGENT/Program.cs:81-149):
    the framework's default 500 applies."""


def dispatch_agent_tool(k8s, raw: str, cfg) -> tuple[int, Any]:
    from .json_extract import extract_json_object

    text = extract_json_object(raw) if cfg.agent.agent_strip_fences else raw
    try:
        call = parse_record(text, AGENT_CALL_ACTION)
        if call is None or is_blank(call["action"]):
            return 400, {"error": "Output del modello non valido", "data": raw}
    except NetJsonError as ex:
        return 400, {"error": "JSON Parse error", "cause": str(ex), "data": raw}
    action = call["action"].lower()
    d = cfg.agent.default_namespace
    try:
        if action == "list_pods":
            ns = d if is_blank(call["namespace"]) else call["namespace"]
            pods = k8s.list_namespaced_pod(ns)["items"]
            lst = [{"ns": (p.get("metadata") or {}).get("namespace"), "name": (p.get("metadata") or {}).get("name"),
                    "phase": (p.get("status") or {}).get("phase"), "node": (p.get("spec") or {}).get("nodeName")}
                   for p in pods]
            # the response echoes the UN-defaulted namespace (quirk A.7.3)
            return 200, {"action": call["action"], "ns": call["namespace"], "pods": lst}
        if action == "get_logs":
            ns = d if is_blank(call["namespace"]) else call["namespace"]
            if is_blank(call["pod"]):
                return 400, {"error": "Missing pod name"}
            container = None if is_blank(call["container"]) else call["container"]
            logs = k8s.read_namespaced_pod_log(call["pod"], ns, container, None)
            return 200, {"action": call["action"], "ns": ns, "pod": call["pod"], "logs": logs}
        if action == "scale_deployment":
            ns = d if is_blank(call["namespace"]) else call["namespace"]
            if is_blank(call["name"]) or call["replicas"] is None:
                return 400, {"error": "Missing name or replicas for scale_deployment"}
            scale = k8s.read_namespaced_deployment_scale(call["name"], ns)
            scale.setdefault("spec", {})["replicas"] = call["replicas"]
            updated = k8s.replace_namespaced_deployment_scale(call["name"], ns, scale)
            return 200, {"action": call["action"], "ns": ns, "deployment": call["name"],
                         "replicas": (updated.get("spec") or {}).get("replicas")}
        return 400, {"error": "Azione non supportata"}
    except Exception as ex:
        raise UnhandledK8sError(str(ex)) from ex
