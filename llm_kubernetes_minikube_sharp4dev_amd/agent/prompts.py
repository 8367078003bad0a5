"""Prompts of the two agents, as the reference intends them (UTF-8 text of the
Windows-1252 source), and the prompt templates.

* ``AGENT_SYSTEM``      — ``Minimal_Agent_RAG/Program.cs:39-46`` (C# raw string: the
  closing delimiter's 4-space indent is removed, so lines keep 4 spaces).
* ``RAG_AGENT_SYSTEM``  — ``Minimal_RAG/Program.cs:136-149``.
* ``agent_prompt``      — ``"{system}\\nUtente: {prompt}\\nRisposta JSON:"`` (Program.cs:48).
* ``json_prompt``       — ``"{system}\\nUtente:\\n{userJson}\\nRispondi SOLO con JSON valido:"``
  (``Helpers.cs:113``), ``userJson`` serialized like System.Text.Json defaults.
"""
from __future__ import annotations

from .dotnet_json import dumps as net_dumps

_AGENT_LINES = [
    "Sei un assistente DevOps per Kubernetes. Rispondi SOLO in JSON",
    "Scegli uno tra: list_pods, get_logs e scale_deployment.",
    '- list_pods:        {"action":"list_pods","namespace": "..."}',
    '- get_logs:         {"action":"get_logs","namespace":"...","pod":"...","container":"opzionale"}',
    '- scale_deployment: {"action":"scale_deployment","namespace":"...","name":"...","replicas":"NUM"}',
    "Nessun testo al di fuori del JSON",
]
AGENT_SYSTEM = "\n".join("    " + l for l in _AGENT_LINES)

RAG_AGENT_SYSTEM = "\n".join([
    "Sei un agente DevOps RAG-only. Puoi scegliere UN SOLO tool tra:",
    "- list_pods {namespace}",
    "- get_logs {namespace, pod, container?}",
    "- scale_deployment {namespace, name, replicas}",
    "- cluster_context {}",
    "- final_answer {}",
    "",
    "Regole:",
    "- Usa SOLO le informazioni contenute nell'array 'evidence'. Se una richiesta non è supportata dai "
    "runbook presenti in evidence, scegli 'final_answer' spiegando che manca evidenza.",
    "- Non inventare valori. Se mancano 'namespace' o 'name', richiedi informazioni con 'final_answer'.",
    "- Per 'scale_deployment' serve evidenza esplicita (runbook di scaling) e namespace ammesso.",
    'Rispondi SOLO con JSON: {"action":"...", "namespace":"...", "name":"...", "replicas":N, '
    '"pod":"...", "container":"..."}.',
])

FINAL_ANSWER_MESSAGE = ("In base ai runbook recuperati non è possibile eseguire un’azione operativa. "
                        "Fornisci namespace e deployment, oppure aggiungi un runbook pertinente.")


def agent_prompt(prompt: str, system: str = AGENT_SYSTEM) -> str:
    return f"{system}\nUtente: {prompt}\nRisposta JSON:"


def json_prompt(system: str, payload) -> str:
    return f"{system}\nUtente:\n{net_dumps(payload)}\nRispondi SOLO con JSON valido:"


def rag_agent_input(user: str, evidence: list, text_chars: int = 1500) -> dict:
    """The anonymous ``input`` object of ``Minimal_RAG/Program.cs:151-161``; member
    order and casing as declared: user, evidence[{Id, Source, Score, text}]."""
    return {
        "user": user,
        "evidence": [{"Id": h.id, "Source": h.source, "Score": h.score,
                      "text": h.text[:text_chars] if len(h.text) > text_chars else h.text} for h in evidence],
    }
