"""LLM-output hardening of ``Helpers.AskOllamaJsonAsync`` (``Helpers.cs:119-128``):
trim whitespace, trim backticks, keep the text between the first ``{`` and the last
``}`` when both exist in that order, otherwise return the raw string (the caller's
deserialize then fails -> 400).  ``/agent`` does NOT do this (quirk A.7.4)."""
from __future__ import annotations

from ..rag.chunking import net_trim


def extract_json_object(raw: str) -> str:
    s = net_trim(raw).strip("`")
    start = s.find("{")
    end = s.rfind("}")
    if start >= 0 and end > start:
        s = s[start:end + 1]
    return s
