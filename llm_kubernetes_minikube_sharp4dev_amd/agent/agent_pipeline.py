"""Batched ``/agent`` (Minimal_Agent, BASELINE.json config 3) and the mixed
agent + RAG session load (config 5), with the request-level interface of
:class:`agent.rag_pipeline.ContinuousLoad`.

``/agent`` per request (``Minimal_Agent_RAG/Program.cs:34-151``): prompt =
``"{system}\nUtente: {prompt}\nRisposta JSON:"`` sent through the model's chat template
(Ollama applies it to ``/api/generate``), streamed output concatenated WITHOUT fence
stripping, strict case-insensitive ``CallAction`` parse, then one k8s action
(no namespace allowlist).  An unhandled k8s error is the 500 of ASP.NET's developer
exception page.
"""
from __future__ import annotations

import time

from .prompts import agent_prompt
from .rag_pipeline import RagAgentResult
from .tools import UnhandledK8sError, dispatch_agent_tool


class AgentPipeline:
    def __init__(self, llm, tokenizer, k8s, cfg, chat_style: str = "llama3"):
        self.llm, self.tok, self.k8s, self.cfg, self.chat_style = llm, tokenizer, k8s, cfg, chat_style

    def plan_requests(self, prompts: list[str]):
        t0 = time.perf_counter()
        ids = self.tok.chat_prompt_batch([agent_prompt(p) for p in prompts], style=self.chat_style)
        return [(p, i, "agent") for p, i in zip(prompts, ids)], {"prompt_s": time.perf_counter() - t0}

    def finish_request(self, prompt: str, out_ids: list, ctx) -> RagAgentResult:
        raw = self.tok.decode(out_ids)
        try:
            status, body = dispatch_agent_tool(self.k8s, raw, self.cfg)
        except UnhandledK8sError as e:
            status, body = 500, f"An unhandled exception has occurred: {e}"
        return RagAgentResult(prompt, status, body, [], 0, len(out_ids), raw)


class MixedPipeline:
    """Concurrent multi-session load: requests alternate between ``/agent_rag`` and
    ``/agent`` (tagged by position), sharing one continuous-batching engine."""

    def __init__(self, rag, agent, agent_every: int = 2):
        self.rag, self.agent, self.every = rag, agent, max(1, agent_every)
        self.llm = rag.llm
        self._n = 0

    def plan_requests(self, prompts: list[str]):
        kinds = []
        for _ in prompts:
            kinds.append("agent" if self._n % self.every == self.every - 1 else "rag")
            self._n += 1
        rq = [p for p, k in zip(prompts, kinds) if k == "rag"]
        aq = [p for p, k in zip(prompts, kinds) if k == "agent"]
        rr, t1 = self.rag.plan_requests(rq) if rq else ([], {})
        ar, t2 = self.agent.plan_requests(aq) if aq else ([], {})
        ri, ai = iter(rr), iter(ar)
        out = []
        for k in kinds:
            if k == "rag":
                p, ids, ctx = next(ri)
                out.append((p, ids, ("rag", ctx)))
            else:
                p, ids, ctx = next(ai)
                out.append((p, ids, ("agent", ctx)))
        tim = {k: t1.get(k, 0.0) + t2.get(k, 0.0) for k in set(t1) | set(t2)}
        return out, tim

    def finish_request(self, prompt: str, out_ids: list, ctx) -> RagAgentResult:
        if ctx is None:
            return self.rag.finish_request(prompt, out_ids, None)
        kind, inner = ctx
        return (self.rag if kind == "rag" else self.agent).finish_request(prompt, out_ids, inner)
