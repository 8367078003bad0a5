"""Batched ``/agent_rag`` pipeline (retrieve -> gate -> augment -> generate -> gate ->
act), the headline workload, running fully in-process on MI355X:

  query embeddings (encoder kernels) -> cosine top-6 (HIP kNN, corpus in HBM)
  -> citations ``score >= max(0.35, 0.6*best)`` -> evidence JSON (System.Text.Json
  escaping) -> Llama-3 chat template -> continuous-batching engine (flash prefill
  with the shared system-prompt prefix served from the prefix cache, hipGraph
  decode) -> JSON extraction -> typed tool call -> RAG gating -> k8s action.

The same per-request semantics as ``Minimal_RAG/Program.cs:106-316``; the HTTP app
(`apps.rag_app`) serves single requests through it, the benchmark runs batches.
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Optional

import torch

from .json_extract import extract_json_object
from .policy import select_citations
from .prompts import RAG_AGENT_SYSTEM, json_prompt, rag_agent_input
from .tools import dispatch_rag_tool


@dataclass
class RagAgentResult:
    prompt: str
    status: int = 200
    body: Any = None
    citations: list = field(default_factory=list)
    prompt_tokens: int = 0
    output_tokens: int = 0
    raw: str = ""
    timings: dict = field(default_factory=dict)


NO_EVIDENCE_NOTE = "Nessuna evidenza trovata nei runbook."


class RagAgentPipeline:
    def __init__(self, index, llm, tokenizer, k8s, cfg, chat_style: str = "llama3"):
        self.index = index
        self.llm = llm
        self.tok = tokenizer
        self.k8s = k8s
        self.cfg = cfg
        self.chat_style = chat_style
        # running totals over planned LLM requests: prompt-body characters and prompt tokens
        # (chat template included) -- bench.py reports their ratio as chars_per_token
        self.planned_chars = 0
        self.planned_tokens = 0
        self.planned_requests = 0
        self.planned_evidence = 0  # evidence chunks that passed the citation gate

    def plan_launch(self, prompts: list[str]) -> dict:
        """Enqueue retrieval for a batch of user prompts without waiting on the device: the
        query encoder and the kNN kernel run on the current stream, the top-k lands in
        pinned memory behind an event (:meth:`RagIndex.search_vectors_async`)."""
        t0 = time.perf_counter()
        r = self.cfg.rag
        embedder = self.index.embedder
        if hasattr(embedder, "embed_tensor"):
            qv = embedder.embed_tensor(prompts)
        else:
            qv = embedder.embed(prompts)
        t1 = time.perf_counter()
        ev0 = ev1 = None
        if isinstance(qv, torch.Tensor) and qv.is_cuda:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        pending = self.index.search_vectors_async(qv, r.agent_topk)
        if ev1 is not None:
            ev1.record()
        return {"prompts": prompts, "pending": pending, "t": (t0, t1, time.perf_counter()), "ev": (ev0, ev1)}

    def plan_ready(self, h: dict) -> bool:
        return h["pending"].ready()

    def plan_finish(self, h: dict):
        """Gating + prompt construction once the launched search has landed."""
        t0, t1, t2 = h["t"]
        res = h["pending"].result()
        t2w = time.perf_counter()
        r = self.cfg.rag
        plans = []
        texts = []
        for p, rr in zip(h["prompts"], res):
            hits = self.index.hits(rr)
            if not hits:
                plans.append((p, None, [], []))
                continue
            citations, evidence = select_citations(hits, r.evidence_min_score, r.citation_best_ratio)
            full = json_prompt(RAG_AGENT_SYSTEM, rag_agent_input(p, evidence, r.evidence_text_chars))
            plans.append((p, full, citations, evidence))
            texts.append(full)
        ids = iter(self.tok.chat_prompt_batch(texts, style=self.chat_style)) if texts else iter(())
        out = []
        for p, full, cit, ev in plans:
            pid = next(ids) if full is not None else None
            if pid is not None:
                self.planned_chars += len(full)
                self.planned_tokens += len(pid)
                self.planned_requests += 1
                self.planned_evidence += len(ev)
            out.append((p, pid, cit, ev))
        t3 = time.perf_counter()
        # embed_s / knn_s: host time blocked in each stage (launch, plus the wait for the
        # top-k); knn_gpu_s: the kNN's device time in situ (event to event on its stream,
        # including any wait for CUs held by a concurrent engine step)
        tim = {"embed_s": t1 - t0, "knn_s": (t2 - t1) + h["pending"].wait_s,
               "prompt_s": t3 - t2w}
        ev0, ev1 = h["ev"]
        if ev0 is not None:
            ev1.synchronize()
            tim["knn_gpu_s"] = ev0.elapsed_time(ev1) / 1e3
        return out, tim

    def plan(self, prompts: list[str]):
        """Retrieval + gating + prompt construction for a batch of user prompts."""
        return self.plan_finish(self.plan_launch(prompts))

    # ---- request-level interface used by ContinuousLoad (shared with AgentPipeline)
    def plan_requests(self, prompts: list[str]):
        """[(prompt, token ids or None (no evidence -> answered without the LLM), ctx)], timings"""
        return self.requests_of(*self.plan(prompts))

    @staticmethod
    def requests_of(plans, tim):
        return [(p, ids, (cit, ev)) for p, ids, cit, ev in plans], tim

    def finish_request(self, prompt: str, out_ids: list, ctx) -> RagAgentResult:
        if ctx is None:
            return RagAgentResult(prompt, 200, {"result": None, "citations": [], "note": NO_EVIDENCE_NOTE})
        return self.finish(prompt, out_ids, *ctx)

    def finish(self, prompt: str, out_ids: list, citations, evidence) -> RagAgentResult:
        raw = self.tok.decode(out_ids)
        tool_json = extract_json_object(raw)
        status, body = dispatch_rag_tool(self.k8s, tool_json, citations, evidence, self.cfg)
        return RagAgentResult(prompt, status, body, citations, 0, len(out_ids), raw)

    def run_batch(self, prompts: list[str], params) -> list[RagAgentResult]:
        """Synchronous batch through an in-process LLMEngine."""
        plans, tim = self.plan(prompts)
        todo = [(i, ids) for i, (_, ids, _, _) in enumerate(plans) if ids is not None]
        seqs = {}
        for i, ids in todo:
            seqs[i] = self.llm.add_request(ids, params.__class__(**{**params.__dict__}))
        t0 = time.perf_counter()
        self.llm.run_until_done(list(seqs.values()))
        tgen = time.perf_counter() - t0
        results = []
        for i, (p, ids, cit, ev) in enumerate(plans):
            if ids is None:
                results.append(RagAgentResult(p, 200, {"result": None, "citations": [], "note": NO_EVIDENCE_NOTE}))
                continue
            s = seqs[i]
            r = self.finish(p, s.output_ids, cit, ev)
            r.prompt_tokens = len(ids)
            r.timings = {**tim, "generate_s": tgen, **s.metrics()}
            results.append(r)
        return results

    def run_continuous(self, next_queries, params, concurrency: int, n_complete: int,
                       admit_chunk: int = 16, on_done=None) -> list[RagAgentResult]:
        """One-shot closed-loop run (see :class:`ContinuousLoad`); drains at the end."""
        load = ContinuousLoad(self, next_queries, params, concurrency, admit_chunk)
        out = load.run(n_complete, on_done)
        load.drain()
        return out


class ContinuousLoad:
    """Closed-loop serving load: keep ``concurrency`` requests in flight in the
    continuous-batching engine; as requests finish, new ones are retrieved and
    admitted (in chunks of ``admit_chunk`` so the query-encoder / kNN launches are
    batched).  Decode tokens of running requests share every step with other
    requests' chunked prefill, so the weights streamed for decode are amortised by
    prefill compute.  ``run`` can be called repeatedly (warm-up, then the timed
    window) without draining the in-flight requests in between; latency is measured
    from the moment a slot frees and its replacement's retrieval starts, to completion.

    Admission planning (query encoder + kNN on a side HIP stream, gating, prompt
    JSON, tokenisation) runs inline on the engine thread between pipelined steps
    (the device is then still busy with the step launched before it), or with
    ``threaded=True`` on a planner thread, as an HTTP front-end's handler threads
    would, proceeding while the engine thread waits on the device.  Measured on
    MI355X (1024 completions, A/B twice): inline 100.4 q/s, threaded 99.4 -- GIL
    hand-offs cost the engine thread more than the overlap gains."""

    def __init__(self, pipe: RagAgentPipeline, next_queries, params, concurrency: int, admit_chunk: int = 16,
                 threaded: bool = False, deferred: Optional[bool] = None):
        self.pipe, self.next_queries, self.params = pipe, next_queries, params
        self.concurrency, self.admit_chunk = concurrency, admit_chunk
        self.inflight: dict = {}
        self.host_s = {"plan": 0.0, "step": 0.0, "finish": 0.0}  # wall time by phase
        self.threaded = threaded
        # deferred=True: retrieval is launched without waiting; its requests are admitted at
        # the first loop iteration after its top-k landed (no host block on the device, one
        # engine step later than a blocking plan).  LK_ADMIT_DEFERRED=1 selects it.
        self.deferred = (os.environ.get("LK_ADMIT_DEFERRED", "0") == "1") if deferred is None else deferred
        self.deferred = self.deferred and hasattr(pipe, "plan_launch")  # pipelines without retrieval: inline
        self._launched: list = []  # (t_adm, plan handle) in launch order
        self._todo: "queue.Queue" = queue.Queue()
        self._ready: "queue.Queue" = queue.Queue()
        self._planning = 0  # queries submitted to the planner and not yet admitted
        self._thread = None
        self._error = None

    # ---- planner
    def _side_stream(self):
        dev = getattr(getattr(self.pipe.llm, "model", None), "device", None)
        if dev is None or dev.type != "cuda":
            return None
        if getattr(self, "_side", None) is None:
            # stream priority knob for the retrieval kernels: a high-priority stream
            # (-1) measured slower on MI355X (98.7 vs 100.8 q/s, kNN 10.4 vs 5.5 ms)
            prio = int(os.environ.get("LK_ADMIT_STREAM_PRIORITY", "0"))
            self._side = torch.cuda.Stream(dev, priority=prio)
        return self._side

    def _plan(self, qs):
        side = self._side_stream()
        t_adm = time.perf_counter()
        if side is not None:
            with torch.cuda.stream(side):
                reqs, tim = self.pipe.plan_requests(qs)
        else:
            reqs, tim = self.pipe.plan_requests(qs)
        return t_adm, time.perf_counter() - t_adm, reqs, tim

    def _launch_plan(self, qs):
        side = self._side_stream()
        t_adm = time.perf_counter()
        if side is not None:
            with torch.cuda.stream(side):
                h = self.pipe.plan_launch(qs)
        else:
            h = self.pipe.plan_launch(qs)
        self.host_s["plan"] += time.perf_counter() - t_adm
        self._launched.append((t_adm, h))

    def _finish_launched(self, block: bool):
        """Plans whose top-k landed (all of them when ``block``), in launch order."""
        while self._launched and (block or self.pipe.plan_ready(self._launched[0][1])):
            t_adm, h = self._launched.pop(0)
            t0 = time.perf_counter()
            reqs, tim = self.pipe.requests_of(*self.pipe.plan_finish(h))
            self._ready.put((t_adm, time.perf_counter() - t0, reqs, tim))

    def _planner(self):
        while True:
            qs = self._todo.get()
            if qs is None:
                return
            try:
                self._ready.put(self._plan(qs))
            except BaseException as e:  # surfaced on the engine thread
                self._error = e
                self._ready.put(None)

    def _submit(self, qs):
        self._planning += len(qs)
        if self.deferred and not self.threaded:
            self._launch_plan(qs)
            return
        if not self.threaded:
            self._ready.put(self._plan(qs))
            return
        if self._thread is None:
            self._thread = threading.Thread(target=self._planner, name="lk-admission", daemon=True)
            self._thread.start()
        self._todo.put(qs)

    def _admit_ready(self, done, block: bool):
        if self._launched:
            self._finish_launched(block)
        while True:
            try:
                item = self._ready.get(block=block)
            except queue.Empty:
                return
            block = False
            if item is None:
                raise RuntimeError("admission planner failed") from self._error
            t_adm, dt, reqs, tim = item
            self.host_s["plan"] += dt
            self._planning -= len(reqs)
            for p, ids, ctx in reqs:
                if ids is None:
                    done.append(self.pipe.finish_request(p, [], None))
                    continue
                seq = self.pipe.llm.add_request(ids, self.params.__class__(**{**self.params.__dict__}))
                seq.arrival = t_adm
                self.inflight[seq.req_id] = (seq, p, ids, ctx, tim)

    def run(self, n_complete: int, on_done=None) -> list[RagAgentResult]:
        """Pipelined engine steps (``LLMEngine.step_pipelined``: step N+1's forward is
        enqueued before the host waits for step N) with admission planned on the
        planner thread meanwhile."""
        pipe = self.pipe
        llm = pipe.llm
        done: list[RagAgentResult] = []
        old_switch = sys.getswitchinterval()
        # the engine thread re-takes the GIL within 0.5 ms of its device wait returning
        sys.setswitchinterval(min(old_switch, 0.0005))

        def reap():
            for rid in [r for r, v in self.inflight.items() if v[0].finished]:
                seq, p, ids, ctx, tim = self.inflight.pop(rid)
                r = pipe.finish_request(p, seq.output_ids, ctx)
                r.prompt_tokens = len(ids)
                r.timings = {**tim, **seq.metrics(), "e2e_s": time.perf_counter() - seq.arrival}
                done.append(r)
                if on_done is not None:
                    on_done(r)

        try:
            while len(done) < n_complete:
                free = self.concurrency - len(self.inflight) - self._planning
                note = ""
                if free >= min(self.admit_chunk, self.concurrency) or (not self.inflight and not self._planning):
                    self._submit(self.next_queries(free))
                    note = "plan"
                # nothing to run: wait for the planner instead of spinning
                n_in = len(self.inflight)
                self._admit_ready(done, block=not llm.has_work() and not self.inflight)
                if len(self.inflight) != n_in:
                    note += "+admit"
                if note:  # step traces tag the launch that follows this host work (bench.py)
                    llm.trace_note = note
                t_st = time.perf_counter()
                if llm.has_work():
                    llm.step_pipelined()
                else:
                    llm.flush()
                t_fin = time.perf_counter()
                self.host_s["step"] += t_fin - t_st
                reap()
                self.host_s["finish"] += time.perf_counter() - t_fin
            llm.flush()
            reap()
        finally:
            sys.setswitchinterval(old_switch)
        return done

    def drain(self):
        if self._thread is not None:
            self._todo.put(None)
            self._thread.join()
            self._thread = None
        while not self._ready.empty():
            self._ready.get()
        self._launched.clear()
        self._planning = 0
        for seq, *_ in self.inflight.values():
            self.pipe.llm.abort(seq.req_id)
        self.inflight.clear()
