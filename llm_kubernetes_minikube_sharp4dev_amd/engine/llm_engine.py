"""The generation engine: request admission, the step loop, stop conditions and
streaming callbacks.  ``AsyncLLMEngine`` runs the step loop on a background thread
for the HTTP server (one engine per GPU / TP group; DP replicas are routed by
``parallel.router``)."""
from __future__ import annotations

import asyncio
import collections
import os
import threading
import time
from typing import Callable, Optional

import torch

from ..utils import metrics as M
from ..utils.logging import get_logger
from .block_manager import make_allocator
from .model_runner import ModelRunner
from .sampling import Sampler, SamplingParams
from .scheduler import Scheduler
from .sequence import Sequence, Status

log = get_logger("engine")


def _plain_greedy(p: SamplingParams) -> bool:
    return p.is_greedy and p.logits_processor is None and (p.repeat_penalty == 1.0 or p.repeat_last_n == 0)


# order of the pipelined step's phases: "csl" (default) collect -> sample -> launch, or the
# round-2 "lcs" launch -> collect -> sample (A/B knob)
PIPELINE_ORDER = os.environ.get("LK_PIPELINE", "csl")

# grammar jump-forward (LK_JUMP_FORWARD=0 disables): tokens a request's grammar leaves exactly
# one choice for are appended by the host as soon as the token before them is known, and run
# through the model together as one extend chunk instead of one decode step each
JUMP_FORWARD = os.environ.get("LK_JUMP_FORWARD", "1") != "0"

# engine steps between polls of the stream-K GEMM's give-up word
GEMM_HEALTH_EVERY = int(os.environ.get("LK_GEMM_HEALTH_EVERY", "512"))


def _jump_ok(p: SamplingParams) -> bool:
    """Forced tokens can be appended without sampling: a grammar is set, and no repeat
    penalty reads the device history ring the sampler kernel appends to (host-appended
    tokens would be missing from it)."""
    return p.logits_processor is not None and (p.repeat_penalty == 1.0 or p.repeat_last_n == 0)


def _small_buckets() -> tuple:
    """LK_SMALL_STEP_ALIGN: "1" = the decode GEMMs' row buckets (64, 128, 192, 256), or an
    explicit comma list; unset / "0" = off (Scheduler.small_buckets)."""
    v = os.environ.get("LK_SMALL_STEP_ALIGN", "0")
    if v in ("", "0"):
        return ()
    if v == "1":
        return (64, 128, 192, 256)
    return tuple(int(x) for x in v.split(","))


class LLMEngine:
    def __init__(self, model, tokenizer=None, block_size: int = 16, max_model_len: int = 8192,
                 max_num_seqs: int = 256, max_num_batched_tokens: int = 65536,
                 enable_prefix_caching: bool = True, use_graphs: bool = True, num_blocks: Optional[int] = None,
                 kv_cache_gb: Optional[float] = None, gpu_memory_fraction: float = 0.85, seed: int = 0,
                 eos_ids: Optional[set] = None, _runner: Optional[ModelRunner] = None, token_align: int = 256,
                 token_align_wave: int = 0, prefill_hold: Optional[int] = None):
        self.model = model
        self.tokenizer = tokenizer
        self.runner = _runner or ModelRunner(model, block_size, max_model_len, max_num_seqs, num_blocks,
                                             kv_cache_gb, gpu_memory_fraction, use_graphs)
        self.allocator = make_allocator(self.runner.num_blocks, block_size, enable_prefix_caching)
        if prefill_hold is None:
            # new prefill waits up to 4 steps for a full 4096-token step while >= 64 decode rows keep
            # the GPU busy: the prefill GEMMs cost ~10 % less per row at 4,096 rows than at ~2,500
            # (RAG bench, same box: 109.90 / 109.80 vs 108.92 / 108.73 q/s, p50 / p90 -10 / -15 ms,
            # p99 +10 ms; agent workload q/s neutral, profiles/r5_prefill_hold/)
            prefill_hold = int(os.environ.get("LK_PREFILL_HOLD", "4"))
        self.scheduler = Scheduler(self.allocator, block_size, max_num_seqs, max_num_batched_tokens, max_model_len,
                                   token_align, token_align_wave, prefill_hold,
                                   int(os.environ.get("LK_HOLD_MIN_DECODE", "64")),
                                   float(os.environ.get("LK_HOLD_FILL", "1.0")),
                                   _small_buckets(), int(os.environ.get("LK_HOLD_SMALL", "0")))
        self.sampler = Sampler(model.cfg.vocab_size, seed, history_len=max_model_len)
        self.max_model_len = max_model_len
        if eos_ids is None:
            eos_ids = set(tokenizer.eos_ids) if tokenizer is not None else set(model.cfg.eos_token_ids)
        self.eos_ids = set(eos_ids)
        self.lock = threading.RLock()
        # new requests land here without the engine lock (the lock is held across a step's
        # device wait: an HTTP event loop admitting a request must not stall behind it);
        # the step loop moves them into the scheduler at its next launch
        self._inbox: collections.deque = collections.deque()
        self.steps = 0
        self.launches = 0
        self._inflight = None  # the launched-and-sampled step not yet collected (step_pipelined)
        self._pending = None   # the launched step not yet sampled (step_pipelined, LK_PIPELINE=csl)
        # optional per-step trace: (prefill tokens, decode rows, wall seconds) -- bench.py
        self.step_trace: Optional[list] = None
        self._trace_end_ev = None  # the last traced step's ids-copy event (device idle before the next)
        self._trace_lazy = None    # (trace index, start, end) of a rowless step timed at the next one
        self._last_ids_ev = None   # the most recently recorded ids-copy event (starvation check)
        self.trace_note = ""       # caller's tag for the host work before the next launch (bench)

    # ------------------------------------------------------------------ API
    def add_request(self, prompt_ids: list, params: Optional[SamplingParams] = None,
                    req_id: Optional[str] = None, on_token: Optional[Callable] = None) -> Sequence:
        params = params or SamplingParams()
        seq = Sequence(list(prompt_ids), params)
        if req_id:
            seq.req_id = req_id
        seq.on_token = on_token
        seq.step_arrival = self.launches
        budget = self.max_model_len - len(seq.prompt_ids)
        if budget <= 0:
            raise ValueError("prompt longer than max_model_len")
        params.max_tokens = min(params.max_tokens, budget)
        self._inbox.append(seq)  # deque.append is atomic: no lock on the caller's thread
        M.REQUESTS.inc()
        return seq

    def _drain_inbox(self):
        """Move newly added requests into the scheduler (caller holds ``self.lock``)."""
        while self._inbox:
            self.scheduler.add(self._inbox.popleft())

    def abort(self, req_id: str) -> bool:
        with self.lock:
            self._drain_inbox()
            return self.scheduler.abort(req_id)

    def has_work(self) -> bool:
        return bool(self._inbox) or self.scheduler.has_work()

    # ------------------------------------------------------------------ step
    # A step is three phases: _launch (schedule, build the inputs, enqueue the forward),
    # _sample (grammar masks on the host + the sampling kernels, then a non-blocking
    # copy of the ids to pinned memory and an event), _collect (wait for that event,
    # append the tokens, stop conditions, callbacks, prefix-cache publishing).
    #
    #   step()            launch -> sample -> collect: every token is on the host when
    #                     it returns (server / tests / run_until_done).
    #   step_pipelined()  launch(N+1) -> collect(N) -> sample(N+1): the forward of step
    #                     N+1 is enqueued before the host waits for step N, its decode
    #                     inputs gathered on the device from step N's ids, so the GPU
    #                     never idles across the host's per-step work (stop checks,
    #                     grammar masks, scheduling, input building, admission).  A
    #                     request finishing by length is not stepped speculatively; one
    #                     stopping on EOS / a stop string wastes one row of one step.
    #                     Default order (LK_PIPELINE=csl): collect(N) -> sample(N+1) ->
    #                     launch(N+2), the same one-step-in-flight invariant rotated so that
    #                     the caller's per-step work (reaping finished requests, admission)
    #                     runs AFTER the next forward is enqueued: the device then holds two
    #                     forwards of work while the host does it, instead of waiting for it
    #                     (a kernel trace of the headline showed ~0.7 ms of device idle per
    #                     7 ms decode step with the lcs order, profiles/r3_gaps/).

    @torch.inference_mode()
    def step(self) -> list:
        """One synchronous scheduler iteration.  Returns the sequences that got a token."""
        out = self.flush()
        nxt = self._launch()
        if nxt is None:
            return out
        return out + self._collect(self._sample(nxt))

    @torch.inference_mode()
    def step_pipelined(self) -> list:
        """One pipelined iteration; returns the sequences that got a token (from the
        PREVIOUS launch).  Call :meth:`flush` when done.  Under tensor parallelism the
        worker ranks gather the in-flight inputs from their own copy of greedy ids, or
        from the driver's sampled ids broadcast over the TP group."""
        if PIPELINE_ORDER == "lcs":
            nxt = self._launch()
            out = self._collect(self._inflight) if self._inflight is not None else []
            self._inflight = self._sample(nxt) if nxt is not None else None
            return out
        out = self._collect(self._inflight) if self._inflight is not None else []
        self._inflight = self._sample(self._pending) if self._pending is not None else None
        self._pending = self._launch()
        return out

    @property
    def in_flight(self) -> bool:
        """A pipelined step is launched and not yet collected."""
        return self._inflight is not None or self._pending is not None

    @torch.inference_mode()
    def flush(self) -> list:
        """Collect the in-flight pipelined step(s), if any."""
        out = []
        if self._inflight is not None:
            p, self._inflight = self._inflight, None
            out = self._collect(p)
        if self._pending is not None:
            p, self._pending = self._pending, None
            out += self._collect(self._sample(p))
        return out

    def _launch(self):
        with self.lock:
            ts = time.perf_counter()
            self._drain_inbox()
            batch = self.scheduler.schedule()
            # requests that could never fit were finished by the scheduler
            if batch.empty:
                return None
            t0 = time.perf_counter()
            # plain greedy steps get token ids straight from the model (no fp32 logits;
            # under TP an all-gather of (max, argmax) pairs instead of the vocab)
            greedy = all(_plain_greedy(sq.params) for sq, _, _ in batch.items)
            ev0 = None
            # traced runs: did the device already finish everything queued before this launch
            # (then all of this launch's host preparation is device idle)?
            starved = (self.step_trace is not None and self._last_ids_ev is not None
                       and self._last_ids_ev.query())
            if self.step_trace is not None and self.model.device.type == "cuda":
                ev0 = torch.cuda.Event(enable_timing=True)  # GPU-side step start (after earlier work)
                ev0.record()
            rows, out = self.runner.forward_logits(batch.items, greedy)
            note, self.trace_note = self.trace_note, ""
            for seq, start, n in batch.items:
                seq.num_computed = start + n
                seq.steps_run += 1
                if seq.step_first is None:
                    seq.step_first = self.launches
            self.launches += 1
            return [batch, rows, out, greedy, ts, t0, time.perf_counter(), (ev0, note, starved)]

    def _sample(self, launched):
        batch, rows, out, greedy, ts, t0, t1, ev0n = launched
        ev0 = ev0n[0]
        host = ev = ids = None
        if rows:
            seqs = [s for s, _ in rows]
            ids = out if greedy else self.sampler(out, [s.params for s in seqs], [s.output_ids for s in seqs],
                                                  [s.req_id for s in seqs])
            if ids.is_cuda:
                host = torch.empty(ids.shape, dtype=ids.dtype, pin_memory=True)
                host.copy_(ids, non_blocking=True)
                ev = torch.cuda.Event(enable_timing=ev0 is not None)
                ev.record()
                self._last_ids_ev = ev
            else:
                host = ids
            for i, s in enumerate(seqs):
                if not s.discard_rows:  # a row whose token jump-forward already appended stays out
                    s.num_inflight, s.inflight_row = 1, i
            self.runner.prev_ids = ids
            self.runner.prev_sampled_rows = 0 if greedy else len(rows)
        elif ev0 is not None:
            # a step with no sampled rows (a prompt chunk that does not end its prompt): its end
            # still bounds the traced GPU time, so the next step's idle is not charged with it
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
        return (batch, rows, host, ev, ts, t0, t1, time.perf_counter(), ev0n)

    def _collect(self, pending) -> list:
        batch, rows, host, ev, ts, t0, t1, t1s, (ev0, launched_note, starved) = pending
        t2 = time.perf_counter()
        if rows and ev is not None:
            ev.synchronize()  # outside the lock: aborts and admissions never wait on the device
        with self.lock:
            out = []
            if rows:
                ids = host.tolist()
                now = t2 = time.perf_counter()
                for (seq, _), tid in zip(rows, ids):
                    if seq.discard_rows:
                        # the row predicted a token jump-forward appended meanwhile: its KV
                        # write (the previous token) is what the step was for
                        seq.discard_rows -= 1
                        continue
                    seq.num_inflight, seq.inflight_row = 0, -1
                    if seq.finished:
                        continue  # aborted, or stopped while this step was in flight
                    self._append(seq, int(tid), now)
                    if JUMP_FORWARD and not seq.finished and _jump_ok(seq.params):
                        self._jump(seq, now)
                    out.append(seq)
            for seq, _, _ in batch.items:
                if not seq.finished:
                    self.scheduler.publish_blocks(seq)
            self.steps += 1
            if self.steps % GEMM_HEALTH_EVERY == 0 and self.model.device.type == "cuda":
                self._check_gemm_health(self.model.device)
            if self.step_trace is not None:
                t3 = time.perf_counter()
                ndec = len(batch.items) - sum(1 for sq, st, n in batch.items if st < len(sq.prompt_ids))
                npre = sum(n for sq, st, n in batch.items if st < len(sq.prompt_ids))
                # (a rowless step's end event is not waited for: its GPU time is filled in at the
                # next traced step, whose own wait has completed it)
                done = bool(rows) and ev is not None  # this step's end was waited for
                if self._trace_lazy is not None and done:
                    k, e0, e1, pe = self._trace_lazy
                    if k < len(self.step_trace):
                        t = self.step_trace[k]
                        idl = max(0.0, pe.elapsed_time(e0) / 1e3) if pe is not None else 0.0
                        self.step_trace[k] = t[:7] + (e0.elapsed_time(e1) / 1e3, idl) + t[9:]
                    self._trace_lazy = None
                gpu = ev0.elapsed_time(ev) / 1e3 if (ev0 is not None and done) else 0.0
                # device idle between the previous traced step's ids copy and this step's start
                # marker: > 0 when the host reached this launch after the device ran dry
                idle = 0.0
                if ev0 is not None and ev is not None and not rows:
                    if self._trace_lazy is None:
                        self._trace_lazy = (len(self.step_trace), ev0, ev, self._trace_end_ev)
                elif ev0 is not None and self._trace_end_ev is not None and done:
                    idle = max(0.0, self._trace_end_ev.elapsed_time(ev0) / 1e3)
                if ev is not None:
                    self._trace_end_ev = ev
                # (prefill tokens, decode rows, step s, schedule s, prepare+launch s, sample+sync s, post s,
                #  GPU s from the step's first kernel to its ids copy, device idle before it, caller tag,
                #  device already idle when the launch began, total token rows of the step)
                self.step_trace.append((npre, ndec, t3 - t0, t0 - ts, t1 - t0,
                                        (t2 - t1) if rows else 0.0, (t3 - t2) if rows else 0.0, gpu, idle,
                                        launched_note, starved, batch.num_tokens))
            M.STEP_TOKENS.observe(batch.num_tokens)
            M.STEP_TIME.observe(time.perf_counter() - t0)
            M.KV_USAGE.set(self.allocator.usage())
            M.RUNNING.set(len(self.scheduler.running))
            return out

    @staticmethod
    def _check_gemm_health(device=None):
        """Fail loudly if a stream-K prefill GEMM gave up waiting for a partial tile since the
        last check (csrc/gemm.hip poisons such a tile with NaN; never expected: the wait is a
        bound instead of a hang), or a token id outside the vocabulary reached the embedding
        (csrc/step_ops.hip counts them).  Two 4-byte device reads per GEMM_HEALTH_EVERY steps."""
        from .. import ops

        if not ops.available():
            return
        errs = int(ops.lib().gemm_streamk(-1))
        if errs:
            raise RuntimeError(f"stream-K GEMM: {errs} partial-tile wait(s) timed out; outputs were poisoned")
        import torch

        with torch.cuda.device(device if device is not None else torch.cuda.current_device()):
            bad = int(ops.lib().embed_errors())  # this engine's device's counter
        if bad:
            raise RuntimeError(f"embedding: {bad} token id(s) outside the vocabulary were looked up (a tokenizer / "
                               f"model vocab mismatch); their rows were zero")

    def _jump(self, seq: Sequence, now: float):
        """Grammar jump-forward: append the tokens ``seq``'s grammar allows exactly one choice
        for (literal keys, punctuation, the rest of a unique tool name), so the model runs
        them as one extend chunk -- every forced token still gets its forward pass (its KV
        feeds the next sampled token) -- instead of spending a decode step on each.  The
        output is the one step-by-step decoding gives: a one-id mask makes that id the draw.
        A request's last token is always left to the sampler, so no forward pass of the
        step-by-step run is dropped.  If the step already in flight is computing the KV of
        the token just collected, that row's prediction is discarded at its collect."""
        p = seq.params
        inflight_kv = seq.num_computed >= seq.length  # the launched step writes the last token's KV
        room = min(p.max_tokens - len(seq.output_ids), self.max_model_len - seq.length) - 1
        n = 0
        while n < room:
            allowed = p.logits_processor(seq.output_ids)
            if allowed is None or len(allowed) != 1:
                break
            tid = int(allowed[0])
            if tid in self.eos_ids and not p.ignore_eos:
                break  # an end of sequence stays a sampled stop
            self._append(seq, tid, now)
            n += 1
            if seq.finished:  # a stop string completed
                return
        if n:
            seq.jumped += n
            if inflight_kv:
                seq.discard_rows += 1

    def _append(self, seq: Sequence, tid: int, now: float):
        if seq.first_token_at is None:
            seq.first_token_at = now
        seq.output_ids.append(tid)
        p = seq.params
        reason = None
        n = len(seq.output_ids)
        if not p.ignore_eos and tid in self.eos_ids and n > p.min_tokens:
            reason = "stop"
        elif n >= p.max_tokens:
            reason = "length"
        elif seq.length >= self.max_model_len:
            reason = "length"
        if p.stop and self.tokenizer is not None and reason is None:
            tail = self.tokenizer.decode(seq.output_ids[-32:])
            if any(s and s in tail for s in p.stop):
                reason = "stop"
        if reason:
            seq.step_finish = self.launches
            self.scheduler.finish(seq, reason)
            self.sampler.release(seq.req_id)
            M.GEN_TOKENS.inc(n)
        if seq.on_token is not None:
            try:
                seq.on_token(seq, tid, reason is not None)
            except Exception:  # pragma: no cover - a client callback must not kill the loop
                log.exception("on_token callback failed")

    def run_until_done(self, seqs: Optional[list] = None, max_steps: int = 10_000_000):
        steps = 0
        while self.has_work() and steps < max_steps:
            self.step()
            steps += 1
            if seqs is not None and all(s.finished for s in seqs):
                break

    def generate(self, prompts: list, params: Optional[SamplingParams] = None) -> list:
        """Synchronous batch generation over token-id prompts (list of lists)."""
        seqs = [self.add_request(p, params if params is not None else SamplingParams.greedy()) for p in prompts]
        self.run_until_done(seqs)
        return seqs


class _LoopMux:
    """Token hand-off from the engine thread to one asyncio loop: the tokens of a whole
    engine step (one per running stream) are queued under a lock and delivered by ONE
    ``call_soon_threadsafe`` wake-up, not one self-pipe write and loop wake-up per stream
    per token (128 per step at the serving point)."""

    def __init__(self, loop):
        self.loop = loop
        self.lock = threading.Lock()
        self.pending: list = []
        self.scheduled = False

    def push(self, q, item):
        with self.lock:
            self.pending.append((q, item))
            if self.scheduled:
                return
            self.scheduled = True
        self.loop.call_soon_threadsafe(self._drain)

    def _drain(self):
        with self.lock:
            items, self.pending, self.scheduled = self.pending, [], False
        for q, it in items:
            q.put_nowait(it)


class AsyncLLMEngine:
    """Background step loop + asyncio streaming for the HTTP front-end."""

    def __init__(self, engine: LLMEngine, request_timeout_s: Optional[float] = None, stall_s: float = 120.0):
        import sys

        from ..utils.watchdog import StepWatchdog

        # the step loop shares the GIL with the HTTP event loop: a short switch interval lets
        # it take the GIL back within ~0.2 ms of its GPU waits instead of the default 5 ms
        sys.setswitchinterval(min(sys.getswitchinterval(), 2e-4))
        self._muxes: dict = {}
        self.engine = engine
        self.request_timeout_s = request_timeout_s
        self._wake = threading.Event()
        self._stop = False
        self.watchdog = StepWatchdog("engine", stall_s=stall_s, on_stall=lambda dt: self._fail_all("stalled"))
        # LK_STEP_TRACE=N: trace every step (LLMEngine.step_trace) and log a summary per N traced
        # steps -- GPU time, device idle before launches, host time -- so a served engine's step
        # loop can be checked for a starved device the way bench.py's in-process runs are
        self._trace_every = int(os.environ.get("LK_STEP_TRACE", "0") or 0)
        if self._trace_every > 0:
            self.engine.step_trace = []
        self._thread = threading.Thread(target=self._loop, name="lk-engine", daemon=True)
        self._thread.start()

    def _log_trace(self):
        tr = self.engine.step_trace
        if not tr or len(tr) < self._trace_every:
            return
        self.engine.step_trace = []
        n = len(tr)
        log.info("step trace: %d steps (%d decode-only), GPU %.1f ms, device idle before launch %.1f ms "
                 "(%d launches found it idle), host step %.1f ms, mean prefill %d rows / decode %d rows",
                 n, sum(1 for t in tr if t[0] == 0), 1e3 * sum(t[7] for t in tr), 1e3 * sum(t[8] for t in tr),
                 sum(1 for t in tr if t[10]), 1e3 * sum(t[2] for t in tr), sum(t[0] for t in tr) // n,
                 sum(t[1] for t in tr) // n)

    @property
    def healthy(self) -> bool:
        return self.watchdog.healthy and self._thread.is_alive()

    def _fail_all(self, why: str):
        """Finish every in-flight request with an error token (-1) so no client hangs."""
        with self.engine.lock:
            self.engine._drain_inbox()
            for s in list(self.engine.scheduler.running) + list(self.engine.scheduler.waiting):
                self.engine.scheduler.abort(s.req_id)
                s.error = why
                if s.on_token:
                    s.on_token(s, -1, True)

    def _loop(self):
        from ..utils.pyprof import thread_profile

        with thread_profile("engine"):
            self._loop_body()

    def _loop_body(self):
        while not self._stop:
            if not self.engine.has_work():
                if self.engine.in_flight:
                    with self.watchdog.busy():
                        self.engine.flush()
                    continue
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                with self.watchdog.busy():
                    self.engine.step_pipelined()
                self.watchdog.beat()
                if self._trace_every:
                    self._log_trace()
            except Exception:  # pragma: no cover
                log.exception("engine step failed; aborting in-flight requests")
                self._fail_all("engine step failed")

    def shutdown(self):
        self._stop = True
        self._wake.set()
        self.watchdog.stop()
        if self._thread.is_alive() and self._thread is not threading.current_thread():
            self._thread.join(timeout=10)

    async def stream(self, prompt_ids: list, params: SamplingParams, req_id: Optional[str] = None,
                     timeout_s: Optional[float] = None):
        """Async generator of (token_id, finished, seq).  A request still running after
        ``timeout_s`` (default: the engine's ``request_timeout_s``) is aborted and
        ``asyncio.TimeoutError`` raised; a client that stops iterating (HTTP disconnect)
        aborts its request."""
        loop = asyncio.get_running_loop()
        q: asyncio.Queue = asyncio.Queue()
        timeout_s = timeout_s if timeout_s is not None else self.request_timeout_s
        deadline = loop.time() + timeout_s if timeout_s else None
        mux = self._muxes.get(id(loop))
        if mux is None or mux.loop is not loop:
            mux = self._muxes[id(loop)] = _LoopMux(loop)

        def cb(seq, tid, fin):
            mux.push(q, (tid, fin, seq))

        seq = self.engine.add_request(prompt_ids, params, req_id, cb)
        self._wake.set()
        try:
            while True:
                if deadline is None:
                    tid, fin, s = await q.get()
                else:
                    tid, fin, s = await asyncio.wait_for(q.get(), max(0.0, deadline - loop.time()))
                yield tid, fin, s
                if fin:
                    break
        finally:
            if not seq.finished:
                self.engine.abort(seq.req_id)

    async def generate(self, prompt_ids: list, params: SamplingParams, req_id: Optional[str] = None,
                       timeout_s: Optional[float] = None):
        last = None
        async for _, fin, s in self.stream(prompt_ids, params, req_id, timeout_s):
            last = s
        return last
