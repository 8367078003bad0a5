"""Continuous-batching scheduler with chunked prefill, prefix caching and
recompute preemption.

Each step has a token budget (``max_num_batched_tokens``).  Running decode
sequences are served first (1 token each, so latency-bound agent loops never wait
behind a long RAG prefill), then running prefill chunks, then new requests are
admitted FIFO while the budget and the KV block pool allow.  When the pool runs
dry the most recently admitted sequence is preempted (its blocks are freed and it
is recomputed later — usually mostly from the prefix cache).
"""
from __future__ import annotations

import os

import time
from collections import deque
from dataclasses import dataclass, field

from .block_manager import NoFreeBlocks
from .sequence import Sequence, Status


@dataclass
class ScheduledBatch:
    items: list = field(default_factory=list)   # (seq, start, n_tokens)

    @property
    def empty(self) -> bool:
        return not self.items

    @property
    def num_tokens(self) -> int:
        return sum(n for _, _, n in self.items)


class Scheduler:
    def __init__(self, allocator, block_size: int, max_num_seqs: int = 256,
                 max_num_batched_tokens: int = 65536, max_model_len: int = 8192, token_align: int = 256,
                 token_align_wave: int = 0, prefill_hold: int = 0, hold_min_decode: int = 64,
                 hold_fill: float = 1.0, small_buckets: tuple = (), hold_small: int = 0):
        self.alloc = allocator
        # weight-streaming steps (<= small_buckets[-1] rows): prompt prefill is trimmed so the
        # step stays in the row bucket its decode / extend rows already need (the decode GEMMs'
        # cost steps up with the padded row count, 64 / 128 / 192 / 256); the trimmed prompt
        # tokens lead the next step.  () = off
        self.small_buckets = tuple(sorted(small_buckets))
        # prefill hold-back: while at least hold_min_decode decode rows keep the GPU busy, new
        # prefill waits (up to prefill_hold consecutive steps) until it fills the step's token
        # budget (hold_fill x max_num_batched_tokens): the prefill GEMMs then run on whole waves
        # of 256x256 tiles instead of a partial step's 1.3-1.8 waves, and the small remainders
        # of an admission chunk ride in the next full step instead of a step of their own
        self.prefill_hold = prefill_hold
        self.hold_min_decode = hold_min_decode
        self.hold_fill = hold_fill
        # ... except that a held step may still take prompt tokens up to hold_small rows in total:
        # it streams every weight once anyway (the weight-streaming GEMMs serve <= 256 rows), so a
        # few hundred prompt rows ride in it for about half their cost in a full step
        self.hold_small = hold_small
        self._held = 0  # consecutive steps that held prefill back
        # mixed steps: trim prefill chunks so the step's row count is a multiple of the
        # prefill GEMM's 256-row macro tile (a 3852-row step runs 16 row tiles, the 16th
        # nearly empty); the trimmed tokens lead the next step
        self.token_align = token_align
        # ... and, past token_align_wave rows, to a multiple of it: with 256 x 256 tiles a
        # 4096-row step fills the chip's 256 CUs exactly once on the N = 4096 projections
        # (o / down), a 5120-row step runs 1.25 waves of them
        self.token_align_wave = token_align_wave
        # ... but only in steps with at least this many decode rows: they guarantee the next step
        # runs anyway, so the trimmed tokens ride in it.  A step of (almost) only prefill -- low
        # load, e.g. one request in flight -- would otherwise split a prompt's last chunk into a
        # step of its own: one more weight pass on the request's critical path (batch 1: a 627-row
        # prompt ran as 512 + 115 rows, ~4 ms of its time to first token)
        self.align_min_decode = int(os.environ.get("LK_ALIGN_MIN_DECODE", "32"))
        self.bs = block_size
        self.max_num_seqs = max_num_seqs
        self.max_tokens = max_num_batched_tokens
        self.max_model_len = max_model_len
        self.waiting: deque[Sequence] = deque()
        self.running: list[Sequence] = []

    def add(self, seq: Sequence):
        if len(seq.prompt_ids) >= self.max_model_len:
            raise ValueError(f"prompt of {len(seq.prompt_ids)} tokens exceeds max_model_len={self.max_model_len}")
        self.waiting.append(seq)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    # -------------------------------------------------------------- blocks
    def _ensure(self, seq: Sequence, total_tokens: int) -> bool:
        need = (total_tokens + self.bs - 1) // self.bs - len(seq.block_table)
        got = []
        try:
            for _ in range(need):
                got.append(self.alloc.allocate())
        except NoFreeBlocks:
            self.alloc.free_all(got)
            return False
        seq.block_table.extend(got)
        return True

    def release(self, seq: Sequence):
        self.alloc.free_all(seq.block_table)
        seq.block_table = []

    def _preempt(self, seq: Sequence):
        self.release(seq)
        seq.num_computed = 0
        seq.num_hashed_blocks = 0
        seq.last_hash = 0
        seq.status = Status.WAITING
        seq.num_preemptions += 1
        self.waiting.appendleft(seq)

    def _admit_prefix(self, seq: Sequence):
        if seq.num_computed == 0 and not seq.block_table:
            ids = seq.tokens(0, seq.length)
            blocks, parent = self.alloc.match_prefix(ids)
            if blocks:
                seq.block_table = list(blocks)
                seq.num_computed = len(blocks) * self.bs
                seq.num_hashed_blocks = len(blocks)
                seq.last_hash = parent
                seq.num_cached_prefix = max(seq.num_cached_prefix, seq.num_computed)

    # -------------------------------------------------------------- schedule
    @staticmethod
    def _generating(seq: Sequence) -> bool:
        """Decode rows and extend chunks of generated tokens (not prompt prefill)."""
        return seq.is_decode or (seq.num_computed >= len(seq.prompt_ids) and seq.output_ids)

    def _hold_prefill(self) -> bool:
        if not self.prefill_hold or self._held >= self.prefill_hold:
            return False
        dec = pre = 0
        for s in self.running:
            if s.done_after_inflight:
                continue
            if self._generating(s):
                dec += s.pending
            else:
                pre += s.pending
        if dec < self.hold_min_decode or not (pre or self.waiting):
            return False
        room = self.max_num_seqs - len(self.running)
        for k, s in enumerate(self.waiting):
            if k >= room:
                break
            pre += s.length - s.num_computed
        return dec + pre < self.hold_fill * self.max_tokens

    def schedule(self) -> ScheduledBatch:
        batch = ScheduledBatch()
        budget = self.max_tokens
        # decode first, then extend chunks of generated tokens, then in-flight prefill chunks
        # (stable within each class)
        self.running.sort(key=lambda s: 0 if s.is_decode else (1 if self._generating(s) else 2))
        hold = self._hold_prefill()
        self._held = self._held + 1 if hold else 0
        i = 0
        while i < len(self.running) and budget > 0:
            seq = self.running[i]
            if seq.done_after_inflight or seq.length + seq.num_inflight >= self.max_model_len:
                i += 1  # finishes when its in-flight token is collected
                continue
            cap = budget
            if hold and not self._generating(seq):
                cap = min(budget, self.hold_small - (self.max_tokens - budget))
                if cap <= 0:
                    break  # prefill chunks sort last: all held this step
            n = min(seq.pending, cap)
            if not self._ensure(seq, seq.num_computed + n):
                victim = self.running.pop()
                self._preempt(victim)
                if victim is seq:
                    break
                continue
            batch.items.append((seq, seq.num_computed, n))
            budget -= n
            i += 1

        def admit_cap() -> int:
            return min(budget, self.hold_small - (self.max_tokens - budget)) if hold else budget

        while self.waiting and admit_cap() > 0 and len(self.running) < self.max_num_seqs:
            seq = self.waiting[0]
            if seq.num_inflight:
                break  # preempted with a token in flight: re-admit once it is collected
            self._admit_prefix(seq)
            n = min(seq.pending, admit_cap())
            if not self._ensure(seq, seq.num_computed + n):
                if not self.running and not batch.items:
                    # nothing else holds blocks: this request can never fit
                    self.waiting.popleft()
                    self.release(seq)
                    seq.status = Status.FINISHED
                    seq.finish_reason = "error: kv cache too small"
                break
            self.waiting.popleft()
            seq.status = Status.RUNNING
            if seq.prefill_started_at is None:
                seq.prefill_started_at = time.perf_counter()
            self.running.append(seq)
            batch.items.append((seq, seq.num_computed, n))
            budget -= n
        self._align(batch)
        self._align_small(batch)
        return batch

    def _align_small(self, batch: ScheduledBatch):
        if not self.small_buckets:
            return
        total = batch.num_tokens
        if total > self.small_buckets[-1]:
            return
        fixed = sum(n for seq, _, n in batch.items if self._generating(seq))
        if fixed == 0 or fixed == total:  # a pure prefill step, or nothing to trim
            return
        cap = next(b for b in self.small_buckets if b >= fixed)
        ex = total - cap
        if ex <= 0:
            return
        for k in range(len(batch.items) - 1, -1, -1):
            seq, st, n = batch.items[k]
            if self._generating(seq):
                continue
            cut = min(ex, n)
            if cut == n:
                del batch.items[k]  # the whole chunk waits for the next step (its blocks stay reserved)
            else:
                batch.items[k] = (seq, st, n - cut)
            ex -= cut
            if not ex:
                return

    def _align(self, batch: ScheduledBatch):
        a = self.token_align
        if not a:
            return
        total = batch.num_tokens
        if sum(1 for _, _, n in batch.items if n == 1) < self.align_min_decode:
            return
        if self.token_align_wave and total > self.token_align_wave:
            a = self.token_align_wave
        ex = total % a
        if total <= a or not ex:
            return
        for k in range(len(batch.items) - 1, -1, -1):
            seq, st, n = batch.items[k]
            if n > 1:  # a prefill chunk (decode rows are 1 token)
                cut = min(ex, n - 1)
                batch.items[k] = (seq, st, n - cut)
                ex -= cut
                if not ex:
                    return

    def publish_blocks(self, seq: Sequence):
        """Register newly completed full blocks in the prefix cache (only blocks whose
        token values the host already holds)."""
        full = min(seq.num_computed, seq.length) // self.bs
        while seq.num_hashed_blocks < full and seq.num_hashed_blocks < len(seq.block_table):
            j = seq.num_hashed_blocks
            toks = seq.tokens(j * self.bs, (j + 1) * self.bs)
            seq.last_hash = self.alloc.register(seq.block_table[j], seq.last_hash, toks)
            seq.num_hashed_blocks += 1

    def finish(self, seq: Sequence, reason: str):
        seq.status = Status.FINISHED
        seq.finish_reason = reason
        seq.finished_at = time.perf_counter()
        if seq in self.running:
            self.running.remove(seq)
        self.release(seq)

    def abort(self, req_id: str) -> bool:
        for q in (self.running, self.waiting):
            for s in list(q):
                if s.req_id == req_id:
                    if s in self.running:
                        self.running.remove(s)
                    else:
                        self.waiting.remove(s)
                    self.release(s)
                    s.status = Status.FINISHED
                    s.finish_reason = "abort"
                    s.finished_at = time.perf_counter()
                    return True
        return False
