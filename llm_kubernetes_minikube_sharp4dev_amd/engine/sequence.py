"""Request / sequence state for the continuous-batching engine."""
from __future__ import annotations

import enum
import itertools
import time
from dataclasses import dataclass, field
from typing import Callable, Optional

from .sampling import SamplingParams

_ids = itertools.count()


class Status(enum.Enum):
    WAITING = 0
    RUNNING = 1
    FINISHED = 2


@dataclass
class Sequence:
    prompt_ids: list
    params: SamplingParams
    req_id: str = field(default_factory=lambda: f"req-{next(_ids)}")
    output_ids: list = field(default_factory=list)
    block_table: list = field(default_factory=list)
    num_computed: int = 0          # tokens whose K/V are in the cache
    num_cached_prefix: int = 0     # tokens served by the prefix cache at admission
    num_hashed_blocks: int = 0     # full blocks already published to the prefix cache
    last_hash: int = 0
    # pipelined stepping (LLMEngine.step_pipelined): a token sampled on the device whose
    # value the host has not collected yet, and its row in that step's id tensor
    num_inflight: int = 0
    inflight_row: int = -1
    # grammar jump-forward (LLMEngine._jump): output tokens appended without sampling, and
    # launched rows whose predictions are void because such tokens were appended meanwhile
    jumped: int = 0
    discard_rows: int = 0
    status: Status = Status.WAITING
    finish_reason: Optional[str] = None
    arrival: float = field(default_factory=time.perf_counter)
    first_token_at: Optional[float] = None
    finished_at: Optional[float] = None
    prefill_started_at: Optional[float] = None
    num_preemptions: int = 0
    # engine-step accounting (LLMEngine launch counter): arrival, first scheduled, finish
    step_arrival: int = 0
    step_first: Optional[int] = None
    step_finish: Optional[int] = None
    steps_run: int = 0
    text: str = ""
    on_token: Optional[Callable] = None    # callback(seq, token_id, finished)
    user: dict = field(default_factory=dict)

    @property
    def length(self) -> int:
        return len(self.prompt_ids) + len(self.output_ids)

    @property
    def pending(self) -> int:
        """Tokens not yet run through the model (an in-flight sampled token counts)."""
        return self.length + self.num_inflight - self.num_computed

    def token_at(self, i: int) -> int:
        n = len(self.prompt_ids)
        return self.prompt_ids[i] if i < n else self.output_ids[i - n]

    def tokens(self, start: int, end: int) -> list:
        n = len(self.prompt_ids)
        if end <= n:
            return self.prompt_ids[start:end]
        if start >= n:
            return self.output_ids[start - n:end - n]
        return self.prompt_ids[start:] + self.output_ids[: end - n]

    @property
    def is_decode(self) -> bool:
        return self.pending == 1 and len(self.output_ids) + self.num_inflight > 0

    @property
    def done_after_inflight(self) -> bool:
        """The in-flight token is this request's last by length (max_tokens): the
        pipelined scheduler does not run a speculative step for it."""
        return self.num_inflight > 0 and len(self.output_ids) + self.num_inflight >= self.params.max_tokens

    @property
    def finished(self) -> bool:
        return self.status == Status.FINISHED

    def metrics(self) -> dict:
        end = self.finished_at or time.perf_counter()
        ttft = (self.first_token_at - self.arrival) if self.first_token_at else None
        n = len(self.output_ids)
        tpot = ((end - self.first_token_at) / (n - 1)) if (self.first_token_at and n > 1) else None
        return {"e2e_s": end - self.arrival, "ttft_s": ttft, "tpot_s": tpot, "prompt_tokens": len(self.prompt_ids),
                "output_tokens": n, "jumped_tokens": self.jumped, "cached_prefix_tokens": self.num_cached_prefix,
                "preemptions": self.num_preemptions,
                "steps_queued": (self.step_first - self.step_arrival) if self.step_first is not None else None,
                "steps_in_system": (self.step_finish - self.step_arrival) if self.step_finish is not None else None,
                "steps_run": self.steps_run}
