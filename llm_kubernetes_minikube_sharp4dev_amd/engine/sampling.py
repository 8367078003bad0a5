"""Sampling parameters (Ollama ``options`` semantics) and the batched sampler.

Fast paths: an all-greedy batch is one HIP argmax kernel over the logits; a batch
with temperatures but no top-k/top-p/penalty is one HIP Gumbel-max kernel.  Anything
else -- Ollama's defaults (temperature 0.8, top-k 40, top-p 0.9, repeat penalty 1.1 over
the last 64 tokens, which is what an OllamaSharp client gets: it sends no options) -- is
``ops.sample``: two HIP launches (csrc/sampling.hip lk_sample) driven by one int32
parameter row per sequence, with each sequence's generated tokens kept in a device
history ring that the kernel itself appends to (the host never builds a penalty
window, and with pipelined steps the ring already holds the token the host has not
collected yet).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Callable, Optional

import numpy as np
import torch

from .. import ops


@dataclass
class SamplingParams:
    temperature: float = 0.8
    top_k: int = 40
    top_p: float = 0.9
    repeat_penalty: float = 1.1
    repeat_last_n: int = 64
    seed: Optional[int] = None
    max_tokens: int = 256
    min_tokens: int = 0
    stop: list = field(default_factory=list)
    ignore_eos: bool = False
    # callable(generated_ids) -> allowed token-id tensor/list or None (constrained decoding)
    logits_processor: Optional[Callable] = None

    @classmethod
    def greedy(cls, max_tokens: int = 256, **kw) -> "SamplingParams":
        return cls(temperature=0.0, top_k=0, top_p=1.0, repeat_penalty=1.0, max_tokens=max_tokens, **kw)

    @classmethod
    def from_ollama(cls, options: Optional[dict], defaults=None, num_predict_default: int = 256) -> "SamplingParams":
        """Map an Ollama ``options`` dict (temperature, top_k, top_p, repeat_penalty,
        repeat_last_n, seed, num_predict, stop) onto SamplingParams."""
        o = dict(options or {})
        d = defaults
        sp = cls(
            temperature=float(o.get("temperature", d.temperature if d else 0.8)),
            top_k=int(o.get("top_k", d.top_k if d else 40)),
            top_p=float(o.get("top_p", d.top_p if d else 0.9)),
            repeat_penalty=float(o.get("repeat_penalty", d.repeat_penalty if d else 1.1)),
            repeat_last_n=int(o.get("repeat_last_n", d.repeat_last_n if d else 64)),
            seed=o.get("seed"),
        )
        n = int(o.get("num_predict", d.num_predict if d else -1))
        sp.max_tokens = num_predict_default if n is None or n < 0 else n
        stop = o.get("stop") or []
        sp.stop = [stop] if isinstance(stop, str) else list(stop)
        return sp

    @property
    def is_greedy(self) -> bool:
        return self.temperature <= 0.0 or self.top_k == 1


# grammar-constrained rows select over their allowed ids only (LK_SPARSE_SELECT=0: dense
# -inf mask over [rows, V] + full-row select, the path CPU tensors and top-k/top-p take)
SPARSE_SELECT = os.environ.get("LK_SPARSE_SELECT", "1") != "0"


class Sampler:
    def __init__(self, vocab_size: int, seed: int = 0, history_len: int = 256):
        self.vocab_size = vocab_size
        self.seed = seed
        # the device history ring holds a sequence's whole output (up to max_model_len), so
        # repeat_last_n > 256 and -1 (Ollama: the whole context) penalise the full history
        self.RING = max(256, -(-min(int(history_len), 32768) // 256) * 256)
        self.step = 0
        # processors return the same cached list objects for recurring grammar states:
        # memoise their int64 arrays (id -> (list, array); the list reference keeps the id valid)
        self._arr_cache: dict = {}

    def _as_array(self, allowed, V: int):
        """int64 array of the in-vocabulary ids of ``allowed`` (memoised for the recurring
        cached lists of a grammar)."""
        if isinstance(allowed, np.ndarray):
            a = allowed.astype(np.int64, copy=False)
            return a[(a >= 0) & (a < V)] if len(a) and (a.min() < 0 or a.max() >= V) else a
        hit = self._arr_cache.get(id(allowed))
        if hit is not None and hit[0] is allowed:
            return hit[1]
        a = np.asarray(allowed, dtype=np.int64)
        if len(a) and (a.min() < 0 or a.max() >= V):
            a = a[(a >= 0) & (a < V)]
        # every list, short ones too: the grammar states recur (literal / EOS lists)
        if len(self._arr_cache) > 8192:
            self._arr_cache.clear()
        self._arr_cache[id(allowed)] = (allowed, a)
        return a

    def _plan(self, rows: dict, B: int, dev) -> torch.Tensor:
        """Device int32 [B flags | B+1 offsets | allowed ids] of the constrained rows
        (flag 0 = unconstrained row) for the HIP select_allowed kernel.  Staged through a small
        ring of pinned buffers: a pageable host->device copy makes the host wait until the
        device queue reaches it (behind the step's forward), which would stall the pipelined
        engine's next launch."""
        order = sorted(rows)
        flags = np.zeros(B, dtype=np.int32)
        counts = np.zeros(B + 1, dtype=np.int64)
        for i in order:
            flags[i] = 1
            counts[i + 1] = len(rows[i])
        offs = np.cumsum(counts)
        ids = np.concatenate([rows[i] for i in order])
        plan = np.concatenate([flags, offs.astype(np.int32), ids.astype(np.int32)])
        if dev.type != "cuda":
            return torch.from_numpy(plan)
        ring = getattr(self, "_plan_ring", None)
        if ring is None:
            ring = self._plan_ring = [[None, None] for _ in range(4)]  # [pinned int32 buffer, event]
            self._plan_k = 0
        self._plan_k = (self._plan_k + 1) % len(ring)
        slot = ring[self._plan_k]
        if slot[1] is not None:
            slot[1].synchronize()  # the copy that last read this buffer has run
        if slot[0] is None or slot[0].numel() < plan.size:
            slot[0] = torch.empty(max(2 * plan.size, 1 << 14), dtype=torch.int32, pin_memory=True)
        slot[0][: plan.size].numpy()[:] = plan
        out = torch.empty(plan.size, dtype=torch.int32, device=dev)
        out.copy_(slot[0][: plan.size], non_blocking=True)
        slot[1] = torch.cuda.Event()
        slot[1].record()
        return out

    # ---------------------------------------------------------------- device sampler state
    RING = 256        # default history window per sequence (repeat_last_n is clamped to it)
    SLOTS = 1024      # sequences with a live ring (>= 2x max_num_seqs; LRU-evicted beyond)

    def _ring(self, dev):
        if getattr(self, "_hist", None) is None or self._hist.device != dev:
            self._hist = torch.zeros((self.SLOTS, self.RING), dtype=torch.int32, device=dev)
            self._hist_len = torch.zeros(self.SLOTS, dtype=torch.int32, device=dev)
            self._slot_of: dict = {}   # key -> (slot, request salt)
            self._lru: dict = {}       # key -> last step seen
            self._free = list(range(self.SLOTS - 1, -1, -1))
            self._assigned = 0
        return self._hist, self._hist_len

    def _slot(self, key, live: set):
        """(slot, reset, request salt) of sequence ``key``; a new key takes a free slot or,
        with none left, the least recently used one not in this batch."""
        hit = self._slot_of.get(key)
        if hit is not None:
            self._lru[key] = self.step
            return hit[0], 0, hit[1]
        if self._free:
            slot = self._free.pop()
        else:
            victim = min((k for k in self._lru if k not in live), key=self._lru.get)
            slot = self._slot_of.pop(victim)[0]
            self._lru.pop(victim)
        self._assigned += 1
        self._slot_of[key] = (slot, self._assigned)
        self._lru[key] = self.step
        return slot, 1, self._assigned

    def release(self, key):
        """Forget a finished sequence's ring (its slot is reused)."""
        hit = getattr(self, "_slot_of", {}).pop(key, None)
        if hit is not None:
            self._lru.pop(key, None)
            self._free.append(hit[0])

    def _device_sample(self, logits, params, keys):
        dev = logits.device
        hist, hist_len = self._ring(dev)
        B = logits.shape[0]
        prm = np.zeros((B, 8), dtype=np.int32)
        f = prm.view(np.float32)
        live = set(keys)
        seed = self.seed
        for i, (p, key) in enumerate(zip(params, keys)):
            slot, reset, salt = self._slot(key, live)
            f[i, 0] = 0.0 if p.is_greedy else p.temperature
            f[i, 1] = p.top_p
            f[i, 2] = p.repeat_penalty
            prm[i, 3] = p.top_k
            prm[i, 4] = min(p.repeat_last_n, self.RING) if p.repeat_last_n >= 0 else self.RING
            prm[i, 5] = slot
            prm[i, 6] = reset
            prm[i, 7] = (int(p.seed) if p.seed is not None else salt) & 0x7FFFFFFF
        prm_t = torch.from_numpy(prm)
        if dev.type == "cuda":
            prm_t = prm_t.pin_memory().to(dev, non_blocking=True)
        lg = logits if logits.dtype == torch.float32 and logits.is_contiguous() else logits.float().contiguous()
        return ops.sample(lg, prm_t, hist, hist_len, seed)

    def __call__(self, logits: torch.Tensor, params: list, histories: list, keys: Optional[list] = None) -> torch.Tensor:
        """logits [B, V] (f32) -> int32 token ids [B] (on logits.device).  ``keys``: a stable
        id per row's sequence (its history ring); default the row index."""
        self.step += 1
        B = logits.shape[0]
        dev = logits.device
        keys = list(keys) if keys is not None else list(range(B))
        # constrained decoding: on the GPU the select kernel scans only each row's allowed
        # ids (one host->device copy of the id lists); otherwise everything outside the
        # allowed set is masked -- one copy of the flat (row * V + token) positions and one
        # index_fill for the whole batch.  (An advanced-index assignment of a Python
        # scalar, mask[r, t] = 0.0, blocks the host until the device queue drains --
        # measured 15 ms behind a queued forward -- serialising the step pipelining.)
        V = logits.shape[1]
        rows = {}
        for i, p in enumerate(params):
            if p.logits_processor is not None:
                allowed = p.logits_processor(histories[i])
                if allowed is not None:
                    rows[i] = self._as_array(allowed, V)
        need_filter = any((not p.is_greedy) and (0 < p.top_k < V or p.top_p < 1.0) for p in params)
        need_penalty = any(p.repeat_penalty != 1.0 and p.repeat_last_n != 0 for p in params)
        plan = None
        if rows and not need_filter and not need_penalty and SPARSE_SELECT and ops.use_hip(logits):
            # selection straight over each row's allowed ids (HIP select_allowed): no mask
            plan = self._plan(rows, B, dev)
        elif rows:
            crow = list(rows)
            flat = [rows[i] + j * V for j, i in enumerate(crow)]
            idx = torch.from_numpy(np.concatenate(flat)).to(dev, non_blocking=True)
            mask = torch.full((len(crow), V), float("-inf"), device=dev, dtype=logits.dtype)
            mask.view(-1).index_fill_(0, idx, 0.0)
            sel = torch.from_numpy(np.asarray(crow, dtype=np.int64)).to(dev, non_blocking=True)
            logits.index_add_(0, sel, mask)
        if need_filter or need_penalty:
            # Ollama's chain (penalty -> top-k -> temperature -> top-p -> draw) in one fused kernel
            return self._device_sample(logits, params, keys)
        if all(p.is_greedy for p in params):
            if plan is not None:
                return ops.lib().select_allowed(logits, plan)
            return ops.select_tokens(logits)
        temps = torch.tensor([0.0 if p.is_greedy else p.temperature for p in params], dtype=torch.float32)
        seed = self.seed
        for p in params:
            if p.seed is not None:
                seed = int(p.seed)
                break
        if plan is not None:
            return ops.lib().select_allowed(logits, plan, temps.to(dev), seed, self.step)
        return ops.select_tokens(logits, temps.to(dev), seed=seed, step=self.step)
