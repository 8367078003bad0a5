"""Paged-KV block allocator with hash-chained prefix caching.

Every full block of a sequence gets a content hash chained over its prefix
(hash(parent_hash, block tokens)); a freed block stays addressable by its hash
until the allocator needs it again (LRU over free cached blocks).  All
``/agent_rag`` prompts share the same system-prompt prefix (``Minimal_RAG/
Program.cs:136-149``), so its KV is computed once and re-used by every request.

A C++ implementation with identical semantics lives in ``native`` (``_runtime``);
:func:`make_allocator` prefers it when built.
"""
from __future__ import annotations

from collections import OrderedDict, deque
from typing import Optional


def chain_hash(parent: int, tokens) -> int:
    h = 1469598103934665603 ^ (parent & 0xFFFFFFFFFFFFFFFF)
    for t in tokens:
        h ^= (int(t) + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


class NoFreeBlocks(RuntimeError):
    pass


class BlockAllocator:
    def __init__(self, num_blocks: int, block_size: int, prefix_caching: bool = True):
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.prefix_caching = prefix_caching
        self.ref = [0] * num_blocks
        self.free = deque(range(num_blocks))           # never-used or uncached blocks
        self.cached_free: OrderedDict[int, int] = OrderedDict()  # block -> hash (LRU order)
        self.hash_to_block: dict[int, int] = {}
        self.block_hash: dict[int, int] = {}
        self.hits = 0
        self.queries = 0

    # --------------------------------------------------------------- capacity
    @property
    def num_free(self) -> int:
        return len(self.free) + len(self.cached_free)

    def usage(self) -> float:
        return 1.0 - self.num_free / max(1, self.num_blocks)

    # --------------------------------------------------------------- alloc/free
    def allocate(self) -> int:
        if self.free:
            b = self.free.popleft()
        elif self.cached_free:
            b, h = self.cached_free.popitem(last=False)  # evict LRU cached block
            self.hash_to_block.pop(h, None)
            self.block_hash.pop(b, None)
        else:
            raise NoFreeBlocks()
        self.ref[b] = 1
        return b

    def free_block(self, b: int):
        self.ref[b] -= 1
        if self.ref[b] > 0:
            return
        h = self.block_hash.get(b)
        if h is not None and self.prefix_caching:
            self.cached_free[b] = h
        else:
            self.block_hash.pop(b, None)
            self.free.append(b)

    def free_all(self, blocks):
        for b in reversed(blocks):
            self.free_block(b)

    # --------------------------------------------------------------- prefix cache
    def match_prefix(self, tokens) -> tuple[list[int], int]:
        """Return (blocks, parent_hash) for the longest cached run of FULL blocks of
        ``tokens``; the blocks' refcounts are taken."""
        if not self.prefix_caching:
            return [], 0
        bs = self.block_size
        out, parent = [], 0
        nfull = len(tokens) // bs
        # never match the whole prompt: the last token must be recomputed for logits
        if nfull * bs == len(tokens):
            nfull -= 1
        for i in range(nfull):
            h = chain_hash(parent, tokens[i * bs:(i + 1) * bs])
            self.queries += 1
            b = self.hash_to_block.get(h)
            if b is None:
                break
            self.hits += 1
            if self.ref[b] == 0:
                self.cached_free.pop(b, None)
            self.ref[b] += 1
            out.append(b)
            parent = h
        return out, parent

    def register(self, block: int, parent: int, tokens) -> int:
        """Publish a just-filled block under its chained hash; returns the hash."""
        h = chain_hash(parent, tokens)
        if self.prefix_caching and h not in self.hash_to_block:
            self.hash_to_block[h] = block
            self.block_hash[block] = h
        return h


def make_allocator(num_blocks: int, block_size: int, prefix_caching: bool = True, prefer_native: bool = True):
    if prefer_native:
        try:
            from ..native import runtime

            if runtime.available():
                return runtime.NativeBlockAllocator(num_blocks, block_size, prefix_caching)
        except Exception:
            pass
    return BlockAllocator(num_blocks, block_size, prefix_caching)
