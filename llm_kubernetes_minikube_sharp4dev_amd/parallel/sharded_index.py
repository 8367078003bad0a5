"""Corpus-sharded brute-force kNN across ranks (BASELINE.json config 4: 1M-doc kNN
resident in HBM; at 8 GPUs each holds 1/8 of the matrix).

Each rank scores its shard with the fused HIP cosine/top-k kernel, indices are
offset to global ids, the per-rank top-k (score, id) lists are all-gathered
(``nq x k`` pairs per rank: a few KiB, latency-bound on xGMI) and merged by the HIP
merge kernel with the same (score desc, id asc) order as a single-GPU search — so
sharded and unsharded results are identical (test_parallel_cpu)."""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from .. import ops


def shard_bounds(n: int, rank: int, world: int) -> tuple[int, int]:
    per = (n + world - 1) // world
    return min(n, rank * per), min(n, (rank + 1) * per)


class ShardedKnnIndex:
    def __init__(self, corpus_shard: torch.Tensor, offset: int, group=None, norms: Optional[torch.Tensor] = None):
        self.corpus = corpus_shard.contiguous()
        self.norms = norms if norms is not None else ops.row_norms(self.corpus)
        self.offset = offset
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    @classmethod
    def from_full(cls, corpus: torch.Tensor, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        lo, hi = shard_bounds(corpus.shape[0], rank, world)
        return cls(corpus[lo:hi], lo, group)

    def search(self, queries: torch.Tensor, k: int):
        q = queries.to(self.corpus.device, self.corpus.dtype).contiguous()
        qn = ops.row_norms(q)
        if self.corpus.shape[0]:
            s, i = ops.knn_topk(self.corpus, self.norms, q, qn, k)
            s, i = s.to(q.device), i.to(q.device)
            i = torch.where(i >= 0, i + self.offset, i)
        else:
            s = torch.full((q.shape[0], k), float("-inf"), device=q.device)
            i = torch.full((q.shape[0], k), -1, dtype=torch.int32, device=q.device)
        if self.world == 1:
            return s, i
        ss = [torch.empty_like(s) for _ in range(self.world)]
        ii = [torch.empty_like(i) for _ in range(self.world)]
        dist.all_gather(ss, s.contiguous(), group=self.group)
        dist.all_gather(ii, i.contiguous(), group=self.group)
        return ops.knn_merge(torch.cat(ss, 1), torch.cat(ii, 1), k)
