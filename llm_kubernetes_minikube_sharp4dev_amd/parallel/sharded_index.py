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
    """One rank's contiguous row shard of the corpus.  ``group``: the process group whose ranks
    hold the other shards (the device group's all-gather), or ``host_group``: a CPU (gloo) group
    over which the per-rank top-k lists travel as host tensors -- the TP engine's control group,
    so the exchange never enters the device stream the step collectives are ordered on."""

    def __init__(self, corpus_shard: torch.Tensor, offset: int, group=None, norms: Optional[torch.Tensor] = None,
                 host_group=None):
        self.corpus = corpus_shard.contiguous()
        self.norms = norms if norms is not None else ops.row_norms(self.corpus)
        self.offset = offset
        self.group = group
        self.host_group = host_group
        g = host_group if host_group is not None else group
        self.world = dist.get_world_size(g) if dist.is_initialized() else 1

    @classmethod
    def from_full(cls, corpus: torch.Tensor, group=None):
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        lo, hi = shard_bounds(corpus.shape[0], rank, world)
        return cls(corpus[lo:hi], lo, group)

    @classmethod
    def for_tp(cls, corpus: torch.Tensor, tp):
        """Rank tp.rank's shard of a TP group (the exchange over its CPU control group)."""
        lo, hi = shard_bounds(corpus.shape[0], tp.rank, tp.size)
        return cls(corpus[lo:hi].clone(), lo, None, host_group=tp.ctrl if tp.size > 1 else None)

    def local(self, queries: torch.Tensor, k: int):
        """This shard's top-k (scores f32, GLOBAL ids int32; -1 pads)."""
        q = queries.to(self.corpus.device, self.corpus.dtype).contiguous()
        qn = ops.row_norms(q)
        if self.corpus.shape[0]:
            s, i = ops.knn_topk(self.corpus, self.norms, q, qn, k)
            s, i = s.to(q.device), i.to(q.device)
            i = torch.where(i >= 0, i + self.offset, i)
        else:
            s = torch.full((q.shape[0], k), float("-inf"), device=q.device)
            i = torch.full((q.shape[0], k), -1, dtype=torch.int32, device=q.device)
        return s, i

    def search(self, queries: torch.Tensor, k: int):
        if self.host_group is not None:
            s, i = self.local(queries, k)
            if self.world == 1:
                return s, i
            ss = [torch.empty_like(s, device="cpu") for _ in range(self.world)]
            ii = [torch.empty_like(i, device="cpu") for _ in range(self.world)]
            dist.all_gather(ss, s.cpu(), group=self.host_group)
            dist.all_gather(ii, i.cpu(), group=self.host_group)
            dev = queries.device if queries.is_cuda else s.device
            return ops.knn_merge(torch.cat(ss, 1).to(dev), torch.cat(ii, 1).to(dev), k)
        return self._search_group(queries, k)

    def _search_group(self, queries: torch.Tensor, k: int):
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
