"""Micro-batching of concurrent embedding requests.

OllamaSharp-style clients embed ONE text per HTTP request (``Embedder.cs:34``); at 128
concurrent ``/agent_rag`` sessions that is 128 independent tiny encoder passes.
:class:`MicroBatcher` collects the requests that arrive within ``max_wait_s`` of the
first one and runs them as one packed varlen encoder forward on a worker thread, then
hands every request its own rows.  Up to ``max_inflight`` batches run at once: on a GPU
shared with the LLM engine a batch's latency is mostly its kernels waiting for CUs held
by the engine's step, so a second batch waiting alongside it (its own HIP stream) beats
queueing behind it."""
from __future__ import annotations

import asyncio
import concurrent.futures
from typing import Callable, Optional


class MicroBatcher:
    def __init__(self, fn: Callable[[list], "object"], max_items: int = 256, max_wait_s: float = 0.002,
                 max_inflight: int = 1):
        self.fn = fn                    # list of texts -> [len, D] tensor / array (rows in order)
        self.max_items = max_items
        self.max_wait_s = max_wait_s
        self.max_inflight = max(1, max_inflight)
        self._sem: Optional[asyncio.Semaphore] = None
        # the batches run on their own threads, never queued behind other work in the
        # event loop's default executor
        self._pool = concurrent.futures.ThreadPoolExecutor(self.max_inflight, thread_name_prefix="lk-batch")
        self._q: Optional[asyncio.Queue] = None
        self._task: Optional[asyncio.Task] = None
        self.batches = 0
        self.items = 0

    def _ensure(self):
        if self._task is None or self._task.done():
            self._q = asyncio.Queue()
            self._sem = asyncio.Semaphore(self.max_inflight)
            self._task = asyncio.get_running_loop().create_task(self._run())

    async def submit(self, texts: list):
        self._ensure()
        fut = asyncio.get_running_loop().create_future()
        await self._q.put((texts, fut))
        return await fut

    async def _run(self):
        loop = asyncio.get_running_loop()
        while True:
            first = await self._q.get()
            await self._sem.acquire()  # a batch slot; requests keep queueing meanwhile
            group = [first]
            n = len(first[0])
            deadline = loop.time() + self.max_wait_s
            while n < self.max_items:
                try:
                    item = self._q.get_nowait() if loop.time() >= deadline else \
                        await asyncio.wait_for(self._q.get(), deadline - loop.time())
                except (asyncio.TimeoutError, asyncio.QueueEmpty):
                    break
                group.append(item)
                n += len(item[0])
            loop.create_task(self._batch(group))

    async def _batch(self, group):
        texts = [t for g in group for t in g[0]]
        try:
            out = await asyncio.get_running_loop().run_in_executor(self._pool, self.fn, texts)
        except Exception as e:  # every waiter sees the failure
            for _, f in group:
                if not f.done():
                    f.set_exception(e)
            return
        finally:
            self._sem.release()
        self.batches += 1
        self.items += len(texts)
        r = 0
        for g, f in group:
            if not f.done():
                f.set_result(out[r:r + len(g)])
            r += len(g)
