"""serving.batcher.MicroBatcher: requests arriving together share one call, every caller
gets its own rows in order, up to max_inflight batches overlap, failures reach every
waiter of the failed batch only."""
import asyncio
import threading
import time

import numpy as np
import pytest

from llm_kubernetes_minikube_sharp4dev_amd.serving.batcher import MicroBatcher


def _fn_factory(delay=0.05, fail_on=None):
    calls, live, peak = [], [0], [0]
    lock = threading.Lock()

    def fn(texts):
        with lock:
            live[0] += 1
            peak[0] = max(peak[0], live[0])
            calls.append(list(texts))
        time.sleep(delay)
        with lock:
            live[0] -= 1
        if fail_on is not None and fail_on in texts:
            raise RuntimeError("boom")
        return np.array([[float(t.split("-")[1])] for t in texts])

    return fn, calls, peak


@pytest.mark.parametrize("inflight", [1, 2])
def test_rows_in_order_and_overlap(inflight):
    fn, calls, peak = _fn_factory()
    b = MicroBatcher(fn, max_items=8, max_wait_s=0.005, max_inflight=inflight)

    async def main():
        return await asyncio.gather(*(b.submit([f"t-{i}", f"t-{i + 1000}"]) for i in range(24)))

    out = asyncio.run(main())
    for i, rows in enumerate(out):
        assert rows[:, 0].tolist() == [float(i), float(i + 1000)]
    assert len(calls) < 24                      # requests were batched
    assert all(len(c) <= 8 + 1 for c in calls)  # max_items bounds a batch (a request is never split)
    assert peak[0] <= inflight
    if inflight == 2:
        assert peak[0] == 2                     # batches overlapped


def test_failure_reaches_only_its_batch():
    fn, calls, _ = _fn_factory(delay=0.02, fail_on="t-3")
    b = MicroBatcher(fn, max_items=1, max_wait_s=0.0, max_inflight=2)

    async def main():
        return await asyncio.gather(*(b.submit([f"t-{i}"]) for i in range(6)), return_exceptions=True)

    res = asyncio.run(main())
    assert isinstance(res[3], RuntimeError)
    assert all(not isinstance(r, Exception) for i, r in enumerate(res) if i != 3)
