"""C++ block allocator == Python block allocator, operation by operation."""
import random

import pytest

from llm_kubernetes_minikube_sharp4dev_amd.engine.block_manager import BlockAllocator, NoFreeBlocks, chain_hash
from llm_kubernetes_minikube_sharp4dev_amd.native import runtime


@pytest.fixture(scope="module")
def native():
    try:
        runtime.build()
    except Exception as e:  # toolchain missing: the Python allocator is the fallback
        pytest.skip(f"native build unavailable: {e}")
    return runtime


def test_chain_hash_matches(native):
    m = native.load()
    for toks in ([], [1, 2, 3], list(range(16)), [128000, 7, 99999]):
        for parent in (0, 12345678901234567, 2**64 - 1):
            assert m.chain_hash(parent, toks) == chain_hash(parent, toks)


def test_random_ops_equivalent(native):
    rng = random.Random(0)
    py = BlockAllocator(24, 4, True)
    nat = native.NativeBlockAllocator(24, 4, True)
    owned_py, owned_nat = [], []
    prefixes = [[rng.randrange(50) for _ in range(rng.randrange(1, 20))] for _ in range(6)]
    for step in range(2000):
        op = rng.random()
        if op < 0.35:
            try:
                a = py.allocate()
            except NoFreeBlocks:
                a = None
            try:
                b = nat.allocate()
            except NoFreeBlocks:
                b = None
            assert a == b
            if a is not None:
                owned_py.append(a)
                owned_nat.append(b)
        elif op < 0.6 and owned_py:
            i = rng.randrange(len(owned_py))
            py.free_block(owned_py.pop(i))
            nat.free_block(owned_nat.pop(i))
        elif op < 0.8 and owned_py:
            toks = rng.choice(prefixes)
            blk = owned_py[rng.randrange(len(owned_py))]
            parent = rng.choice([0, 7])
            assert py.register(blk, parent, toks[:4]) == nat.register(blk, parent, toks[:4])
        else:
            toks = rng.choice(prefixes)
            a, pa = py.match_prefix(toks)
            b, pb = nat.match_prefix(toks)
            assert (a, pa) == (b, pb)
            owned_py.extend(a)
            owned_nat.extend(b)
        assert py.num_free == nat.num_free
    assert py.hits == nat.hits and py.queries == nat.queries


def test_slots_for(native):
    m = native.load()
    s, p = m.slots_for([5, 2, 9], 14, 4, 8)
    assert list(p) == [14, 15, 16, 17] and list(s) == [2 * 8 + 6, 2 * 8 + 7, 9 * 8 + 0, 9 * 8 + 1]
    with pytest.raises(IndexError):
        m.slots_for([1], 0, 9, 8)
