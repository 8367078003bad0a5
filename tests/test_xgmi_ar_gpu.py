"""K14 one-shot all-reduce over IPC-mapped peer buffers: two processes share the box's
single MI355X (each maps the other's staging / signal buffers through HIP IPC, as the
ranks of an 8-GPU node map their peers' over xGMI).  Exact sums of small integers
(bf16-representable), several sizes, in place, and replayed from a captured hipGraph."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _vals(n, r, it=0):
    return ((torch.arange(n) * (r + 1) + it) % 64).to(torch.bfloat16)


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce

    tp = TPGroup(rank, world, dist.group.WORLD, ctrl=dist.group.WORLD, ranks=list(range(world)))
    ar = XgmiAllReduce(tp, 1 << 20)
    ok = []
    for n in (8, 4096, 24576, 8 * 4096 * 3, 1 << 19):
        x = _vals(n, rank).cuda()
        assert ar.eligible(x)
        ar.all_reduce_(x)
        torch.cuda.synchronize()
        want = sum(_vals(n, r).float() for r in range(world))
        ok.append(bool(torch.equal(x.float().cpu(), want)))
    # hipGraph: capture once, replay with new inputs (epochs advance on the device)
    buf = torch.zeros(8192, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        buf.copy_(_vals(8192, rank, 99).cuda())
        ar.all_reduce_(buf)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ar.all_reduce_(buf)
    for it in range(3):
        buf.copy_(_vals(8192, rank, it).cuda())
        g.replay()
        torch.cuda.synchronize()
        want = sum(_vals(8192, r, it).float() for r in range(world))
        ok.append(bool(torch.equal(buf.float().cpu(), want)))
    ok.append(ar.error() == 0)
    torch.save(ok, os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_xgmi_allreduce_two_processes():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        for r in range(2):
            ok = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)
            assert all(ok), f"rank {r}: {ok}"


def _timeout_worker(rank, world, port, out_dir):
    """Rank 1 skips the call (a dead / desynchronised peer): rank 0's kernel must give up
    after its bounded spin, set the error word and return -- no hung device."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce

    tp = TPGroup(rank, world, dist.group.WORLD, ctrl=dist.group.WORLD, ranks=list(range(world)))
    ar = XgmiAllReduce(tp, 1 << 20)
    x = _vals(4096, rank).cuda()
    ar.all_reduce_(x)  # one good call first
    torch.cuda.synchronize()
    res = {"first_ok": ar.error() == 0}
    dist.barrier()
    if rank == 0:
        t0 = time.time()
        ar.all_reduce_(x)  # the peer never arrives
        torch.cuda.synchronize()
        res.update(seconds=time.time() - t0, error=ar.error())
    torch.save(res, os.path.join(out_dir, f"t{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_xgmi_allreduce_missing_peer_times_out_with_error():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_timeout_worker, args=(2, _free_port(), d), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "t0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "t1.pt"), weights_only=True)
    assert r0["first_ok"] and r1["first_ok"]
    assert r0["error"] == 1 and r0["seconds"] < 60, r0
