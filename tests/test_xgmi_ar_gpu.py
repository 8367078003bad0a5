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
# up to 8 ranks share the ONE device here: keep every rank's spinning workgroups co-resident
os.environ.setdefault("LK_XGMI_AR_BLOCKS", "32")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _vals(n, r, it=0, mod=32):
    # sums over up to 8 ranks stay below 256: exact in bf16
    return ((torch.arange(n) * (r + 1) + it) % mod).to(torch.bfloat16)


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


@pytest.mark.parametrize("world", [2, 8])
def test_xgmi_allreduce_two_processes(world):
    """World 8 = the production TP=8 group's signal layout (kMaxRanks slots per workgroup)."""
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
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


def _fused_worker(rank, world, port, out_dir):
    """Fused all-reduce + residual + RMSNorm vs the unfused chain (same one-shot all-reduce,
    then ops.rmsnorm with the residual): bit-identical outputs and residuals, eager and
    replayed from a hipGraph, at decode row counts and both Llama widths."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from llm_kubernetes_minikube_sharp4dev_amd import ops
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce

    tp = TPGroup(rank, world, dist.group.WORLD, ctrl=dist.group.WORLD, ranks=list(range(world)))
    ar = XgmiAllReduce(tp, 8 << 20)
    tp.xgmi = ar
    ok = []
    for T, H in ((1, 8192), (7, 4096), (64, 8192), (256, 8192), (100, 4096)):
        g = torch.Generator().manual_seed(T * 31 + H)
        xs = [torch.randn(T, H, generator=g).to(torch.bfloat16) for _ in range(world)]
        res0 = torch.randn(T, H, generator=g).to(torch.bfloat16)
        w = (torch.rand(H, generator=g) + 0.5).to(torch.bfloat16).cuda()
        x = xs[rank].cuda()
        # unfused: one-shot all-reduce, then the add + norm kernel
        xu, ru = x.clone(), res0.cuda()
        ar.all_reduce_(xu)
        yu = ops.rmsnorm(xu, w, 1e-5, residual=ru)
        # fused
        rf = res0.cuda()
        yf = tp.all_reduce_rmsnorm(x.clone(), rf, w, 1e-5)
        torch.cuda.synchronize()
        ok.append((T, H, bool(torch.equal(yf.cpu(), yu.cpu())), bool(torch.equal(rf.cpu(), ru.cpu()))))
    # graph capture + replay of the fused call
    T, H = 64, 8192
    xin = torch.zeros(T, H, dtype=torch.bfloat16, device="cuda")
    res = torch.zeros(T, H, dtype=torch.bfloat16, device="cuda")
    w = torch.ones(H, dtype=torch.bfloat16, device="cuda")
    out = torch.empty(T, H, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ar.all_reduce_rmsnorm_(xin, res, w, 1e-5, out)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        ar.all_reduce_rmsnorm_(xin, res, w, 1e-5, out)
    for it in range(3):
        g = torch.Generator().manual_seed(1000 + it)
        xs = [torch.randn(T, H, generator=g).to(torch.bfloat16) for _ in range(world)]
        r0 = torch.randn(T, H, generator=g).to(torch.bfloat16)
        xin.copy_(xs[rank].cuda())
        res.copy_(r0.cuda())
        gr.replay()
        torch.cuda.synchronize()
        tot = sum(v.float() for v in xs).to(torch.bfloat16)
        ru = r0.cuda()
        yu = ops.rmsnorm(tot.cuda(), w, 1e-5, residual=ru)
        ok.append(("graph", it, bool(torch.equal(out.cpu(), yu.cpu())), bool(torch.equal(res.cpu(), ru.cpu()))))
    ok.append(("err", 0, ar.error() == 0, ar.error() == 0))
    torch.save(ok, os.path.join(out_dir, f"f{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_xgmi_allreduce_rmsnorm_fused_bit_identical(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_fused_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            ok = torch.load(os.path.join(d, f"f{r}.pt"), weights_only=True)
            assert all(o[-1] and o[-2] for o in ok), f"rank {r}: {ok}"


def _two_shot_worker(rank, world, port, out_dir):
    """Two-shot (reduce-scatter + all-gather) forms on an odd world (3 processes on the one GPU):
    exact integer sums of the plain all-reduce (row counts below, at and above the world size),
    and the fused residual + RMSNorm form bit-identical to the one-shot fused kernel -- eager,
    interleaved with one-shot calls (shared per-workgroup epochs), and replayed from a hipGraph."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce

    tp = TPGroup(rank, world, dist.group.WORLD, ctrl=dist.group.WORLD, ranks=list(range(world)))
    two = XgmiAllReduce(tp, 16 << 20, two_shot=True)
    one = XgmiAllReduce(tp, 16 << 20, two_shot=False)
    ok = []
    for T, H in ((1, 8192), (2, 4096), (5, 4096), (64, 8192), (1000, 1024)):
        x = _vals(T * H, rank).view(T, H).cuda()
        two.all_reduce_(x)
        torch.cuda.synchronize()
        want = sum(_vals(T * H, r).float() for r in range(world)).view(T, H)
        ok.append(("plain", T, H, bool(torch.equal(x.float().cpu(), want))))
    x = _vals(24576, rank).cuda()  # 1-D message: viewed as rows of 8
    two.all_reduce_(x)
    torch.cuda.synchronize()
    ok.append(("plain1d", 24576, 0, bool(torch.equal(x.float().cpu(), sum(_vals(24576, r).float() for r in range(world))))))
    for T, H in ((3, 8192), (64, 8192), (257, 4096), (1024, 8192)):
        g = torch.Generator().manual_seed(T * 17 + H)
        xs = [torch.randn(T, H, generator=g).to(torch.bfloat16) for _ in range(world)]
        res0 = torch.randn(T, H, generator=g).to(torch.bfloat16)
        w = (torch.rand(H, generator=g) + 0.5).to(torch.bfloat16).cuda()
        r1, r2 = res0.cuda(), res0.cuda()
        y1 = one.all_reduce_rmsnorm_(xs[rank].cuda(), r1, w, 1e-5)
        y2 = two.all_reduce_rmsnorm_(xs[rank].cuda(), r2, w, 1e-5)
        torch.cuda.synchronize()
        ok.append(("fused", T, H, bool(torch.equal(y1.cpu(), y2.cpu())) and bool(torch.equal(r1.cpu(), r2.cpu()))))
    # hipGraph: two-shot fused + a one-shot all-reduce in the same graph, replayed
    T, H = 96, 8192
    xin = torch.zeros(T, H, dtype=torch.bfloat16, device="cuda")
    small = torch.zeros(4096, dtype=torch.bfloat16, device="cuda")
    res = torch.zeros(T, H, dtype=torch.bfloat16, device="cuda")
    w = torch.ones(H, dtype=torch.bfloat16, device="cuda")
    out = torch.empty(T, H, dtype=torch.bfloat16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        two.all_reduce_rmsnorm_(xin, res, w, 1e-5, out)
        one.all_reduce_(small)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        two.all_reduce_rmsnorm_(xin, res, w, 1e-5, out)
        one.all_reduce_(small)
    for it in range(3):
        g = torch.Generator().manual_seed(2000 + it)
        xs = [torch.randn(T, H, generator=g).to(torch.bfloat16) for _ in range(world)]
        r0 = torch.randn(T, H, generator=g).to(torch.bfloat16)
        xin.copy_(xs[rank].cuda())
        res.copy_(r0.cuda())
        small.copy_(_vals(4096, rank, it).cuda())
        gr.replay()
        torch.cuda.synchronize()
        ref_r = r0.cuda()
        ref_y = one.all_reduce_rmsnorm_(xs[rank].cuda(), ref_r, w, 1e-5)
        torch.cuda.synchronize()
        want_small = sum(_vals(4096, r, it).float() for r in range(world))
        ok.append(("graph", it, 0, bool(torch.equal(out.cpu(), ref_y.cpu())) and bool(torch.equal(res.cpu(), ref_r.cpu()))
                   and bool(torch.equal(small.float().cpu(), want_small))))
    ok.append(("err", 0, 0, two.error() == 0 and one.error() == 0))
    torch.save(ok, os.path.join(out_dir, f"s{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [3, 8])
def test_xgmi_two_shot_allreduce_and_fused_norm(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_two_shot_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            ok = torch.load(os.path.join(d, f"s{r}.pt"), weights_only=True)
            assert all(o[-1] for o in ok), f"rank {r}: {ok}"


def _gather_worker(rank, world, port, out_dir):
    """IPC all-gather / broadcast of raw bytes (any dtype, sizes not a multiple of 16 B), the
    TPGroup routes that use them (all_gather_cat / all_gather_rows / broadcast_ / greedy_ids) in
    IPC-only mode, eager and replayed from a hipGraph."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.tp import TPGroup
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.xgmi_ar import XgmiAllReduce

    tp = TPGroup(rank, world, dist.group.WORLD, ctrl=dist.group.WORLD, ranks=list(range(world)), ipc_only=True)
    tp.xgmi = XgmiAllReduce(tp, 4 << 20, rccl=False)
    ok = []
    for shape, dt in (((5,), torch.float32), ((3, 7), torch.int64), ((64, 1000), torch.bfloat16), ((1,), torch.int32)):
        x = (torch.arange(int(torch.tensor(shape).prod())).view(shape) * (rank + 1)).to(dt).cuda()
        g = tp.xgmi.all_gather(x)
        want = torch.stack([(torch.arange(x.numel()).view(shape) * (r + 1)).to(dt) for r in range(world)])
        ok.append(("gather", str(dt), bool(torch.equal(g.cpu(), want))))
        cat = tp.all_gather_cat(x, dim=-1)
        ok.append(("cat", str(dt), bool(torch.equal(cat.cpu(), torch.cat(list(want), dim=-1)))))
        b = x.clone()
        tp.broadcast_(b)
        ok.append(("bcast", str(dt), bool(torch.equal(b.cpu(), want[0]))))
    rows = tp.all_gather_rows(torch.full((3, 16), float(rank), device="cuda", dtype=torch.bfloat16))
    ok.append(("rows", "", bool(torch.equal(rows.float().cpu(), torch.arange(world).repeat_interleave(3)[:, None].float().expand(-1, 16)))))
    # vocab-parallel greedy: rank r holds vocab slice [r*V, (r+1)*V), the max planted on rank world-1
    V = 96
    lg = torch.randn(4, V, generator=torch.Generator().manual_seed(rank)).to(torch.bfloat16).cuda()
    if rank == world - 1:
        lg[:, 17] = 50.0
    ids = tp.greedy_ids(lg, vocab_lo=rank * V)
    ok.append(("greedy", "", bool(torch.equal(ids.cpu(), torch.full((4,), (world - 1) * V + 17, dtype=torch.int32)))))
    # hipGraph: broadcast + all-gather captured and replayed with new inputs
    src = torch.zeros(40, dtype=torch.float32, device="cuda")
    dst = torch.zeros(40, dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        tp.xgmi.broadcast_(src)
        tp.xgmi.state.gather(src.view(torch.uint8)[:144].clone(), torch.empty(144 * world, dtype=torch.uint8, device="cuda"), -1)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        tp.xgmi.broadcast_(src)
        dst.copy_(src * 2)
    for it in range(3):
        src.copy_(torch.arange(40, dtype=torch.float32, device="cuda") + 100 * rank + it)
        gr.replay()
        torch.cuda.synchronize()
        ok.append(("graph", it, bool(torch.equal(dst.cpu(), 2 * (torch.arange(40, dtype=torch.float32) + it)))))
    ok.append(("err", "", tp.xgmi.error() == 0))
    torch.save(ok, os.path.join(out_dir, f"g{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_xgmi_gather_broadcast(world):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_gather_worker, args=(world, _free_port(), d), nprocs=world, join=True)
        for r in range(world):
            ok = torch.load(os.path.join(d, f"g{r}.pt"), weights_only=True)
            assert all(o[-1] for o in ok), f"rank {r}: {ok}"
