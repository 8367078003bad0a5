"""RCCL (torch.distributed backend "nccl" on ROCm) on the box's MI355X: the collectives the TP /
DP / sharded-kNN paths issue (all-reduce, reduce-scatter, all-gather, broadcast, object
all-gather) run through RCCL in a world of one rank per GPU -- here the single GPU, so the
world is 1 -- eagerly and captured in a hipGraph (the decode graphs capture the TP
all-reduces).  Multi-rank RCCL needs more than one GPU (the round driver's 8-GPU run); the
gloo CPU tests cover the multi-rank logic."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    res = {"backend": dist.get_backend()}
    x = torch.arange(8192, device=dev, dtype=torch.float32).to(torch.bfloat16)
    y = x.clone()
    dist.all_reduce(y)
    res["all_reduce"] = bool(torch.equal(x, y))
    rs = torch.empty(8192, device=dev, dtype=torch.bfloat16)
    dist.reduce_scatter_tensor(rs, x)
    res["reduce_scatter"] = bool(torch.equal(rs, x))
    ag = torch.empty(8192, device=dev, dtype=torch.bfloat16)
    dist.all_gather_into_tensor(ag, x)
    res["all_gather"] = bool(torch.equal(ag, x))
    b = x.clone()
    dist.broadcast(b, src=0)
    res["broadcast"] = bool(torch.equal(b, x))
    objs = [None]
    dist.all_gather_object(objs, {"rank": 0})
    res["all_gather_object"] = objs == [{"rank": 0}]
    # the TP decode graphs capture RCCL all-reduces: capture + replay
    buf = torch.ones(64, 8192, device=dev, dtype=torch.bfloat16)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dist.all_reduce(buf)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    # captured as the engine captures its decode graphs (engine/model_runner.py): with the
    # default "global" capture mode the process group's watchdog thread, polling the events of
    # earlier eager collectives, hits hipErrorStreamCaptureUnsupported and aborts the process
    # (seen on MI355X / ROCm 7, first run of this test); "thread_local" confines the capture
    # rules to the capturing thread
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        dist.all_reduce(buf)
        buf.mul_(2)
    buf.fill_(3)
    g.replay()
    torch.cuda.synchronize()
    res["graph_all_reduce"] = bool((buf == 6).all())
    # the sharded kNN exchange over the RCCL group: local top-k -> all_gather -> HIP merge
    from llm_kubernetes_minikube_sharp4dev_amd import ops
    from llm_kubernetes_minikube_sharp4dev_amd.parallel.sharded_index import ShardedKnnIndex

    corpus = torch.randn(5000, 768, device=dev).to(torch.bfloat16)
    q = torch.randn(4, 768, device=dev).to(torch.bfloat16)
    sc, ids = ShardedKnnIndex.from_full(corpus).search(q, 6)
    ss, ii = [torch.empty_like(sc)], [torch.empty_like(ids)]
    dist.all_gather(ss, sc.contiguous())
    dist.all_gather(ii, ids.contiguous())
    ms, mi = ops.knn_merge(torch.cat(ss, 1), torch.cat(ii, 1), 6)
    s2, i2 = ops.knn_topk(corpus, ops.row_norms(corpus), q, ops.row_norms(q), 6)
    res["sharded_knn"] = bool(torch.equal(mi.cpu().long(), i2.cpu().long()))
    torch.save(res, out)
    dist.destroy_process_group()


def test_rccl_collectives_and_graph_capture_on_mi355x():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "r.pt")
        mp.spawn(_worker, args=(_port(), out), nprocs=1, join=True)
        res = torch.load(out, weights_only=True)
    assert res.pop("backend") == "nccl"
    assert all(res.values()), res
