"""bench.py contract on the CPU (gloo): one JSON line with the required fields, for a
single rank and for 2-rank DP / TP launches through torch.distributed.run (the same
launcher and rendezvous the driver uses on the 8-GPU node)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REQUIRED = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(extra, nproc=1, timeout=600, self_launch=False):
    args = ["--device", "cpu", "--model", "llama-tiny", "--embedder", "bert-tiny", "--docs", "8", "--batch", "2",
            "--steps", "1", "--warmup", "1", "--max-new-tokens", "3", *extra]
    if nproc == 1 or self_launch:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py"), *args]
        if self_launch:
            cmd += ["--gpus", str(nproc)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
               "--gpus", str(nproc), *args]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert REQUIRED <= set(d)
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    return d


@pytest.mark.parametrize("workload", ["rag", "agent"])
def test_bench_single_rank_json(workload):
    d = _run(["--workload", workload])
    assert d["n_gpus"] == 1 and d["value"] > 0 and d["config"]["parallelism"] == "dp1"


def test_bench_two_rank_dp():
    d = _run([], nproc=2)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4


def test_bench_four_rank_dp():
    """The driver's N=4 launch shape (torchrun, one rank per device, rank-0 JSON over all ranks):
    four replicas share the index build and report the whole-job aggregate."""
    d = _run([], nproc=4)
    assert d["n_gpus"] == 4 and d["config"]["parallelism"] == "dp4" and d["config"]["global_batch"] == 8
    assert d["value"] > 0 and d["ms_per_step"] > 0


def test_bench_self_launch_two_ranks():
    """The driver's plain ``python bench.py --gpus 2`` (no torchrun): bench.py starts both rank
    processes itself, and the single JSON line is the 2-replica whole-job aggregate."""
    d = _run([], nproc=2, self_launch=True)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2" and d["config"]["global_batch"] == 4
    dist = d["config"]["distributed"]
    assert dist["world_size"] == 2 and len(dist["per_replica"]) == 2
    assert all(r["completions"] > 0 for r in dist["per_replica"])


def test_bench_self_launch_tp2():
    """``python bench.py --gpus 2 --tp 2`` (no launcher): one TP group of the two self-launched
    ranks, the sharded kNN equal to the single scan."""
    d = _run(["--tp", "2"], nproc=2, self_launch=True)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "tp2" and d["value"] > 0
    assert d["config"]["knn"]["matches_single_scan"] is True


def test_bench_refuses_gpus_world_mismatch():
    """--gpus 2 inside a launcher that started WORLD_SIZE=1 is refused before any work."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, cwd="/tmp",
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr and not r.stdout.strip()


def test_bench_self_launch_propagates_rank_failure():
    """A rank that fails ends the self-launched job with a non-zero exit and no JSON line."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "2",
                        "--model", "no-such-model", "--embedder", "bert-tiny", "--docs", "8"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_bench_two_rank_tp():
    """--tp 2: the corpus is sharded over the TP group (each rank scans half, the leader merges) and
    the sharded top-k equals the single full scan."""
    d = _run(["--tp", "2"], nproc=2)
    assert d["config"]["parallelism"] == "tp2" and d["config"]["global_batch"] == 2 and d["value"] > 0
    knn = d["config"]["knn"]
    assert knn["mode"].startswith("sharded over tp2") and knn["matches_single_scan"] is True, knn


def test_bench_refuses_forced_reference_on_gpu_device():
    """--device cuda with LK_FORCE_REFERENCE=1 would time the torch reference ops: refused
    before any GPU or corpus work."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1"], capture_output=True,
                       text=True, timeout=120, cwd="/tmp", env=dict(os.environ, LK_FORCE_REFERENCE="1"))
    assert r.returncode != 0 and "LK_FORCE_REFERENCE" in r.stderr


def test_http_bench_cpu_plumbing():
    """bench.py --via-http plumbing: Ollama-compatible server + Minimal_RAG app processes,
    /agent_rag driven over HTTP at two concurrency levels (tiny CPU models)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "benchmarks", "http_bench.py"), "--docs", "8",
                        "--concurrency", "1,2", "--requests", "2,4", "--model", "llama-tiny", "--embedder", "bert-tiny",
                        "--max-new-tokens", "3"], capture_output=True, text=True, timeout=600, cwd="/tmp",
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert set(d["config"]["levels"]) == {"1", "2"} and d["value"] > 0
    assert sum(d["config"]["levels"]["2"]["http_status_counts"].values()) == 4


def test_tp_sim_estimate_counts_only_exposed_collectives():
    """--tp-sim's collective estimate: a prefill-sized step's post-attention half runs as a
    pipeline over row chunks (models/llama.py _post_attn_pipelined), so only the collective time
    the pipeline exposes is added; decode-sized steps count every tail whole."""
    import importlib.util

    from llm_kubernetes_minikube_sharp4dev_amd.models.configs import decoder_config
    from llm_kubernetes_minikube_sharp4dev_amd.models.llama import overlap_chunks

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    floor = b._collective_floor(None, 8192)  # the measured per-call floor (profiles/r4_tp_collectives)
    lc = decoder_config("llama-3-70b")
    assert overlap_chunks(64) is None and overlap_chunks(2048) is None
    assert overlap_chunks(4096) == [(0, 2048), (2048, 4096)]
    for up in (True, False):
        serial = lambda rows: (2 * lc.num_layers + 1) * b._per_call_us(floor, rows, lc.hidden, 8, up)  # noqa: E731
        assert abs(b._exposed_step_us(floor, 64, lc, 8, up) - serial(64)) < 1e-6
        exposed = b._exposed_step_us(floor, 4096, lc, 8, up)
        assert 0 < exposed < 0.7 * serial(4096), (up, exposed, serial(4096))  # (2 chunks: ~0.62 / ~0.5)
