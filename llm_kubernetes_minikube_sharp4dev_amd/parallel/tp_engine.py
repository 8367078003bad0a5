"""Tensor-parallel generation (Llama-3-70B TP=8 over xGMI, BASELINE.json config 4).

One process per GPU.  Rank 0 owns the scheduler, the block allocator and the
sampler; every step it broadcasts the host-side :class:`StepInputs` to the other
ranks over a small CPU (gloo) control group -- a fixed-layout int64 header plus one
int32 payload, block tables trimmed to their live width (``encode_msg``) -- then all ranks run the same forward
in lockstep — weights and KV heads sharded, two RCCL all-reduces per layer, vocab
all-gather for the logits.  Decode hipGraphs are captured on every rank for the
same batch buckets (RCCL calls inside the graph), so a TP decode step is one graph
replay per GPU.

    tp = init_distributed()                    # torchrun, backend nccl (RCCL)
    model = build_decoder("llama-3-70b", device=f"cuda:{rank}", tp=tp)
    if rank == 0:
        engine = make_tp_engine(model, tp, ...); engine.generate(...); shutdown(engine)
    else:
        run_tp_worker(model, tp, ...)
"""
from __future__ import annotations

import os
import time
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine.model_runner import ModelRunner
from ..utils.logging import get_logger
from .tp import TPGroup

log = get_logger("tp")


_CMDS = ("stop", "step", "capture", "barrier", "knn", "shard")
# StepInputs array fields in wire order (lists travel as int32 arrays; gather = (dst, src))
_FIELDS = ("ids", "positions", "slots", "q_lens", "ctx_lens", "tables_p", "ctx_d", "tables_d", "logits_rows",
           "gather_dst", "gather_src")
_NF = 5                                   # header slots per field: present, dtype, dim0, dim1, sent dim1
_HDR = 10 + _NF * len(_FIELDS)


def _live_width(t: np.ndarray) -> int:
    """Columns up to the last non-zero one: block tables are zero-padded to the bucket's
    full width (up to max_model_len / block_size); only the live part travels."""
    if t.size == 0:
        return 0
    nz = np.flatnonzero(t.any(axis=0))
    return int(nz[-1]) + 1 if nz.size else 0


def encode_msg(cmd: str, arg=None) -> tuple[np.ndarray, np.ndarray]:
    """(int64 header [_HDR], int32 payload) of a control message: a fixed-layout tensor
    pair instead of a pickled object (no pickling, no per-step Python object graph)."""
    h = np.zeros(_HDR, dtype=np.int64)
    h[0] = _CMDS.index(cmd)
    parts = []
    if cmd == "capture":
        h[7], h[8] = int(arg[0]), int(bool(arg[1]))
    elif cmd == "knn":  # (queries [nq, D] bf16 / f32 host tensor, k): raw bytes travel as int32 words
        q, k = arg
        if q.dtype not in (torch.bfloat16, torch.float32):
            raise TypeError("sharded kNN queries must be bf16 or f32")
        raw = q.contiguous().view(-1).view(torch.uint8).numpy()
        h[2], h[7], h[8], h[9] = int(q.dtype == torch.float32), q.shape[0], q.shape[1], int(k)
        parts.append(np.frombuffer(np.ascontiguousarray(np.pad(raw, (0, (-raw.size) % 4))).tobytes(), dtype=np.int32))
    elif cmd == "shard":  # (rows, dim, f32): the corpus rows follow as one scatter over the control group
        h[7], h[8], h[2] = int(arg[0]), int(arg[1]), int(bool(arg[2]))
    elif cmd == "step":
        si = arg
        h[2], h[3], h[4], h[5], h[6] = si.num_decode, si.decode_graph, int(si.greedy), si.shared_len, si.prev_bcast
        vals = {f: getattr(si, f, None) for f in _FIELDS[:9]}
        vals["gather_dst"], vals["gather_src"] = si.gather if si.gather is not None else (None, None)
        for k, f in enumerate(_FIELDS):
            v = vals[f]
            b = 10 + _NF * k
            if v is None:
                continue
            a = np.asarray(v)
            h[b], h[b + 1] = 1, 1 if a.dtype == np.int64 else 0
            h[b + 2] = a.shape[0] if a.ndim else 0
            if a.ndim == 2:
                w = _live_width(a) if f in ("tables_p", "tables_d") else a.shape[1]
                h[b + 3], h[b + 4] = a.shape[1], w
                a = a[:, :w]
            parts.append(np.ascontiguousarray(a, dtype=np.int32).reshape(-1))
    payload = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)
    h[1] = payload.size
    return h, payload


def decode_msg(h: np.ndarray, payload: np.ndarray):
    from ..engine.model_runner import StepInputs

    cmd = _CMDS[int(h[0])]
    if cmd == "capture":
        return cmd, (int(h[7]), bool(h[8]))
    if cmd == "knn":
        nq, d, k = int(h[7]), int(h[8]), int(h[9])
        dt, esz = (torch.float32, 4) if h[2] else (torch.bfloat16, 2)
        raw = torch.from_numpy(payload.copy().view(np.uint8)[: nq * d * esz].copy())
        return cmd, (raw.view(dt).view(nq, d), k)
    if cmd == "shard":
        return cmd, (int(h[7]), int(h[8]), bool(h[2]))
    if cmd != "step":
        return cmd, None
    out, off = {}, 0
    for k, f in enumerate(_FIELDS):
        b = 10 + _NF * k
        if not h[b]:
            out[f] = None
            continue
        dt = np.int64 if h[b + 1] else np.int32
        d0, d1, w = int(h[b + 2]), int(h[b + 3]), int(h[b + 4])
        if d1:
            a = np.zeros((d0, d1), dtype=dt)
            a[:, :w] = payload[off:off + d0 * w].reshape(d0, w)
            off += d0 * w
        else:
            a = payload[off:off + d0].astype(dt)
            off += d0
        out[f] = a
    gather = (out.pop("gather_dst"), out.pop("gather_src"))
    si = StepInputs(ids=out["ids"], positions=out["positions"], slots=out["slots"], num_decode=int(h[2]),
                    decode_graph=int(h[3]), q_lens=out["q_lens"].tolist() if out["q_lens"] is not None else [],
                    ctx_lens=out["ctx_lens"].tolist() if out["ctx_lens"] is not None else [],
                    tables_p=out["tables_p"], ctx_d=out["ctx_d"], tables_d=out["tables_d"],
                    logits_rows=out["logits_rows"] if out["logits_rows"] is not None else np.zeros(0, np.int64),
                    greedy=bool(h[4]), gather=gather if gather[0] is not None else None,
                    shared_len=int(h[5]), prev_bcast=int(h[6]))
    return cmd, si


class _ShmChannel:
    """Single-producer / multi-consumer message slots in POSIX shared memory for the TP
    ranks of one node (TP never spans nodes here: one process per GPU, TP within the
    node's xGMI mesh).  Two slots alternate; the driver writes a message's bytes, then its
    sequence number; a worker spins on the sequence number, copies the message out and
    acknowledges it; the driver reuses a slot only once every worker acknowledged the
    message two back.  x86 keeps stores (and loads) in program order, so a worker that
    sees the new sequence number sees the complete message.  Idle workers back off from
    spinning to 50 us - 1 ms sleeps."""

    SLOT = 8 << 20
    ACKS = 64

    def __init__(self, name: str, create: bool, worker_index: int = -1, n_workers: int = 0):
        import mmap

        size = 64 + 8 * self.ACKS + 2 * self.SLOT
        self.path = os.path.join("/dev/shm", name)
        fd = os.open(self.path, (os.O_CREAT | os.O_EXCL | os.O_RDWR) if create else os.O_RDWR, 0o600)
        try:
            if create:
                os.ftruncate(fd, size)
            self.mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        buf = self.mm
        self.seq = np.ndarray((1,), dtype=np.uint64, buffer=buf, offset=0)
        self.acks = np.ndarray((self.ACKS,), dtype=np.uint64, buffer=buf, offset=64)
        self.slots = [np.ndarray((self.SLOT,), dtype=np.uint8, buffer=buf, offset=64 + 8 * self.ACKS + i * self.SLOT)
                      for i in range(2)]
        if create:
            self.seq[0] = 0
            self.acks[:] = 0
        self.me, self.n_workers, self.next = worker_index, n_workers, 1
        self.created = create
        # a follower whose parent (the serving supervisor, or the leader that spawned it) is
        # gone stops waiting: the leader can no longer send it "stop"
        self.ppid = os.getppid()
        # a worker that stops acknowledging (crash, hang) fails the driver's step instead of
        # spinning it forever: the engine's failure path then ends the in-flight requests
        self.timeout_s = float(os.environ.get("LK_TP_CTRL_TIMEOUT_S", "120"))

    def send(self, h: np.ndarray, payload: np.ndarray):
        n = int(self.seq[0]) + 1
        nbytes = h.nbytes + payload.nbytes
        if nbytes > self.SLOT:
            raise ValueError(f"control message of {nbytes} B exceeds the {self.SLOT} B slot")
        spins, t0 = 0, 0.0
        while n > 2 and int(self.acks[: self.n_workers].min()) < n - 2:  # slot still being read
            spins += 1
            if spins > 2000:
                time.sleep(5e-5)
                if t0 == 0.0:
                    t0 = time.monotonic()
                elif spins % 1000 == 0 and time.monotonic() - t0 > self.timeout_s:
                    late = [i for i in range(self.n_workers) if int(self.acks[i]) < n - 2]
                    raise RuntimeError(
                        f"TP control channel: worker(s) {late} did not take message {n - 2} within "
                        f"{self.timeout_s:.0f} s (LK_TP_CTRL_TIMEOUT_S); a rank crashed or hung")
        slot = self.slots[n & 1]
        slot[: h.nbytes] = h.view(np.uint8)
        slot[h.nbytes: nbytes] = payload.view(np.uint8)
        self.seq[0] = n  # publish last

    def recv(self) -> tuple[np.ndarray, np.ndarray]:
        spins, sleep = 0, 5e-5
        while int(self.seq[0]) < self.next:
            spins += 1
            if spins > 20000:
                time.sleep(sleep)
                sleep = min(sleep * 1.5, 1e-3)
                if spins % 4096 == 0 and os.getppid() != self.ppid:
                    raise RuntimeError("TP control channel: the parent process is gone; leaving")
        slot = self.slots[self.next & 1]
        h = slot[: _HDR * 8].view(np.int64).copy()
        n = int(h[1])
        payload = slot[_HDR * 8: _HDR * 8 + 4 * n].view(np.int32).copy()
        self.acks[self.me] = self.next
        self.next += 1
        return h, payload

    def close(self):
        self.seq = self.acks = self.slots = None  # drop the views before unmapping
        try:
            self.mm.close()
        except BufferError:
            pass
        if self.created:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass


class _Ctrl:
    """Driver -> worker control channel of one TP group.  Messages are a fixed int64 header
    plus an exact-size int32 payload (``encode_msg``).  Transport: a shared-memory slot
    pair (``_ShmChannel``) when the group's ranks share a host, else two gloo broadcasts.
    ``LK_TP_CTRL=gloo`` forces the broadcasts."""

    def __init__(self, tp: TPGroup):
        self.tp = tp
        self.seconds = 0.0   # driver-side time spent in the control hop
        self.messages = 0
        self.shm = None
        if tp.size > 1 and tp.ctrl is not None:
            self.group, self.src = tp.ctrl, tp.ranks[0]
        elif tp.size > 1:
            ranks = dist.get_process_group_ranks(tp.group) if tp.group is not None else list(range(tp.size))
            self.group = dist.new_group(ranks, backend="gloo")
            self.src = ranks[0]
        else:
            self.group, self.src = None, 0
        self._h = torch.zeros(_HDR, dtype=torch.int64)
        if tp.size > 1 and os.environ.get("LK_TP_CTRL", "shm") == "shm":
            self._setup_shm()

    def _setup_shm(self):
        import socket
        import uuid

        box = [None, socket.gethostname()]
        if self.tp.rank == 0:
            import atexit

            name = f"lk_tpctrl_{os.getpid()}_{uuid.uuid4().hex[:8]}"
            self.shm = _ShmChannel(name, True, n_workers=self.tp.size - 1)
            box[0] = name
            path = self.shm.path
            atexit.register(lambda: os.path.exists(path) and os.unlink(path))  # a driver that dies
        dist.broadcast_object_list(box, src=self.src, group=self.group)
        same = [None] * self.tp.size
        dist.all_gather_object(same, socket.gethostname() == box[1], group=self.group)
        if not all(same):  # ranks on another host: broadcasts
            if self.shm is not None:
                self.shm.close()
                self.shm = None
            return
        if self.tp.rank > 0:
            self.shm = _ShmChannel(box[0], False, worker_index=self.tp.rank - 1)
        dist.barrier(group=self.group)  # every worker attached before the driver may unlink

    def send(self, cmd: str, arg=None):
        if self.tp.size == 1:
            return
        t0 = time.perf_counter()
        h, payload = encode_msg(cmd, arg)
        if self.shm is not None:
            self.shm.send(h, payload)
        else:
            self._h.copy_(torch.from_numpy(h))
            dist.broadcast(self._h, src=self.src, group=self.group)
            if payload.size:
                dist.broadcast(torch.from_numpy(payload), src=self.src, group=self.group)
        self.seconds += time.perf_counter() - t0
        self.messages += 1
        if cmd == "stop":
            self.close()

    def recv(self):
        if self.shm is not None:
            h, payload = self.shm.recv()
        else:
            dist.broadcast(self._h, src=self.src, group=self.group)
            h = self._h.numpy().copy()
            payload = np.zeros(int(h[1]), dtype=np.int32)
            if payload.size:
                dist.broadcast(torch.from_numpy(payload), src=self.src, group=self.group)
        msg = decode_msg(h, payload)
        if msg[0] == "stop":
            self.close()
        return msg

    def close(self):
        if self.shm is not None:
            # the driver unlinks only after the workers saw "stop" (their ack of it)
            if self.shm.created:
                n = int(self.shm.seq[0])
                t0 = time.time()
                while int(self.shm.acks[: self.shm.n_workers].min()) < n and time.time() - t0 < 30:
                    time.sleep(1e-4)
            self.shm.close()
            self.shm = None


def _agree_num_blocks(model, tp: TPGroup, **kw) -> int:
    """Size the KV pool from this rank's free memory, then take the group minimum
    (rank 0's allocator hands out block ids that every rank must hold) -- a host-side
    agreement over the CPU control group."""
    keys = ("block_size", "max_model_len", "max_num_seqs", "kv_cache_gb", "gpu_memory_fraction")
    n = torch.tensor([ModelRunner.plan_num_blocks(model, **{k: kw[k] for k in keys if k in kw})], dtype=torch.int64)
    if tp.size > 1:
        if tp.ctrl is not None:
            dist.all_reduce(n, op=dist.ReduceOp.MIN, group=tp.ctrl)
        else:
            if torch.cuda.is_available() and model.device.type == "cuda":
                n = n.to(model.device)
            dist.all_reduce(n, op=dist.ReduceOp.MIN, group=tp.group)
    return int(n.item())


def tune_collectives(model, tp: TPGroup):
    """Self-check the group's IPC collectives against the reference on the real peers, then
    measure the all-reduce algorithms at the model's hidden size (every rank in lockstep; the
    leader's table is used by all): xgmi_ar.XgmiAllReduce.self_check / tune.  A group whose
    IPC all-gather or handshakes failed the check leaves the IPC path (RCCL only); without a
    usable RCCL communicator (several ranks on one device) that is an error."""
    x = getattr(tp, "xgmi", None)
    if x is None or x.table or tp.size == 1:
        return
    if not (torch.cuda.is_available() and model.device.type == "cuda"):
        return
    if not x.check and os.environ.get("LK_XGMI_SELFCHECK", "1") != "0":
        t0 = time.perf_counter()
        rep = x.self_check(model.cfg.hidden)
        rep["seconds"] = round(time.perf_counter() - t0, 2)
        if tp.rank == 0 or rep["vetoed_buckets"] or rep["ipc_disabled"]:
            log.info("TP collectives self-check (rank %d): %s", tp.rank, rep)
        if rep["ipc_disabled"]:
            if not x.rccl:
                raise RuntimeError(f"IPC collectives failed their start-up self-check and the group has no "
                                   f"RCCL communicator to fall back to: {rep}")
            log.warning("IPC collectives disabled for this TP group (self-check): %s", rep["reasons_on_rank"])
            tp.xgmi_check = rep
            tp.xgmi = None
            return
    if os.environ.get("LK_XGMI_TUNE", "1") == "0":
        return
    t0 = time.perf_counter()
    x.tune(model.cfg.hidden)
    x.tune_s = time.perf_counter() - t0
    if tp.rank == 0:
        log.info("TP collectives (measured in %.1f s): %s", x.tune_s, x.describe())


def make_tp_runner(model, tp: TPGroup, **runner_kw) -> tuple[ModelRunner, _Ctrl]:
    tune_collectives(model, tp)
    ctrl = _Ctrl(tp)
    nb = runner_kw.pop("num_blocks", None)
    if nb is None:
        nb = _agree_num_blocks(model, tp, **runner_kw)
    runner = ModelRunner(model, num_blocks=nb, **runner_kw)
    return runner, ctrl


def make_tp_engine(model, tp: TPGroup, tokenizer=None, engine_kw: Optional[dict] = None, **runner_kw):
    """Rank 0: an LLMEngine whose runner broadcasts each step to the TP workers."""
    from ..engine.llm_engine import LLMEngine

    runner, ctrl = make_tp_runner(model, tp, **runner_kw)
    ekw = dict(engine_kw or {})
    eng = LLMEngine.__new__(LLMEngine)
    LLMEngine.__init__(eng, model, tokenizer, block_size=runner.bs, max_model_len=runner.max_model_len,
                       max_num_seqs=runner.max_num_seqs, num_blocks=runner.num_blocks, use_graphs=runner.use_graphs,
                       _runner=runner, **ekw)
    runner.step_hook = lambda si: ctrl.send("step", si)
    eng.tp_ctrl = ctrl
    return eng


@torch.inference_mode()
def tp_capture_all(engine, max_batch: Optional[int] = None, variants=(False, True)):
    """Capture decode graphs on every rank in lockstep -- under inference mode like the workers'
    side and ModelRunner.capture_all: a graph captured earlier in the process under inference mode
    (the batch-1 query-encoder graphs) leaves the CUDA generator's graph-state tensors as inference
    tensors, which a capture outside inference mode may not update (capture_begin raised)."""
    r = engine.runner
    for B in r.graph_sizes:
        for v in variants:
            if (max_batch is None or B <= max_batch) and (B, v) not in r.graphs:
                engine.tp_ctrl.send("capture", (B, v))
                r.capture(B, v)


def shutdown_tp(engine):
    engine.tp_ctrl.send("stop")


def tp_knn_search(engine, shard, queries: torch.Tensor, k: int):
    """Leader side of the sharded kNN (every TP rank scans 1/T of the corpus): broadcast the
    queries over the control channel, search this rank's shard, gather every rank's top-k over
    the CPU control group and merge with the HIP merge (stable (score desc, id asc) order:
    identical to one full scan).  The workers answer in order with their steps, so the exchange
    never interleaves with the step collectives on the device.  A served index searches from
    HTTP threads while the engine thread steps: the engine lock keeps the control channel's
    messages (one producer) and the control group's collectives in one order."""
    q = queries.to(shard.corpus.dtype)
    ctrl = getattr(engine, "tp_ctrl", None)
    lock = getattr(engine, "lock", None)
    with lock if lock is not None else _NoLock():
        if ctrl is not None and ctrl.tp.size > 1:
            ctrl.send("knn", (q.cpu(), k))
        return shard.search(q.to(shard.corpus.device), k)


class _NoLock:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _scatter_rows(ctrl, n: int, d: int, f32: bool, host: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Rows [lo, hi) of an n x d corpus to each rank of the control group (one gloo scatter of
    equal padded slices from the leader; bf16 travels as int16 words).  Returns this rank's rows."""
    from .sharded_index import shard_bounds

    tp = ctrl.tp
    per = (n + tp.size - 1) // tp.size
    wire = torch.float32 if f32 else torch.int16
    buf = torch.zeros((per, d), dtype=wire)
    parts = None
    if host is not None:
        h = host.contiguous() if f32 else host.to(torch.bfloat16).contiguous().view(torch.int16)
        parts = []
        for r in range(tp.size):
            lo, hi = shard_bounds(n, r, tp.size)
            p = torch.zeros((per, d), dtype=wire)
            p[: hi - lo] = h[lo:hi]
            parts.append(p)
    dist.scatter(buf, parts, src=ctrl.src, group=ctrl.group)
    lo, hi = shard_bounds(n, tp.rank, tp.size)
    rows = buf[: hi - lo]
    return rows if f32 else rows.view(torch.bfloat16)


def _shard_index(ctrl, rows: torch.Tensor, n: int, device):
    from .sharded_index import ShardedKnnIndex, shard_bounds

    lo, _ = shard_bounds(n, ctrl.tp.rank, ctrl.tp.size)
    return ShardedKnnIndex(rows.to(device).contiguous(), lo, None, host_group=ctrl.group if ctrl.tp.size > 1 else None)


def tp_shard_corpus(engine, corpus: torch.Tensor, device=None):
    """Leader: distribute an n x d corpus over the TP group (each rank keeps rows
    shard_bounds(n, rank, T); workers get a "shard" command, then their rows by one scatter)
    and return the leader's ShardedKnnIndex (``tp_knn_search(engine, shard, ...)`` searches the
    whole group).  bf16 on the GPU (the single-GPU index's dtype), f32 on the CPU."""
    ctrl = engine.tp_ctrl
    dev = torch.device(device) if device is not None else engine_device(engine)
    f32 = dev.type != "cuda"
    n, d = corpus.shape
    host = corpus.detach().to("cpu", torch.float32 if f32 else torch.bfloat16)
    lock = getattr(engine, "lock", None)
    with lock if lock is not None else _NoLock():
        ctrl.send("shard", (n, d, f32))
        rows = _scatter_rows(ctrl, n, d, f32, host)
    return _shard_index(ctrl, rows, n, dev)


def engine_device(engine):
    m = getattr(engine, "model", None)
    return m.device if m is not None else getattr(engine, "device", torch.device("cpu"))


class KnnGroup:
    """Leader handle of a TP group that holds only corpus shards (``rag-app --tp T``: no
    model; the workers run ``run_tp_worker(None, tp)``): ``tp_shard_corpus`` /
    ``tp_knn_search`` accept it in place of an engine."""

    def __init__(self, tp: TPGroup, device):
        import threading

        self.tp = tp
        self.device = torch.device(device)
        self.model = None
        self.tp_ctrl = _Ctrl(tp)
        self.lock = threading.Lock()

    def shutdown(self):
        with self.lock:
            self.tp_ctrl.send("stop")


def tp_barrier(engine):
    """World barrier (after a device sync) from the TP driver while its workers sit in
    run_tp_worker: they receive a "barrier" command and join the same barrier."""
    ctrl = getattr(engine, "tp_ctrl", None)
    if ctrl is not None:
        ctrl.send("barrier")
    if torch.cuda.is_available() and engine.model.device.type == "cuda":
        torch.cuda.synchronize()
    dist.barrier()


@torch.inference_mode()
def run_tp_worker(model, tp: TPGroup, knn=None, device=None, **runner_kw):
    """Ranks > 0: execute whatever rank 0 schedules until it says stop (``knn``: this rank's
    ShardedKnnIndex, answering the leader's sharded searches; a "shard" command replaces it with
    rows the leader scatters).  ``model=None``: a kNN-only rank (the leader is a KnnGroup)."""
    from ..utils.watchdog import StepWatchdog

    stall_s = float(runner_kw.pop("stall_s", 600.0)) if "stall_s" in runner_kw else 600.0
    if model is not None:
        runner, ctrl = make_tp_runner(model, tp, **runner_kw)
        device = model.device
    else:
        runner, ctrl = None, _Ctrl(tp)
        device = torch.device(device) if device is not None else torch.device("cpu")
    on_gpu = torch.cuda.is_available() and device.type == "cuda"
    wd = StepWatchdog(f"tp-worker-{tp.rank}", stall_s=stall_s)
    n = 0
    pending: list = []
    while True:
        cmd, arg = ctrl.recv()  # idle wait for the driver: not a stall
        wd.beat()
        if cmd == "stop":
            for ev in pending:
                ev.synchronize()
            break
        if cmd in ("capture", "step") and runner is None:
            raise RuntimeError(f"kNN-only TP worker got a {cmd!r} command")
        if cmd == "capture":
            runner.capture(*arg)
        elif cmd == "barrier":
            if on_gpu:
                torch.cuda.synchronize()
            dist.barrier()
        elif cmd == "shard":
            rows, d, f32 = arg
            knn = _shard_index(ctrl, _scatter_rows(ctrl, rows, d, f32), rows, device)
        elif cmd == "knn":
            if knn is None:
                raise RuntimeError("TP worker got a sharded kNN search but holds no corpus shard")
            q, k = arg
            knn.search(q.to(knn.corpus.device), k)
        elif cmd == "step":
            with wd.busy():  # a step that never returns (dead peer in an all-reduce) is a stall
                runner.execute(arg)
                if on_gpu:
                    # keep <= 2 steps in flight (the driver pipelines: step N+1's inputs
                    # arrive before step N is done, so the device never idles waiting here)
                    ev = torch.cuda.Event()
                    ev.record()
                    pending.append(ev)
                    if len(pending) > 2:
                        pending.pop(0).synchronize()
            n += 1
    wd.stop()
    log.info("tp worker rank %d done after %d steps", tp.rank, n)
    return n
