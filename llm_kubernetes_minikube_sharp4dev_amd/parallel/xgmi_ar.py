"""xGMI collectives over IPC-mapped peer memory (K14, csrc/xgmi_allreduce.hip).

Each rank exports an IPC staging (two regions) + signal buffer; the handles are exchanged
once over the TP group's CPU (gloo) control group, every rank maps its peers' buffers, and
every call is ONE kernel with per-workgroup flag handshakes (hipGraph-capturable: the epochs
live in device memory):

* one-shot all-reduce (decode-sized messages): stage -> handshake -> read and sum every rank's
  copy -> handshake.  Latency-optimal; each of the 7 links carries the whole message S.
* two-shot all-reduce (prefill-sized messages): reduce-scatter + all-gather through the same
  mappings, 2S/world per link (S/4 on 8 ranks) for one more handshake.  Bit-identical to
  one-shot.
* all-gather / broadcast of raw bytes (``gather``): the vocab-parallel argmax pairs, sampled
  ids, logits of sampled rows -- so a TP group can run with no RCCL call at all (several ranks
  on ONE device, where RCCL refuses the communicator: the one-GPU multi-rank tests).

The all-reduces have a fused residual + RMSNorm form (:meth:`XgmiAllReduce.all_reduce_rmsnorm_`),
the tail of every row-parallel projection.

Before any of it routes production traffic, :meth:`XgmiAllReduce.self_check` runs every
all-reduce form (one-shot, two-shot, fused with the residual + RMSNorm tail) per row bucket and
the all-gather on the real peers against a reference (RCCL where the group has a communicator,
else a gloo all-reduce of host copies), on small-integer data whose sums are exact in bf16 in any
order -- so the all-reduce and residual results must be bit-identical; the normalised output
within one bf16 rounding.  A mismatch routes that (bucket, algorithm) away from the IPC kernel
with the reason logged; a handshake timeout or a broken all-gather takes the group off the IPC
path.  Every rank applies the MAX of the flags (one agreement over the control group), and the
outcome is reported (``self.check``, the bench JSON's ``tp_collectives.self_check``).

Which algorithm serves a message is MEASURED at attach time (:meth:`XgmiAllReduce.tune`): for
each row bucket the fused tail is timed as one-shot, two-shot and (when the group has a usable
RCCL communicator) RCCL all-reduce + the norm kernel; the leader's fastest choice per bucket is
broadcast so every rank routes alike (a rank taking RCCL while another takes the IPC kernel
would deadlock).  ``LK_XGMI_TUNE=0`` keeps the static rule (two-shot from
``LK_XGMI_2SHOT_MIN_KB`` on >= 4 ranks).  Staging region size: ``LK_XGMI_AR_MB`` (default 64 MB
= a 4096-token x 8192 bf16 prefill message); larger all-reduces run in chunks.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..ops import lib

ALGOS = ("ipc1", "ipc2", "rccl")
TUNE_ROWS = (1, 4, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096)


def _default_bytes() -> int:
    return int(float(os.environ.get("LK_XGMI_AR_MB", "64")) * (1 << 20)) // 16 * 16


class XgmiAllReduce:
    def __init__(self, tp, max_bytes: int | None = None, two_shot: bool | None = None, rccl: bool = True):
        self.tp = tp
        self.max_bytes = max_bytes if max_bytes is not None else _default_bytes()
        # None: measured table / static rule; True / False: always / never two-shot
        self.two_shot = two_shot
        self.two_shot_min = int(float(os.environ.get("LK_XGMI_2SHOT_MIN_KB", "1024")) * 1024)
        self.rccl = rccl          # the group's device communicator is usable (not several ranks per device)
        self.table: dict = {}     # rows bucket -> algorithm (tune())
        self.timings: dict = {}   # rows bucket -> {algorithm: us} (leader's measurement)
        self.bad: dict = {}       # rows bucket -> {algorithms the self-check failed}
        self.gather_ok = True     # the IPC all-gather / broadcast matched the reference
        self.check: dict = {}     # self_check() report
        self.state = lib().XgmiAr(tp.rank, tp.size, self.max_bytes)
        mine = self.state.handles()
        blobs = [None] * tp.size
        group = tp.ctrl if tp.ctrl is not None else tp.group
        dist.all_gather_object(blobs, mine, group=group)
        self.state.open(blobs)

    # ------------------------------------------------------------------ routing
    def eligible(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous() and t.numel() % 8 == 0
                and t.numel() * 2 <= self.max_bytes and t.data_ptr() % 16 == 0)

    def _bucket(self, rows: int):
        for b in sorted(self.table):
            if rows <= b:
                return b
        return max(self.table) if self.table else None

    def algo(self, rows: int, nbytes: int) -> str:
        """Algorithm for a message of ``rows`` rows / ``nbytes`` bytes: forced, measured, or the
        static rule."""
        if self.two_shot is not None:
            return "ipc2" if self.two_shot else "ipc1"
        b = self._bucket(rows)
        if b is not None:
            a = self.table[b]
            return a if (a != "rccl" or self.rccl) else "ipc1"
        a = "ipc2" if self.tp.size >= 4 and nbytes >= self.two_shot_min else "ipc1"
        bad = self.bad.get(self._check_bucket(rows), ())
        if a in bad:  # untuned group: the self-check still vetoes a failing kernel
            a = "rccl" if self.rccl else next((o for o in ("ipc1", "ipc2") if o not in bad), a)
        return a

    def _check_bucket(self, rows: int):
        ks = sorted(self.bad)
        return next((b for b in ks if rows <= b), ks[-1] if ks else None)

    def use_two_shot(self, t: torch.Tensor) -> bool:
        rows = t.shape[0] if t.dim() >= 2 else 1
        return self.algo(rows, t.numel() * 2) == "ipc2"

    # ------------------------------------------------------------------ collectives
    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if not self.eligible(t):  # too large / odd: chunks of the staging size (IPC-only groups)
            return self._all_reduce_chunked(t)
        if self.use_two_shot(t):
            v = t.view(-1, t.shape[-1]) if t.dim() >= 2 and t.shape[-1] % 8 == 0 else t.view(-1, 8)
            self.state.all_reduce2(v, v)
        else:
            self.state.all_reduce(t, t)
        return t

    def _all_reduce_chunked(self, t: torch.Tensor) -> torch.Tensor:
        if t.dtype != torch.bfloat16:
            raise TypeError("IPC all-reduce: bf16 only")
        flat = t.contiguous().view(-1)
        pad = (-flat.numel()) % 8
        work = torch.nn.functional.pad(flat, (0, pad)) if pad else flat.clone()
        step = self.max_bytes // 2 // 8 * 8
        # the chunks are staging-sized: no row bucket applies, so an algorithm the self-check
        # vetoed in ANY bucket is not used
        vetoed = set().union(*self.bad.values()) if self.bad else set()
        algo = next((a for a in ("ipc1", "ipc2") if a not in vetoed), None)
        if algo is None:
            raise RuntimeError("IPC all-reduce: every IPC algorithm failed the start-up self-check")
        for s in range(0, work.numel(), step):
            piece = work[s:s + step]
            if algo == "ipc2":
                v = piece.view(-1, 8)
                self.state.all_reduce2(v, v)
            else:
                self.state.all_reduce(piece, piece)
        t.copy_(work[: flat.numel()].view_as(t))
        return t

    def eligible_rows(self, x: torch.Tensor, residual: torch.Tensor) -> bool:
        return (self.eligible(x) and x.dim() == 2 and residual.is_contiguous() and residual.shape == x.shape
                and residual.dtype == torch.bfloat16 and x.shape[1] % 8 == 0)

    def all_reduce_rmsnorm_(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                            out: torch.Tensor | None = None, algo: str | None = None) -> torch.Tensor:
        """RMSNorm(allreduce(x) + residual) * w in ONE kernel (residual updated in place):
        the TP decode layer's "row-parallel GEMM -> all-reduce -> add -> norm" tail."""
        if out is None:
            out = torch.empty_like(x)
        algo = algo or ("ipc2" if self.use_two_shot(x) else "ipc1")
        if algo == "ipc2":
            self.state.all_reduce2(x, out, residual, w.contiguous(), float(eps))
        else:
            self.state.all_reduce_rmsnorm(x, residual, w.contiguous(), float(eps), out)
        return out

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape]: every rank's t (any dtype), rank order."""
        nb = t.numel() * t.element_size()
        pad = (-nb) % 16
        src = t.contiguous().view(-1).view(torch.uint8)
        if pad or src.data_ptr() % 16:
            src = torch.nn.functional.pad(src, (0, pad))
        if src.numel() > self.max_bytes:
            raise ValueError(f"IPC all-gather of {src.numel()} B exceeds the {self.max_bytes} B staging region")
        out = torch.empty(self.tp.size * src.numel(), dtype=torch.uint8, device=t.device)
        self.state.gather(src, out, -1)
        out = out.view(self.tp.size, -1)[:, :nb].contiguous()
        return out.view(t.dtype).view(self.tp.size, *t.shape)

    def broadcast_(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        """In place: rank ``root``'s t on every rank."""
        nb = t.numel() * t.element_size()
        if nb % 16 == 0 and t.is_contiguous() and t.data_ptr() % 16 == 0 and nb <= self.max_bytes:
            b = t.view(-1).view(torch.uint8)
            self.state.gather(b, b, root)
            return t
        src = torch.nn.functional.pad(t.contiguous().view(-1).view(torch.uint8), (0, (-nb) % 16))
        if src.numel() > self.max_bytes:
            raise ValueError(f"IPC broadcast of {src.numel()} B exceeds the {self.max_bytes} B staging region")
        self.state.gather(src, src, root)
        t.copy_(src[:nb].view(t.dtype).view_as(t))
        return t

    def error(self) -> int:
        """Non-zero if a handshake ever timed out (a peer missing a call)."""
        return self.state.error()

    # ------------------------------------------------------------------ start-up measurement
    @torch.inference_mode()
    def tune(self, hidden: int, rows=TUNE_ROWS, iters: int = 8, norm_eps: float = 1e-5) -> dict:
        """Time the fused all-reduce + residual + RMSNorm tail per row bucket as one-shot,
        two-shot and (if the group has a usable RCCL communicator) RCCL + the norm kernel, on
        every rank in lockstep; keep the LEADER's fastest per bucket and broadcast it so every
        rank routes identically.  Returns {rows: {algo: us}} (the leader's medians)."""
        from .. import ops

        dev = torch.device("cuda", torch.cuda.current_device())
        algos = [a for a in ALGOS if a != "rccl" or self.rccl]
        res: dict = {}
        for T in rows:
            if T * hidden * 2 > self.max_bytes:
                break
            x = torch.randn(T, hidden, device=dev, dtype=torch.bfloat16)
            r = torch.randn(T, hidden, device=dev, dtype=torch.bfloat16)
            w = torch.ones(hidden, device=dev, dtype=torch.bfloat16)
            out = torch.empty_like(x)

            def run(a):
                if a == "rccl":
                    y = x.clone()
                    dist.all_reduce(y, group=self.tp.group)
                    ops.rmsnorm(y, w, norm_eps, residual=r)
                else:
                    self.all_reduce_rmsnorm_(x, r, w, norm_eps, out, algo=a)

            ts = {a: [] for a in algos}
            for a in algos:  # warm-up (and RCCL communicator set-up) in lockstep
                run(a)
            torch.cuda.synchronize()
            for _ in range(3):
                for a in algos:
                    dist.barrier(group=self.tp.ctrl if self.tp.ctrl is not None else self.tp.group)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(iters):
                        run(a)
                    e1.record()
                    e1.synchronize()
                    ts[a].append(e0.elapsed_time(e1) * 1e3 / iters)
            res[T] = {a: round(sorted(v)[len(v) // 2], 1) for a, v in ts.items()}
        box = [res]
        group = self.tp.ctrl if self.tp.ctrl is not None else self.tp.group
        dist.broadcast_object_list(box, src=self.tp.ranks[0] if self.tp.ranks else 0, group=group)
        self.timings = box[0]
        self.table = route_table(self.timings, self.bad, self.rccl)
        if self.error():
            raise RuntimeError("xGMI collective handshake timed out during tuning")
        return self.timings

    # ------------------------------------------------------------------ start-up self-check
    def _reference_all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        """The trusted all-reduce: RCCL on the device, else gloo on host copies."""
        if self.rccl:
            y = t.clone()
            dist.all_reduce(y, group=self.tp.group)
            return y
        y = t.float().cpu()
        dist.all_reduce(y, group=self.tp.ctrl if self.tp.ctrl is not None else self.tp.group)
        return y.to(t.dtype).to(t.device)

    def _reference_all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self.rccl:
            parts = [torch.empty_like(t) for _ in range(self.tp.size)]
            dist.all_gather(parts, t.contiguous(), group=self.tp.group)
            return torch.stack(parts)
        parts = [torch.empty_like(t.cpu()) for _ in range(self.tp.size)]
        dist.all_gather(parts, t.cpu().contiguous(), group=self.tp.ctrl if self.tp.ctrl is not None else self.tp.group)
        return torch.stack(parts).to(t.device)

    @torch.inference_mode()
    def self_check(self, hidden: int, rows=TUNE_ROWS, eps: float = 1e-5) -> dict:
        """Run every IPC collective on the real peers against the reference (see the module
        doc); record per-bucket failures in ``self.bad`` / ``self.gather_ok`` after a MAX
        agreement over the group, and return the report (also kept in ``self.check``)."""
        from .. import ops

        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
        buckets = [T for T in rows if T * hidden * 2 <= self.max_bytes]
        algos = ("ipc1", "ipc2")
        flags = torch.zeros(len(buckets) * 2 + 2, dtype=torch.int64)  # per (bucket, algo); gather; timeout
        why: dict = {}
        w = (torch.arange(hidden, device=dev) % 7 + 1).to(torch.bfloat16) / 4  # non-unit norm weight
        for bi, T in enumerate(buckets):
            g = torch.Generator().manual_seed(7919 * (self.tp.rank + 1) + T)
            x = torch.randint(-4, 5, (T, hidden), generator=g).to(torch.bfloat16).to(dev)
            r = torch.randint(-4, 5, (T, hidden), generator=g).to(torch.bfloat16).to(dev)
            ref = self._reference_all_reduce(x)
            r_ref = r.clone()
            out_ref = ops.rmsnorm(ref.clone(), w, eps, residual=r_ref)
            for ai, a in enumerate(algos):
                bad = []
                y = x.clone()
                if a == "ipc2":
                    v = y.view(-1, y.shape[-1])
                    self.state.all_reduce2(v, v)
                else:
                    self.state.all_reduce(y, y)
                if not torch.equal(y, ref):
                    bad.append(f"all-reduce differs in {int((y != ref).sum())} of {y.numel()} elements")
                rr = r.clone()
                out = self.all_reduce_rmsnorm_(x.clone(), rr, w, eps, algo=a)
                if not torch.equal(rr, r_ref):
                    bad.append("fused tail: residual differs")
                if not torch.allclose(out.float(), out_ref.float(), rtol=2 ** -7, atol=1e-3):
                    bad.append(f"fused tail: norm output off by {float((out.float() - out_ref.float()).abs().max()):.3g}")
                if bad:
                    flags[bi * 2 + ai] = 1
                    why[f"{T}/{a}"] = "; ".join(bad)
        probe = torch.arange(1000, dtype=torch.int32, device=dev) * (self.tp.rank + 3)
        got = self.all_gather(probe)
        if not torch.equal(got.cpu(), self._reference_all_gather(probe).cpu()):
            flags[-2] = 1
            why["all_gather"] = "IPC all-gather differs from the reference"
        if self.error():
            flags[-1] = 1
            why["handshake"] = "an IPC handshake timed out (a peer never arrived)"
        dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=self.tp.ctrl if self.tp.ctrl is not None else self.tp.group)
        self.bad = {T: {a for ai, a in enumerate(algos) if flags[bi * 2 + ai]} for bi, T in enumerate(buckets)}
        self.gather_ok = not bool(flags[-2])
        report = {"reference": "rccl" if self.rccl else "gloo (host copies)",
                  "buckets": {str(T): {a: ("FAILED" if a in self.bad[T] else "ok") for a in algos} for T in buckets},
                  "all_gather": "ok" if self.gather_ok else "FAILED",
                  "handshake_timeout": bool(flags[-1]),
                  "reasons_on_rank": why}
        vetoed = sorted(T for T, s in self.bad.items() if s)
        report["vetoed_buckets"] = vetoed
        # buckets where BOTH IPC forms failed: without an RCCL communicator to route them to,
        # the group's all-reduce is known to be wrong there -> the group is unusable
        unusable = sorted(T for T, s in self.bad.items() if set(algos) <= s)
        report["unusable_buckets"] = unusable
        report["ipc_disabled"] = bool(flags[-1]) or (not self.gather_ok) or (bool(unusable) and not self.rccl)
        if self.table:  # re-route an already-tuned table
            self.table = route_table(self.timings, self.bad, self.rccl)
        self.check = report
        return report

    def describe(self) -> str:
        return "; ".join(f"<= {T} rows: {a} ({', '.join(f'{k} {v} us' for k, v in self.timings.get(T, {}).items())})"
                         for T, a in sorted(self.table.items()))


def route_table(timings: dict, bad: dict, rccl: bool) -> dict:
    """Per row bucket the fastest algorithm the self-check did not veto; a bucket where every
    IPC form failed goes to RCCL.  Without a communicator such a bucket is an error: the
    self-check reports it (``unusable_buckets``, ``ipc_disabled``) and ``tune_collectives``
    raises before any table is built; called anyway, this raises too."""
    table = {}
    for T, v in timings.items():
        veto = bad.get(T) or bad.get(int(T)) or set()
        ok = {a: t for a, t in v.items() if a not in veto and (a != "rccl" or rccl)}
        if not ok:
            if not rccl:
                raise RuntimeError(f"all-reduce bucket <= {T} rows: every IPC algorithm failed the self-check "
                                   f"and the group has no RCCL communicator")
            ok = {"rccl": 0.0}
        table[T] = min(ok, key=ok.get)
    return table


def attach(tp, max_bytes: int | None = None, rccl: bool = True, tune_hidden: int | None = None) -> XgmiAllReduce:
    """Route this TP group's eligible collectives through the xGMI kernels; with ``tune_hidden``
    measure the per-bucket algorithm table first (LK_XGMI_TUNE=0 skips it)."""
    tp.xgmi = XgmiAllReduce(tp, max_bytes, rccl=rccl)
    if tune_hidden and os.environ.get("LK_XGMI_TUNE", "1") != "0":
        t0 = time.perf_counter()
        tp.xgmi.tune(tune_hidden)
        tp.xgmi.tune_s = time.perf_counter() - t0
    return tp.xgmi
