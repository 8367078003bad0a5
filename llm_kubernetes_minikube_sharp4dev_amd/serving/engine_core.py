"""Engine core: the GPU process of a split server.

The Ollama HTTP surface (JSON parsing, chat templates, tokenisation, incremental
detokenisation, NDJSON framing -- ~5k chunks/s at 128 concurrent .NET sessions) used to share
one Python process, and its GIL, with the engine's step loop.  In the split layout
(``serve --frontends F``) this process keeps only the engines; F front-end processes
(:mod:`.remote`, SO_REUSEPORT on :11434) do the HTTP work and talk to it over a Unix socket
with a compact binary protocol:

  frame  = u32 little-endian length + msgpack body
  client -> core  ["gen", rid, model, ids, sampling-dict, format] | ["abort", rid]
                  | ["embed", rid, model, texts] | ["load", rid, model]
  core -> client  ["tok", [[rid, [ids..], finished, reason, cached_prefix, error], ...], stats]
                  | ["emb", rid, f32 bytes, rows, dim] | ["load", rid, meta] | ["err", rid, msg]

Every engine step's tokens for one connection leave as ONE frame (the engine thread appends
them, a writer thread per connection drains and sends), so the core's Python work per step is
one msgpack pack per front-end, not one HTTP write per stream.  ``stats`` (free KV blocks,
waiting / running requests) rides on every token frame: the front-ends route each request to
the core with the most headroom (:class:`.remote.CorePool`).
"""
from __future__ import annotations

import concurrent.futures
import os
import socket
import struct
import threading
from typing import Optional

import msgpack

from ..engine.sampling import SamplingParams
from ..utils.logging import get_logger

log = get_logger("serving.core")
_HDR = struct.Struct("<I")


def send_frame(sock: socket.socket, obj, lock: Optional[threading.Lock] = None):
    body = msgpack.packb(obj, use_bin_type=True)
    data = _HDR.pack(len(body)) + body
    if lock is None:
        sock.sendall(data)
    else:
        with lock:
            sock.sendall(data)


def recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("peer closed")
        buf += chunk
    return bytes(buf)


def recv_frame(sock: socket.socket):
    (n,) = _HDR.unpack(recv_exact(sock, 4))
    return msgpack.unpackb(recv_exact(sock, n), raw=False)


SP_FIELDS = ("temperature", "top_k", "top_p", "repeat_penalty", "repeat_last_n", "seed", "max_tokens",
             "min_tokens", "stop", "ignore_eos")


def sp_to_wire(sp: SamplingParams) -> dict:
    return {k: getattr(sp, k) for k in SP_FIELDS}


def _accounting(seq) -> dict:
    """Per-request engine accounting sent with a request's last token (front-ends report it)."""
    q = (seq.step_first - seq.step_arrival) if getattr(seq, "step_first", None) is not None else None
    return {"cached": seq.num_cached_prefix, "preempt": getattr(seq, "num_preemptions", 0),
            "queued": q, "run": getattr(seq, "steps_run", None), "jumped": getattr(seq, "jumped", 0)}


def _count_request(seq):
    """The finished request's accounting as per-request counters in this (core) process."""
    from ..utils import tracing

    a = _accounting(seq)
    n = len(seq.prompt_ids)
    for name, v in (("req_prompt_tokens", n), ("req_cached_prefix_tokens", a["cached"]),
                    ("req_uncached_prompt_tokens", n - a["cached"]), ("req_output_tokens", len(seq.output_ids)),
                    ("req_preemptions", a["preempt"]), ("req_steps_queued", a["queued"]),
                    ("req_steps_run", a["run"]), ("req_jumped_tokens", a["jumped"])):
        if v is not None:
            tracing.count("core", name, v)


class _Conn:
    """One front-end connection: a reader thread (ops in) and a writer thread that sends the
    tokens the engine appended since the last frame as one frame."""

    def __init__(self, core: "EngineCore", sock: socket.socket, cid: int):
        self.core, self.sock, self.cid = core, sock, cid
        self.lock = threading.Lock()
        self.pending: list = []
        self.other: list = []
        self.wake = threading.Event()
        self.alive = True
        self.reqs: dict = {}  # rid -> (engine handle, engine req id)
        threading.Thread(target=self._reader, name=f"lk-core-rd{cid}", daemon=True).start()
        threading.Thread(target=self._writer, name=f"lk-core-wr{cid}", daemon=True).start()

    # -- engine thread side ------------------------------------------------------
    def on_token(self, rid, seq, tid, fin):
        if fin:
            _count_request(seq)
        # a finished request carries its engine accounting (cached prefix, preemptions, steps)
        item = [rid, tid, fin, (seq.finish_reason or "stop") if fin else None,
                _accounting(seq) if fin else None, getattr(seq, "error", None) if tid < 0 else None]
        with self.lock:
            self.pending.append(item)
        self.wake.set()

    def post(self, msg):
        with self.lock:
            self.other.append(msg)
        self.wake.set()

    # -- threads -----------------------------------------------------------------
    def _writer(self):
        try:
            while self.alive:
                self.wake.wait(0.5)
                self.wake.clear()
                with self.lock:
                    toks, self.pending = self.pending, []
                    other, self.other = self.other, []
                for m in other:
                    send_frame(self.sock, m)
                if toks:
                    # coalesce per request: [rid, [ids], fin, reason, cached, error]
                    by: dict = {}
                    order = []
                    for rid, tid, fin, reason, cached, err in toks:
                        e = by.get(rid)
                        if e is None:
                            e = by[rid] = [rid, [], False, None, None, None]
                            order.append(rid)
                        if tid >= 0:
                            e[1].append(tid)
                        if fin:
                            e[2], e[3], e[4], e[5] = True, reason, cached, err
                            self.reqs.pop(rid, None)
                    send_frame(self.sock, ["tok", [by[r] for r in order], self.core.stats()])
        except (OSError, ConnectionError):
            pass
        finally:
            self.close()

    def _reader(self):
        try:
            while self.alive:
                msg = recv_frame(self.sock)
                self.core.dispatch(self, msg)
        except (OSError, ConnectionError, ValueError):
            pass
        finally:
            self.close()

    def close(self):
        if not self.alive:
            return
        self.alive = False
        self.wake.set()
        for rid, (h, erid) in list(self.reqs.items()):  # a vanished front-end frees its requests
            h.engine.abort(erid)
        self.reqs.clear()
        try:
            self.sock.close()
        except OSError:
            pass


def _tp_size(engine) -> int:
    """Ranks of the engine's tensor-parallel group (1: a single-GPU engine)."""
    ctrl = getattr(engine, "tp_ctrl", None)
    return int(ctrl.tp.size) if ctrl is not None else 1


class EngineCore:
    """Serve ``manager``'s engines (loaded in this process, on its GPU) to front-end
    processes over a Unix socket at ``path``."""

    def __init__(self, manager, path: str):
        self.mgr = manager
        self.path = path
        self._pool = concurrent.futures.ThreadPoolExecutor(4, thread_name_prefix="lk-core-emb")
        self._ids = 0
        self._conns: list = []
        if os.path.exists(path):
            os.unlink(path)
        self.srv = socket.socket(socket.AF_UNIX, socket.SOCK_STREAM)
        self.srv.bind(path)
        self.srv.listen(64)
        self._t = threading.Thread(target=self._accept, name="lk-core-accept", daemon=True)
        self._t.start()
        log.info("engine core listening on %s", path)

    def stats(self) -> list:
        """[free KV blocks, waiting, running] of the first loaded generator (racy reads: a hint)."""
        for h in self.mgr.generators.values():
            e = h.engine
            try:
                return [int(e.allocator.num_free), len(e.scheduler.waiting) + len(e._inbox), len(e.scheduler.running)]
            except Exception:  # pragma: no cover
                break
        return [0, 0, 0]

    def _accept(self):
        while True:
            try:
                s, _ = self.srv.accept()
            except OSError:
                return
            self._ids += 1
            self._conns.append(_Conn(self, s, self._ids))

    def _meta(self, h) -> dict:
        return {"name": h.name, "preset": h.preset, "max_model_len": h.engine.max_model_len,
                "eos_ids": sorted(int(t) for t in h.engine.eos_ids), "chat_style": h.chat_style,
                "load_s": h.load_s, "vocab_size": int(h.engine.model.cfg.vocab_size), "tp": _tp_size(h.engine)}

    def dispatch(self, conn: _Conn, msg):
        op = msg[0]
        if op == "gen":
            _, rid, model, ids, spd, fmt = msg
            try:
                h = self.mgr.generator(model)
            except KeyError as e:
                conn.post(["err", rid, str(e)])
                return
            sp = SamplingParams(**spd)
            if fmt:
                from ..engine.constrained import json_logits_processor

                sp.logits_processor = json_logits_processor(h.tokenizer, fmt if isinstance(fmt, dict) else None)
            erid = f"c{conn.cid}-{rid}"
            conn.reqs[rid] = (h, erid)
            h.engine.add_request(list(ids), sp, erid, lambda seq, tid, fin, rid=rid: conn.on_token(rid, seq, tid, fin))
            h.async_engine._wake.set()
        elif op == "abort":
            ent = conn.reqs.pop(msg[1], None)
            if ent is not None:
                ent[0].engine.abort(ent[1])
        elif op == "embed":
            _, rid, model, texts = msg
            self._pool.submit(self._embed, conn, rid, model, texts)
        elif op == "load":
            _, rid, model = msg
            self._pool.submit(self._load, conn, rid, model)
        elif op == "spans":  # this process's span / counter summary (front-end /debug/spans)
            from ..utils import tracing

            conn.post(["spans", msg[1], tracing.summary(float(msg[2]) if len(msg) > 2 else 0.0)])

    def _embed(self, conn, rid, model, texts):
        try:
            h = self.mgr.embedder(model)
            v = h.engine.embed_cpu(list(texts))
            v = v.float().numpy() if hasattr(v, "numpy") else v
            import numpy as np

            v = np.ascontiguousarray(v, dtype=np.float32)
            conn.post(["emb", rid, v.tobytes(), int(v.shape[0]), int(v.shape[1]) if v.ndim > 1 else 0])
        except Exception as e:  # noqa: BLE001 - reported to the client
            conn.post(["err", rid, f"{type(e).__name__}: {e}"])

    def _load(self, conn, rid, model):
        try:
            kind, _ = self.mgr.resolve(model)
            if kind == "generate":
                conn.post(["load", rid, {"kind": kind, **self._meta(self.mgr.generator(model))}])
            else:
                h = self.mgr.embedder(model)
                conn.post(["load", rid, {"kind": kind, "name": h.name, "preset": h.preset, "load_s": h.load_s}])
        except Exception as e:  # noqa: BLE001
            conn.post(["err", rid, f"{type(e).__name__}: {e}"])

    def close(self):
        try:
            self.srv.close()
        finally:
            for c in self._conns:
                c.close()
            if os.path.exists(self.path):
                os.unlink(self.path)
