"""Front-end side of the split server: the Ollama HTTP app (``ollama_server.create_app``)
running in a process WITHOUT the GPU, driving one or more engine cores (:mod:`.engine_core`)
over Unix sockets.

* :class:`CoreClient` -- one connection to one engine core (asyncio; one reader task routes
  the per-step token frames to the requests' queues);
* :class:`CorePool` -- every core this front-end knows (one per GPU replica): a request goes
  to the core with the fewest requests outstanding from this front-end plus the core's own
  waiting queue, ties to the most free KV blocks (the stats each token frame carries).  F
  front-end processes share :11434 through SO_REUSEPORT, so with 8 GPUs no single Python
  loop sees every NDJSON chunk (the single-proxy router did);
* :class:`RemoteModelManager` -- the :class:`.model_manager.ModelManager` surface the HTTP
  app uses, with handles whose ``async_engine.stream`` / ``engine.embed_cpu`` go to the cores.
  Tokenisation, chat templates and detokenisation run here, in the front-end.
"""
from __future__ import annotations

import asyncio
import itertools
import os
import time
from dataclasses import dataclass, field
from typing import Optional

import msgpack
import numpy as np

from ..config import Config
from ..engine.sampling import SamplingParams
from ..models.tokenizer import load_tokenizer
from ..utils.logging import get_logger
from .engine_core import _HDR, sp_to_wire
from .model_manager import ModelManager

log = get_logger("serving.remote")


@dataclass
class _SeqView:
    """What the HTTP app reads off a finished engine sequence."""
    output_ids: list = field(default_factory=list)
    num_cached_prefix: int = 0
    finish_reason: Optional[str] = None
    error: Optional[str] = None
    arrival: float = field(default_factory=time.time)
    first_token_at: Optional[float] = None
    finished: bool = False
    num_preemptions: int = 0
    steps_queued: Optional[int] = None
    steps_run: Optional[int] = None
    jumped: int = 0

    def set_accounting(self, acc):
        if isinstance(acc, dict):
            self.num_cached_prefix = acc.get("cached") or 0
            self.num_preemptions = acc.get("preempt") or 0
            self.steps_queued, self.steps_run = acc.get("queued"), acc.get("run")
            self.jumped = acc.get("jumped") or 0
        else:  # (older cores: the cached-prefix count alone)
            self.num_cached_prefix = acc or 0


class CoreClient:
    def __init__(self, path: str):
        self.path = path
        self.reader = self.writer = None
        self.queues: dict = {}    # rid -> asyncio.Queue of token batches
        self.futs: dict = {}      # rid -> Future (embed / load / err)
        self.outstanding = 0
        self.served = 0
        self.stats = [0, 0, 0]    # free KV blocks, waiting, running (last frame)
        self._rid = itertools.count(1)
        self._task = None
        self.loop = None
        self.connected = False
        self.frames = 0           # token frames received (health: the core is stepping)

    async def connect(self, retries: int = 600):
        for i in range(retries):
            try:
                self.reader, self.writer = await asyncio.open_unix_connection(self.path, limit=1 << 24)
                break
            except (FileNotFoundError, ConnectionRefusedError):
                await asyncio.sleep(0.5)
        else:
            raise ConnectionError(f"engine core at {self.path} not reachable")
        self.connected = True
        self.loop = asyncio.get_running_loop()
        self._task = self.loop.create_task(self._read())

    def send(self, msg):
        body = msgpack.packb(msg, use_bin_type=True)
        self.writer.write(_HDR.pack(len(body)) + body)

    async def _read(self):
        try:
            while True:
                n = _HDR.unpack(await self.reader.readexactly(4))[0]
                msg = msgpack.unpackb(await self.reader.readexactly(n), raw=False)
                op = msg[0]
                if op == "tok":
                    self.frames += 1
                    for item in msg[1]:
                        q = self.queues.get(item[0])
                        if q is not None:
                            q.put_nowait(item)
                    self.stats = msg[2]
                else:
                    f = self.futs.pop(msg[1], None)
                    if f is not None and not f.done():
                        if op == "err":
                            f.set_exception(RuntimeError(msg[2]))
                        else:
                            f.set_result(msg)
                    elif op == "err" and msg[1] in self.queues:
                        self.queues[msg[1]].put_nowait([msg[1], [], True, "stop", 0, msg[2]])
        except (asyncio.IncompleteReadError, ConnectionError):
            self.connected = False
            log.error("engine core %s disconnected", self.path)
            for rid, q in list(self.queues.items()):
                q.put_nowait([rid, [], True, "stop", 0, "engine core disconnected"])
            for f in self.futs.values():
                if not f.done():
                    f.set_exception(ConnectionError("engine core disconnected"))

    async def request(self, op: str, *args):
        rid = next(self._rid)
        f = self.loop.create_future()
        self.futs[rid] = f
        self.send([op, rid, *args])
        return await f

    async def stream(self, model: str, ids: list, sp: SamplingParams, timeout_s: Optional[float] = None):
        rid = next(self._rid)
        q: asyncio.Queue = asyncio.Queue()
        self.queues[rid] = q
        self.outstanding += 1
        self.served += 1
        view = _SeqView()
        self.send(["gen", rid, model, list(ids), sp_to_wire(sp), getattr(sp, "format", None)])
        # the request timeout is one timer that drops a sentinel into the queue (asyncio.wait_for
        # per token costs a task per token: the front-end's largest per-chunk cost)
        timer = self.loop.call_later(timeout_s, q.put_nowait, None) if timeout_s else None
        done = False
        try:
            while True:
                item = await q.get()
                if item is None:
                    raise asyncio.TimeoutError()
                _, toks, fin, reason, cached, err = item
                if toks and view.first_token_at is None:
                    view.first_token_at = time.time()
                for i, t in enumerate(toks):
                    view.output_ids.append(t)
                    last = fin and i == len(toks) - 1
                    if last:
                        view.finished, view.finish_reason = True, reason
                        view.set_accounting(cached)
                    yield t, last, view
                if fin:
                    done = True
                    if err or not toks:
                        view.finished, view.finish_reason, view.error = True, reason, err
                        view.set_accounting(cached)
                        yield -1 if err else (toks[-1] if toks else -1), True, view
                    break
        finally:
            if timer is not None:
                timer.cancel()
            self.queues.pop(rid, None)
            self.outstanding -= 1
            if not done:
                self.send(["abort", rid])


class CorePool:
    """The engine cores one front-end routes over (one per GPU replica)."""

    def __init__(self, paths: list[str]):
        self.clients = [CoreClient(p) for p in paths]
        self._rr = itertools.count()

    async def connect(self):
        await asyncio.gather(*(c.connect() for c in self.clients))

    def pick(self) -> CoreClient:
        if len(self.clients) == 1:
            return self.clients[0]
        best = min(c.outstanding + c.stats[1] for c in self.clients)
        cands = [c for c in self.clients if c.outstanding + c.stats[1] == best]
        if len(cands) > 1:
            most = max(c.stats[0] for c in cands)
            cands = [c for c in cands if c.stats[0] == most]
        return cands[next(self._rr) % len(cands)]


class _RemoteWatchdog:
    """The /health view of a remote engine core: the front-end cannot see the core's step
    loop, so ``steps`` counts the token frames received (one per engine step with output) and
    ``stalls`` the cores whose connection dropped."""

    def __init__(self, owner: "_RemoteAsync"):
        self.owner = owner  # the pool is read through the handle (tests swap it)

    @property
    def steps(self) -> int:
        return sum(c.frames for c in self.owner.pool.clients)

    @property
    def stalls(self) -> int:
        return sum(0 if c.connected else 1 for c in self.owner.pool.clients)


class _RemoteAsync:
    def __init__(self, pool: CorePool, model: str, timeout_s: Optional[float]):
        self.pool, self.model, self.request_timeout_s = pool, model, timeout_s
        self.watchdog = _RemoteWatchdog(self)

    @property
    def healthy(self) -> bool:
        """Every engine core connection is up (a core that died closed its socket)."""
        return all(c.connected for c in self.pool.clients)

    async def stream(self, prompt_ids: list, params: SamplingParams, req_id=None, timeout_s=None):
        c = self.pool.pick()
        async for item in c.stream(self.model, prompt_ids, params, timeout_s or self.request_timeout_s):
            yield item

    async def generate(self, prompt_ids: list, params: SamplingParams, req_id=None, timeout_s=None):
        last = None
        async for _, _, s in self.stream(prompt_ids, params, req_id, timeout_s):
            last = s
        return last

    def shutdown(self):
        pass


@dataclass
class _EngineView:
    max_model_len: int
    eos_ids: set
    model: Optional[object] = None


@dataclass
class RemoteGeneratorHandle:
    name: str
    preset: str
    engine: _EngineView
    async_engine: _RemoteAsync
    tokenizer: object
    chat_style: str
    loaded_at: float = field(default_factory=time.time)
    load_s: float = 0.0
    tp: int = 1  # ranks of the cores' tensor-parallel groups (serve --tp)


class _RemoteEmbed:
    def __init__(self, pool: CorePool, model: str, tokenizer=None, max_len: int = 512):
        self.pool, self.model = pool, model
        self.tok, self.max_len = tokenizer, max_len

    def tokenize(self, texts: list) -> list:
        """Token ids as the core's encoder sees them (front-end side: /api/embed reports
        prompt_eval_count without a round trip)."""
        return self.tok.encode_for_embedding(list(texts), self.max_len)

    def embed_cpu(self, texts: list) -> np.ndarray:
        """Blocking (called from the HTTP app's embedding batcher threads, never from the
        core connection's own event loop: that would wait on a coroutine the blocked loop can
        never run)."""
        if not texts:  # nothing to encode: no round trip (the empty /api/embed input)
            return np.zeros((0, 0), np.float32)
        c = self.pool.pick()
        try:
            running = asyncio.get_running_loop()
        except RuntimeError:
            running = None
        if running is not None and running is c.loop:
            raise RuntimeError("_RemoteEmbed.embed_cpu called on the core connection's event loop; "
                               "use embed_async")
        fut = asyncio.run_coroutine_threadsafe(c.request("embed", self.model, list(texts)), c.loop)
        return self._decode(fut.result())

    async def embed_async(self, texts: list) -> np.ndarray:
        """Non-blocking form for callers on the core connection's loop."""
        if not texts:
            return np.zeros((0, 0), np.float32)
        return self._decode(await self.pool.pick().request("embed", self.model, list(texts)))

    @staticmethod
    def _decode(msg) -> np.ndarray:
        _, _, data, rows, dim = msg
        return np.frombuffer(data, dtype=np.float32).reshape(rows, dim) if rows else np.zeros((0, 0), np.float32)


@dataclass
class RemoteEmbedderHandle:
    name: str
    preset: str
    engine: _RemoteEmbed
    loaded_at: float = field(default_factory=time.time)
    load_s: float = 0.0


class RemoteModelManager(ModelManager):
    """ModelManager whose models live in engine-core processes.  Never touches the GPU."""

    def __init__(self, core_paths: list[str], cfg: Optional[Config] = None, aliases: Optional[dict] = None,
                 checkpoints: Optional[dict] = None):
        import threading

        self.cfg = cfg or Config()
        self.device = None
        self.aliases = dict(aliases or {})
        self.checkpoints = dict(checkpoints or {})
        self.engine_overrides = {}
        self.generators: dict = {}
        self.embedders: dict = {}
        self.lock = threading.RLock()
        self.pool = CorePool(core_paths)

    def _load_remote(self, name: str) -> dict:
        c = self.pool.clients[0]
        fut = asyncio.run_coroutine_threadsafe(c.request("load", name), c.loop)
        for other in self.pool.clients[1:]:  # every replica loads it (results are identical)
            asyncio.run_coroutine_threadsafe(other.request("load", name), other.loop).result()
        return fut.result()[2]

    def generator(self, name: str):
        with self.lock:
            if name in self.generators:
                return self.generators[name]
            kind, preset = self.resolve(name)
            if kind != "generate":
                raise KeyError(f"model '{name}' does not support generate")
            meta = self._load_remote(name)
            ck = self.checkpoints.get(name) or self.checkpoints.get(preset)
            h = RemoteGeneratorHandle(name, preset, _EngineView(meta["max_model_len"], set(meta["eos_ids"])),
                                      _RemoteAsync(self.pool, name, self.cfg.agent.request_timeout_s),
                                      load_tokenizer(ck), meta["chat_style"], load_s=meta["load_s"],
                                      tp=int(meta.get("tp", 1)))
            self.generators[name] = h
            return h

    def embedder(self, name: str):
        with self.lock:
            if name in self.embedders:
                return self.embedders[name]
            kind, preset = self.resolve(name)
            if kind != "embed":
                raise KeyError(f"model '{name}' does not support embeddings")
            meta = self._load_remote(name)
            from ..models.configs import ENCODERS

            ck = self.checkpoints.get(name) or self.checkpoints.get(preset)
            h = RemoteEmbedderHandle(name, preset, _RemoteEmbed(self.pool, name, load_tokenizer(ck),
                                                                ENCODERS[preset].max_position),
                                     load_s=meta["load_s"])
            self.embedders[name] = h
            return h

    def shutdown(self):
        pass


def create_frontend_app(core_paths: list[str], cfg: Optional[Config] = None, aliases=None, checkpoints=None,
                        preload: Optional[list] = None):
    """The Ollama HTTP app over remote engine cores (connects at startup)."""
    from .ollama_server import create_app

    mgr = RemoteModelManager(core_paths, cfg, aliases, checkpoints)
    app = create_app(mgr)

    @app.on_event("startup")
    async def _connect():
        await mgr.pool.connect()
        for m in preload or []:
            kind, _ = mgr.resolve(m)
            await asyncio.to_thread(mgr.generator if kind == "generate" else mgr.embedder, m)

    return app


def reuseport_socket(host: str, port: int):
    import socket

    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
    s.bind((host, port))
    s.listen(4096)
    s.set_inheritable(True)
    return s


def core_socket_path(port: int, idx: int) -> str:
    return os.path.join(os.environ.get("LK_CORE_DIR", "/tmp"), f"lk-core-{port}-{idx}.sock")
