"""Command line.

  serve           Ollama-compatible server on :11434.  On GPUs the split server by default --
                  one engine-core process per GPU + 2 HTTP front-end processes sharing the
                  port (SO_REUSEPORT), each routing over every core; ``--frontends F`` sets F;
                  ``--frontends 0``: one process on one GPU / the CPU, and with ``--gpus N``
                  the round-2 layout (N replica servers + one proxy)
                  ``--tp T``: every engine core is a tensor-parallel group of T processes
                  (rank 0 the core the front-ends talk to, T-1 follower ranks)
  serve-core      one engine core (GPU process of the split server)
  tp-worker       follower rank of a TP group (started by serve / all / rag-app --tp)
  serve-frontend  one HTTP front-end of the split server
  rag-app         Minimal_RAG port (:5103): /health, /rag/search, /agent_rag
  agent-app       Minimal_Agent port (:5217): /health, /agent
  all             server + both apps in one process sharing the engines (in-process
                  LLM/embedding calls, no HTTP hop)
  index           build / refresh the persisted RAG index of a knowledge folder
  fake-apiserver  in-memory kube-apiserver (echoserver fixture) for demos/tests
  router          DP router in front of existing replicas
"""
from __future__ import annotations

import argparse
import asyncio
import os
import subprocess
import sys
import time


def _kv(items):
    out = {}
    for it in items or []:
        k, _, v = it.partition("=")
        out[k] = v
    return out


def _cfg(args):
    from .config import load_config

    cfg = load_config(getattr(args, "config", None))
    if getattr(args, "knowledge", None):
        cfg.rag.knowledge_dir = args.knowledge
    if getattr(args, "kubeconfig", None):
        cfg.agent.kubeconfig = args.kubeconfig
        cfg.agent.fake_cluster = False
    if getattr(args, "index_cache", None):
        cfg.rag.cache_dir = args.index_cache
    return cfg


def _uvicorn(app, host, port, name="http"):
    import uvicorn

    from .utils.pyprof import thread_profile

    with thread_profile(f"loop_{name}") as dump:  # LK_PYPROFILE=<dir>: the event loop's profile
        if getattr(app, "router", None) is not None:
            app.router.on_shutdown.append(dump)
        # keep-alive well past a long generation (uvicorn's 5 s default closes pooled client
        # connections mid-burst), a deep accept queue for bursts of concurrent clients, and a
        # bounded graceful shutdown so a SIGTERM always returns
        uvicorn.run(app, host=host, port=port, log_level="warning", timeout_keep_alive=120,
                    backlog=4096, timeout_graceful_shutdown=5)


def _resolve_tp(args):
    if getattr(args, "tp", None) is None:
        args.tp = _cfg(args).engine.tp_size
    return args.tp


def cmd_serve(args):
    if _resolve_tp(args) > 1:
        if args.frontends == 0:
            raise SystemExit("serve --tp needs the split server (--frontends >= 1): the TP leader is an engine core")
        args.frontends = args.frontends or 2
        return _serve_split(args)
    if args.frontends is None:
        # on GPUs the split server (engine core per GPU + 2 SO_REUSEPORT front-ends) by default:
        # no single Python loop relays every replica's NDJSON chunks, and HTTP framing and
        # (de)tokenisation leave the GPU process (one MI355X at 128 sessions: 93.95 vs 87.31 q/s,
        # profiles/r3_http_split/); on the CPU the one-process server.  device_count() does not
        # initialise the GPU, so the cores can still be started as fresh processes.
        import torch

        on_gpu = args.device != "cpu" and torch.cuda.device_count() > 0
        args.frontends = 2 if (args.gpus > 1 or on_gpu) else 0
    if args.frontends > 0:
        return _serve_split(args)
    if args.gpus > 1:  # --frontends 0: the round-2 single-proxy router over replica servers
        return _serve_replicas(args)
    from .serving.model_manager import ModelManager
    from .serving.ollama_server import create_app

    cfg = _cfg(args)
    mgr = ModelManager(cfg, device=args.device, aliases=_kv(args.alias), checkpoints=_kv(args.checkpoint))
    for m in args.preload or []:
        kind, _ = mgr.resolve(m)
        (mgr.generator if kind == "generate" else mgr.embedder)(m)
    _uvicorn(create_app(mgr), args.host, args.port, "server")


def _model_args(args) -> list:
    g = lambda k: getattr(args, k, None) or []  # noqa: E731
    return sum([["--alias", a] for a in g("alias")], []) + sum([["--checkpoint", c] for c in g("checkpoint")], []) + \
        sum([["--preload", p] for p in g("preload")], []) + (["--config", args.config] if getattr(args, "config", None) else [])


def _supervise(procs, late=()):
    """Block until a child exits (then stop the rest) or a signal arrives.  ``late``: TP
    follower ranks, stopped by their leader (which ``procs`` holds) and terminated only if
    still running after it."""
    import signal

    stop = []
    signal.signal(signal.SIGTERM, lambda *a: stop.append(1))
    late = list(late)
    try:
        while not stop and all(p.poll() is None for p in list(procs) + late):
            time.sleep(0.5)
    except KeyboardInterrupt:
        pass
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
        t0 = time.time()
        while time.time() - t0 < 20 and any(p.poll() is None for p in late):
            time.sleep(0.1)
        for p in late:
            if p.poll() is None:
                p.terminate()
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                p.kill()
    return 0


def _serve_split(args):
    """Engine core(s) + HTTP front-ends.  One GPU: this process is the core and starts the
    front-ends; ``--gpus N``: N core processes (one per GPU) and the front-ends, supervised by
    this process, which never touches the GPU."""
    from .serving.remote import core_socket_path

    mod = "llm_kubernetes_minikube_sharp4dev_amd"
    T = args.tp
    gpus = T if (T > 1 and args.gpus == 1) else args.gpus  # --tp T alone: one group over GPUs 0..T-1
    if gpus % T:
        raise SystemExit(f"--tp {T} must divide --gpus {args.gpus}")
    n_cores = 1 if (T > 1 and args.one_device) else gpus // T
    paths = [core_socket_path(args.port, g) for g in range(n_cores)]
    fe_env = dict(os.environ, HIP_VISIBLE_DEVICES="-1", CUDA_VISIBLE_DEVICES="-1", ROCR_VISIBLE_DEVICES="-1")
    fe_cmd = [sys.executable, "-m", mod, "serve-frontend", "--host", args.host, "--port", str(args.port),
              "--cores", ",".join(paths)] + _model_args(args)
    if T > 1:
        # one TP group per core: rank 0 = the engine core the front-ends route to, ranks 1..T-1
        # follower processes; every rank a fresh process (this supervisor never touches the GPU)
        from .parallel.launch import free_port, rank_env

        dev = ["--device", args.device] if args.device else []
        leaders, followers = [], []
        for g in range(n_cores):
            port = free_port()
            for r in range(T):
                local = 0 if args.one_device else g * T + r
                argv = (["serve-core", "--socket", paths[g]] if r == 0 else ["tp-worker"]) + ["--tp", str(T)]
                p = subprocess.Popen([sys.executable, "-m", mod] + argv + dev + _model_args(args),
                                     env=rank_env(r, T, local, port, args.one_device))
                (leaders if r == 0 else followers).append(p)
        fes = [subprocess.Popen(fe_cmd, env=fe_env) for _ in range(args.frontends)]
        return _supervise(leaders + fes, followers)
    if args.gpus == 1:
        from .serving.engine_core import EngineCore

        mgr = _manager(args)
        core = EngineCore(mgr, paths[0])
        fes = [subprocess.Popen(fe_cmd, env=fe_env) for _ in range(args.frontends)]
        try:
            return _supervise(fes)
        finally:
            core.close()
            mgr.shutdown()
    procs = []
    for g in range(args.gpus):
        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(g), CUDA_VISIBLE_DEVICES=str(g))
        procs.append(subprocess.Popen([sys.executable, "-m", mod, "serve-core", "--socket", paths[g]] +
                                      _model_args(args), env=env))
    procs += [subprocess.Popen(fe_cmd, env=fe_env) for _ in range(args.frontends)]
    return _supervise(procs)


def _manager(args, tp=None, device=None):
    from .serving.model_manager import ModelManager

    mgr = ModelManager(_cfg(args), device=device or getattr(args, "device", None), aliases=_kv(args.alias),
                       checkpoints=_kv(args.checkpoint), tp=tp)
    if mgr.tp is not None:  # the followers are already building this model: load it first
        mgr.generator(mgr.tp_generator_name(args.preload))
    for m in args.preload or []:
        kind, _ = mgr.resolve(m)
        (mgr.generator if kind == "generate" else mgr.embedder)(m)
    return mgr


def cmd_serve_core(args):
    import signal

    from .serving.engine_core import EngineCore

    # block SIGTERM / SIGINT BEFORE any thread starts (engine loop, socket, embed threads
    # inherit the mask): otherwise the supervisor's terminate() can land on one of them with
    # the default action and kill the process without the cleanup below, and Ctrl-C goes to
    # Python's handler instead of sigwait
    sigs = {signal.SIGTERM, signal.SIGINT}
    signal.pthread_sigmask(signal.SIG_BLOCK, sigs)
    tp = dev = None
    if args.tp > 1:  # rank 0 of a TP group (serve --tp): the group's engine core
        from .parallel.launch import init_tp_rank

        tp, dev = init_tp_rank(args.tp, args.device)
        if tp.rank != 0:
            raise SystemExit("serve-core is rank 0 of its TP group; followers run tp-worker")
    mgr = _manager(args, tp, dev)
    core = EngineCore(mgr, args.socket)
    try:
        signal.sigwait(sigs)
    finally:
        core.close()
        mgr.shutdown()
        if tp is not None:
            import torch.distributed as dist

            dist.destroy_process_group()


def cmd_tp_worker(args):
    """Follower rank (1..T-1) of a TP group: this rank's shards of the leader's generator
    (``run_tp_worker``), or with ``--knn-only`` only a corpus shard (``rag-app --tp``)."""
    import torch.distributed as dist

    from .parallel.launch import init_tp_rank
    from .serving.model_manager import ModelManager

    tp, dev = init_tp_rank(args.tp, args.device)
    if tp.rank == 0:
        raise SystemExit("tp-worker runs ranks 1..T-1; rank 0 is the leader")
    if args.knn_only:
        from .parallel.tp_engine import run_tp_worker

        run_tp_worker(None, tp, device=dev)
    else:
        mgr = ModelManager(_cfg(args), device=str(dev), aliases=_kv(args.alias), checkpoints=_kv(args.checkpoint),
                           tp=tp)
        mgr.run_tp_worker(mgr.tp_generator_name(args.preload))
    dist.destroy_process_group()


def cmd_serve_frontend(args):
    import uvicorn

    from .serving.remote import create_frontend_app, reuseport_socket

    app = create_frontend_app(args.cores.split(","), _cfg(args), _kv(args.alias), _kv(args.checkpoint),
                              preload=args.preload)
    from .utils.pyprof import thread_profile

    sock = reuseport_socket(args.host, args.port)
    cfg = uvicorn.Config(app, log_level="warning", timeout_keep_alive=120, backlog=4096, timeout_graceful_shutdown=5)
    with thread_profile(f"frontend_{os.getpid()}") as dump:  # LK_PYPROFILE=<dir>
        app.router.on_shutdown.append(dump)
        uvicorn.Server(cfg).run(sockets=[sock])


def _serve_replicas(args):
    """One process per GPU (HIP_VISIBLE_DEVICES) + router; this parent never touches
    the GPU itself."""
    procs, urls = [], []
    base = args.port + 1
    for g in range(args.gpus):
        env = dict(os.environ, HIP_VISIBLE_DEVICES=str(g), CUDA_VISIBLE_DEVICES=str(g))
        cmd = [sys.executable, "-m", "llm_kubernetes_minikube_sharp4dev_amd", "serve", "--host", "127.0.0.1",
               "--port", str(base + g)] + sum([["--alias", a] for a in args.alias or []], []) + \
            sum([["--checkpoint", c] for c in args.checkpoint or []], []) + \
            sum([["--preload", p] for p in args.preload or []], [])
        if args.config:
            cmd += ["--config", args.config]
        procs.append(subprocess.Popen(cmd, env=env))
        urls.append(f"http://127.0.0.1:{base + g}")
    try:
        from .parallel.router import create_router_app

        _uvicorn(create_router_app(urls), args.host, args.port)
    finally:
        for p in procs:
            p.terminate()


def _backends(args, cfg, mgr=None):
    from .k8s.client import make_client
    from .rag.embedder import LocalEmbedder, OllamaEmbedder
    from .serving.backends import LocalGenerate, OllamaHTTPGenerate

    k8s = make_client(cfg)
    if mgr is not None:
        emb = LocalEmbedder(mgr.embedder(cfg.rag.embed_model).engine)
        llm = LocalGenerate(mgr, cfg.agent.gen_model)
    else:
        emb = OllamaEmbedder(cfg.agent.embedder_url, cfg.rag.embed_model)
        llm = OllamaHTTPGenerate(cfg.agent.ollama_url, cfg.agent.gen_model)
    return emb, llm, k8s


def cmd_rag_app(args):
    from .apps.rag_app import create_rag_app
    from .rag.index import RagIndex

    cfg = _cfg(args)
    if args.ollama_url:
        cfg.agent.ollama_url = cfg.agent.embedder_url = args.ollama_url
    group = None
    if _resolve_tp(args) > 1:  # the corpus sharded over T processes that hold nothing else
        from .parallel.tp_engine import KnnGroup

        tp, dev, workers = _lead_tp_group(args, ["tp-worker", "--tp", str(args.tp), "--knn-only"]
                                          + (["--device", args.device] if args.device else []))
        group = KnnGroup(tp, dev)
    emb, llm, k8s = _backends(args, cfg)
    try:
        if args.synthetic_docs:
            idx = _synthetic_index(args, emb)
            app = create_rag_app(cfg, idx, llm, k8s, build_index=False)
        else:
            idx = RagIndex(emb, backend=cfg.rag.index_backend, device=_index_device(args, group))
            app = create_rag_app(cfg, idx, llm, k8s)
        if group is not None:
            _shard_served_index(idx, group)
            _serve_apps([(app, args.port)], args.host)
        else:
            _uvicorn(app, args.host, args.port, "rag_app")
    finally:
        if group is not None:
            _end_tp_group(group.shutdown, workers)


def _serve_apps(apps, host):
    """Run uvicorn servers [(app, port)] on an event loop in a worker thread until SIGTERM /
    SIGINT reaches this (main) thread, then stop them all and return -- so the caller's
    cleanup (a TP leader stopping its followers) always runs.  (uvicorn serving on the main
    thread installs its own handlers and re-raises the signal after its shutdown, which would
    end the process before that cleanup; with several servers only one of them would stop.)"""
    import signal
    import threading

    import uvicorn

    servers = [uvicorn.Server(uvicorn.Config(a, host=host, port=p, log_level="warning", timeout_keep_alive=120,
                                             backlog=4096, timeout_graceful_shutdown=5)) for a, p in apps]

    async def main():
        await asyncio.gather(*(s.serve() for s in servers))

    th = threading.Thread(target=lambda: asyncio.run(main()), name="lk-http", daemon=True)
    stop = threading.Event()
    prev = {sg: signal.signal(sg, lambda *a: stop.set()) for sg in (signal.SIGTERM, signal.SIGINT)}
    th.start()
    try:
        while th.is_alive() and not stop.wait(0.5):
            pass
    finally:
        for sv in servers:
            sv.should_exit = True
        th.join(timeout=15)
        for sg, h in prev.items():
            signal.signal(sg, h)


def _index_device(args, group=None):
    if group is not None:
        return str(group.device)
    return "cpu" if getattr(args, "device", None) == "cpu" else None


def _lead_tp_group(args, worker_argv):
    """This process becomes rank 0 of a fresh TP group of ``args.tp`` ranks: start ranks
    1..T-1 (``python -m <pkg> <worker_argv> <model args>``) as new processes BEFORE this one
    touches the GPU, then join the group.  -> (TPGroup, device, worker processes)."""
    from .parallel.launch import free_port, init_tp_rank, rank_env, spawn_ranks

    port = free_port()
    os.environ.update(rank_env(0, args.tp, 0, port, args.one_device, base={}))
    argv = list(worker_argv) + _model_args(args)
    workers = spawn_ranks(lambda r: argv, args.tp, port, one_device=args.one_device)
    try:
        tp, dev = init_tp_rank(args.tp, getattr(args, "device", None))
    except BaseException:
        for w in workers:
            w.terminate()
        raise
    return tp, dev, workers


def _end_tp_group(stop_fn, workers, wait_s: float = 30.0):
    """Leader exit: tell the followers to stop, give them ``wait_s`` to leave, then end them."""
    try:
        stop_fn()
    finally:
        t0 = time.time()
        while time.time() - t0 < wait_s and any(w.poll() is None for w in workers):
            time.sleep(0.1)
        for w in workers:
            if w.poll() is None:
                w.terminate()


def _shard_served_index(idx, engine):
    """Spread a built RagIndex's corpus over the engine's TP group (``tp_shard_corpus``) and
    route its searches through the sharded scan (``tp_knn_search``: same hits as one scan)."""
    import torch

    from .parallel.tp_engine import tp_knn_search, tp_shard_corpus

    if len(idx) == 0:
        return None
    corpus = idx._gpu[0] if idx._gpu is not None else torch.from_numpy(idx.matrix())
    shard = tp_shard_corpus(engine, corpus)
    idx.set_sharded(lambda q, k: tp_knn_search(engine, shard, q, k), dim=corpus.shape[1])
    print(f"[rag] {len(idx)} chunks sharded over tp{engine.tp_ctrl.tp.size} "
          f"({shard.corpus.shape[0]} rows on the leader)", flush=True)
    return shard


def _synthetic_index(args, query_embedder):
    """Benchmark bootstrap (benchmarks/http_bench.py): the synthetic runbook corpus of
    bench.py, bulk-embedded ONCE on this process's GPU by an in-process encoder of the same
    preset and seed as the serving process's embedder (the batched replacement of the
    reference's serial per-chunk HTTP embedding, ``RagIndex.cs:47``), kNN on the GPU; every
    request's query embedding still goes through ``query_embedder`` (HTTP /api/embeddings)."""
    import torch

    from .config import Config
    from .engine.embed_engine import EmbeddingEngine
    from .models import build_encoder
    from .models.tokenizer import builtin_tokenizer
    from .rag.corpus import build_chunks
    from .rag.index import RagChunk, RagIndex

    chunks = build_chunks(args.synthetic_docs, 0, workers=8)
    dev = torch.device("cuda" if torch.cuda.is_available() and getattr(args, "device", None) != "cpu" else "cpu")
    enc = build_encoder(args.bulk_embed, device=dev, seed=Config().engine.seed,
                        dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32)
    eng = EmbeddingEngine(enc, builtin_tokenizer(), name=args.bulk_embed, max_tokens_per_batch=131072)
    corpus = eng.embed([c[2] for c in chunks]).to(torch.bfloat16 if dev.type == "cuda" else torch.float32)
    idx = RagIndex(query_embedder, backend="gpu" if dev.type == "cuda" else "exact", device=str(dev))
    idx.chunks = [RagChunk(i, s, t) for i, s, t in chunks]
    if dev.type == "cuda":
        idx.set_gpu_corpus(corpus.contiguous())
    else:
        idx._emb = list(corpus.float().numpy())
    del enc, eng
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    print(f"[rag-app] synthetic index: {len(chunks)} chunks", flush=True)
    return idx


def cmd_agent_app(args):
    from .apps.agent_app import create_agent_app

    cfg = _cfg(args)
    if args.ollama_url:
        cfg.agent.ollama_url = args.ollama_url
    _, llm, k8s = _backends(args, cfg)
    _uvicorn(create_agent_app(cfg, llm, k8s), args.host, args.port)


def cmd_all(args):
    from .apps.agent_app import create_agent_app
    from .apps.rag_app import create_rag_app
    from .rag.index import RagIndex
    from .serving.model_manager import ModelManager
    from .serving.ollama_server import create_app

    cfg = _cfg(args)
    tp = dev = None
    workers = []
    if _resolve_tp(args) > 1:  # this process = rank 0 (engines, apps, the leader's corpus shard)
        args.preload = [cfg.agent.gen_model]
        tp, dev, workers = _lead_tp_group(args, ["tp-worker", "--tp", str(args.tp)]
                                          + (["--device", args.device] if args.device else []))
    mgr = ModelManager(cfg, device=str(dev) if dev is not None else args.device, aliases=_kv(args.alias),
                       checkpoints=_kv(args.checkpoint), tp=tp)
    try:
        if tp is not None:
            mgr.generator(cfg.agent.gen_model)  # the followers are building it
        emb, llm, k8s = _backends(args, cfg, mgr)
        idx = RagIndex(emb, backend=cfg.rag.index_backend, device=_index_device(args, None) if dev is None else str(dev))
        rag = create_rag_app(cfg, idx, llm, k8s)
        if tp is not None:
            _shard_served_index(idx, mgr.generator(cfg.agent.gen_model).engine)
        apps = [(create_app(mgr), cfg.server.ollama_port), (rag, cfg.server.rag_port),
                (create_agent_app(cfg, llm, k8s), cfg.server.agent_port)]
        _serve_apps(apps, args.host)
    finally:
        if tp is not None:
            _end_tp_group(mgr.shutdown, workers)


def cmd_index(args):
    from .rag.embedder import OllamaEmbedder
    from .rag.index import RagIndex

    cfg = _cfg(args)
    if args.local:
        from .serving.model_manager import ModelManager
        from .rag.embedder import LocalEmbedder

        emb = LocalEmbedder(ModelManager(cfg).embedder(cfg.rag.embed_model).engine)
    else:
        emb = OllamaEmbedder(args.ollama_url or cfg.agent.embedder_url, cfg.rag.embed_model)
    idx = RagIndex(emb, backend="exact")
    t0 = time.time()
    stats = idx.build_incremental(cfg.rag.knowledge_dir, args.index_cache or ".lk_index")
    print({**stats, "seconds": round(time.time() - t0, 2)})


def cmd_fake_apiserver(args):
    from .k8s.fake import FakeCluster, make_apiserver_app

    _uvicorn(make_apiserver_app(FakeCluster.default(fault_rate=args.fault_rate, latency_s=args.latency)),
             args.host, args.port)


def cmd_router(args):
    from .parallel.router import create_router_app

    _uvicorn(create_router_app(args.backends.split(",")), args.host, args.port)


def _tp_args(p):
    p.add_argument("--tp", type=int, default=None,
                   help="(default: engine.tp_size of the config, 1) tensor-parallel degree: the generator's weights / KV heads / vocab and the RAG corpus "
                        "sharded over T processes (one per GPU, RCCL + IPC xGMI collectives)")
    p.add_argument("--one-device", action="store_true",
                   help="with --tp: every rank on GPU 0 (gloo + IPC collectives; rehearses TP on a one-GPU box)")


def main(argv=None):
    # a long-running server that dies in native code (a HIP runtime abort, a segfault in an
    # extension thread) leaves every thread's Python stack in its log
    import faulthandler

    faulthandler.enable(all_threads=True)
    # GIL hand-off interval of the serving processes (Python's default is 5 ms: an event loop
    # waking up while the engine thread runs Python waits up to that long for the GIL, per hop)
    sw = os.environ.get("LK_GIL_SWITCH_US")
    if sw:
        sys.setswitchinterval(float(sw) / 1e6)
    ap = argparse.ArgumentParser(prog="llm_kubernetes_minikube_sharp4dev_amd")
    sub = ap.add_subparsers(dest="cmd", required=True)

    def common(p, port):
        p.add_argument("--host", default="127.0.0.1")
        p.add_argument("--port", type=int, default=port)
        p.add_argument("--config", default=None)
        return p

    p = common(sub.add_parser("serve"), 11434)
    p.add_argument("--device", default=None)
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--alias", action="append", help="client-name=preset (e.g. llama3.1:8b=opt-125m)")
    p.add_argument("--checkpoint", action="append", help="name-or-preset=safetensors dir")
    p.add_argument("--preload", action="append")
    p.add_argument("--frontends", type=int, default=None,
                   help="split server: HTTP front-end processes (SO_REUSEPORT) in front of the engine core(s); "
                        "default 2 on GPUs, 0 (one process) on the CPU; 0 with --gpus > 1 = single-proxy router")
    _tp_args(p)
    p.set_defaults(fn=cmd_serve)
    p = common(sub.add_parser("serve-core"), 0)
    p.add_argument("--socket", required=True)
    p.add_argument("--device", default=None)
    p.add_argument("--alias", action="append")
    p.add_argument("--checkpoint", action="append")
    p.add_argument("--preload", action="append")
    p.add_argument("--tp", type=int, default=1, help="rank 0 of a TP group of this size (env RANK / WORLD_SIZE / MASTER_*)")
    p.set_defaults(fn=cmd_serve_core)
    p = common(sub.add_parser("tp-worker"), 0)
    p.add_argument("--tp", type=int, required=True)
    p.add_argument("--device", default=None)
    p.add_argument("--knn-only", action="store_true", help="hold only a corpus shard (rag-app --tp)")
    p.add_argument("--alias", action="append")
    p.add_argument("--checkpoint", action="append")
    p.add_argument("--preload", action="append")
    p.set_defaults(fn=cmd_tp_worker)
    p = common(sub.add_parser("serve-frontend"), 11434)
    p.add_argument("--cores", required=True, help="comma-separated engine-core socket paths")
    p.add_argument("--alias", action="append")
    p.add_argument("--checkpoint", action="append")
    p.add_argument("--preload", action="append")
    p.set_defaults(fn=cmd_serve_frontend)
    for name, port, fn in (("rag-app", 5103, cmd_rag_app), ("agent-app", 5217, cmd_agent_app)):
        p = common(sub.add_parser(name), port)
        p.add_argument("--ollama-url", default=None)
        p.add_argument("--knowledge", default=None)
        p.add_argument("--kubeconfig", default=None)
        p.add_argument("--index-cache", default=None)
        if name == "rag-app":
            p.add_argument("--synthetic-docs", type=int, default=0,
                           help="index bench.py's synthetic corpus of this many documents instead of --knowledge")
            p.add_argument("--bulk-embed", default="bge-base",
                           help="encoder preset for the one-off bulk index build (same seed as the server's)")
            p.add_argument("--device", default=None)
            p.add_argument("--alias", action="append")
            p.add_argument("--checkpoint", action="append")
            _tp_args(p)
        p.set_defaults(fn=fn)
    p = common(sub.add_parser("all"), 0)
    p.add_argument("--device", default=None)
    p.add_argument("--alias", action="append")
    p.add_argument("--checkpoint", action="append")
    p.add_argument("--knowledge", default=None)
    p.add_argument("--kubeconfig", default=None)
    p.add_argument("--index-cache", default=None)
    _tp_args(p)
    p.set_defaults(fn=cmd_all)
    p = sub.add_parser("index")
    p.add_argument("--config", default=None)
    p.add_argument("--knowledge", default=None)
    p.add_argument("--index-cache", default=None)
    p.add_argument("--ollama-url", default=None)
    p.add_argument("--local", action="store_true")
    p.set_defaults(fn=cmd_index)
    p = common(sub.add_parser("fake-apiserver"), 8001)
    p.add_argument("--fault-rate", type=float, default=0.0)
    p.add_argument("--latency", type=float, default=0.0)
    p.set_defaults(fn=cmd_fake_apiserver)
    p = common(sub.add_parser("router"), 11434)
    p.add_argument("--backends", required=True)
    p.set_defaults(fn=cmd_router)
    args = ap.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
