"""Opt-in per-thread Python profiles of the serving loops (``LK_PYPROFILE=<dir>``).

The HTTP path's CPU is split over a few Python threads sharing one GIL: uvicorn's event
loop (request parsing, NDJSON streaming) and the LLM engine thread (scheduling,
admission, detokenisation).  ``cProfile`` observes only the thread it is enabled in, so
each loop wraps itself in :func:`thread_profile` and the summary of each thread lands in
its own text file (top functions by own time), written when the loop exits or when the
yielded ``dump`` is called (uvicorn re-raises SIGTERM after its shutdown, so a server
dumps from its shutdown hook).
"""
from __future__ import annotations

import contextlib
import cProfile
import io
import os
import pstats


@contextlib.contextmanager
def thread_profile(name: str, top: int = 45):
    out_dir = os.environ.get("LK_PYPROFILE")
    if not out_dir:
        yield lambda: None
        return
    prof = cProfile.Profile()
    done = []

    def dump():
        if done:
            return
        done.append(1)
        prof.disable()
        _write(prof, out_dir, name, top)

    prof.enable()
    try:
        yield dump
    finally:
        dump()


def _write(prof, out_dir, name, top):
    os.makedirs(out_dir, exist_ok=True)
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats("tottime").print_stats(top)
    st.sort_stats("cumulative").print_stats(top)
    with open(os.path.join(out_dir, f"pyprof_{name}_{os.getpid()}.txt"), "w") as f:
        f.write(s.getvalue())
