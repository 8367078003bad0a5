"""Engine watchdog (SURVEY §5 failure detection): a stall detector for the step loop
of an engine (single GPU, TP driver or TP worker).

The loop calls :meth:`StepWatchdog.beat` after every step and brackets blocking work
with :meth:`busy`.  If the loop is busy and no beat arrives within ``stall_s`` (a hung
kernel, a collective waiting on a dead rank, a deadlocked RCCL call), the watchdog
logs the stall with every thread's Python stack (``faulthandler``), marks itself
unhealthy (served on ``/health``-style endpoints and ``/metrics``) and calls
``on_stall`` -- the serving engine uses it to fail the in-flight requests so clients
get an error instead of hanging.  RCCL/gloo collectives additionally carry the
process-group timeout (``LK_DIST_TIMEOUT_S``, see ``parallel.tp.init_distributed``).
"""
from __future__ import annotations

import faulthandler
import io
import sys
import threading
import time
from typing import Callable, Optional

from .logging import get_logger

log = get_logger("watchdog")


class StepWatchdog:
    def __init__(self, name: str, stall_s: float = 120.0, on_stall: Optional[Callable[[float], None]] = None,
                 poll_s: Optional[float] = None):
        self.name, self.stall_s, self.on_stall = name, stall_s, on_stall
        self.poll_s = poll_s if poll_s is not None else max(0.05, min(5.0, stall_s / 10))
        self.last_beat = time.monotonic()
        self.steps = 0
        self.stalls = 0
        self.healthy = True
        self._busy = 0
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._reported = False
        self._thread = threading.Thread(target=self._run, name=f"lk-watchdog-{name}", daemon=True)
        self._thread.start()

    def beat(self):
        with self._lock:
            self.last_beat = time.monotonic()
            self.steps += 1
            if self._reported:
                log.warning("%s: step loop recovered after a stall", self.name)
            self._reported = False
            self.healthy = True

    class _Busy:
        def __init__(self, wd):
            self.wd = wd

        def __enter__(self):
            with self.wd._lock:
                if self.wd._busy == 0:
                    self.wd.last_beat = time.monotonic()
                self.wd._busy += 1

        def __exit__(self, *exc):
            with self.wd._lock:
                self.wd._busy -= 1
            return False

    def busy(self):
        """Context manager around work that must make progress (a step, a collective)."""
        return StepWatchdog._Busy(self)

    def stalled_for(self) -> float:
        with self._lock:
            return time.monotonic() - self.last_beat if self._busy else 0.0

    def _run(self):
        while not self._stop.wait(self.poll_s):
            dt = self.stalled_for()
            if dt < self.stall_s or self._reported:
                continue
            self._reported = True
            self.healthy = False
            self.stalls += 1
            buf = io.StringIO()
            try:
                faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            except Exception:  # pragma: no cover - stderr without a fileno (pytest capture)
                import traceback

                for tid, frame in sys._current_frames().items():
                    buf.write(f"thread {tid}:\n" + "".join(traceback.format_stack(frame)))
            log.error("%s: no step progress for %.1f s (stall #%d)%s", self.name, dt, self.stalls,
                      ("\n" + buf.getvalue()) if buf.getvalue() else "")
            if self.on_stall is not None:
                try:
                    self.on_stall(dt)
                except Exception:  # pragma: no cover
                    log.exception("on_stall callback failed")

    def stop(self):
        self._stop.set()
