"""Loader for the in-tree HIP kernel library ``_C`` (built by ``csrc/build.py``).

Policy: tensors on the GPU ALWAYS go through the HIP kernels.  If the extension is
missing while a GPU is present, :func:`lib` raises — there is no silent eager
fallback on the device (set ``LK_FORCE_REFERENCE=1`` to opt into the torch
reference implementations explicitly, e.g. for A/B numerics).  CPU tensors use the
fp32 torch references in :mod:`.reference`.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def force_reference() -> bool:
    return os.environ.get("LK_FORCE_REFERENCE", "0") not in ("", "0", "false", "False")


def try_lib():
    """Return the extension module or None (never raises)."""
    global _mod, _err
    if _mod is not None:
        return _mod
    with _lock:
        if _mod is None and _err is None:
            try:
                import torch  # noqa: F401  (loads libamdhip64 / libtorch first)

                alt = os.environ.get("LK_LIB_PATH")
                if not alt:
                    verify_stamp()
                if alt:  # A/B knob: another build of this extension (e.g. the previous commit's)
                    spec = importlib.util.spec_from_file_location("llm_kubernetes_minikube_sharp4dev_amd._C", alt)
                    _mod = importlib.util.module_from_spec(spec)
                    spec.loader.exec_module(_mod)
                else:
                    _mod = importlib.import_module("llm_kubernetes_minikube_sharp4dev_amd._C")
                if os.environ.get("LK_WS_ROT"):  # weight-streaming GEMM K-step rotation override
                    _mod.ws_set_rot(int(os.environ["LK_WS_ROT"]))
            except Exception as e:  # pragma: no cover - depends on build state
                _err = e
    return _mod


def _csrc_build():
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[2]
    if not (root / "csrc" / "build.py").exists():
        return None
    sys.path.insert(0, str(root / "csrc"))
    try:
        import build as _b  # csrc/build.py
    finally:
        sys.path.pop(0)
    return _b


def verify_stamp() -> str | None:
    """Refuse a ``_C`` whose embedded source stamp differs from the sources in this tree
    (a stale binary would otherwise run silently).  ``LK_EXT_AUTOBUILD=1`` rebuilds first;
    ``LK_ALLOW_STALE_EXT=1`` skips the check.  Returns the stamp (None: no csrc/ tree)."""
    b = _csrc_build()
    if b is None or os.environ.get("LK_ALLOW_STALE_EXT", "0") == "1":
        return None
    from ..utils import provenance

    expected = b.tree_hash()
    if os.environ.get("LK_EXT_AUTOBUILD", "0") == "1" and provenance.read_stamp(b.so_path()) != expected:
        b.build()
    return provenance.check(b.so_path(), expected, "HIP kernel library _C", "python csrc/build.py")


def lib():
    m = try_lib()
    if m is None:
        raise RuntimeError(
            "HIP kernel library `_C` is not built/loadable "
            f"({_err!r}); run `python csrc/build.py` (gfx950)."
        )
    return m


def available() -> bool:
    return try_lib() is not None


def use_hip(t) -> bool:
    """True when tensor ``t`` must take the HIP path."""
    return bool(getattr(t, "is_cuda", False)) and not force_reference()


def build_if_needed(verbose: bool = False):
    """Compile the library in-tree (used by __graft_entry__.build and tests)."""
    return _csrc_build().build(verbose=verbose)
