"""Native (C++) runtime: build + load ``_runtime`` (csrc/runtime/*.cpp, pybind11).

:class:`NativeBlockAllocator` is a drop-in for ``engine.block_manager.BlockAllocator``
(the scheduler's per-step hot path); it raises the same ``NoFreeBlocks`` type.
"""
from __future__ import annotations

import importlib
import importlib.util
import os
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
SRC = ROOT / "csrc" / "runtime"
_mod = None


def so_path() -> Path:
    return Path(__file__).resolve().parent / f"_runtime{sysconfig.get_config_var('EXT_SUFFIX') or '.so'}"


def sanitized_so_path() -> Path:
    return ROOT / "build" / "asan" / so_path().name


def _opt(sanitize: bool) -> list:
    return (["-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"]
            if sanitize else ["-O3"])


def tree_hash(sanitize: bool = False) -> str:
    """Content hash of csrc/runtime's sources + flags: the stamp the built module carries."""
    from ..utils.provenance import content_hash

    deps = sorted(SRC.glob("*.cpp")) + sorted(SRC.glob("*.h"))
    return content_hash(deps, " ".join(_opt(sanitize) + ["-std=c++17"]), root=ROOT)


def build(verbose: bool = False, sanitize: bool = False) -> Path:
    """Compile csrc/runtime/*.cpp into the package (``sanitize=True``: an ASan + UBSan build
    under build/asan/, loaded by setting LK_NATIVE_RUNTIME_SO and preloading libasan).
    Rebuilds whenever the embedded source stamp differs from the tree's (content, not mtime)."""
    import pybind11

    from ..utils.provenance import read_stamp

    out = sanitized_so_path() if sanitize else so_path()
    out.parent.mkdir(parents=True, exist_ok=True)
    srcs = sorted(SRC.glob("*.cpp"))
    stamp = tree_hash(sanitize)
    if out.exists() and read_stamp(out) == stamp:
        return out
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, *_opt(sanitize), "-shared", "-fPIC", "-std=c++17", "-Wall", "-pthread", f"-I{pybind11.get_include()}",
           f"-I{sysconfig.get_paths()['include']}", f'-DLK_SOURCE_STAMP="LKSTAMP:{stamp}"', *map(str, srcs),
           "-o", str(out)]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native runtime build failed:\n{r.stderr}")
    print(f"[build] linked {out.relative_to(ROOT)}", flush=True)
    return out


def load():
    global _mod
    if _mod is None:
        alt = os.environ.get("LK_NATIVE_RUNTIME_SO")  # e.g. the ASan/UBSan build
        if alt:
            spec = importlib.util.spec_from_file_location("llm_kubernetes_minikube_sharp4dev_amd.native._runtime", alt)
            _mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(_mod)
        else:
            if SRC.exists() and os.environ.get("LK_ALLOW_STALE_EXT", "0") != "1":
                from ..utils.provenance import check

                check(so_path(), tree_hash(), "native runtime _runtime", "python -m llm_kubernetes_minikube_sharp4dev_amd.native.runtime")
            _mod = importlib.import_module("llm_kubernetes_minikube_sharp4dev_amd.native._runtime")
    return _mod


def available() -> bool:
    try:
        load()
        return True
    except Exception:
        return False


class NativeBlockAllocator:
    """Thin adapter so the native allocator raises the engine's NoFreeBlocks type."""

    def __init__(self, num_blocks: int, block_size: int, prefix_caching: bool = True):
        m = load()
        self._a = m.BlockAllocator(num_blocks, block_size, prefix_caching)
        self._native_exc = m.NoFreeBlocks
        self.num_blocks = num_blocks
        self.block_size = block_size
        self.prefix_caching = prefix_caching

    def allocate(self) -> int:
        from ..engine.block_manager import NoFreeBlocks

        try:
            return self._a.allocate()
        except self._native_exc:
            raise NoFreeBlocks() from None

    def free_block(self, b: int):
        self._a.free_block(b)

    def free_all(self, blocks):
        self._a.free_all(list(blocks))

    def match_prefix(self, tokens):
        blocks, parent = self._a.match_prefix([int(t) for t in tokens])
        return list(blocks), parent

    def register(self, block: int, parent: int, tokens) -> int:
        return self._a.register(block, parent, [int(t) for t in tokens])

    @property
    def num_free(self) -> int:
        return self._a.num_free

    def usage(self) -> float:
        return self._a.usage()

    @property
    def hits(self):
        return self._a.hits

    @property
    def queries(self):
        return self._a.queries

    @property
    def ref(self):
        a = self._a

        class _R:
            def __getitem__(self, b):
                return a.ref(b)

        return _R()


if __name__ == "__main__":  # pragma: no cover
    build(verbose=True)
    _mod = None
    print("native runtime available:", available())
    sys.exit(0)
