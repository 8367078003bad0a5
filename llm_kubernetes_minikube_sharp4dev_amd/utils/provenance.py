"""Build provenance of the native libraries (``_C`` kernels, ``native/_runtime``).

Each library embeds ``LKSTAMP:<hash>`` at link time, where the hash covers the content of
every source / header it is built from and the code-generation flags (``csrc/build.py``,
``native/runtime.py``).  The loaders compare that stamp with a hash of the sources in the
tree BEFORE importing the library (a Python extension cannot be re-imported once loaded),
so a stale binary -- built from other sources than the ones next to it -- fails loudly
instead of running silently.  Object caching in ``csrc/build.py`` keys on the same
content hashes, not on mtimes.
"""
from __future__ import annotations

import hashlib
import mmap
import re
from pathlib import Path
from typing import Iterable, Optional

STAMP_PREFIX = b"LKSTAMP:"
_STAMP_RE = re.compile(re.escape(STAMP_PREFIX) + rb"([0-9a-f]{16})")


def content_hash(files: Iterable[Path], extra: str = "", root: Optional[Path] = None) -> str:
    """16-hex sha256 over (relative path, bytes) of ``files`` (sorted) and ``extra``."""
    h = hashlib.sha256()
    for f in sorted(Path(p) for p in files):
        name = str(f.relative_to(root)) if root is not None else f.name
        h.update(name.encode())
        h.update(b"\0")
        h.update(f.read_bytes())
        h.update(b"\0")
    h.update(extra.encode())
    return h.hexdigest()[:16]


def read_stamp(so: Path) -> Optional[str]:
    """The LKSTAMP hash embedded in a built library, or None (missing file / no stamp)."""
    try:
        with open(so, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
            i = m.find(STAMP_PREFIX)
            while i >= 0:
                hit = _STAMP_RE.match(m, i)
                if hit:
                    return hit.group(1).decode()
                i = m.find(STAMP_PREFIX, i + 1)
    except (OSError, ValueError):
        return None
    return None


class StaleLibraryError(RuntimeError):
    pass


def check(so: Path, expected: str, what: str, rebuild_hint: str) -> str:
    """Raise StaleLibraryError unless ``so`` carries the stamp ``expected``."""
    got = read_stamp(so)
    if got != expected:
        raise StaleLibraryError(
            f"{what} at {so} is stale or unstamped: built from sources {got or '<none>'}, the tree's "
            f"sources hash to {expected}. Rebuild it ({rebuild_hint}); LK_ALLOW_STALE_EXT=1 loads it anyway.")
    return got
