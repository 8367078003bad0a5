"""Build provenance: the native libraries embed a content hash of their sources + flags and
refuse to load when the tree's sources hash differently."""
import shutil
import sys
from pathlib import Path

import pytest

from llm_kubernetes_minikube_sharp4dev_amd.ops import _ext
from llm_kubernetes_minikube_sharp4dev_amd.utils import provenance

ROOT = Path(__file__).resolve().parents[1]


def _build_mod():
    sys.path.insert(0, str(ROOT / "csrc"))
    try:
        import build
    finally:
        sys.path.pop(0)
    return build


def test_built_library_carries_the_tree_stamp():
    b = _build_mod()
    if not b.so_path().exists():
        pytest.skip("extension not built")
    assert provenance.read_stamp(b.so_path()) == b.tree_hash()
    assert _ext.verify_stamp() == b.tree_hash()


def test_content_hash_tracks_content_not_mtime(tmp_path):
    f = tmp_path / "k.hip"
    f.write_text("__global__ void k() {}\n")
    h0 = provenance.content_hash([f], "-O3", root=tmp_path)
    f.touch()
    assert provenance.content_hash([f], "-O3", root=tmp_path) == h0
    f.write_text("__global__ void k() { /* edit */ }\n")
    assert provenance.content_hash([f], "-O3", root=tmp_path) != h0
    assert provenance.content_hash([f], "-O2", root=tmp_path) != provenance.content_hash([f], "-O3", root=tmp_path)


def test_stale_library_is_refused(tmp_path, monkeypatch):
    b = _build_mod()
    if not b.so_path().exists():
        pytest.skip("extension not built")
    so = tmp_path / b.so_path().name
    shutil.copy(b.so_path(), so)

    class Edited:  # the tree after a source edit that was not rebuilt
        @staticmethod
        def tree_hash():
            return "0123456789abcdef"

        @staticmethod
        def so_path():
            return so

    monkeypatch.setattr(_ext, "_csrc_build", lambda: Edited)
    with pytest.raises(provenance.StaleLibraryError, match="stale"):
        _ext.verify_stamp()
    monkeypatch.setenv("LK_ALLOW_STALE_EXT", "1")
    assert _ext.verify_stamp() is None


def test_unstamped_binary_reads_none(tmp_path):
    p = tmp_path / "x.so"
    p.write_bytes(b"\x7fELF....LKSTAMP:unstamped....")
    assert provenance.read_stamp(p) is None
    p.write_bytes(b"junk LKSTAMP:0011223344556677 tail")
    assert provenance.read_stamp(p) == "0011223344556677"


def test_native_runtime_stamp_matches():
    from llm_kubernetes_minikube_sharp4dev_amd.native import runtime

    if not runtime.so_path().exists():
        pytest.skip("runtime not built")
    assert provenance.read_stamp(runtime.so_path()) == runtime.tree_hash()
