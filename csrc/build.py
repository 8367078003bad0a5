"""In-tree build of the gfx950 kernel library into the package as ``_C*.so``.

Compiles every ``csrc/*.hip`` with ``hipcc --offload-arch=gfx950`` straight from
source (no hipify step: the kernels are written for CDNA4 directly), compiles the
torch bindings, and links one Python extension module next to the package
``__init__``.  Object files are cached under ``build/`` and only rebuilt when the
source, a header or the flags changed (content hashes, not mtimes), so iterating on one
kernel recompiles one file.  The linked library embeds ``LKSTAMP:<hash>`` of every source,
header and flag (``tree_hash``); ``ops._ext`` refuses to load a library whose stamp does not
match the sources next to it (utils/provenance.py).

    python csrc/build.py            # incremental
    python csrc/build.py --clean    # from scratch
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "csrc"
PKG = ROOT / "llm_kubernetes_minikube_sharp4dev_amd"
ARCH = os.environ.get("LK_OFFLOAD_ARCH", "gfx950")
EXT_NAME = "_C"


def _torch_paths():
    import torch
    import torch.utils.cpp_extension as ce

    inc = [Path(p) for p in ce.include_paths()]
    lib = Path(torch.__file__).parent / "lib"
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found")


def _provenance():
    sys.path.insert(0, str(ROOT))
    try:
        from llm_kubernetes_minikube_sharp4dev_amd.utils import provenance
    finally:
        sys.path.pop(0)
    return provenance


def _codegen_flags(debug: bool = False) -> tuple[list[str], list[str]]:
    """Flags that shape the generated code (no include paths of the local install)."""
    common = ["-O3", "-fPIC", "-std=c++17"]
    if debug:
        common += ["-DLK_DEBUG", "-g"]
    kern = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast"]
    bind = common + [f"--offload-arch={ARCH}", "-DTORCH_API_INCLUDE_EXTENSION_H", f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
                     "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1"]
    return kern, bind


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip")) + [CSRC / "bindings.cpp"] + sorted(CSRC.glob("*.h"))


def tree_hash(debug: bool = False) -> str:
    """Content hash of every source / header of ``_C`` plus its code-generation flags: the
    stamp the linked library must carry."""
    kern, bind = _codegen_flags(debug)
    return _provenance().content_hash(sources(), " ".join(kern) + "|" + " ".join(bind), root=ROOT)


def so_path() -> Path:
    return PKG / f"{EXT_NAME}{sysconfig.get_config_var('EXT_SUFFIX') or '.so'}"


def _job_key(src: Path, headers: list[Path], cmd: list[str]) -> str:
    # flags without the local include paths (same image here and on the GPU box)
    return _provenance().content_hash([src, *headers], " ".join(c for c in cmd if not c.startswith("-I")))


def build(clean: bool = False, jobs: int | None = None, verbose: bool = False, debug: bool = False) -> Path:
    global BUILD
    if debug:  # device asserts (LK_DASSERT) on, separate object cache
        BUILD = ROOT / "build" / "csrc-debug"
    if clean and BUILD.exists():
        shutil.rmtree(BUILD)
    BUILD.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    headers = sorted(CSRC.glob("*.h"))
    common = ["-O3", "-fPIC", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-I{CSRC}"]
    if debug:
        common += ["-DLK_DEBUG", "-g"]
    kern_flags = common + [f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-ffp-contract=fast"]
    bind_flags = common + [
        f"--offload-arch={ARCH}",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
        f"-I{py_inc}",
        "-Wno-unused-result",
        "-Wno-deprecated-declarations",
    ] + [f"-I{p}" for p in inc]

    jobs_list = []
    for src in sorted(CSRC.glob("*.hip")):
        obj = BUILD / (src.stem + ".o")
        jobs_list.append((src, obj, [hipcc, *kern_flags, "-c", str(src), "-o", str(obj)]))
    bsrc = CSRC / "bindings.cpp"
    bobj = BUILD / "bindings.o"
    jobs_list.append((bsrc, bobj, [hipcc, *bind_flags, "-x", "hip", "-c", str(bsrc), "-o", str(bobj)]))

    def stale(job):
        src, obj, cmd = job
        key = obj.with_suffix(".o.key")
        return not obj.exists() or not key.exists() or key.read_text() != _job_key(src, headers, cmd)

    todo = [j for j in jobs_list if stale(j)]
    n = jobs or min(8, max(1, (os.cpu_count() or 4)))

    def run(job):
        src, obj, cmd = job
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src.name}\n{r.stdout}\n{r.stderr}")
        obj.with_suffix(".o.key").write_text(_job_key(src, headers, cmd))
        return src.name

    if todo:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for name in ex.map(run, todo):
                print(f"[build] compiled {name}", flush=True)

    out = so_path()
    stamp = tree_hash(debug)
    stamp_src = BUILD / "stamp.cpp"
    stamp_src.write_text('// generated by csrc/build.py: provenance of the linked library\n'
                         f'extern "C" __attribute__((used, visibility("default"))) const char lk_source_stamp[] = '
                         f'"LKSTAMP:{stamp}";\n')
    stamp_obj = BUILD / "stamp.o"
    r = subprocess.run([hipcc, "-O2", "-fPIC", "-c", str(stamp_src), "-o", str(stamp_obj)], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"stamp compile failed\n{r.stderr}")
    objs = [j[1] for j in jobs_list] + [stamp_obj]
    prov = _provenance()
    if not out.exists() or todo or prov.read_stamp(out) != stamp:
        link = [
            hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(out),
            f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            f"-Wl,-rpath,{lib}",
        ]
        if verbose:
            print(" ".join(link), flush=True)
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        print(f"[build] linked {out.relative_to(ROOT)} (stamp {stamp})", flush=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("--debug", action="store_true", help="device bounds checks (LK_DASSERT), -g")
    a = ap.parse_args(argv)
    build(a.clean, a.jobs, a.verbose, a.debug)


if __name__ == "__main__":
    sys.exit(main())
