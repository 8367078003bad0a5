"""In-tree build of the gfx950 kernel library into the package as ``_C*.so``.

Compiles every ``csrc/*.hip`` with ``hipcc --offload-arch=gfx950`` straight from
source (no hipify step: the kernels are written for CDNA4 directly), compiles the
torch bindings, and links one Python extension module next to the package
``__init__``.  Object files are cached under ``build/`` and only rebuilt when the
source or a header changed, so iterating on one kernel recompiles one file.

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


def _newer(src: Path, obj: Path, headers: list[Path]) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    return src.stat().st_mtime > t or any(h.stat().st_mtime > t for h in headers)


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

    todo = [j for j in jobs_list if _newer(j[0], j[1], headers)]
    n = jobs or min(8, max(1, (os.cpu_count() or 4)))

    def run(job):
        src, obj, cmd = job
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src.name}\n{r.stdout}\n{r.stderr}")
        return src.name

    if todo:
        with cf.ThreadPoolExecutor(max_workers=n) as ex:
            for name in ex.map(run, todo):
                print(f"[build] compiled {name}", flush=True)

    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    out = PKG / f"{EXT_NAME}{suffix}"
    objs = [j[1] for j in jobs_list]
    if not out.exists() or any(o.stat().st_mtime > out.stat().st_mtime for o in objs):
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
        print(f"[build] linked {out.relative_to(ROOT)}", flush=True)
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
