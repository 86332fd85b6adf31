"""Build the native libraries in-tree (gfx950 only).

* ``_native/libimagent_kernels.so`` - hand-written HIP/CDNA4 kernels
  (``csrc/kernels/*.hip``), hipcc ``--offload-arch=gfx950``.
* ``_native/libimagent_comm.so``    - RCCL communicator + comm stream
  (``csrc/comm``), linked against the ``librccl.so`` bundled with torch (the
  same library c10d's ProcessGroupNCCL uses).
* ``_native/libimagent_runtime.so`` - host runtime (bucket planner / ready
  tracker, ``csrc/runtime``), plain C++.

All three expose a C ABI and are loaded with ctypes (``ops/_lib.py``), so they
do not depend on the torch C++ ABI and compile in seconds. The libraries are
rebuilt only when a source is newer than the output.

Usage: ``python -m imagent_amd.build [--force] [-j N]``
"""

from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
from typing import List

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
OUT = os.path.join(PKG_DIR, "_native")
ARCH = os.environ.get("IMAGENT_OFFLOAD_ARCH", "gfx950")


def _torch_lib_dir() -> str:
    import importlib.util
    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _rocm() -> str:
    return os.environ.get("ROCM_PATH", "/opt/rocm")


def _hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(_rocm(), "bin", "hipcc")
    return p


def _newer(srcs: List[str], out: str) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in srcs)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n  " + " ".join(cmd) + "\n" + r.stdout)


def _compile_hip_object(src: str, obj: str, extra: List[str]) -> str:
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", src, "-o", obj,
           "-munsafe-fp-atomics", "-Wno-unused-result"] + extra
    _run(cmd)
    return obj


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    out = os.path.join(OUT, "libimagent_kernels.so")
    if not force and not _newer(srcs + hdrs, out):
        return out
    objdir = os.path.join(OUT, "obj")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda so: _compile_hip_object(so[0], so[1], []), zip(srcs, objs)))
    tl = _torch_lib_dir()
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs +
         [f"-L{tl}", f"-Wl,-rpath,{tl}"])
    return out


def build_comm(force: bool = False) -> str:
    src = os.path.join(CSRC, "comm", "rccl_comm.cpp")
    out = os.path.join(OUT, "libimagent_comm.so")
    if not force and not _newer([src], out):
        return out
    os.makedirs(OUT, exist_ok=True)
    tl = _torch_lib_dir()
    rccl = os.path.join(tl, "librccl.so")
    if not os.path.exists(rccl):
        rccl = os.path.join(_rocm(), "lib", "librccl.so")
    _run([_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-x", "hip", f"--offload-arch={ARCH}",
          f"-I{_rocm()}/include", src, "-x", "none", "-o", out, rccl, f"-Wl,-rpath,{tl}"])
    return out


def build_runtime(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    out = os.path.join(OUT, "libimagent_runtime.so")
    if not force and not _newer(srcs, out):
        return out
    os.makedirs(OUT, exist_ok=True)
    cxx = shutil.which("g++") or "c++"
    _run([cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", out] + srcs)
    return out


def build_all(force: bool = False, jobs: int = 8, verbose: bool = True) -> List[str]:
    outs = [build_runtime(force), build_kernels(force, jobs), build_comm(force)]
    if verbose:
        for o in outs:
            print("built", os.path.relpath(o, os.path.dirname(PKG_DIR)))
    return outs


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=8)
    a = ap.parse_args(argv)
    build_all(a.force, a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
