"""Build the native libraries in-tree (gfx950 only).

* ``_native/libimagent_kernels.so`` - hand-written HIP/CDNA4 kernels
  (``csrc/kernels/*.hip``), hipcc ``--offload-arch=gfx950``.
* ``_native/libimagent_comm.so``    - RCCL communicator + comm stream
  (``csrc/comm``), linked against the ``librccl.so`` bundled with torch (the
  same library c10d's ProcessGroupNCCL uses).
* ``_native/libimagent_runtime.so`` - host runtime (bucket planner / ready
  tracker, ``csrc/runtime``), plain C++.

All three expose a C ABI and are loaded with ctypes (``ops/_lib.py``), so they
do not depend on the torch C++ ABI. A library is rebuilt when the SHA-256 of its
sources, headers and compile command differs from the stamp written next to it
(``<lib>.stamp``) -- content, not mtimes, so a stale ``.so`` that travelled with
a snapshot (newer mtime than an edited source) is never reused.

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


def _digest(srcs: List[str], cmd: List[str]) -> str:
    import hashlib
    h = hashlib.sha256()
    # paths enter by file name only: the tree is built here and run from another directory on the GPU box
    h.update("\0".join(os.path.basename(c) if os.path.isabs(c) else c for c in cmd).encode())
    for s in sorted(srcs):
        h.update(os.path.basename(s).encode() + b"\0")
        with open(s, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _stale(srcs: List[str], out: str, cmd: List[str]) -> bool:
    """True when ``out`` is missing or was built from other sources / flags."""
    if not os.path.exists(out) or not os.path.exists(out + ".stamp"):
        return True
    with open(out + ".stamp") as f:
        return f.read().strip() != _digest(srcs, cmd)


def _stamp(srcs: List[str], out: str, cmd: List[str]) -> None:
    with open(out + ".stamp", "w") as f:
        f.write(_digest(srcs, cmd) + "\n")


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed:\n  " + " ".join(cmd) + "\n" + r.stdout)


HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-Wno-unused-result"]


def _compile_hip_object(src: str, obj: str, extra: List[str]) -> str:
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-c", src, "-o", obj] + HIP_FLAGS + extra
    _run(cmd)
    return obj


def build_kernels(force: bool = False, jobs: int = 8) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    out = os.path.join(OUT, "libimagent_kernels.so")
    key = ["kernels", ARCH] + HIP_FLAGS
    if not force and not _stale(srcs + hdrs, out, key):
        return out
    objdir = os.path.join(OUT, "obj")
    os.makedirs(objdir, exist_ok=True)
    objs = [os.path.join(objdir, os.path.basename(s) + ".o") for s in srcs]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda so: _compile_hip_object(so[0], so[1], []), zip(srcs, objs)))
    tl = _torch_lib_dir()
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs +
         [f"-L{tl}", f"-Wl,-rpath,{tl}"])
    _stamp(srcs + hdrs, out, key)
    return out


def build_kernels_variant(tag: str, defines: List[str], jobs: int = 8) -> str:
    """An A/B build of the kernels library with extra compile flags (e.g. ``-DEPI_QB=4``) into
    ``_native/ab/<tag>/``; a process loads it instead of the default with ``IMAGENT_KERNELS_LIB=<path>``."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.h")))
    d = os.path.join(OUT, "ab", tag)
    out = os.path.join(d, "libimagent_kernels.so")
    key = ["kernels", ARCH] + HIP_FLAGS + list(defines)
    if not _stale(srcs + hdrs, out, key):
        return out
    os.makedirs(os.path.join(d, "obj"), exist_ok=True)
    objs = [os.path.join(d, "obj", os.path.basename(x) + ".o") for x in srcs]
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(lambda so: _compile_hip_object(so[0], so[1], list(defines)), zip(srcs, objs)))
    tl = _torch_lib_dir()
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs +
         [f"-L{tl}", f"-Wl,-rpath,{tl}"])
    _stamp(srcs + hdrs, out, key)
    return out


def build_comm(force: bool = False) -> str:
    src = os.path.join(CSRC, "comm", "rccl_comm.cpp")
    out = os.path.join(OUT, "libimagent_comm.so")
    tl = _torch_lib_dir()
    rccl = os.path.join(tl, "librccl.so")
    if not os.path.exists(rccl):
        rccl = os.path.join(_rocm(), "lib", "librccl.so")
    cmd = [_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-x", "hip", f"--offload-arch={ARCH}",
           f"-I{_rocm()}/include", src, "-x", "none", "-o", out, rccl, f"-Wl,-rpath,{tl}"]
    key = ["comm"] + cmd  # the whole command line: a flag change rebuilds
    if not force and not _stale([src], out, key):
        return out
    os.makedirs(OUT, exist_ok=True)
    _run(cmd)
    _stamp([src], out, key)
    return out


def build_runtime(force: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    out = os.path.join(OUT, "libimagent_runtime.so")
    cxx = shutil.which("g++") or "c++"
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-pthread", "-o", out] + srcs
    key = ["runtime"] + cmd  # the whole command line: a flag change rebuilds
    if not force and not _stale(srcs, out, key):
        return out
    os.makedirs(OUT, exist_ok=True)
    _run(cmd)
    _stamp(srcs, out, key)
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
