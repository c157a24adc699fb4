"""In-tree native build for drtc_amd (no JIT cache, no hipify).

Two extension modules are produced next to this file:

* ``_hipk``   - the CDNA4 kernels (``csrc/kernels/*.hip``) compiled by hipcc
  for ``--offload-arch=gfx950`` plus their pybind11 bindings.
* ``_native`` - the CPU runtime (``csrc/runtime/*.cpp``): bcrypt, the paged
  KV block allocator / scheduler core and the append-only Raft log store,
  compiled by g++.

Usage: ``python -m drtc_amd._build`` (or ``__graft_entry__.build()``).
Objects are rebuilt only when a source or header is newer than the module.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("DRTC_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _pybind_includes() -> list[str]:
    import pybind11

    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _torch_lib() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


def _build_module(name: str, sources: list[str], headers: list[str], compiler: str,
                  cflags: list[str], ldflags: list[str], jobs: int) -> str:
    os.makedirs(BUILD, exist_ok=True)
    target = os.path.join(HERE, name + EXT)
    objs = []
    todo = []
    for src in sources:
        obj = os.path.join(BUILD, name + "_" + os.path.basename(src) + ".o")
        objs.append(obj)
        if _newer(obj, [src] + headers):
            todo.append([compiler, *cflags, "-c", src, "-o", obj])
    if todo:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(_run, todo))
    if todo or _newer(target, objs):
        _run([compiler, "-shared", *objs, "-o", target, *ldflags])
    return target


def build_hip(jobs: int = 8) -> str:
    kdir = os.path.join(CSRC, "kernels")
    sources = sorted(glob.glob(os.path.join(kdir, "*.hip")) + glob.glob(os.path.join(kdir, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(kdir, "*.h")))
    cflags = [
        f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=fast",
        "-Wno-unused-result", f"-I{kdir}", *_pybind_includes(),
    ]
    # hipBLASLt: link the copy PyTorch ships (it is already loaded when torch
    # is imported first, and the soname resolves to it), headers from /opt/rocm
    tlib = _torch_lib()
    return _build_module("_hipk", sources, headers, HIPCC, cflags,
                         [f"--offload-arch={ARCH}", "-fPIC", f"-L{tlib}", "-l:libhipblaslt.so",
                          f"-Wl,-rpath,{tlib}"], jobs)


def build_native(jobs: int = 8) -> str:
    rdir = os.path.join(CSRC, "runtime")
    sources = sorted(glob.glob(os.path.join(rdir, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(rdir, "*.h")))
    cflags = ["-O2", "-fPIC", "-std=c++17", "-fvisibility=hidden", f"-I{rdir}",
              *_pybind_includes()]
    return _build_module("_native", sources, headers, os.environ.get("CXX", "g++"),
                         cflags, ["-fPIC", "-pthread"], jobs)


def build_all(jobs: int = 8, hip: bool = True) -> list[str]:
    out = [build_native(jobs)]
    if hip:
        out.append(build_hip(jobs))
    return out


if __name__ == "__main__":
    for p in build_all(hip="--no-hip" not in sys.argv):
        print(p)
