"""In-tree build of the native libraries (no JIT cache, no hipify).

* ``libapex_kernels.so`` -- every ``csrc/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` into one shared library with a C ABI (ctypes).
* ``libapex_runtime.so`` -- host C++ runtime (``csrc/runtime/*.cpp``: sum-tree,
  n-step builder, frame ring bookkeeping) built with g++.
* ``libapex_comm.so`` -- the native RCCL communicator (``csrc/comm/rccl_comm.cpp``),
  host code built with hipcc against the RCCL / HIP headers (librccl is dlopen()ed).

Objects are rebuilt only when their source (or a header) is newer.  The
libraries land in ``apex_dqn_amd/ops/_build/`` (``APEX_BUILD_DIR`` overrides it)
which ships to the GPU box with the repo snapshot (git-ignored, not
gpurun-ignored).  Builds hold an exclusive ``fcntl`` lock on ``_build/.lock``: the
ranks of a torchrun job that all find the library missing build it once -- the
first takes the lock and compiles, the others wait and then find it fresh.
"""
from __future__ import annotations

import contextlib
import fcntl
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(PKG, "csrc")
OUT = os.environ.get("APEX_BUILD_DIR") or os.path.join(HERE, "_build")
KERNEL_LIB = os.path.join(OUT, "libapex_kernels.so")
KERNEL_DEBUG_LIB = os.path.join(OUT, "libapex_kernels_debug.so")
RUNTIME_LIB = os.path.join(OUT, "libapex_runtime.so")
COMM_LIB = os.path.join(OUT, "libapex_comm.so")
ARCH = os.environ.get("APEX_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# -amdgpu-mfma-vgpr-form: MFMA accumulators in ArchVGPRs.  With the default
# AGPR form the register allocator rotates the 32 accumulator registers
# between the two pipeline halves of every GEMM main loop (44 v_accvgpr
# moves per 32 MFMAs -- measured in the ISA); VGPR form makes the loops
# MFMA + ds_read + buffer_load only.
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-mllvm", "-amdgpu-mfma-vgpr-form", "-Wno-unused-result", "-I", CSRC]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I", CSRC]


def _newer(src_files: List[str], target: str) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


@contextlib.contextmanager
def build_lock():
    """Exclusive inter-process lock over the build directory (re-entrant per process
    through the depth counter: build_all -> build_kernels)."""
    os.makedirs(OUT, exist_ok=True)
    if _LOCK["depth"] > 0:
        _LOCK["depth"] += 1
        try:
            yield
        finally:
            _LOCK["depth"] -= 1
        return
    with open(os.path.join(OUT, ".lock"), "a+") as f:
        fcntl.flock(f.fileno(), fcntl.LOCK_EX)
        _LOCK["depth"] = 1
        try:
            yield
        finally:
            _LOCK["depth"] = 0
            fcntl.flock(f.fileno(), fcntl.LOCK_UN)


_LOCK = {"depth": 0}


def build_kernels(force: bool = False, jobs: int = 8, verbose: bool = False, debug: bool = False) -> str:
    """``debug=True`` builds ``libapex_kernels_debug.so`` with ``-DAPEX_DEBUG_BOUNDS``
    (device-side index checks in the replay kernels, see csrc/sumtree.hip) and
    ``-DAPEX_PROBE`` (in-kernel phase stamps, csrc/mfma_common.h)."""
    with build_lock():
        return _build_kernels(force, jobs, verbose, debug)


def _build_kernels(force: bool, jobs: int, verbose: bool, debug: bool) -> str:
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.cuh"))
    lib_path = KERNEL_DEBUG_LIB if debug else KERNEL_LIB
    suffix = ".dbg.o" if debug else ".o"
    # APEX_DEBUG_DEFS: extra space-separated -D flags for the diagnostic library only
    # (kernel experiments behind #ifdef, e.g. scripts/probe_conv12.py)
    extra = [f for f in os.environ.get("APEX_DEBUG_DEFS", "").split() if f.startswith("-D")]
    flags = HIP_FLAGS + (["-DAPEX_DEBUG_BOUNDS", "-DAPEX_PROBE"] + extra if debug else [])
    objs = []
    todo = []
    if debug:
        build_kernels(force=force, jobs=jobs)  # sources without debug checks reuse the release objects
    for s in srcs:
        text = open(s).read()
        dbg_src = debug and ("APEX_DEBUG_BOUNDS" in text or "PROBE(" in text)
        o = os.path.join(OUT, os.path.basename(s) + (suffix if dbg_src else ".o"))
        objs.append(o)
        if debug and not dbg_src:
            continue
        if force or _newer([s] + headers + [os.path.abspath(__file__)], o):
            todo.append([HIPCC] + flags + ["-c", s, "-o", o])
    if todo:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(_run, todo))
    if force or todo or _newer(objs, lib_path):
        # link to a temporary name, then rename: a process that maps the library
        # never sees a half-written file
        tmp = lib_path + f".tmp{os.getpid()}"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs)
        os.replace(tmp, lib_path)
    if verbose:
        print(f"built {lib_path} ({len(todo)} objects recompiled)")
    return lib_path


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    with build_lock():
        return _build_runtime(force, verbose)


def _build_runtime(force: bool, verbose: bool) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    if srcs and (force or _newer(srcs + hdrs, RUNTIME_LIB)):
        _run(["g++"] + CXX_FLAGS + ["-shared", "-o", RUNTIME_LIB] + srcs + ["-lpthread"])
        if verbose:
            print(f"built {RUNTIME_LIB}")
    return RUNTIME_LIB


def build_comm(force: bool = False, verbose: bool = False) -> str:
    with build_lock():
        return _build_comm(force, verbose)


def _build_comm(force: bool, verbose: bool) -> str:
    src = os.path.join(CSRC, "comm", "rccl_comm.cpp")
    if force or _newer([src], COMM_LIB):
        _run([HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", "-I", "/opt/rocm/include", src, "-o", COMM_LIB, "-ldl"])
        if verbose:
            print(f"built {COMM_LIB}")
    return COMM_LIB


def build_all(force: bool = False, verbose: bool = True, debug: bool = True) -> None:
    with build_lock():
        build_runtime(force=force, verbose=verbose)
        build_comm(force=force, verbose=verbose)
        build_kernels(force=force, verbose=verbose)
        if debug:
            build_kernels(force=force, verbose=verbose, debug=True)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
