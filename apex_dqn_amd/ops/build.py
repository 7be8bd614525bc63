"""In-tree, content-addressed build of the native libraries (no JIT cache, no hipify).

* ``libapex_kernels.so`` -- every ``csrc/*.hip`` compiled by ``hipcc
  --offload-arch=gfx950`` into one shared library with a C ABI (ctypes).
* ``libapex_runtime.so`` -- host C++ runtime (``csrc/runtime/*.cpp``: sum-tree,
  n-step builder, frame ring bookkeeping) built with g++.
* ``libapex_comm.so`` -- the native RCCL communicator (``csrc/comm/rccl_comm.cpp``),
  host code built with hipcc against the RCCL / HIP headers (librccl is dlopen()ed).

Staleness is decided by CONTENT, never by file times: every object carries a key --
the SHA-256 of its source, every header it may include, the compile flags and the
compiler's ``--version`` text -- in a ``.key`` sidecar, and is recompiled when the
key differs.  Each library's build id (a hash of its objects' keys and the link
line) is compiled INTO the library as a marker string (``APEX_BUILD_ID:<hex>``,
also returned by its exported ``apex_build_id()``); :func:`library_stale` reads it
from the file without loading it, and the loaders (``ops/_lib.py``,
``runtime/native.py``, ``parallel/rccl.py``) rebuild a library whose stamp does not
match the tree -- or refuse it when they may not build.  A checkout or copy that
makes a binary look newer than an edited source therefore cannot run stale code.

The libraries land in ``apex_dqn_amd/ops/_build/`` (``APEX_BUILD_DIR`` overrides it)
which ships to the GPU box with the repo snapshot (git-ignored, not
gpurun-ignored).  Builds hold an exclusive ``fcntl`` lock on ``_build/.lock``: the
ranks of a torchrun job that all find the library missing build it once -- the
first takes the lock and compiles, the others wait and then find it current.
"""
from __future__ import annotations

import contextlib
import fcntl
import glob
import hashlib
import os
import re
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional, Sequence

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
CXX = os.environ.get("CXX_APEX", "g++")
BUILD_SCHEMA = "apex-build-2"      # bump when the key recipe itself changes

# -amdgpu-mfma-vgpr-form: MFMA accumulators in ArchVGPRs.  With the default
# AGPR form the register allocator rotates the 32 accumulator registers
# between the two pipeline halves of every GEMM main loop (44 v_accvgpr
# moves per 32 MFMAs -- measured in the ISA); VGPR form makes the loops
# MFMA + ds_read + buffer_load only.
HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-mllvm", "-amdgpu-mfma-vgpr-form", "-Wno-unused-result", "-I", CSRC]
CXX_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-Wno-unused-function", "-I", CSRC]
COMM_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-I", "/opt/rocm/include"]

_STAMP_RE = re.compile(rb"APEX_BUILD_ID:([0-9a-f]{64})")
_COMPILER_IDS: Dict[str, str] = {}


# ------------------------------------------------------------------ keys
def normalize_compiler_version(text: str) -> str:
    """The version facts of a ``--version`` banner, without what varies between two
    installs of the same compiler (install paths, the configuration file line): the
    lines naming a version, path tokens dropped."""
    keep = []
    for line in text.splitlines():
        if "version" not in line.lower() and not line.startswith(("g++", "gcc", "c++")):
            continue
        toks = [t for t in line.split() if "/" not in t]
        keep.append(" ".join(toks))
    return "\n".join(keep) if keep else text.strip()


def compiler_id(cc: str) -> str:
    """The normalized ``cc --version`` (cached per process): part of every key built with
    ``cc``.  A missing compiler raises: the key would not describe what built the
    shipped objects (and nothing could rebuild them here anyway)."""
    if cc not in _COMPILER_IDS:
        r = subprocess.run([cc, "--version"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           timeout=120)
        _COMPILER_IDS[cc] = normalize_compiler_version(r.stdout)
    return _COMPILER_IDS[cc]


def _digest(files: Sequence[str], extra: Sequence[str]) -> str:
    h = hashlib.sha256(BUILD_SCHEMA.encode())
    for f in files:
        h.update(b"\0file\0" + os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    for e in extra:
        h.update(b"\0arg\0" + e.encode())
    return h.hexdigest()


def _rel_flag(f: str) -> str:
    return f.replace(CSRC, "<csrc>").replace(PKG, "<pkg>")


def read_stamp(lib_path: str) -> Optional[str]:
    """The build id compiled into a library (``APEX_BUILD_ID:<hex>``), read from the
    file without loading it; None if missing / unstamped."""
    try:
        with open(lib_path, "rb") as f:
            m = _STAMP_RE.search(f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def _read_key(path: str) -> Optional[str]:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _write_key(path: str, key: str) -> None:
    tmp = path + f".tmp{os.getpid()}"
    with open(tmp, "w") as f:
        f.write(key + "\n")
    os.replace(tmp, path)


def _stamp_source(lib_id: str, tag: str) -> str:
    """A host source defining the library's stamp (marker string + ``apex_build_id()``)."""
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, f"build_id_{tag}.cpp")
    text = ('extern "C" {\n'
            f'__attribute__((used)) const char apex_build_id_marker_{tag}[] = "APEX_BUILD_ID:{lib_id}";\n'
            f'const char* apex_build_id() {{ return apex_build_id_marker_{tag} + 14; }}\n'
            '}\n')
    with open(path, "w") as f:
        f.write(text)
    return path


# ---------------------------------------------------------------- plans
class _Plan:
    """What one library is built from: objects (source -> key) and its build id."""

    def __init__(self, lib: str, cc: str, flags: List[str], srcs: List[str], hdrs: List[str], tag: str,
                 obj_suffix: str = ".o", link: Optional[List[str]] = None, link_libs: Sequence[str] = ()):
        self.lib, self.cc, self.flags, self.tag = lib, cc, list(flags), tag
        self.link = list(link if link is not None else ["-shared", "-fPIC"])
        self.link_libs = list(link_libs)
        cid = compiler_id(cc)
        hdrs = sorted(hdrs)
        # the checkout's absolute path (an include flag) is not content: the tree builds
        # to the same keys wherever it is copied (a GPU box runs it from a scratch path)
        kflags = [_rel_flag(f) for f in self.flags]
        self.objs = []
        for s in srcs:
            o = os.path.join(OUT, os.path.basename(s) + obj_suffix)
            self.objs.append((s, o, _digest([s] + hdrs, kflags + [cid])))
        h = hashlib.sha256((BUILD_SCHEMA + tag).encode())
        for _, o, k in self.objs:
            h.update(os.path.basename(o).encode() + b"=" + k.encode())
        h.update(" ".join(self.link + self.link_libs + [cid]).encode())
        self.build_id = h.hexdigest()

    def stale_objects(self, force: bool = False):
        return [(s, o, k) for s, o, k in self.objs
                if force or not os.path.exists(o) or _read_key(o + ".key") != k]

    def lib_current(self) -> bool:
        return read_stamp(self.lib) == self.build_id


DEBUG_ONLY_SOURCES = ("cu_steal.hip",)


def kernel_plan(debug: bool = False) -> _Plan:
    """``libapex_kernels(.debug).so``: every csrc/*.hip; the debug library builds the
    sources with debug checks or probes with -DAPEX_DEBUG_BOUNDS -DAPEX_PROBE (plus
    ``APEX_DEBUG_DEFS``), the rest are the release objects."""
    every = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    # benchmark-only kernels (cu_steal.hip: the CU-steal proxy of scripts/bench_cu_steal.py)
    # ship in the diagnostic library only
    srcs = [s for s in every if os.path.basename(s) not in DEBUG_ONLY_SOURCES]
    hdrs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.cuh"))
    if not debug:
        return _Plan(KERNEL_LIB, HIPCC, HIP_FLAGS, srcs, hdrs, "kernels",
                     link=["-shared", "-fPIC", f"--offload-arch={ARCH}"])
    srcs = every
    # APEX_DEBUG_DEFS: extra space-separated -D flags for the diagnostic library only
    # (kernel experiments behind #ifdef, e.g. scripts/archive/probe_conv12.py); part of the keys
    extra = [f for f in os.environ.get("APEX_DEBUG_DEFS", "").split() if f.startswith("-D")]
    dflags = HIP_FLAGS + ["-DAPEX_DEBUG_BOUNDS", "-DAPEX_PROBE"] + extra
    rel = kernel_plan(False)
    dbg_srcs = [s for s in srcs if ("APEX_DEBUG_BOUNDS" in open(s).read() or "PROBE(" in open(s).read()
                                    or os.path.basename(s) in DEBUG_ONLY_SOURCES)]
    dp = _Plan(KERNEL_DEBUG_LIB, HIPCC, dflags, dbg_srcs, hdrs, "kernels_debug", obj_suffix=".dbg.o",
               link=["-shared", "-fPIC", f"--offload-arch={ARCH}"])
    # the release objects of the other sources join the debug library
    objs = {s: (s, o, k) for s, o, k in dp.objs}
    dp.objs = [objs.get(s) or next(x for x in rel.objs if x[0] == s) for s in srcs]
    dp.release_part = [x for x in rel.objs if x[0] not in objs]
    h = hashlib.sha256((BUILD_SCHEMA + "kernels_debug").encode())
    for _, o, k in dp.objs:
        h.update(os.path.basename(o).encode() + b"=" + k.encode())
    h.update(" ".join(dp.link + [compiler_id(HIPCC)]).encode())
    dp.build_id = h.hexdigest()
    return dp


def runtime_plan() -> _Plan:
    srcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    hdrs = glob.glob(os.path.join(CSRC, "runtime", "*.h"))
    return _Plan(RUNTIME_LIB, CXX, CXX_FLAGS, srcs, hdrs, "runtime", obj_suffix=".rt.o",
                 link=["-shared", "-fPIC"], link_libs=["-lpthread"])


def comm_plan() -> _Plan:
    srcs = [os.path.join(CSRC, "comm", "rccl_comm.cpp")]
    return _Plan(COMM_LIB, HIPCC, COMM_FLAGS, srcs, [], "comm", obj_suffix=".comm.o",
                 link=["-shared", "-fPIC"], link_libs=["-ldl"])


_PLANS = {"kernels": lambda: kernel_plan(False), "kernels_debug": lambda: kernel_plan(True),
          "runtime": runtime_plan, "comm": comm_plan}


def library_stale(which: str = "kernels") -> bool:
    """True when the library's compiled-in build id does not match the current tree
    (sources, headers, flags, compiler), or it is missing."""
    return not _PLANS[which]().lib_current()


# ---------------------------------------------------------------- build
def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


def _compile(job) -> None:
    cmd, o, key = job
    tmp = o + f".tmp{os.getpid()}"
    _run(cmd + ["-o", tmp])
    os.replace(tmp, o)
    _write_key(o + ".key", key)


def _build_plan(p: _Plan, force: bool, jobs: int, verbose: bool) -> str:
    os.makedirs(OUT, exist_ok=True)
    todo = [([p.cc] + p.flags + ["-c", s], o, k) for s, o, k in p.stale_objects(force)]
    for rp in getattr(p, "release_part", ()):   # debug library: release objects it links
        s, o, k = rp
        if force or not os.path.exists(o) or _read_key(o + ".key") != k:
            todo.append(([HIPCC] + HIP_FLAGS + ["-c", s], o, k))
    if todo:
        with ThreadPoolExecutor(max_workers=jobs) as ex:
            list(ex.map(_compile, todo))
    if force or todo or not p.lib_current():
        stamp_src = _stamp_source(p.build_id, p.tag)
        stamp_obj = os.path.join(OUT, f"build_id_{p.tag}.o")
        _run([CXX, "-O1", "-fPIC", "-c", stamp_src, "-o", stamp_obj])
        # link to a temporary name, then rename: a process that maps the library
        # never sees a half-written file
        tmp = p.lib + f".tmp{os.getpid()}"
        _run([p.cc] + p.link + ["-o", tmp] + [o for _, o, _ in p.objs] + [stamp_obj] + p.link_libs)
        os.replace(tmp, p.lib)
    if verbose:
        print(f"built {p.lib} ({len(todo)} objects recompiled, id {p.build_id[:12]})")
    return p.lib


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
        return _build_plan(kernel_plan(debug), force, jobs, verbose)


def build_runtime(force: bool = False, verbose: bool = False) -> str:
    with build_lock():
        return _build_plan(runtime_plan(), force, 4, verbose)


def build_comm(force: bool = False, verbose: bool = False) -> str:
    with build_lock():
        return _build_plan(comm_plan(), force, 1, verbose)


def ensure_current(which: str, allow_build: bool = True) -> str:
    """Path of a library whose stamp matches the tree: rebuilt first when stale and
    ``allow_build``; a stale library that may not be rebuilt is refused."""
    p = _PLANS[which]()
    if p.lib_current():
        return p.lib
    if not allow_build:
        raise RuntimeError(f"{p.lib} is stale or missing (build id {read_stamp(p.lib)} != tree {p.build_id}); "
                           f"run `python -m apex_dqn_amd.ops.build`")
    {"kernels": lambda: build_kernels(), "kernels_debug": lambda: build_kernels(debug=True),
     "runtime": build_runtime, "comm": build_comm}[which]()
    if not _PLANS[which]().lib_current():     # pragma: no cover - would be a key-recipe bug
        raise RuntimeError(f"{p.lib}: rebuilt library still does not match the tree")
    return p.lib


def build_all(force: bool = False, verbose: bool = True, debug: bool = True) -> None:
    with build_lock():
        build_runtime(force=force, verbose=verbose)
        build_comm(force=force, verbose=verbose)
        build_kernels(force=force, verbose=verbose)
        if debug:
            build_kernels(force=force, verbose=verbose, debug=True)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
