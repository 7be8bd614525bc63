"""Content-addressed native builds (ops/build.py): an edited source is detected by its
content even when the library on disk is NEWER than the edit (a checkout / copy that
reorders mtimes), the stale library is rebuilt, and the build id compiled into it
matches the tree again.  Runs the real toolchains on throw-away source trees."""
import ctypes
import os
import shutil
import time

import pytest

from apex_dqn_amd.ops import build


def _tree(tmp_path, monkeypatch):
    csrc, out = tmp_path / "csrc", tmp_path / "out"
    (csrc / "runtime").mkdir(parents=True)
    out.mkdir()
    monkeypatch.setattr(build, "CSRC", str(csrc))
    monkeypatch.setattr(build, "OUT", str(out))
    monkeypatch.setattr(build, "RUNTIME_LIB", str(out / "libapex_runtime.so"))
    monkeypatch.setattr(build, "KERNEL_LIB", str(out / "libapex_kernels.so"))
    monkeypatch.setattr(build, "HIP_FLAGS", [f for f in build.HIP_FLAGS if f != build.CSRC] + [str(csrc)])
    return csrc, out


def _call(lib_path, fn):
    cp = lib_path + f".{time.monotonic_ns()}.so"    # dlopen caches by path: load a private copy
    shutil.copy(lib_path, cp)
    f = getattr(ctypes.CDLL(cp), fn)
    f.restype = ctypes.c_int
    return f()


def _age(paths, seconds):
    t = time.time() - seconds
    for p in paths:
        os.utime(p, (t, t))


def test_runtime_rebuilt_on_content_change_with_older_mtime(tmp_path, monkeypatch):
    csrc, out = _tree(tmp_path, monkeypatch)
    src = csrc / "runtime" / "x.cpp"
    src.write_text('extern "C" int apex_probe_value() { return 1; }\n')
    lib = build.ensure_current("runtime")
    assert build.read_stamp(lib) == build.runtime_plan().build_id
    assert not build.library_stale("runtime") and _call(lib, "apex_probe_value") == 1
    # edit the source, then make it look OLDER than the library and its objects
    src.write_text('extern "C" int apex_probe_value() { return 2; }\n')
    _age([str(src)], 3600)
    assert os.path.getmtime(lib) > os.path.getmtime(src)
    assert build.library_stale("runtime")
    with pytest.raises(RuntimeError, match="stale"):
        build.ensure_current("runtime", allow_build=False)
    lib = build.ensure_current("runtime")
    assert not build.library_stale("runtime") and _call(lib, "apex_probe_value") == 2
    # a flag change is a content change too
    monkeypatch.setattr(build, "CXX_FLAGS", build.CXX_FLAGS + ["-DAPEX_SOMETHING=1"])
    assert build.library_stale("runtime")


@pytest.mark.skipif(not os.path.exists(build.HIPCC), reason="hipcc not installed")
def test_kernel_library_header_edit_detected(tmp_path, monkeypatch):
    csrc, out = _tree(tmp_path, monkeypatch)
    (csrc / "v.h").write_text("#define APEX_PROBE_V 7\n")
    (csrc / "k.hip").write_text('#include <hip/hip_runtime.h>\n#include "v.h"\n'
                                '__global__ void probe_k(int* p) { p[0] = APEX_PROBE_V; }\n'
                                'extern "C" int apex_probe_value() { return APEX_PROBE_V; }\n')
    lib = build.ensure_current("kernels")
    assert _call(lib, "apex_probe_value") == 7
    (csrc / "v.h").write_text("#define APEX_PROBE_V 8\n")
    _age([str(csrc / "v.h"), str(csrc / "k.hip")], 3600)
    assert build.library_stale("kernels")
    lib = build.ensure_current("kernels")
    assert not build.library_stale("kernels") and _call(lib, "apex_probe_value") == 8


def test_keys_do_not_depend_on_the_checkout_path(monkeypatch):
    """The same sources under another absolute path (a GPU box runs the tree from a
    scratch directory) build to the same keys: the shipped libraries stay current."""
    ids = build.kernel_plan().build_id, build.runtime_plan().build_id
    import shutil
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        csrc = os.path.join(td, "pkg", "csrc")
        shutil.copytree(build.CSRC, csrc, ignore=shutil.ignore_patterns("__pycache__"))
        monkeypatch.setattr(build, "CSRC", csrc)
        monkeypatch.setattr(build, "PKG", os.path.dirname(csrc))
        monkeypatch.setattr(build, "HIP_FLAGS", [csrc if f.endswith("/csrc") else f for f in build.HIP_FLAGS])
        monkeypatch.setattr(build, "CXX_FLAGS", [csrc if f.endswith("/csrc") else f for f in build.CXX_FLAGS])
        assert (build.kernel_plan().build_id, build.runtime_plan().build_id) == ids
