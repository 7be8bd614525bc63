"""Multi-rank launch hygiene: four ranks that start on a checkout with no built
kernel library build it ONCE (``ops/build.py`` holds an ``fcntl`` lock over the
build directory; the waiters then find the objects' content keys and the library's
build-id stamp current).  A stub compiler
(``HIPCC``) records every invocation, so the test needs no toolchain time."""
import os
import stat
import tempfile

import torch.multiprocessing as mp

STUB = r'''#!/bin/sh
# record the call, then create the -o target like a compiler would (a link
# concatenates its objects, so the build-id stamp object's marker survives)
[ "$1" = "--version" ] && {{ echo "stub hipcc"; exit 0; }}
echo "$PPID $*" >> "{log}"
sleep 0.2
out=""
prev=""
objs=""
for a in "$@"; do
  if [ "$prev" = "-o" ]; then out="$a";
  else case "$a" in *.o) objs="$objs $a";; esac; fi
  prev="$a"
done
[ -n "$out" ] && : > "$out"
case " $* " in *" -shared "*) [ -n "$objs" ] && cat $objs > "$out";; esac
exit 0
'''


def _rank(build_dir, hipcc, q):
    os.environ["APEX_BUILD_DIR"] = build_dir
    os.environ["HIPCC"] = hipcc
    from apex_dqn_amd.ops import build
    q.put(build.build_kernels())


def test_four_ranks_cold_start_build_once():
    with tempfile.TemporaryDirectory() as td:
        log = os.path.join(td, "calls.log")
        hipcc = os.path.join(td, "hipcc")
        with open(hipcc, "w") as f:
            f.write(STUB.format(log=log))
        os.chmod(hipcc, os.stat(hipcc).st_mode | stat.S_IEXEC)
        bdir = os.path.join(td, "build")
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        procs = [ctx.Process(target=_rank, args=(bdir, hipcc, q)) for _ in range(4)]
        for p in procs:
            p.start()
        libs = [q.get(timeout=120) for _ in procs]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        assert len(set(libs)) == 1 and os.path.exists(libs[0])
        calls = open(log).read().splitlines()
        here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        from apex_dqn_amd.ops.build import DEBUG_ONLY_SOURCES    # (built into the debug library only)
        n_src = len([f for f in os.listdir(os.path.join(here, "apex_dqn_amd", "csrc"))
                     if f.endswith(".hip") and f not in DEBUG_ONLY_SOURCES])
        compiles = [c for c in calls if " -c " in c]
        links = [c for c in calls if " -shared " in c]
        assert len(compiles) == n_src, calls          # every source compiled exactly once
        assert len(links) == 1, links                 # one link, by one rank
        assert len({c.split()[0] for c in compiles + links}) == 1   # all by the same process
