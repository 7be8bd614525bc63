"""Out-of-process probe of the data-parallel step's HIP-graph capture (W > 1).

The DP step of the fused NatureCNN learner is captured into HIP graphs with RCCL
collectives inside (``learner/dp_step.py``, ``parallel/rccl.py``).  A capture that
crashes natively (round 5 found stream patterns that segfault inside
``hipStreamEndCapture``, ``profiles/r5_dp_capture_probe.txt``) cannot be caught in
process, and at W > 1 RCCL's P2P / proxy path is only exercised once there are peers.
So before the parent process makes ANY HIP call, every rank spawns ONE fresh child
(``subprocess``; never an exec of the parent) that

* joins its own rendezvous -- the same TCP store as torch.distributed (the torchrun
  agent's store, or rank 0's), under the key prefix ``apex_capture_probe/<restart>`` --
  with an RCCL process group for host-side collectives and its own native RCCL
  communicator for the step, as the parent will have,
* builds each learner variant the parent will run on a small synthetic replay,
  captures the DP step's graphs and replays them once, checks the update is finite,
* writes a per-variant verdict into the store and exits.

Each parent waits for its child (a deadline, and a failure flag any rank may raise
kills the child at once), publishes the child's exit status, and reads every rank's.
A variant keeps its graphs only if every rank's child exited 0 and captured it; else
every parent runs that variant's eager DP step (``learner.graph_fallback``).  The
reference has a single learner process and no such step (``main.py:37-47``).

Test hooks: ``APEX_CAPTURE_PROBE_INJECT=abort`` makes the child abort (SIGABRT) after
its captures, ``=hang`` makes it sleep past the deadline (``abort@1``: on rank 1 only);
``APEX_CAPTURE_PROBE_DRY=1`` skips the GPU work (the CPU test of the rendezvous and the
agreement).
"""
from __future__ import annotations

import datetime
import json
import os
import subprocess
import sys
import time
from typing import Any, Dict, List, Optional

PREFIX = "apex_capture_probe"
CHILD_MODULE = "apex_dqn_amd.runtime.capture_probe"
_KEEP: list = []      # the parent's store client / server stays up for the process group init


def _store(rank: int, world: int, timeout_s: float, client: bool = False):
    """The rendezvous store torch.distributed's ``env://`` uses: the torchrun agent's
    (TORCHELASTIC_USE_AGENT_STORE) as a client, else rank 0 hosts it.  ``multi_tenant``
    lets the later process-group init of this process share the same server."""
    from torch.distributed import TCPStore
    addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29511"))
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true"
    master = (not client) and (not agent) and rank == 0
    return TCPStore(addr, port, None, is_master=master, timeout=datetime.timedelta(seconds=timeout_s),
                    multi_tenant=True)


def _prefix() -> str:
    return f"{PREFIX}/{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}"


def run_probe(variants: List[Dict[str, Any]], rank: int, world: int, local_rank: int,
              timeout: float = 120.0, log=None) -> Dict[str, Any]:
    """Parent side (call before any HIP call).  ``variants``: the learners the parent will
    build, each ``{"name", "cfg" (ApexConfig dict), "steps"}``.  Returns
    ``{"rc": [exit status per rank], "ok": {name: bool}, "seconds": s}``."""
    t0 = time.time()
    pre = _prefix()
    store = _store(rank, world, max(timeout, 60.0) + 60.0)
    spec = dict(rank=rank, world=world, local_rank=local_rank, prefix=pre, variants=variants)
    env = dict(os.environ)
    env["APEX_CAPTURE_PROBE_SPEC"] = json.dumps(spec)
    env.setdefault("GLOO_SOCKET_IFNAME", "lo")
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    out = open(os.devnull, "wb") if log is None else log
    child = subprocess.Popen([sys.executable, "-X", "faulthandler", "-u", "-m", CHILD_MODULE],
                             env=env, cwd=root, stdout=out, stderr=subprocess.STDOUT)
    fail_key = f"{pre}/failed"
    rc: Optional[int] = None
    deadline = time.time() + float(timeout)
    while rc is None:
        rc = child.poll()
        if rc is not None:
            break
        if time.time() > deadline or store.check([fail_key]):
            child.kill()            # a peer failed (its RCCL init / collectives would block) or deadline
            child.wait()
            rc = 124 if time.time() > deadline else 125
            break
        time.sleep(0.05)
    if rc != 0:
        store.set(fail_key, str(rank))
    store.set(f"{pre}/rc/{rank}", str(rc))
    rcs = [int(store.get(f"{pre}/rc/{r}").decode()) for r in range(world)]
    ok = {v["name"]: False for v in variants}
    if all(x == 0 for x in rcs):
        got = [json.loads(store.get(f"{pre}/result/{r}").decode()) for r in range(world)]
        ok = {name: all(bool(g.get(name, False)) for g in got) for name in ok}
    if log is None:
        out.close()
    _KEEP.append(store)
    return {"rc": rcs, "ok": ok, "seconds": round(time.time() - t0, 2)}


def _synthetic_replay(cfg, device, seed: int):
    """A small replay shard with the config's frame stack, prefilled with random frames."""
    import numpy as np
    from ..replay.gpu_replay import GpuReplayShard
    C, A = cfg.frame_stack, cfg.env_conf.action_dim
    cap = max(4096, 4 * cfg.Learner.replay_sample_size)
    rp = GpuReplayShard(cap, cap, cap + 512, C, device=device, seed=seed)
    rng = np.random.default_rng(seed)
    K = cap - 256
    seqs = rp.append_frames(rng.integers(0, 255, (K + C + 8, 84, 84), dtype=np.uint8))
    st = np.stack([seqs[i:i + C] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, A, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    return rp


def _child() -> int:
    spec = json.loads(os.environ["APEX_CAPTURE_PROBE_SPEC"])
    rank, world, pre = int(spec["rank"]), int(spec["world"]), spec["prefix"]
    inject = os.environ.get("APEX_CAPTURE_PROBE_INJECT", "")
    if "@" in inject:
        inject, only = inject.split("@", 1)
        inject = inject if int(only) == rank else ""
    dry = os.environ.get("APEX_CAPTURE_PROBE_DRY", "") == "1"
    import torch
    import torch.distributed as dist
    from ..config import ApexConfig
    from ..parallel.dist import Comm
    store = _store(rank, world, 120.0, client=True)
    res = {v["name"]: True for v in spec["variants"]} if dry else {}
    dev = torch.device("cuda", int(spec["local_rank"])) if not dry else torch.device("cpu")
    # the parent's arrangement: an RCCL process group (host-side collectives, the native
    # communicator's id exchange) beside the native communicator of the step
    kw = {} if dry else {"device_id": dev}
    if not dry:
        torch.cuda.set_device(dev)
    dist.init_process_group("gloo" if dry else "nccl", store=dist.PrefixStore(pre + "/pg", store), rank=rank,
                            world_size=world, timeout=datetime.timedelta(seconds=120), **kw)
    comm = Comm(rank, world, dev)
    for v in ([] if dry else spec["variants"]):
        cfg = ApexConfig.from_dict(v["cfg"])
        rp = _synthetic_replay(cfg, dev, 17 + rank)
        from ..learner.fused_learner import FusedNatureLearner
        L = FusedNatureLearner(cfg, dev, rp, comm=comm)
        p0 = L.p32.clone()
        L.prepare_graphs(multi=True)
        L.steps(max(1, int(v.get("steps", 1))))
        torch.cuda.synchronize(dev)
        ok = L._graphs_enabled() and bool(torch.isfinite(L.p32).all()) and not torch.equal(L.p32, p0)
        res[v["name"]] = bool(ok)
        print(f"[capture probe rank {rank}] {v['name']}: graphs={L._graphs_enabled()} "
              f"fallback={L.graph_fallback} ok={ok}", flush=True)
        del L, rp
        torch.cuda.empty_cache()
    if inject == "abort":
        os.abort()
    if inject == "hang":
        time.sleep(3600)
    nat = getattr(comm, "_native", None)
    if nat is not None:
        nat.check()
        nat.close()
    store.set(f"{pre}/result/{rank}", json.dumps(res))
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(_child())
