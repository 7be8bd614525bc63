"""Bisect a crash in the DP step's graph capture: each variant captures the DP step in a
subprocess of its own (faulthandler on) and reports its exit code.

    python scripts/probe_dp_capture.py [variant ...]
"""
import os
import subprocess
import sys

# in order; the first failing variant ends the run (a crash is not retried on the GPU)
VARIANTS = ["emu_noshard", "emu_shard", "native_w1", "native_w1_shard", "native_w1_ar_shard", "native_w1_inject",
            "torch_w1", "torch_w1_shard", "torch_w1_ar_shard"]


def child(name: str) -> None:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    import numpy as np
    import torch
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm, EmulatedComm
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    shard = "off" if name in ("emu_noshard", "native_w1", "torch_w1") else "on"
    rt = {"use_graphs": True, "graph_steps": 1, "dp_shard_update": shard}
    if name.startswith(("native", "torch")):
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29733", WORLD_SIZE="1", RANK="0")
        comm = Comm.from_env(device=dev, force=True)
        rt.update(force_dp=True, comm_backend=name.split("_")[0],
                  dp_fc_exchange="allreduce" if "_ar" in name else "factors")
        rows = 512
    else:
        comm = EmulatedComm(8, 0, dev)
        rows = 512
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": rows}, "Runtime": rt})
    rp = GpuReplayShard(8000, 8000, 8100, 4, device=dev, seed=1)
    rng = np.random.default_rng(2)
    seqs = rp.append_frames(rng.integers(0, 255, (7000, 84, 84), dtype=np.uint8))
    K = 6000
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    L = FusedNatureLearner(cfg, dev, rp, comm=comm)
    L._inject_capture_failure = name.endswith("inject")
    print(name, "B", L.B, "shard", L._shard, "coll", L.coll.name, "graphs", L._graphs_enabled(), flush=True)
    L._body()
    torch.cuda.synchronize()
    print(name, "eager ok", flush=True)
    L.step()
    torch.cuda.synchronize()
    print(name, "capture + replay ok", bool(torch.isfinite(L.p32).all()), "fallback", L.graph_fallback, flush=True)


def main() -> None:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    names = sys.argv[1:] or VARIANTS
    for n in names:
        r = subprocess.run([sys.executable, "-X", "faulthandler", "-u", os.path.abspath(__file__), "--child", n],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120)
        lines = [ln for ln in r.stdout.splitlines() if ln.strip() and "amdgpu.ids" not in ln]
        print(f"== {n}: rc={r.returncode}", flush=True)
        for ln in lines[-14:]:
            print("   ", ln, flush=True)
        if r.returncode != 0:
            print("stopping at the first failure", flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
