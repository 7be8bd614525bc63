"""BASELINE config 4 on one MI355X: the Atari 2M-transition prioritized replay.

The reference keeps ``soft_capacity`` transitions in one Python list (``replay.py:44-57,
71-80``, ``parameters.json:28``); here a replay shard is an HBM frame ring + records +
64-ary sum tree (``replay/gpu_replay.py``).  For each shard size -- the 100k shard every
other bench uses, a 312.5k shard (one of 8 ranks' share of a 2M replay with 25 %
headroom, ``ApexConfig.shard_capacity``) and the whole 2.5M-slot replay on ONE GPU -- this
script measures on synthetic frames:

* the learner's grad-steps/s at batch 512 (bench.py's harness: HIP graphs, warm-up, the
  eviction + rebuild at its 100-step cadence inside the timed window);
* ``remove_to_fit`` + exact tree ``rebuild`` at that size, with the eviction sized to the
  inserts of 100 learner steps at the end-to-end rate (500k frames/s at ~2.3k steps/s
  is ~22k transitions per 100 steps), and its cost amortised over 100 steps;
* actor insert throughput (frame append + n-step records, 256 transitions per call);
* HBM in use against the device's capacity.

    python scripts/bench_replay_2m.py --out gpurun_out/replay_2m.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def build(cap: int, soft: int, device, actions: int = 4):
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    frames_cap = cap + 4096
    rp = GpuReplayShard(cap, soft, frames_cap, 4, alpha=0.6, beta=0.4, device=device, seed=1)
    # synthetic frames straight into HBM (chunked: one randint buffer of the whole ring
    # would double the peak), then records over them
    g = torch.Generator(device=device).manual_seed(1000)
    step = 1 << 18
    for s in range(0, frames_cap, step):
        n = min(step, frames_cap - s)
        rp.frames[s:s + n].copy_(torch.randint(0, 256, (n, 84, 84), generator=g, device=device, dtype=torch.uint8))
    rp.frame_head = frames_cap
    rng = np.random.default_rng(0)
    chunk = 1 << 16
    for s in range(0, cap, chunk):
        K = min(chunk, cap - s)
        base = rng.integers(0, frames_cap - 8, size=K)
        st = base[:, None] + np.arange(4)[None]
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, actions, K),
                       R=rng.normal(size=K).astype(np.float32), Gamma=np.full(K, 0.99 ** 3, np.float32),
                       priority=rng.random(K).astype(np.float32) + 0.01))
    rp.rebuild()
    torch.cuda.synchronize()
    return rp


def replay_bytes(rp) -> dict:
    t = {"frames": rp.frames, "tree_leaf": rp.leaf, "tree_nodes": rp.nodes}
    rec = sum(x.numel() * x.element_size() for x in (rp.obs, rp.nxt, rp.act, rp.rew, rp.gam, rp.gen))
    out = {k: v.numel() * v.element_size() for k, v in t.items()}
    out["records"] = rec
    out["total"] = sum(out.values())
    return out


def time_evict_rebuild(rp, n_new: int, reps: int = 5) -> dict:
    """Insert ``n_new`` transitions past the soft capacity, then time remove_to_fit
    (FIFO zeroing of the evicted leaves) and rebuild (exact recompute of every level)."""
    rng = np.random.default_rng(7)
    ev, rb = [], []
    for _ in range(reps):
        base = rng.integers(0, rp.F - 8, size=n_new)
        st = base[:, None] + np.arange(4)[None]
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, n_new), R=np.zeros(n_new, np.float32),
                       Gamma=np.full(n_new, 0.97, np.float32), priority=rng.random(n_new).astype(np.float32) + 0.01))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n_ev = rp.remove_to_fit()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        rp.rebuild()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        ev.append((t1 - t0) * 1e3)
        rb.append((t2 - t1) * 1e3)
    return {"evicted_per_call": int(n_ev), "remove_to_fit_ms": float(np.median(ev)),
            "rebuild_ms": float(np.median(rb))}


def time_inserts(rp, n_calls: int = 200, K: int = 256) -> dict:
    """Actor-side insert path: append K new frames + K n-step records per call."""
    rng = np.random.default_rng(9)
    frames = rng.integers(0, 255, (K, 84, 84), dtype=np.uint8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n_calls):
        seqs = rp.append_frames(frames)
        st = np.maximum(seqs[:, None] - 3 + np.arange(4)[None], 0)
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, K), R=np.zeros(K, np.float32),
                       Gamma=np.full(K, 0.97, np.float32), priority=np.ones(K, np.float32)))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"transitions_per_s": n_calls * K / dt, "frames_per_s": n_calls * K / dt, "calls": n_calls, "K": K}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="100000,312500,2500000")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--evict-per-100", type=int, default=22000)
    ap.add_argument("--out", default="gpurun_out/replay_2m.json")
    args = ap.parse_args()
    import bench
    from apex_dqn_amd.parallel.dist import Comm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm(0, 1, dev)
    free0, total = torch.cuda.mem_get_info(dev)
    res = {"device_hbm_bytes": total, "sizes": []}
    bargs = bench.parser().parse_args(["--no-bf16-extra"])
    for cap in [int(x) for x in args.sizes.split(",")]:
        soft = int(cap / 1.25) if cap > 100000 else cap        # 2M soft / 2.5M physical (25 % headroom)
        t0 = time.perf_counter()
        rp = build(cap, soft, dev)
        rp.remove_to_fit()                  # down to the soft capacity before timing
        rp.rebuild()
        torch.cuda.synchronize()
        build_s = time.perf_counter() - t0
        bargs.replay = cap
        cfg, L = bench.make_learner(bargs, "fp32", dev, comm, 0, rp)
        cfg.Learner.remove_old_xp_freq = 100
        r = bench.measure(cfg, L, rp, comm, args.warmup, args.steps, prep_warm=4)
        step_ms = 1e3 * r["dt"] / args.steps
        er = time_evict_rebuild(rp, args.evict_per_100)
        ins = time_inserts(rp)
        free, _ = torch.cuda.mem_get_info(dev)
        row = {"capacity": cap, "soft_capacity": soft, "tree_levels": rp.L, "build_s": round(build_s, 1),
               "steps_per_s": round(args.steps / r["dt"], 1), "ms_per_step": round(step_ms, 4),
               "graph_captures_in_timed": r["graph_captures_in_timed"],
               **{k: round(v, 3) if isinstance(v, float) else v for k, v in er.items()},
               "evict_rebuild_share_of_100_steps": round((er["remove_to_fit_ms"] + er["rebuild_ms"]) /
                                                         (100 * step_ms), 5),
               "insert": {k: round(v, 1) if isinstance(v, float) else v for k, v in ins.items()},
               "replay_bytes": replay_bytes(rp), "hbm_used_bytes": int(total - free),
               "hbm_used_fraction": round((total - free) / total, 4)}
        res["sizes"].append(row)
        print(json.dumps(row), flush=True)
        del L, rp
        torch.cuda.empty_cache()
    base = res["sizes"][0]["ms_per_step"]
    for row in res["sizes"]:
        row["step_vs_first"] = round(row["ms_per_step"] / base - 1.0, 4)
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({"steps_vs_100k": [r["step_vs_first"] for r in res["sizes"]]}))


if __name__ == "__main__":
    main()
