"""Is a multi-stream HIP graph launch host-bound?  For each configuration, the host time of
``graph.replay()`` of the learner's multi-update graph (returns once every node is enqueued)
next to the wall time of the same launches with the GPU drained; also the graph's node count
per update.

    python scripts/probe_graph_launch.py --out gpurun_out/graph_launch.jsonl
"""
import argparse
import json
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

CONFIGS = {
    "single_512": [],
    "single_74": ["--batch", "74"],
    "emulated_w8": ["--emulate-world", "8"],
    "emulated_w8_graph1": ["--emulate-world", "8", "--graph-steps", "1"],
}


def probe(name, extra, launches):
    import bench
    from apex_dqn_amd.parallel.dist import Comm, EmulatedComm
    args = bench.parser().parse_args(["--no-bf16-extra"] + extra)
    dev = torch.device("cuda", 0)
    comm = EmulatedComm(args.emulate_world, 0, dev) if args.emulate_world else Comm(0, 1, dev)
    if args.emulate_world:
        args.force_dp = True
    replay = bench.make_replay(args, dev, 0)
    cfg, L = bench.make_learner(args, "fp32", dev, comm, 0, replay)
    for _ in range(3):
        L.steps(L.rt.graph_steps) if hasattr(L, "steps") else L.step()
    L.prepare_graphs()
    g, k = (L._multi, int(L.rt.graph_steps)) if L._multi is not None else (L._graphs, 1)
    torch.cuda.synchronize()
    host = []
    t0 = time.perf_counter()
    for _ in range(launches):
        a = time.perf_counter()
        g.replay()
        host.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    # launches spaced out (GPU drained before each): host enqueue alone
    iso = []
    for _ in range(10):
        torch.cuda.synchronize()
        a = time.perf_counter()
        g.replay()
        iso.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    host.sort()
    iso.sort()
    row = {"config": name, "updates_per_launch": k, "launches": launches,
           "host_us_per_update_median": round(1e6 * host[len(host) // 2] / k, 1),
           "host_us_per_update_drained": round(1e6 * iso[len(iso) // 2] / k, 1),
           "wall_us_per_update": round(1e6 * wall / (launches * k), 1)}
    print(json.dumps(row), flush=True)
    del L, replay
    torch.cuda.empty_cache()
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--launches", type=int, default=40)
    ap.add_argument("--out", default="gpurun_out/graph_launch.jsonl")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        for n in a.configs.split(","):
            f.write(json.dumps(probe(n, CONFIGS[n], a.launches)) + "\n")


if __name__ == "__main__":
    main()
