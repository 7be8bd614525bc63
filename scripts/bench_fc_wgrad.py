"""The fc-wgrad + head-wgrad + priority write-back launch (csrc/sumtree.hip
fc_wgrad_head_prio_kernel) against its parts, at the learner's shapes (B=512):
fc weight-gradient GEMM alone, head wgrad alone, the tree update alone."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from bench_tree import timed  # noqa: E402
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    res = {}
    for dtype in ("bf16", "fp32"):
        args = bench.parser().parse_args(["--batch", os.environ.get("B", "512")])
        from apex_dqn_amd.parallel.dist import Comm
        comm = Comm(0, 1, dev)
        replay = bench.make_replay(args, dev, 0)
        cfg, L = bench.make_learner(args, dtype, dev, comm, 0, replay)
        for _ in range(3):
            L.step()
        torch.cuda.synchronize()
        B, ops, sp = L.B, L.ops, L.split
        S = L.S
        lo = dict(dh_lo=L.dH_lo, x_lo=L.y3_lo[:B], Hon_lo=L.h_lo) if sp else {}
        prio = (replay, S["idx"], S["gen"], L.td_abs)
        r = {}
        r["fused"] = timed(lambda: ops.fc_head_wgrad(L.dH, L.y3[:B], L.G["wfc"], L.G["bfc"], L.h, L.dhead, L.G, prio,
                                                     **lo))
        lo2 = dict(dh_lo=L.dH_lo, x_lo=L.y3_lo[:B]) if sp else {}
        r["fc_gemm_only"] = timed(lambda: ops.fc_wgrad(L.dH, L.y3[:B], L.G["wfc"], L.G["bfc"], **lo2))
        r["tree_update_only"] = timed(lambda: replay.update_priorities(S["idx"], L.td_abs, S["gen"]))
        res[dtype] = {k: round(v, 2) for k, v in r.items()}
        print(dtype, json.dumps(res[dtype]), flush=True)
        del L, replay
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/fc_wgrad_parts.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
