"""Diagnostic: one learner step with the fc epilogue deferred into the head vs the
separate epilogue launch; prints the max |difference| of each step tensor."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))


def main():
    from test_gpu_runtime import _filled_replay
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    dev = torch.device("cuda", 0)
    for dtype, graphs, n in (("fp32", False, 1), ("fp32", True, 1), ("fp32", True, 4), ("fp32", False, 4),
                             ("fp32", True, 9), ("bf16", False, 1)):
        cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                    "Learner": {"replay_sample_size": 128},
                                    "Runtime": {"use_graphs": graphs, "graph_steps": 4, "dtype": dtype}})
        res = []
        for defer in (True, False):
            torch.manual_seed(0)
            rp = _filled_replay(seed=11)
            L = FusedNatureLearner(cfg, dev, rp)
            L._defer_fc_epilogue = defer
            L.steps(n)
            torch.cuda.synchronize()
            d = {"h": L.h[:128].float(), "td": L.td_abs, "dH": L.dH.float(), "g32": L.g32, "p32": L.p32,
                 "idx": L.S["idx"].double()}
            if L.h_lo is not None:
                d["h_lo"] = L.h_lo[:128].float()
                d["dH_lo"] = L.dH_lo.float()
            res.append(d)
        for k in res[0]:
            print(dtype, "graphs" if graphs else "eager", n, k, float((res[0][k] - res[1][k]).abs().max()), flush=True)


if __name__ == "__main__":
    main()
