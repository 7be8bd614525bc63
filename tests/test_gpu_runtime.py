"""GPU runtime: actor head kernel, actor group + HBM replay + fused learner loop
(HIP graphs on), CLI in gpu mode."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_actor_head_kernel_vs_torch():
    from apex_dqn_amd.ops.fused_ops import HipBackend, TorchBackend
    g = torch.Generator(device="cpu").manual_seed(0)
    E, A = 70, 6
    H = torch.relu(torch.randn(E, 1024, generator=g)).to(DEV, torch.bfloat16)
    P = {"wv": (torch.randn(512, generator=g) * 0.05).to(DEV), "bv": torch.randn(1, generator=g).to(DEV),
         "wa": (torch.randn(A, 512, generator=g) * 0.05).to(DEV), "ba": torch.randn(A, generator=g).to(DEV)}
    ctr = torch.zeros(1, dtype=torch.int64, device=DEV)
    out = {}
    for name, be in (("hip", HipBackend()), ("ref", TorchBackend(torch.float32))):
        q = torch.zeros(E, A, device=DEV)
        a = torch.zeros(E, dtype=torch.int32, device=DEV)
        be.actor_head(H, P, torch.zeros(E, device=DEV), ctr, 5, q, a)  # eps = 0: greedy
        out[name] = (q, a)
    torch.testing.assert_close(out["hip"][0], out["ref"][0], rtol=1e-4, atol=1e-4)
    assert torch.equal(out["hip"][1].long(), out["hip"][0].argmax(1))
    q = torch.zeros(E, A, device=DEV)
    acts = []
    for i in range(50):  # eps = 1: uniform over actions
        a = torch.zeros(E, dtype=torch.int32, device=DEV)
        ctr.fill_(i)
        HipBackend().actor_head(H, P, torch.ones(E, device=DEV), ctr, 5, q, a)
        acts.append(a.cpu().numpy())
    counts = np.bincount(np.concatenate(acts), minlength=A)
    assert counts.min() > 0.1 * counts.sum() / A


def test_gpu_loop_with_graphs():
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Actor": {"num_actors": 64, "n_step_transition_batch_size": 64,
                                          "Q_network_sync_freq": 20},
                                "Learner": {"min_replay_mem_size": 2000, "replay_sample_size": 128,
                                            "remove_old_xp_freq": 25, "q_target_sync_freq": 50},
                                "Replay_Memory": {"soft_capacity": 8000},
                                "Runtime": {"log_every": 25, "use_graphs": True}})
    out = train_frames(cfg, DEV, 100)
    L = out["learner"]
    assert L.num_q_updates == 100
    m = L.last_metrics()
    assert np.isfinite(m["loss"]) and m["grad_norm"] > 0
    assert out["actors"].inserted >= 2000


def test_main_cli_gpu_mode(tmp_path):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), "--params-file",
                        os.path.join(ROOT, "parameters.json"), "--mode", "gpu", "--learner-steps", "30",
                        "--set", "Learner.min_replay_mem_size=1000", "--set", "Learner.replay_sample_size=64",
                        "--set", f"Runtime.ckpt_dir={tmp_path}", "--set", "Runtime.ckpt_freq=30",
                        "--set", "Replay_Memory.soft_capacity=5000"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    assert '"learner_steps": 30' in r.stdout
    assert os.path.exists(os.path.join(str(tmp_path), "checkpoint.pt"))
