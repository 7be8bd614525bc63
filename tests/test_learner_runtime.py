"""Learners, envs and runtime loops on CPU (the CartPole plumbing config runs
without a GPU), including fault injection and checkpoint resume."""
import copy
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from apex_dqn_amd.config import ApexConfig
from apex_dqn_amd.envs.vector_envs import AtariPreprocess, CartPoleVec, SyntheticAtariVec, _area_matrix
from apex_dqn_amd.learner.losses import ddqn_loss, huber
from apex_dqn_amd.learner.torch_learner import TorchLearner

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _cp_cfg(**rt):
    d = {"env_conf": {"state_shape": [4], "action_dim": 2, "name": "CartPole-v1"},
         "Actor": {"num_actors": 4, "num_steps": 3, "Q_network_sync_freq": 50, "n_step_transition_batch_size": 8},
         "Learner": {"min_replay_mem_size": 300, "replay_sample_size": 64, "q_target_sync_freq": 100,
                     "remove_old_xp_freq": 50},
         "Replay_Memory": {"soft_capacity": 5000},
         "Runtime": dict({"lr": 1e-3, "log_every": 100}, **rt)}
    return ApexConfig.from_dict(d)


def test_ddqn_loss_manual():
    qt = torch.tensor([[1.0, 2.0], [0.0, 5.0]])
    qn = torch.tensor([[3.0, 1.0], [0.0, 1.0]])
    qg = torch.tensor([[10.0, 20.0], [7.0, 8.0]])
    A = torch.tensor([1, 0])
    R = torch.tensor([1.0, 2.0])
    G = torch.tensor([0.5, 0.0])
    loss, td = ddqn_loss(qt, qn, qg, A, R, G, None, loss="mse")
    # sample0: argmax online = 0 -> target 10 -> G = 1 + 5 = 6; delta = 6 - 2 = 4
    # sample1: terminal -> G = 2; delta = 2 - 0 = 2
    torch.testing.assert_close(td, torch.tensor([4.0, 2.0]))
    assert float(loss) == pytest.approx((0.5 * 16 + 0.5 * 4) / 2)
    assert float(huber(torch.tensor(3.0))) == pytest.approx(2.5)


def test_target_sync_cadence_and_centered_rmsprop():
    cfg = _cp_cfg()
    cfg.Learner.q_target_sync_freq = 3
    L = TorchLearner(cfg, "cpu")
    # target starts equal to online (reference A30: independently initialised)
    for a, b in zip(L.Q.parameters(), L.Q_target.parameters()):
        assert torch.equal(a, b)
    opt = L.optimizer
    assert isinstance(opt, torch.optim.RMSprop)
    g = opt.param_groups[0]
    assert g["centered"] and g["alpha"] == 0.95 and g["weight_decay"] == 0 and g["eps"] == 1.5e-7
    rng = np.random.default_rng(0)
    batch = dict(S_t=rng.normal(size=(8, 4)).astype(np.float32), S_tpn=rng.normal(size=(8, 4)).astype(np.float32),
                 A_t=rng.integers(0, 2, 8), R=rng.normal(size=8).astype(np.float32),
                 Gamma=np.full(8, 0.9, np.float32), weights=np.ones(8, np.float32))
    synced = []
    for i in range(6):
        L.step(batch)
        same = all(torch.equal(a, b) for a, b in zip(L.Q.parameters(), L.Q_target.parameters()))
        synced.append(same)
    # synced exactly at updates 3 and 6 (reference A17 syncs on every step except multiples)
    assert synced == [False, False, True, False, False, True]


def test_checkpoint_resume_bit_identical(tmp_path):
    cfg = _cp_cfg()
    L = TorchLearner(cfg, "cpu")
    rng = np.random.default_rng(1)
    batch = dict(S_t=rng.normal(size=(8, 4)).astype(np.float32), S_tpn=rng.normal(size=(8, 4)).astype(np.float32),
                 A_t=rng.integers(0, 2, 8), R=rng.normal(size=8).astype(np.float32),
                 Gamma=np.full(8, 0.9, np.float32), weights=np.ones(8, np.float32))
    for _ in range(3):
        L.step(batch)
    p = str(tmp_path / "ck.pt")
    L.save(p)
    cfg2 = copy.deepcopy(cfg)
    cfg2.Learner.load_saved_state = p
    L2 = TorchLearner(cfg2, "cpu")
    assert L2.num_q_updates == 3
    L.step(batch)
    L2.step(batch)
    for a, b in zip(L.Q.parameters(), L2.Q.parameters()):
        assert torch.equal(a, b)


def test_envs():
    env = CartPoleVec(8, seed=0)
    obs = env.reset()
    assert obs.shape == (8, 4)
    total_done = 0
    for _ in range(300):
        obs, r, d, info = env.step(np.random.randint(0, 2, 8))
        total_done += d.sum()
    assert total_done > 0
    se = SyntheticAtariVec(5, action_dim=6)
    f = se.reset()
    assert f.shape == (5, 84, 84) and f.dtype == np.uint8
    # area resize: a constant image stays constant; rows of the matrix sum to 1
    m = _area_matrix(84, 210)
    np.testing.assert_allclose(m.sum(1), 1.0)
    pre = AtariPreprocess()
    img = np.full((210, 160, 3), 100, np.uint8)
    out = pre(img)
    assert out.shape == (84, 84) and np.all(out == 100)


def test_inline_cartpole_learns():
    from apex_dqn_amd.runtime.loops import train_inline
    torch.manual_seed(0)
    out = train_inline(_cp_cfg(), 2500, actor_steps_per_update=1)
    assert out["learner"].num_q_updates == 2500
    assert out["mean_return_last"] > 40  # random policy averages ~22


@pytest.mark.slow
def test_multiprocess_topology_with_actor_fault_injection():
    from apex_dqn_amd.runtime.loops import train_multiprocess
    cfg = _cp_cfg(heartbeat_timeout=30.0)
    out = train_multiprocess(cfg, 300, num_procs=2, kill_actor_at=50, max_wall_s=240)
    assert out["learner"].num_q_updates == 300
    assert out["restarts"] >= 1  # the killed actor was detected and restarted
    assert len(out["episodes"]) > 0


def test_gpu_loop_pipeline_on_cpu(tmp_path):
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                "Actor": {"num_actors": 6, "n_step_transition_batch_size": 6,
                                          "Q_network_sync_freq": 5},
                                "Learner": {"min_replay_mem_size": 40, "replay_sample_size": 8,
                                            "remove_old_xp_freq": 4, "q_target_sync_freq": 5},
                                "Replay_Memory": {"soft_capacity": 120},
                                "Runtime": {"replay_capacity": 150, "log_every": 4, "use_graphs": False,
                                            "ckpt_dir": str(tmp_path), "ckpt_freq": 6}})
    from apex_dqn_amd.utils.metrics import MetricsLogger
    mpath = str(tmp_path / "m.jsonl")
    ml = MetricsLogger(mpath)
    out = train_frames(cfg, "cpu", 12, metrics=ml)
    ml.close()
    assert out["learner"].num_q_updates == 12
    import json
    recs = [json.loads(x) for x in open(mpath)]
    lrn = [r for r in recs if r["kind"] == "learner"]
    assert lrn and all(k in lrn[-1] for k in ("loss", "grad_steps_per_s", "env_frames_per_s", "inserts_per_s",
                                              "is_weight_mean", "eps_min", "eps_max", "mean_ep_len", "replay"))
    assert out["replay"].size() <= 120
    assert os.path.exists(os.path.join(str(tmp_path), "checkpoint.pt"))
    ck = torch.load(os.path.join(str(tmp_path), "checkpoint.pt"), weights_only=True)
    from apex_dqn_amd.models.dueling import DuellingDQN
    DuellingDQN((4, 84, 84), 4).load_state_dict(ck["Q_state"])


def test_main_cli_inline_cartpole():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "main.py"), "--params-file",
                        os.path.join(ROOT, "configs", "cartpole.json"), "--mode", "inline", "--learner-steps", "50",
                        "--set", "Learner.min_replay_mem_size=200"],
                       capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    assert '"learner_steps": 50' in r.stdout


@pytest.mark.parametrize("net,hip,kind", [("impala", True, "impala"), ("impala", False, "graph"),
                                           ("nature32", True, "fused")])
def test_image_learner_loops_on_cpu(tmp_path, net, hip, kind):
    """IMPALA-deep (hand-written learner or the graph learner) and nature32 (the
    fused NatureCNN learner, conv1 zero-padded) run the GPU-resident loop with
    the HBM-replay API, flat-buffer params and checkpoint resume -- CPU here."""
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                "Actor": {"num_actors": 6, "n_step_transition_batch_size": 6,
                                          "Q_network_sync_freq": 5},
                                "Learner": {"min_replay_mem_size": 40, "replay_sample_size": 8,
                                            "remove_old_xp_freq": 4, "q_target_sync_freq": 5},
                                "Replay_Memory": {"soft_capacity": 120},
                                "Runtime": {"replay_capacity": 150, "log_every": 0, "use_graphs": False,
                                            "network": net, "ckpt_dir": str(tmp_path), "ckpt_freq": 6,
                                            "use_hip_kernels": hip}})
    out = train_frames(cfg, "cpu", 8)
    L = out["learner"]
    assert getattr(L, "kind", "fused") == kind and L.num_q_updates == 8
    assert np.isfinite(L.last_metrics()["loss"]) and L.last_metrics()["grad_norm"] > 0
    if kind == "graph":   # params are views of the flat buffer; the optimizer moved them
        assert L.Q.state_dict()[next(iter(L.Q.state_dict()))].data_ptr() >= L.p32.data_ptr()
    out2 = train_frames(cfg, "cpu", 10)          # resumes the step-6 checkpoint
    assert out2["learner"].num_q_updates == 10


def _small_image_cfg(**rt):
    return ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                 "Actor": {"num_actors": 6, "n_step_transition_batch_size": 6,
                                           "Q_network_sync_freq": 5},
                                 "Learner": {"min_replay_mem_size": 40, "replay_sample_size": 8,
                                             "remove_old_xp_freq": 4, "q_target_sync_freq": 5},
                                 "Replay_Memory": {"soft_capacity": 120},
                                 "Runtime": {"replay_capacity": 150, "log_every": 4, "use_graphs": False, **rt}})


def test_gpu_loop_async_actor_thread_on_cpu(tmp_path):
    """The actor group steps on its own thread while the learner trains (reference
    main.py:46-58 runs actors and learner concurrently)."""
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    from apex_dqn_amd.utils.metrics import MetricsLogger
    mpath = str(tmp_path / "m.jsonl")
    ml = MetricsLogger(mpath)
    out = train_frames(_small_image_cfg(), "cpu", 16, metrics=ml, async_actors=True)
    ml.close()
    assert out["learner"].num_q_updates == 16
    assert out["actor_steps"] > 0 and out["actors"].inserted >= 40
    import json
    lrn = [json.loads(x) for x in open(mpath) if '"learner"' in x]
    assert lrn and lrn[-1]["actor_thread"] is True and lrn[-1]["actor_restarts"] == 0


def test_actor_T_bounds_env_steps():
    """Actor.T (reference actor.py:104,159) stops the actors; the learner finishes its steps."""
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    cfg = _small_image_cfg()
    cfg.Actor.T = 12
    out = train_frames(cfg, "cpu", 10)
    assert out["actor_steps"] == 12 and out["learner"].num_q_updates == 10
    out = train_frames(cfg, "cpu", 10, async_actors=True)
    # the actor thread never passes T; the learner may finish its 10 updates (and stop
    # the thread) before the thread's last step on a loaded host
    assert out["actor_steps"] <= 12 and out["learner"].num_q_updates == 10


class _FlakyGroup:
    def __init__(self, fail_at=3, sleep_at=None):
        self.n, self.fail_at, self.sleep_at, self.resets = 0, fail_at, sleep_at, 0

    def step(self):
        import time
        self.n += 1
        if self.n == self.fail_at:
            raise ValueError("env crashed")
        if self.sleep_at is not None and self.n >= self.sleep_at:
            time.sleep(0.5)
        time.sleep(0.001)

    def reset_episodes(self):
        self.resets += 1


def test_actor_runner_restarts_crashed_thread_and_detects_stall():
    import time
    from apex_dqn_amd.runtime.actor_thread import ActorRunner
    g = _FlakyGroup(fail_at=3)
    events = []
    r = ActorRunner(g, 50, timeout=5.0, on_event=lambda k, **kw: events.append(k)).start()
    t0 = time.time()
    while not r.done and time.time() - t0 < 20:
        r.check()
        time.sleep(0.005)
    r.stop()
    assert r.done and r.restarts == 1 and g.resets == 1 and events == ["actor_restart"]
    g2 = _FlakyGroup(fail_at=-1, sleep_at=2)
    r2 = ActorRunner(g2, 100, timeout=0.2).start()
    time.sleep(0.8)
    with pytest.raises(RuntimeError, match="stalled"):
        r2.check()
    r2.stop()


def test_loop_watchdog_aborts_on_hung_gpu_work():
    from apex_dqn_amd.runtime.gpu_loop import _wait_event

    class Hung:
        def query(self):
            return False

    class Done:
        def query(self):
            return True

    class FakeComm:
        aborted = False

        def abort(self):
            FakeComm.aborted = True

    _wait_event(Done(), 0.1, FakeComm())
    assert not FakeComm.aborted
    with pytest.raises(RuntimeError, match="watchdog"):
        _wait_event(Hung(), 0.05, FakeComm())
    assert FakeComm.aborted


def test_row_resize_recaptures_with_actor_thread_quiesced(monkeypatch):
    """A DP row resize at an eviction (FusedNatureLearner.refresh_replay_stats -> True:
    the step graphs were dropped) recaptures the graphs while the actor thread is
    stopped -- a capture must not see another thread's launches -- and the thread then
    resumes.  Forced here on the CPU loop with the async actor thread on."""
    import threading
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    calls = {"refresh": 0, "prepare": [], "resized_at": None}
    orig_refresh = FusedNatureLearner.refresh_replay_stats

    def refresh(self):
        orig_refresh(self)
        calls["refresh"] += 1
        if calls["refresh"] == 3:            # the second eviction of the training loop
            calls["resized_at"] = self.num_q_updates
            return True
        return False

    def prepare(self, multi=True):
        alive = any(t.name == "apex-actor" and t.is_alive() for t in threading.enumerate())
        calls["prepare"].append((self.num_q_updates, alive))
        return 0

    monkeypatch.setattr(FusedNatureLearner, "refresh_replay_stats", refresh)
    monkeypatch.setattr(FusedNatureLearner, "prepare_graphs", prepare)
    out = train_frames(_small_image_cfg(), "cpu", 12, async_actors=True)
    assert out["learner"].num_q_updates == 12
    n = calls["resized_at"]
    assert n is not None and n > 0
    # the initial capture (before the thread starts) and the recapture at the resize:
    # the actor thread is never alive during either
    assert [c for c in calls["prepare"] if c[0] == n] == [(n, False)], calls
    assert all(alive is False for _, alive in calls["prepare"]), calls
    assert out["actor_steps"] > 0
