"""n-step builder goldens, terminal handling, keys, initial priorities, actor group."""
import numpy as np
import pytest

from apex_dqn_amd.actors.actor_group import ActorGroup
from apex_dqn_amd.actors.nstep import NStepBuilder, nstep_returns_reference
from apex_dqn_amd.envs.vector_envs import CartPoleVec, SyntheticAtariVec


def _run(rewards, dones, n=3, gamma=0.99, qvals=None):
    T = len(rewards)
    b = NStepBuilder(1, n, gamma, (1,), np.float32)
    A = 2
    q = qvals if qvals is not None else np.zeros((T + 1, A))
    for t in range(T):
        b.step(np.array([[t]], np.float32), q[t:t + 1], np.array([0]), np.array([rewards[t]]),
               np.array([dones[t]]), np.array([[t + 1]], np.float32))
    # one extra step so the last full window's bootstrap completes
    b.step(np.array([[T]], np.float32), q[T:T + 1], np.array([0]), np.array([0.0]), np.array([False]),
           np.array([[T + 1]], np.float32))
    return b.get()


def test_golden_three_step_return():
    out = _run([1.0, 10.0, 100.0, 1000.0], [False] * 4)
    first = np.nonzero(out["S_t"][:, 0] == 0)[0][0]
    # reference double-counts and gives 118.81; correct value 108.91
    assert out["R"][first] == pytest.approx(1 + 0.99 * 10 + 0.99 ** 2 * 100, rel=1e-6)
    assert out["Gamma"][first] == pytest.approx(0.99 ** 3)   # reference uses gamma^(n-1) (A8)
    assert out["S_tpn"][first, 0] == 3
    # sliding window: the next transition starts at t=1 and includes r=1000 (A9 drops it)
    second = np.nonzero(out["S_t"][:, 0] == 1)[0][0]
    assert out["R"][second] == pytest.approx(10 + 0.99 * 100 + 0.99 ** 2 * 1000, rel=1e-6)


@pytest.mark.parametrize("seed", range(5))
def test_matches_scalar_oracle_with_terminals(seed):
    rng = np.random.default_rng(seed)
    T = 60
    rew = rng.normal(size=T)
    done = rng.random(T) < 0.1
    out = _run(list(rew), list(done), n=3, gamma=0.97)
    ref = {t: (R, G) for t, R, G in nstep_returns_reference(rew, done, 0.97, 3)}
    got = {int(s): (R, G) for s, R, G in zip(out["S_t"][:, 0], out["R"], out["Gamma"])}
    for t, (R, G) in ref.items():
        assert t in got, t
        assert got[t][0] == pytest.approx(R, rel=1e-5, abs=1e-5)
        assert got[t][1] == pytest.approx(G, rel=1e-6)
    # terminal transitions never bootstrap (A10)
    for t in np.nonzero(done)[0]:
        assert got[int(t)][1] == 0.0


def test_initial_priorities_use_bootstrap_q():
    q = np.array([[1.0, 2.0], [0.5, 3.0], [0.0, 0.0], [4.0, -1.0], [0.0, 0.0], [0.0, 0.0]])
    out = _run([1.0, 1.0, 1.0, 1.0, 1.0], [False] * 5, n=2, gamma=0.5, qvals=q)
    i0 = np.nonzero(out["S_t"][:, 0] == 0)[0][0]
    # |R + gamma^2 max q(S_2) - q(S_0, a=0)| = |1.5 + 0.25*0 - 1|
    assert out["priority"][i0] == pytest.approx(abs(1.5 + 0.25 * 0.0 - 1.0))
    i1 = np.nonzero(out["S_t"][:, 0] == 1)[0][0]
    assert out["priority"][i1] == pytest.approx(abs(1.5 + 0.25 * 4.0 - 0.5))


def test_keys_unique_across_envs():
    b = NStepBuilder(12, 3, 0.99, (1,), np.float32)
    for t in range(40):
        b.step(np.zeros((12, 1), np.float32), np.zeros((12, 2)), np.zeros(12, np.int64), np.ones(12),
               np.zeros(12, bool), np.zeros((12, 1), np.float32))
    k = b.get()["key"]
    assert len(np.unique(k)) == len(k)  # reference str(id)+str(seq) collides (A11)


def test_actor_group_cartpole_and_frames():
    env = CartPoleVec(4, seed=1)
    g = ActorGroup(env, 4, 3, 0.99, 1, 0.4, 7.0)
    for _ in range(30):
        g.step(lambda obs: np.random.randn(len(obs), 2))
    b = g.drain()
    assert b["S_t"].shape[1:] == (4,) and len(b["A_t"]) > 0
    env2 = SyntheticAtariVec(3, action_dim=6)
    g2 = ActorGroup(env2, 3, 3, 0.99, 4, 0.4, 7.0)
    for _ in range(10):
        g2.step(lambda obs: np.random.randn(len(obs), 6))
    b2 = g2.drain()
    assert b2["S_t"].shape[1:] == (4, 84, 84) and b2["S_t"].dtype == np.uint8
    assert np.all(g2.eps <= 0.4)


def test_interleaved_epsilon_ladder_over_ranks():
    """Env i of rank r is actor i * W + r of the global ladder: every rank holds a mix of
    exploratory and greedy actors, and the union over ranks is the whole ladder."""
    from apex_dqn_amd.actors.gpu_actor import ladder_slice
    from apex_dqn_amd.config import ApexConfig, epsilon_ladder
    cfg = ApexConfig()
    W, E = 4, 8
    sl = [ladder_slice(cfg, E, r, W) for r in range(W)]
    full = epsilon_ladder(W * E, cfg.Actor.epsilon, cfg.Actor.alpha)
    assert sorted(sum(sl, [])) == sorted(full)
    assert all(max(s) > 0.1 and min(s) < 0.01 for s in sl)


def test_pipelined_actor_groups_cpu():
    """Runtime.actor_pipeline's group wrapper (actors/gpu_actor.py PipelinedActorGroups) on
    the CPU backend: two groups of E / 2 envs stepped in turn, consecutive env ids, the
    rank's epsilon-ladder slices, one episode list, inserts from both groups."""
    import torch
    from apex_dqn_amd.actors.gpu_actor import PipelinedActorGroups, ladder_slice, make_gpu_actor_group
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    E = 8
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                "Actor": {"num_actors": E, "n_step_transition_batch_size": 8},
                                "Learner": {"replay_sample_size": 16},
                                "Runtime": {"use_graphs": False, "env_backend": "synthetic"}})
    torch.manual_seed(0)
    rp = GpuReplayShard(600, 600, 700, 4, device="cpu")
    L = FusedNatureLearner(cfg, "cpu", rp)
    grp = make_gpu_actor_group(cfg, L, rp, E, pipeline=2)
    assert isinstance(grp, PipelinedActorGroups) and grp.E == E
    assert [g.global_offset for g in grp.groups] == [0, E // 2]
    np.testing.assert_allclose(grp.eps.numpy(), np.array(ladder_slice(cfg, E, 0, 1, E), dtype=np.float32))
    ins = sum(grp.step() for _ in range(12))
    assert all(g.t == 12 for g in grp.groups)
    assert ins == grp.inserted > 0 and all(g.inserted > 0 for g in grp.groups)
    assert all(g.episodes is grp.episodes for g in grp.groups)
    assert len(set(grp.groups[0].builder.env_ids) & set(grp.groups[1].builder.env_ids)) == 0
    grp.reset_episodes()
    grp.step()
    assert all(g.t == 13 for g in grp.groups)

