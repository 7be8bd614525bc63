"""Sum-tree invariants (hypothesis), host prioritized replay and the HBM shard's
CPU implementation against the numpy oracle."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
from apex_dqn_amd.replay.host_replay import PrioritizedReplay
from apex_dqn_amd.replay.sumtree import SumTree, inverse_cdf_oracle


@settings(max_examples=40, deadline=None)
@given(st.lists(st.floats(min_value=0.0, max_value=100.0, allow_nan=False), min_size=1, max_size=300))
def test_sumtree_root_equals_sum_and_inverse_cdf(vals):
    t = SumTree(len(vals))
    t.update(np.arange(len(vals)), vals)
    assert t.total == pytest.approx(sum(vals), rel=1e-9, abs=1e-9)
    if t.total > 0:
        u = np.random.default_rng(0).random(64) * t.total
        got = t.find_prefix(u)
        ref = inverse_cdf_oracle(np.array(vals), u)
        assert np.all(np.array(vals)[got] > 0)
        # equal except where round-off lands exactly on a boundary
        assert np.mean(got == ref) > 0.95


def test_sumtree_duplicates_last_wins_and_min():
    t = SumTree(10)
    t.update([1, 2, 1, 1], [5.0, 3.0, 7.0, 2.0])
    assert t.get([1])[0] == 2.0 and t.total == 5.0 and t.min_positive == 2.0
    t.update([1], [0.0])
    assert t.min_positive == 3.0


def test_sumtree_sampling_proportional():
    rng = np.random.default_rng(0)
    p = rng.random(50) + 0.01
    t = SumTree(50)
    t.update(np.arange(50), p)
    counts = np.zeros(50)
    for _ in range(400):
        counts += np.bincount(t.sample_stratified(256, rng), minlength=50)
    emp = counts / counts.sum()
    assert np.abs(emp - p / p.sum()).max() < 4e-3


def _batch(K, rng, obs_dim=4):
    return dict(S_t=rng.normal(size=(K, obs_dim)).astype(np.float32),
                S_tpn=rng.normal(size=(K, obs_dim)).astype(np.float32),
                A_t=rng.integers(0, 2, K), R=rng.normal(size=K).astype(np.float32),
                Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32))


def test_host_replay_semantics():
    rng = np.random.default_rng(0)
    r = PrioritizedReplay(100, 0.6, 0.4, capacity=150, is_normalise="global_min")
    r.add(_batch(120, rng))
    assert r.size() == 120
    s = r.sample(32)
    assert s["S_t"].shape == (32, 4) and np.all(s["weights"] <= 1.0 + 1e-6)
    assert s["weights"].max() <= 1.0
    leaf = r.tree.get(s["idx"])
    np.testing.assert_allclose(s["weights"], (leaf / r.tree.min_positive) ** -0.4, rtol=1e-5)
    assert r.remove_to_fit() == 20 and r.size() == 100
    assert np.all(r.tree.get(np.arange(20)) == 0)
    r.set_priorities(np.arange(5), np.ones(5))  # evicted: not resurrected (reference A5 keeps stale keys)
    assert np.all(r.tree.get(np.arange(5)) == 0)
    for _ in range(10):  # never samples evicted slots
        assert np.all(r.sample(64)["idx"] >= 20)


def test_host_replay_is_normalise_modes():
    """batch_max: w_i = (N P(i))^-beta / max over the sampled batch (max weight exactly 1);
    global_min: / max over the whole replay = (p_i / p_min)^-beta (numpy oracle)."""
    rng = np.random.default_rng(1)
    b = _batch(200, rng)
    b["priority"][0] = 0.0           # one leaf at the priority floor: p_min = eps^alpha
    for mode in ("batch_max", "global_min"):
        r = PrioritizedReplay(500, 0.6, 0.4, capacity=600, seed=3, is_normalise=mode)
        r.add(b)
        s = r.sample(64)
        leaf = r.tree.get(s["idx"])
        N, tot = r.size(), r.tree.total
        w = (N * leaf / tot) ** -0.4
        ref = w / (w.max() if mode == "batch_max" else (N * r.tree.min_positive / tot) ** -0.4)
        np.testing.assert_allclose(s["weights"], ref, rtol=1e-5)
        if mode == "batch_max":
            assert abs(s["weights"].max() - 1.0) < 1e-6 and s["weights"].mean() > 0.2
        else:
            assert s["weights"].mean() < 0.05    # the floor leaf shrinks every weight


def _shard_fill(rp, K, seed=0):
    rng = np.random.default_rng(seed)
    seqs = rp.append_frames(rng.integers(0, 255, (K + 8, 84, 84), dtype=np.uint8))
    st_ = np.stack([seqs[i:i + 4] for i in range(K)])
    pr = rng.random(K).astype(np.float32) + 0.01
    rp.insert(dict(S_t=st_, S_tpn=st_ + 3, A_t=rng.integers(0, 4, K), R=rng.normal(size=K),
                   Gamma=np.full(K, 0.97), priority=pr))
    return pr


def test_gpu_shard_cpu_path_matches_oracle():
    rp = GpuReplayShard(500, 400, 700, 4, device="cpu", alpha=0.6, beta=0.4)
    pr = _shard_fill(rp, 450)
    leaf = rp.leaf.double().numpy()
    np.testing.assert_allclose(leaf[:450], (pr.astype(np.float64) + 1e-6) ** 0.6, rtol=1e-6)
    assert rp.total() == pytest.approx(leaf.sum(), rel=1e-9)
    out = rp.sample(64)
    c = np.cumsum(leaf)
    idx = out["idx"].numpy()
    seg = c[-1] / 64
    assert np.all((c[idx] - leaf[idx]) <= (np.arange(64) + 1) * seg + 1e-9)
    assert np.all(c[idx] >= np.arange(64) * seg - 1e-9)
    # eviction + frames
    assert rp.remove_to_fit() == 50 and rp.size() == 400
    fr = rp.gather_frames(out["obs"][:4])
    assert fr.shape == (4, 4, 84, 84)
    # generation check: a stale write-back is ignored
    gen = out["gen"].clone()
    gen[0] += 1
    before = float(rp.leaf[idx[0]])
    rp.update_priorities(out["idx"][:1], torch.tensor([9.0]), gen[:1])
    assert float(rp.leaf[idx[0]]) == before


def test_gpu_shard_frame_ring_guard():
    rp = GpuReplayShard(100, 100, 30, 4, device="cpu")
    _shard_fill(rp, 20)
    # overwrite the frame ring: transitions referencing overwritten frames get evicted
    rp.append_frames(np.zeros((40, 84, 84), np.uint8))
    n = rp.remove_to_fit()
    assert n > 0 and rp.size() == 20 - n
