"""The W replay shards of a data-parallel run are ONE prioritized replay.

* chi-square: the empirical sampling frequency of every item over all shards
  matches the global p^alpha / sum p^alpha (reference ``replay.py:19-31,44-57``)
  for deliberately unequal shards (sizes and priority scales differ per rank);
* every global draw lands in exactly one shard; IS weights use the global min;
* the all-gather of the shard statistics over gloo (W=2, 4) and the partition
  of the draws across real processes;
* the sharded config's per-rank capacity (global FIFO bound = soft_capacity).
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp
from scipy import stats as sstats

from apex_dqn_amd.config import ApexConfig
from apex_dqn_amd.replay.gpu_replay import SHARD_STATS, GpuReplayShard, apex_uniform, global_draw

ALPHA, BETA = 0.6, 0.4


def _shard(rank, n_items, scale, seed=0):
    rp = GpuReplayShard(256, 256, 64, 1, frame_shape=(2, 2), alpha=ALPHA, beta=BETA, device="cpu", seed=seed)
    rng = np.random.default_rng(10 + rank)
    K = n_items
    rp.insert(dict(S_t=np.zeros((K, 1)), S_tpn=np.zeros((K, 1)), A_t=np.zeros(K, np.int64), R=np.zeros(K),
                   Gamma=np.zeros(K), priority=(rng.random(K) + 0.05) * scale))
    return rp


def _link(shards, seed=77):
    """The all-gather, emulated in one process: every shard gets every shard's stats."""
    W = len(shards)
    st = torch.tensor([[s.total(), s.min_leaf(), 0.0] for s in shards], dtype=torch.float64).reshape(-1)
    for r, s in enumerate(shards):
        s.enable_sharding(r, W, seed)
        s.shard_stats.copy_(st)


def test_apex_uniform_matches_kernel_formula():
    u = apex_uniform(5, 7, np.arange(1000))
    assert u.dtype == np.float32 and u.min() >= 0.0 and u.max() < 1.0
    assert abs(float(u.mean()) - 0.5) < 0.03
    # deterministic in (seed, ctr, index), different across counters
    np.testing.assert_array_equal(u, apex_uniform(5, 7, np.arange(1000)))
    assert not np.array_equal(u, apex_uniform(5, 8, np.arange(1000)))


@pytest.mark.parametrize("W", [2, 4])
def test_global_sampling_distribution_chi2(W):
    sizes = [40, 25, 60, 10][:W]
    scales = [1.0, 6.0, 0.3, 20.0][:W]
    shards = [_shard(r, sizes[r], scales[r]) for r in range(W)]
    _link(shards)
    B = 24
    leaf = [s.leaf[:s.live].double().numpy() for s in shards]
    p_all = np.concatenate(leaf)
    P = p_all / p_all.sum()
    counts = np.zeros_like(p_all)
    offs = np.cumsum([0] + sizes)
    n_draws = 0
    for it in range(600):
        M_seen = 0
        for r, s in enumerate(shards):
            s.ctr.fill_(it)
            out = s.sample(B)
            v = (out["gen"] >= 0).numpy()
            M_seen += int(v.sum())
            np.add.at(counts, offs[r] + out["idx"].numpy()[v], 1.0)
        st = shards[0].shard_stats.view(W, SHARD_STATS)[:, :2].numpy()
        M = min(W * B, int(np.floor((B - 2) * st[:, 0].sum() / st[:, 0].max())))
        assert M_seen == M          # each global draw in exactly one shard
        n_draws += M
    expected = n_draws * P
    chi2 = float(((counts - expected) ** 2 / expected).sum())
    crit = sstats.chi2.ppf(0.999, len(P) - 1)
    assert chi2 < crit, (chi2, crit)
    # per-shard mass share matches too
    share = np.array([counts[offs[r]:offs[r + 1]].sum() for r in range(W)]) / n_draws
    np.testing.assert_allclose(share, [P[offs[r]:offs[r + 1]].sum() for r in range(W)], atol=0.01)


def test_sharded_is_weights_use_global_min_and_batch_correction():
    shards = [_shard(0, 30, 1.0), _shard(1, 30, 9.0)]
    _link(shards)
    W, B = 2, 16
    pmin = min(s.min_leaf() for s in shards)
    st = shards[0].shard_stats.view(W, SHARD_STATS)[:, :2].numpy()
    M = min(W * B, int(np.floor((B - 2) * st[:, 0].sum() / st[:, 0].max())))
    for r, s in enumerate(shards):
        out = s.sample(B)
        v = out["gen"] >= 0
        p = s.leaf[out["idx"]].double()
        w_exp = torch.clamp((p / pmin) ** -BETA, max=1.0) * (W * B / M)
        torch.testing.assert_close(out["weights"][v].double(), w_exp[v], rtol=1e-5, atol=1e-7)
        assert torch.all(out["weights"][~v] == 0)


def test_sharded_priority_writeback_ignores_foreign_rows():
    """A row of a sharded draw that fell in another shard (generation -1) sits on the
    first live leaf (u = 0); a VALID row that drew the same leaf earlier in the batch
    must keep its new priority (the foreign row takes no part in the last-writer dedupe)."""
    rp = _shard(0, 20, 1.0)
    idx = torch.tensor([0, 5, 0, 0], dtype=torch.int64)
    gen = rp.gen[idx].clone()
    gen[2:] = -1                      # two foreign rows on leaf 0, after the valid one
    td = torch.tensor([3.0, 0.5, 9.0, 9.0])
    rp.update_priorities(idx, td, gen)
    want = (3.0 + rp.eps) ** ALPHA
    assert abs(float(rp.leaf[0]) - want) < 1e-5 * want
    assert abs(float(rp.leaf[5]) - (0.5 + rp.eps) ** ALPHA) < 1e-5


def test_global_draw_partition_is_rank_consistent():
    st = np.array([[3.0, 0.1], [0.0, np.inf], [11.0, 0.2], [5.0, 0.05]])
    B = 10
    got = []
    for r in range(4):
        u, valid, wscale, pm = global_draw(st, r, B, seed=3, ctr=9)
        assert pm == pytest.approx(0.05)
        assert np.all(u[valid] >= 0) and np.all(u[valid] < st[r, 0])
        got.append(int(valid.sum()))
    M = min(4 * B, int(np.floor((B - 2) * st[:, 0].sum() / st[:, 0].max())))
    assert sum(got) == M and got[1] == 0


def _gloo_worker(rank, world, path, q):
    from apex_dqn_amd.parallel.dist import Comm
    torch.set_num_threads(1)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo")
    rp = _shard(rank, 20 + 7 * rank, float(rank + 1) ** 2)
    rp.enable_sharding(rank, world, 123)
    rp.gather_shard_stats()
    res = []
    for it in range(20):
        rp.ctr.fill_(it)
        out = rp.sample(12)
        res.append(int((out["gen"] >= 0).sum()))
    q.put((rank, rp.shard_stats.view(world, SHARD_STATS)[:, :2].numpy().copy(), (rp.total(), rp.min_leaf()), res))
    comm.shutdown()


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4])
def test_shard_stats_allgather_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as td:
        procs = [ctx.Process(target=_gloo_worker, args=(r, world, os.path.join(td, "st"), q)) for r in range(world)]
        for p in procs:
            p.start()
        res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    own = np.array([r[2] for r in res])
    for _, st, _, _ in res:
        np.testing.assert_allclose(st, own, rtol=1e-6)
    T = own[:, 0]
    M = min(world * 12, int(np.floor(10 * T.sum() / T.max())))
    for it in range(20):
        assert sum(r[3][it] for r in res) == M


def test_sharded_config_capacity_per_rank(monkeypatch):
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = ApexConfig.load(os.path.join(here, "configs", "atari_2m_sharded.json"))
    soft, cap = cfg.shard_capacity(8)
    assert soft == 250_000 and cap == 312_500
    assert cfg.shard_capacity(1) == (2_000_000, 2_500_000)
    assert cfg.shard_capacity(3)[0] * 3 >= 2_000_000
    import apex_dqn_amd.runtime.gpu_loop as gl
    seen = {}

    class Probe:
        def __init__(self, cap, soft, frame_cap, C, **kw):
            seen.update(cap=cap, soft=soft, frame_cap=frame_cap)

    monkeypatch.setattr(gl, "GpuReplayShard", Probe)
    gl.build_replay(cfg, "cpu", 45, world=8)
    assert seen["soft"] == 250_000 and seen["cap"] == 312_500
    # frame ring sized for the shard, not the global replay: ~2.8 GB of uint8 frames per rank
    assert seen["frame_cap"] * 84 * 84 < 3.0e9
