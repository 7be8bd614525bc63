"""Global-batch data parallelism (``Runtime.batch_scope = "global"``) on the gloo fake
cluster: W ranks that each compute their share of ONE global prioritized draw of B
samples take the same update as one rank with batch B over the same replay contents
and RNG counter ("W ranks with batch B/W must match 1 rank with batch B").

The one-rank run holds the W shards concatenated in rank order (leaves, records and
frame rings), so the global stratified draw -- identical uniforms, identical strata --
picks the same transitions; the parameters after several updates agree to fp32
round-off (only the order of the gradient sums differs).
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from apex_dqn_amd.config import ApexConfig

CAP, FR = 300, 400
BG, STEPS = 16, 3


def _cfg(slack, exchange="auto", seed=0, shard="auto", adaptive=True):
    return ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 5, "name": "Synthetic"},
                                 "Learner": {"replay_sample_size": BG, "q_target_sync_freq": 2},
                                 "Runtime": {"use_graphs": False, "grad_clip": 40.0, "force_dp": True, "seed": seed,
                                             "batch_scope": "global", "dp_batch_slack": slack,
                                             "dp_fc_exchange": exchange, "dp_shard_update": shard,
                                             "dp_rows_adaptive": adaptive}})


def _computed(L):
    """Mask of the gradient entries this rank computes: all of them, or with the sharded
    update (learner/dp_step.py) the conv + head range and its own fc rows."""
    m = np.ones(L.g32.numel(), bool)
    if L._shard:
        off = L.layout.offsets
        m[off["wfc"]:] = False
        o = off["wfc"] + L._fc_r0 * 3136
        m[o:o + L._fc_S * 3136] = True
        m[off["bfc"] + L._fc_r0:off["bfc"] + L._fc_r0 + L._fc_S] = True
    return m


def _shard(rank):
    """Rank ``rank``'s replay shard: deliberately unequal priority mass per shard."""
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    rp = GpuReplayShard(CAP, CAP, FR, 4, device="cpu", seed=rank + 3)
    rng = np.random.default_rng(100 + rank)
    seqs = rp.append_frames(rng.integers(0, 255, (120, 84, 84), dtype=np.uint8))
    K = 100
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 5, K), R=rng.normal(size=K),
                   Gamma=np.where(rng.random(K) < 0.2, 0.0, 0.97), priority=rng.random(K) * (1 + 0.5 * rank)))
    return rp


def _concat(world):
    """One replay holding the ``world`` shards back to back (rank order)."""
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    shards = [_shard(r) for r in range(world)]
    rp = GpuReplayShard(CAP * world, CAP * world, FR * world, 4, device="cpu", seed=3)
    rp.frames.copy_(torch.cat([s.frames for s in shards]))
    for name in ("act", "rew", "gam", "gen", "leaf"):
        getattr(rp, name).copy_(torch.cat([getattr(s, name) for s in shards]))
    rp.obs.copy_(torch.cat([s.obs + r * FR for r, s in enumerate(shards)]))
    rp.nxt.copy_(torch.cat([s.nxt + r * FR for r, s in enumerate(shards)]))
    rp.live = rp.head = CAP * world
    rp._torch_rebuild()
    return rp


def _worker(rank, world, concat, slack, path, q, exchange="auto", shard="auto", adaptive=True):
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    torch.set_num_threads(2)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo", force=True)
    torch.manual_seed(1234)          # identical initial parameters in every run
    rp = _concat(concat) if concat else _shard(rank)
    # per-rank Runtime.seed (as bench.py sets it): the draw's seed is rank 0's on every rank
    L = FusedNatureLearner(_cfg(slack, exchange, seed=7 * rank, shard=shard, adaptive=adaptive), "cpu", rp,
                           comm=comm)
    assert L._fc_factors == (exchange != "allreduce")
    assert L._shard == (world > 1 and shard != "off")
    mask = _computed(L)
    draws, grads = [], []
    p0 = L.p32.numpy().copy()
    for _ in range(STEPS):
        if adaptive:
            L.refresh_replay_stats()     # (the loop's eviction-cadence check, here every update)
        L._sample()
        valid = L.S["gen"] >= 0
        # global leaf id of every row this rank drew (the concatenated replay's numbering)
        draws.append((L.S["idx"][valid] + (0 if concat else rank * CAP)).tolist())
        L.step()
        grads.append(np.where(mask, L.g32.numpy(), np.nan))
    L.materialize()              # (sharded: every rank's fp32 rows gathered)
    q.put((rank, L.B, int(L.valid_rows_total.item()), draws, grads, L.p32.numpy().copy(), L.t32.numpy().copy(), p0))
    comm.shutdown()


def _run(world, concat, slack, exchange="auto", shard="auto", adaptive=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "store")
        procs = [ctx.Process(target=_worker, args=(r, world, concat, slack, path, q, exchange, shard, adaptive)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    return sorted(res, key=lambda r: r[0])


def test_dp_batch_rows():
    cfg = ApexConfig.from_dict({"Learner": {"replay_sample_size": 512}})
    assert [cfg.dp_batch(w) for w in (1, 2, 4, 8)] == [(512, 512), (290, 512), (146, 512), (74, 512)]
    assert cfg.dp_batch(8, dp=False) == (512, 512)
    cfg.Runtime.batch_scope = "per_rank"
    assert cfg.dp_batch(8) == (512, 8 * 512)


@pytest.mark.slow
@pytest.mark.parametrize("world,exchange,shard", [(2, "factors", "auto"), (4, "factors", "auto"),
                                                  (2, "allreduce", "auto"), (4, "allreduce", "auto"),
                                                  (2, "factors", "off"), (2, "allreduce", "off")])
def test_global_batch_dp_equals_one_rank(world, exchange, shard):
    """``exchange``: the fc gradient as all-gathered factor rows (every rank forms the
    global batch's gradient, or with the sharded update its own fc rows) or all-reduced
    (sharded: reduce-scattered) -- every variant equals the one-rank update."""
    slack = 1.0
    multi = _run(world, 0, slack, exchange, shard)
    one = _run(1, world, slack, "allreduce")[0]
    rows = multi[0][1]
    assert rows == int(np.ceil(BG / world * (1 + slack))) + 2 and one[1] == BG
    # every update drew exactly BG samples over the shards, and one rank drew the same BG
    assert sum(r[2] for r in multi) == STEPS * BG == one[2]
    for s in range(STEPS):
        glob = [i for r in multi for i in r[3][s]]
        assert glob == one[3][s], (s, glob, one[3][s])
    # the same updates: all-reduced gradient and parameters to fp32 round-off
    for r in multi:
        for s in range(STEPS):
            g1, gw = one[4][s], r[4][s]
            m = ~np.isnan(gw)
            assert np.abs(gw[m] - g1[m]).max() <= 2e-6 * np.abs(g1).max() + 1e-10, s
        # parameters: RMSprop divides by sqrt(centered variance), which amplifies the
        # summation-order round-off of the first updates a little
        upd = np.abs(one[5] - one[7]).max()
        dp = np.abs(r[5] - one[5]).max()
        assert dp <= 1e-3 * upd, (dp, upd)
        assert np.array_equal(r[5], multi[0][5])            # replicas bit-identical
        assert np.abs(r[6] - one[6]).max() <= 1e-3 * upd


@pytest.mark.slow
def test_default_slack_adaptive_rows_keep_the_global_batch():
    """At the default slack (0.125) a 2-rank buffer holds 11 rows, enough while no shard
    carries more than 9 / 16 of the priority mass; the priority write-backs push rank 1's
    share past that.  Without the adaptive buffer the draw shrinks (M < 16, a different
    update); with it (``Runtime.dp_rows_adaptive``, learner/dp_step.py; checked here before
    every update, in the loops at the eviction cadence) both ranks grow to the same larger
    buffer and the updates equal the one-rank update over the concatenated replay."""
    fixed = _run(2, 0, 0.125, "factors", "auto", adaptive=False)
    assert fixed[0][1] == 11 and sum(r[2] for r in fixed) < STEPS * BG      # the draw shrank
    multi = _run(2, 0, 0.125, "factors", "auto", adaptive=True)
    one = _run(1, 2, 0.125, "allreduce")[0]
    rows = multi[0][1]
    assert rows > 11 and multi[1][1] == rows
    assert sum(r[2] for r in multi) == STEPS * BG == one[2]
    for s in range(STEPS):
        assert [i for r in multi for i in r[3][s]] == one[3][s]
    upd = np.abs(one[5] - one[7]).max()
    for r in multi:
        assert np.abs(r[5] - one[5]).max() <= 1e-3 * upd
