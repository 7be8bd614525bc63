"""Data-parallel learner over gloo (CPU, world_size 2 and 4): the fake cluster.

Checks that the bucketed, overlapped gradient all-reduce of the fused learner
equals the mean of the per-rank gradients on the same globally drawn batches,
that parameters stay bit-identical across ranks, and that the shards' statistics
are all-gathered (one global prioritized replay, replay/gpu_replay.py).
"""
import os
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from apex_dqn_amd.config import ApexConfig


def _cfg(ar="fp32", force_dp=False):
    return ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 5, "name": "Synthetic"},
                                 "Learner": {"replay_sample_size": 6},
                                 "Runtime": {"use_graphs": False, "grad_clip": 40.0, "allreduce_dtype": ar,
                                             "force_dp": force_dp, "batch_scope": "per_rank"}})


def _replay(rank):
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    rp = GpuReplayShard(300, 300, 400, 4, device="cpu", seed=rank + 3)
    rng = np.random.default_rng(100 + rank)
    seqs = rp.append_frames(rng.integers(0, 255, (120, 84, 84), dtype=np.uint8))
    K = 100
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 5, K), R=rng.normal(size=K),
                   Gamma=np.full(K, 0.97), priority=rng.random(K) * (rank + 1)))
    return rp


def _worker(rank, world, path, q, ar="fp32"):
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    torch.set_num_threads(2)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo", force=world == 1)
    cfg = _cfg(ar, force_dp=world == 1)   # world 1: the DP step forced on one rank
    torch.manual_seed(1234 + rank)  # different local init: rank 0's params must be broadcast
    rp = _replay(rank)
    L = FusedNatureLearner(cfg, "cpu", rp, comm=comm)
    stats = rp.shard_stats.view(world, 3)[:, :2].clone()
    own = (rp.total(), rp.min_leaf())
    # the global draw of step 1 (what L.step() consumes: presampled, version unchanged)
    L._sample()
    # local reference gradient on an identical replay copy and the SAME batch, single
    # rank, scale 1/B: the DP gradient is the mean of these over the ranks
    torch.manual_seed(0)
    rp2 = _replay(rank)
    Lref = FusedNatureLearner(cfg, "cpu", rp2, comm=None)
    Lref.p32.copy_(L.p32)
    Lref.pbf.copy_(L.pbf)
    Lref.sync_target()
    for k, v in L.S.items():
        Lref.S[k].copy_(v)
    Lref.slots.copy_(L.slots)
    Lref._sample_ver = rp2.version
    Lref._seg1()
    Lref._seg2()
    g_local = Lref.g32.clone()
    n_valid = int((L.S["gen"] >= 0).sum())
    L.step()
    counted = int(L.valid_rows_total.item())     # the head's device-side count (bench.py's M)
    g_dp = L.g32.clone()
    for _ in range(3):
        L.step()
    L.materialize()              # sharded fc update (learner/dp_step.py): gather the fp32 rows
    gl = [torch.zeros_like(g_local) for _ in range(world)]
    torch.distributed.all_gather(gl, g_local)
    g_mean = torch.stack(gl).mean(0)
    if L._shard:                 # the gradient rows this rank computed: conv + head, its fc rows
        keep = torch.zeros_like(g_dp, dtype=torch.bool)
        off = L.layout.offsets
        keep[:off["wfc"]] = True
        o = off["wfc"] + L._fc_r0 * 3136
        keep[o:o + L._fc_S * 3136] = True
        keep[off["bfc"] + L._fc_r0:off["bfc"] + L._fc_r0 + L._fc_S] = True
        g_dp, g_mean = g_dp[keep], g_mean[keep]
    pl = [torch.zeros_like(L.p32) for _ in range(world)]
    torch.distributed.all_gather(pl, L.p32.clone())
    perr = max([float((pl[0] - p).abs().max()) for p in pl[1:]], default=0.0)
    q.put((rank, float((g_dp - g_mean).abs().max()), float(g_mean.abs().max()), perr, stats.numpy(),
           own, n_valid, counted))
    comm.shutdown()


@pytest.mark.slow
@pytest.mark.parametrize("ar,world", [("fp32", 1), ("fp32", 2), ("bf16", 2), ("fp32", 4)])
def test_dp_learner_gloo(ar, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "store")
        procs = [ctx.Process(target=_worker, args=(r, world, path, q, ar)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=240) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    tol = 1e-6 if ar == "fp32" else 1e-2          # bf16 payload: ~3 significant digits
    res.sort(key=lambda r: r[0])
    own = np.array([r[5] for r in res])
    for rank, gerr, gmax, perr, stats, _, nv, counted in res:
        assert counted == nv                          # the counted rows are the rows drawn
        assert gerr <= tol * max(gmax, 1e-6) + 1e-9, (rank, gerr, gmax)
        assert perr == 0.0
        # every rank holds every shard's (total, min p) in rank order
        np.testing.assert_allclose(stats, own, rtol=1e-6)
    # every one of the M global draws landed in exactly one shard
    B, T = 6, own[:, 0]
    M = min(world * B, B if world == 1 else int(np.floor((B - 2) * T.sum() / T.max())))
    assert sum(r[6] for r in res) == M


def _elastic_target(comm, attempt, ckdir, out_dir, fail_at):
    """2-rank gloo training; rank 1 crashes at learner step ``fail_at`` on the
    first attempt (fault injection).  Checkpoints every 4 steps."""
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    torch.set_num_threads(2)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                "Actor": {"num_actors": 8, "n_step_transition_batch_size": 4,
                                          "Q_network_sync_freq": 5},
                                "Learner": {"min_replay_mem_size": 40, "replay_sample_size": 8,
                                            "remove_old_xp_freq": 4, "q_target_sync_freq": 5},
                                "Replay_Memory": {"soft_capacity": 120},
                                "Runtime": {"replay_capacity": 150, "log_every": 0, "use_graphs": False,
                                            "ckpt_dir": ckdir, "ckpt_freq": 4}})
    if attempt == 0 and comm.rank == 1:
        import apex_dqn_amd.learner.fused_learner as fl
        orig = fl.FusedNatureLearner.step

        def faulty(self):
            if self.num_q_updates == fail_at:
                os._exit(17)          # hard crash of one learner rank
            return orig(self)
        fl.FusedNatureLearner.step = faulty
    out = train_frames(cfg, "cpu", 12, comm=comm)
    L = out["learner"]
    torch.save({"n": L.num_q_updates, "p": L.p32.clone()}, os.path.join(out_dir, f"rank{comm.rank}.pt"))


@pytest.mark.slow
def test_elastic_restart_resumes_from_checkpoint():
    from apex_dqn_amd.runtime.launch import run_elastic
    with tempfile.TemporaryDirectory() as ck, tempfile.TemporaryDirectory() as out:
        res = run_elastic(_elastic_target, 2, args=(ck, out, 6), max_restarts=2, timeout_s=600)
        assert res["attempts"] == 2 and res["failures"][0]["ranks"][0][0] == 1
        r0 = torch.load(os.path.join(out, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(out, "rank1.pt"), weights_only=True)
        assert r0["n"] == r1["n"] == 12
        assert torch.equal(r0["p"], r1["p"])   # replicas identical after the restart


def _replica_worker(rank, world, path, q):
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    torch.set_num_threads(2)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo")
    L = FusedNatureLearner(_cfg(), "cpu", _replay(rank), comm=comm)
    L.step()
    ok_before = L.check_replicas()
    if rank == 1:                       # a corrupted replica
        L.p32[123] += 1e-3
        L.rms_v[7] += 1.0
    ok_corrupt = L.check_replicas()
    pl = [torch.zeros_like(L.p32) for _ in range(world)]
    torch.distributed.all_gather(pl, L.p32.clone())
    same = all(torch.equal(pl[0], p) for p in pl[1:])
    q.put((rank, ok_before, ok_corrupt, same, L.check_replicas()))
    comm.shutdown()


@pytest.mark.slow
def test_replica_check_detects_and_repairs_divergence():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as td:
        procs = [ctx.Process(target=_replica_worker, args=(r, 2, os.path.join(td, "s"), q)) for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=240) for _ in range(2)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    for _, ok_before, ok_corrupt, same, ok_after in res:
        assert ok_before and not ok_corrupt and same and ok_after



def _probe_parent(rank, world, port, env, q):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **env)
    from apex_dqn_amd.runtime.capture_probe import run_probe
    variants = [{"name": "headline", "cfg": {}}, {"name": "bf16", "cfg": {}}]
    q.put((rank, run_probe(variants, rank, world, 0, timeout=60.0)))


@pytest.mark.parametrize("inject", ["", "abort@1"])
def test_capture_probe_rendezvous_and_agreement(inject):
    """runtime/capture_probe.py across 2 parent processes (dry children: no GPU work):
    every parent spawns one child, the children meet in their own gloo group through the
    parents' TCP store under the probe's key prefix, and every parent reads every rank's
    exit status.  A child that aborts on rank 1 fails the probe on BOTH ranks (the other
    rank's child is killed through the store's failure flag or exits cleanly): every
    variant then runs eagerly everywhere."""
    import random
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + random.randint(0, 150)
    env = {"APEX_CAPTURE_PROBE_DRY": "1", "APEX_CAPTURE_PROBE_INJECT": inject}
    ps = [ctx.Process(target=_probe_parent, args=(r, 2, port, env, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in ps:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert out[0]["rc"] == out[1]["rc"] and out[0]["ok"] == out[1]["ok"]
    if not inject:
        assert out[0]["rc"] == [0, 0] and out[0]["ok"] == {"headline": True, "bf16": True}
    else:
        assert out[0]["rc"][1] == -6 and out[0]["ok"] == {"headline": False, "bf16": False}
    assert max(o["seconds"] for o in out.values()) < 60
