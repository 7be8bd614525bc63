"""GPU runtime: actor head kernel, actor group + HBM replay + fused learner loop
(HIP graphs on), CLI in gpu mode."""
import json
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


def _dp_gpu_worker(rank, world, path, q, exchange="auto"):
    """One rank of a 2-process data-parallel learner sharing cuda:0 (gloo carries
    the CUDA-tensor all-reduces; RCCL refuses two ranks on one GPU).  Exercises the
    DP step exactly as on a node: three captured HIP-graph segments, async bucket
    all-reduces waited on the compute stream, the all-gathered shard statistics of
    the global prioritized replay."""
    import numpy as np
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.init(rank, world, f"file://{path}", backend="gloo", device=dev)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 128},
                                "Runtime": {"use_graphs": True, "dp_fc_exchange": exchange}})
    rp = GpuReplayShard(2000, 2000, 2600, 4, device=dev, seed=rank + 3)
    rng = np.random.default_rng(100 + rank)
    seqs = rp.append_frames(rng.integers(0, 255, (1200, 84, 84), dtype=np.uint8))
    K = 1000
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01 * (rank + 1)))
    torch.manual_seed(1234 + rank)            # different local init: rank 0's params are broadcast
    L = FusedNatureLearner(cfg, dev, rp, comm=comm)
    assert L._fc_factors == (exchange != "allreduce")
    drawn = []
    for _ in range(4):
        if L._sample_ver != rp.version:
            L._sample()
        torch.cuda.synchronize()
        drawn.append((int((L.S["weights"] > 0).sum()), int((L.S["gen"] >= 0).sum())))
        L.step()
    torch.cuda.synchronize()
    assert L._shard                     # (the fc optimizer sharded by rows: gather the fp32 rows)
    L.materialize()
    pl = [torch.zeros_like(L.p32) for _ in range(world)]
    torch.distributed.all_gather(pl, L.p32.clone())
    ok_finite = bool(torch.isfinite(L.p32).all())
    q.put((rank, float((pl[0] - pl[1]).abs().max()), ok_finite, float(L.gnorm[0]), rp.shard_stats.cpu().tolist(),
           drawn))
    comm.shutdown()


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["factors", "allreduce"])
def test_dp_learner_two_ranks_on_one_gpu(tmp_path, exchange):
    """Global-batch DP step (128 samples over two shards, 74 rows per rank) with the fc
    gradient exchanged as all-gathered factor rows (HIP row pack, strided fc wgrad of
    the gathered batch, clip-norm partials of the all-reduced regions) or all-reduced."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "store")
    procs = [ctx.Process(target=_dp_gpu_worker, args=(r, 2, path, q, exchange)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    for rank, perr, finite, gnorm, ratio, _ in res:
        assert perr == 0.0 and finite and gnorm > 0      # replicas bit-identical after 4 DP steps
    assert res[0][4] == res[1][4]                        # same shard statistics on both ranks
    # every update drew exactly the global batch over the two shards (rows with IS weight > 0
    # = rows with a valid generation)
    for t in range(4):
        (w0, g0), (w1, g1) = res[0][5][t], res[1][5][t]
        assert w0 == g0 and w1 == g1 and w0 + w1 == 128, (t, res[0][5], res[1][5])


def _forced_dp_worker(path, q, dtype):
    """One process: the same update as a single-rank step and as the forced DP step
    (world 1 process group, factored fc exchange), from identical state and batch."""
    import numpy as np
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.init(0, 1, f"file://{path}", backend="gloo", device=dev, force=True)
    out = {}
    for dp in (False, True):
        cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                    "Learner": {"replay_sample_size": 256},
                                    "Runtime": {"use_graphs": False, "presample": True, "dtype": dtype,
                                                "force_dp": dp, "dp_fc_exchange": "factors"}})
        # the sharded draw at world 1 is the single-rank draw with the shard seed
        # ((Runtime.seed << 20) ^ 0x5EED): the same seed here gives both runs one batch
        rp = GpuReplayShard(4000, 4000, 4100, 4, device=dev, seed=0x5EED)
        rng = np.random.default_rng(9)
        seqs = rp.append_frames(rng.integers(0, 255, (3000, 84, 84), dtype=np.uint8))
        K = 2800
        st = np.stack([seqs[i:i + 4] for i in range(K)])
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K).astype(np.float32),
                       Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
        torch.manual_seed(3)
        L = FusedNatureLearner(cfg, dev, rp, comm=comm if dp else None)
        assert L._fc_factors == dp
        L.step()
        L.step()
        torch.cuda.synchronize()
        out[dp] = (L.g32.cpu().numpy(), L.p32.cpu().numpy(), float(L.gnorm[0]))
    comm.shutdown()
    (g0, p0, n0), (g1, p1, n1) = out[False], out[True]
    q.put((float(np.abs(g1 - g0).max()), float(np.abs(g0).max()), float(np.abs(p1 - p0).max()),
           float(np.abs(p0).max()), n0, n1))


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_forced_dp_factored_step_matches_single_rank(tmp_path, dtype):
    """The factored DP step on one rank (all-gather = copy) takes the single-rank update:
    gradient, clip norm and parameters agree (the fc gradient runs on the strided
    gathered rows instead of inside the fused fc + head + priority launch: summation
    order only)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_dp_worker, args=(str(tmp_path / "store"), q, dtype))
    p.start()
    gerr, gmax, perr, pmax, n0, n1 = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    assert gerr <= 1e-5 * gmax, (gerr, gmax)
    assert abs(n1 - n0) <= 1e-5 * n0, (n0, n1)
    assert perr <= 1e-6 * pmax + 1e-9, (perr, pmax)


@pytest.mark.parametrize("hip,dtype,kind", [(True, "bf16", "impala"), (False, "bf16", "graph"),
                                            (True, "fp32", "impala"), (False, "fp32", "graph")])
def test_impala_loop_with_hip_graph(hip, dtype, kind):
    """IMPALA-deep on the GPU loop (actors + HBM replay + graph-captured step): the
    hand-written learner -- csrc/impala_split.hip (fp32: split operands, fp32-class actors)
    or csrc/impala.hip (bf16 operands) -- and the torch-autograd graph learner
    (use_hip_kernels off)."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.runtime.gpu_loop import train_frames
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Actor": {"num_actors": 16, "n_step_transition_batch_size": 16,
                                          "Q_network_sync_freq": 10},
                                "Learner": {"min_replay_mem_size": 300, "replay_sample_size": 64,
                                            "remove_old_xp_freq": 10, "q_target_sync_freq": 20},
                                "Replay_Memory": {"soft_capacity": 2000},
                                "Runtime": {"replay_capacity": 2500, "log_every": 0, "use_graphs": True,
                                            "network": "impala", "use_hip_kernels": hip, "dtype": dtype}})
    out = train_frames(cfg, DEV, 30)
    L = out["learner"]
    assert L.kind == kind and L.num_q_updates == 30 and L._graphs is not None
    m = L.last_metrics()
    assert np.isfinite(m["loss"]) and m["grad_norm"] > 0


def test_fused_norm_equals_gradient_norm():
    """Single-rank fused learner: the clip norm summed by the gradient producers
    (fc wgrad epilogue partials + grad_finalize blocks + norm_total) must equal the
    norm of the final flat gradient, step after step (graph replays)."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 256},
                                "Runtime": {"use_graphs": True, "grad_clip": 1e-3}})
    rp = GpuReplayShard(3000, 3000, 3600, 4, device=DEV, seed=5)
    rng = np.random.default_rng(5)
    seqs = rp.append_frames(rng.integers(0, 255, (2000, 84, 84), dtype=np.uint8))
    K = 1800
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    L = FusedNatureLearner(cfg, DEV, rp)
    assert L._fuse_norm
    for _ in range(3):
        L.step()
        torch.cuda.synchronize()
        # the reported norm is that of the gradient the optimizer applies: g32 times the
        # batch-max IS scale (learner/is_norm.py)
        true = float(L.g32.double().norm()) * L.is_scale()
        assert abs(float(L.gnorm[0]) - true) <= 1e-4 * true + 1e-12, (float(L.gnorm[0]), true)


def _filled_replay(seed=5, K=1800):
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    rp = GpuReplayShard(3000, 3000, 3600, 4, device=DEV, seed=seed)
    rng = np.random.default_rng(seed)
    seqs = rp.append_frames(rng.integers(0, 255, (2000, 84, 84), dtype=np.uint8))
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K).astype(np.float32),
                   Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
    return rp


def test_gpu_resume_matches_uninterrupted_run(tmp_path):
    """Checkpoint at update 4, resume in a fresh learner on the replay as it was at
    that update: updates 5..9 are bit-identical to the uninterrupted run (params,
    RMSprop state, target net, sampling counter; graphs on, pre-sampling on)."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 128, "q_target_sync_freq": 3},
                                "Runtime": {"use_graphs": True}})
    rp = _filled_replay()
    L = FusedNatureLearner(cfg, DEV, rp)
    for _ in range(4):
        L.step()
    torch.cuda.synchronize()
    ck = str(tmp_path / "ck.pt")
    L.save(ck)
    tree = [t.clone() for t in (rp.leaf, rp.nodes, rp.min_bits, rp.ctr)]
    for _ in range(5):
        L.step()
    torch.cuda.synchronize()
    rp2 = _filled_replay()
    for dst, src in zip((rp2.leaf, rp2.nodes, rp2.min_bits, rp2.ctr), tree):
        dst.copy_(src)
    cfg2 = ApexConfig.from_dict({**cfg.to_dict(), "Learner": {**cfg.to_dict()["Learner"], "load_saved_state": ck}})
    L2 = FusedNatureLearner(cfg2, DEV, rp2)
    assert L2.num_q_updates == 4
    for _ in range(5):
        L2.step()
    torch.cuda.synchronize()
    for a, b in ((L.p32, L2.p32), (L.rms_v, L2.rms_v), (L.rms_m, L2.rms_m), (L.t32, L2.t32),
                 (rp.leaf, rp2.leaf), (rp.ctr, rp2.ctr)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [32, 48])
def test_fused_learner_unaligned_batch(B):
    """Batches whose online/target split is not a 128-row tile boundary (2B % 128 != 0)
    run each forward layer as two launches; the step matches the torch backend."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard

    def make(backend):
        cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                    "Learner": {"replay_sample_size": B}, "Runtime": {"use_graphs": True}})
        rp = GpuReplayShard(1024, 1024, 2048, 4, device=DEV, seed=1)
        rng = np.random.default_rng(0)
        seqs = rp.append_frames(rng.integers(0, 255, (600, 84, 84), dtype=np.uint8))
        K = 512
        st = np.stack([seqs[i:i + 4] for i in range(K)])
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K),
                       Gamma=np.full(K, 0.97), priority=rng.random(K)))
        torch.manual_seed(0)
        return FusedNatureLearner(cfg, DEV, rp, backend=backend)
    Lh, Lt = make("hip"), make("torch")
    Lt.p32.copy_(Lh.p32); Lt._refresh_bf16(); Lt.sync_target()
    Lh._step_body(); Lt._step_body()
    torch.cuda.synchronize()
    torch.testing.assert_close(Lh.td_abs, Lt.td_abs, rtol=5e-2, atol=5e-2)
    Lh.step()
    torch.cuda.synchronize()
    assert np.isfinite(Lh.last_metrics()["loss"])


_BENCH_KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
               "vs_baseline", "dtype", "data", "config"}


def _bench_json(stdout: str) -> dict:
    import json
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout[-2000:]
    out = json.loads(lines[0])
    assert _BENCH_KEYS <= set(out), set(out)
    return out


def test_bench_contract_one_gpu():
    """bench.py prints exactly one JSON line with the driver's keys; the headline is
    the fp32 (reference-precision) learner, bf16 rides along as value_bf16, and no
    HIP graph is captured inside either timed window (warmup 5 < graph_steps 20:
    the 20-update graph is captured by prepare_graphs, before the clock starts)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "30", "--warmup", "5",
                        "--replay", "20000"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _bench_json(r.stdout)
    assert out["n_gpus"] == 1 and out["steps"] == 30 and out["value"] > 0
    assert out["config"]["global_batch"] == 512 and out["dtype"] == "fp32"
    assert out["value_bf16"] > 0
    assert out["graph_captures_in_timed"] == 0 and out["graph_captures_in_timed_bf16"] == 0
    assert out["prep_graph_captures"] == 2


def test_bench_two_ranks_gloo_rehearsal():
    """The driver's N>1 launch (torch.distributed.run, one rank per device) rehearsed
    with 2 ranks on this one GPU over gloo: every DP code path of the bench runs and
    rank 0 alone prints the whole-job JSON line (RCCL itself refuses 2 ranks on 1 GPU)."""
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29541", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "20", "--warmup", "5", "--replay", "20000",
                        "--dist-backend", "gloo", "--no-bf16-extra"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    out = _bench_json(r.stdout)
    print(r.stdout[-3000:])
    # default: one global 512-sample update per step (strong scaling), each rank computing
    # its share (290 rows at W = 2); the per-rank scope rides along as value_weak
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 512 and out["config"]["parallelism"] == "dp2"
    assert out["scaling"] == "strong" and out["config"]["per_rank_rows"] == 290
    assert out["samples_per_dp_step"] == 512.0 and out["value"] == out["value_strong"] > 0
    assert out["value_weak"] > 0 and out["per_rank_rows_weak"] == 512 and out["samples_per_dp_step_weak"] > 512
    assert out["graph_captures_in_timed"] == 0
    # what the collectives themselves report: the process group's rank count, the checked
    # all-reduce of rank + 1 (1 + 2 = 3), and whether the DP step ran as captured graphs
    # (gloo: eager by design) -- the fields the driver's first N-GPU run is judged by
    assert out["comm_world"] == 2 and out["init_allreduce"] == 3.0 and out["init_allreduce_ok"] is True
    assert out["dp_graphs"] is False and out["graph_fallback"] is None
    assert out["config"]["dp_collectives"] == "torch" and out["config"]["dp_shard_update"] is True
    # the self-checks after the timed region: replicas bit-identical across the 2 ranks;
    # gloo runs the eager DP step, so there is no capture to probe or to compare
    assert out["replicas_identical"] is True
    assert out["dp_capture_probe"] == "not run (eager DP step)" and out["graph_matches_eager"] is None
    assert len(out["param_sha256"]) == 16


def _bench_force_dp(extra_env, port, tmp):
    env = dict(os.environ, **extra_env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--force-dp", "--capture-probe", "on",
                        "--steps", "20", "--warmup", "5", "--replay", "20000", "--no-bf16-extra", "--prep-warm", "0",
                        "--capture-probe-timeout", "120", "--capture-probe-log", str(tmp)],
                       capture_output=True, text=True, timeout=400, cwd=ROOT,
                       env=dict(env, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
    log = open(os.path.join(str(tmp), "capture_probe_rank0.log"), errors="replace").read()
    print(log[-3000:])
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    return _bench_json(r.stdout)


@pytest.mark.gpu
def test_capture_probe_abort_falls_back_to_identical_eager_updates(tmp_path):
    """bench.py's out-of-process DP capture probe (runtime/capture_probe.py) at world 1
    (--force-dp: the DP step over a one-rank RCCL communicator).  Clean: the child
    captures and replays, the parent keeps its graphs, and one captured update equals
    the eager one bit for bit.  With the child forced to abort (SIGABRT after its
    captures) the parent runs the eager DP step instead -- and ends at the same fp32
    weights as the captured run."""
    import random
    port = 29900 + random.randint(0, 90)
    a = _bench_force_dp({}, port, tmp_path)
    b = _bench_force_dp({"APEX_CAPTURE_PROBE_INJECT": "abort"}, port + 1, tmp_path)
    print(json.dumps({k: a.get(k) for k in ("dp_capture_probe", "graph_matches_eager", "param_sha256")}))
    print(json.dumps({k: b.get(k) for k in ("dp_capture_probe", "graph_fallback", "param_sha256")}))
    assert a["dp_capture_probe"]["rc"] == [0] and a["dp_capture_probe"]["ok"] == {"headline": True}
    assert a["dp_graphs"] is True and a["graph_fallback"] is None and a["graph_captures_in_timed"] == 0
    assert a["graph_matches_eager"] is True and a["replicas_identical"] is True
    assert a["dp_capture_probe"]["seconds"] < 60
    assert b["dp_capture_probe"]["rc"] == [-6] and b["dp_capture_probe"]["ok"] == {"headline": False}
    assert b["dp_graphs"] is False and "capture probe" in b["graph_fallback"]
    assert b["graph_matches_eager"] is None
    assert a["param_sha256"] == b["param_sha256"]


def _native_rccl_worker(q, port):
    import os
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0")
    import torch
    from apex_dqn_amd.parallel.dist import Comm
    from apex_dqn_amd.parallel.rccl import make_collectives
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.from_env(device=dev, force=True)
    coll = make_collectives(comm, "native", dev)
    nc = comm._native
    out = {"version": nc.version}
    x = torch.arange(1000, dtype=torch.float32, device=dev)
    w = coll.all_reduce(x)
    w.wait()
    g_out = torch.zeros(4, dtype=torch.float64, device=dev)
    coll.all_gather_into(g_out, torch.tensor([1.5, 2.5, 3.5, 4.5], dtype=torch.float64, device=dev)).wait()
    b = torch.full((7,), 3.0, device=dev, dtype=torch.bfloat16)
    nc.broadcast_(b, 0)
    # captured: all-reduce on the comm stream inside a HIP graph, replayed twice
    y = torch.ones(4096, device=dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        coll.all_reduce(y).wait()
    torch.cuda.current_stream(dev).wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y.mul_(2.0)
        coll.all_reduce(y).wait()
        y.add_(1.0)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    nc.check()
    out.update(x_ok=bool(torch.equal(x, torch.arange(1000, dtype=torch.float32, device=dev))),
               gather=g_out.cpu().tolist(), bcast=float(b.float().min()), bmax=float(b.float().max()), y=float(y[0]))
    comm.shutdown()
    q.put(out)


@pytest.mark.gpu
def test_native_rccl_communicator_world1():
    """csrc/comm/rccl_comm.cpp over the process's librccl: init from a unique id,
    all-reduce / all-gather / broadcast on explicit streams, capture in a HIP graph,
    async-error check (world 1: one rank per GPU, the box has one)."""
    import random
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_native_rccl_worker, args=(q, 29600 + random.randint(0, 300)))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert out["version"] > 0 and out["x_ok"]
    assert out["gather"] == [1.5, 2.5, 3.5, 4.5] and out["bcast"] == out["bmax"] == 3.0
    assert out["y"] == 7.0          # (1*2+1)*2+1: two replays of mul / all-reduce / add


def test_rewarm_preserves_state():
    """learner.rewarm (bench.py's untimed warm replays before the timed window) keeps no
    update: after it the next updates equal those of a learner that never rewarmed."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 128},
                                "Runtime": {"use_graphs": True, "graph_steps": 4}})
    outs = []
    for warm in (0, 3):
        torch.manual_seed(0)
        rp = _filled_replay(seed=7)
        L = FusedNatureLearner(cfg, DEV, rp)
        L.steps(5)
        if warm:
            L.rewarm(warm)
        assert L.num_q_updates == 5
        L.steps(8)
        torch.cuda.synchronize()
        outs.append((L.p32.clone(), L.rms_v.clone(), rp.leaf.clone(), rp.ctr.clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_fc_epilogue_in_head_matches_separate_launch(dtype):
    """The fc forward's split-K epilogue (and the conv2 weight pack) folded into the DDQN
    head launch (ops.fc_fwd(defer_head=True) + head_common.h load_row_part): the stream
    activations h are computed with the same sums, bias, ReLU and rounding as the
    separate epilogue launch (bit-identical at equal parameters: scripts/archive/diag_fc_head.py);
    the head's dot products compile to a different instruction order, so |delta| and the
    update agree to fp32 rounding.  (Later updates are not compared: early centered-RMSprop
    steps scale a gradient difference by up to lr / eps ~ 400, so ulp-level differences
    compound within a few updates -- scripts/archive/diag_fc_head.py.)"""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 128},
                                "Runtime": {"use_graphs": True, "graph_steps": 4, "dtype": dtype}})
    outs = []
    for defer in (True, False):
        torch.manual_seed(0)
        rp = _filled_replay(seed=11)
        L = FusedNatureLearner(cfg, DEV, rp)
        L._defer_fc_epilogue = defer
        L.step()                      # the one-update graph (captured + replayed)
        torch.cuda.synchronize()
        outs.append((L.h[:128].clone(), L.g32.clone(), L.rms_v.clone(), L.td_abs.clone(), L.p32.clone()))
        del L
    assert torch.equal(outs[0][0], outs[1][0])     # h: same parameters, same sums and rounding
    for a, b in zip(outs[0][1:4], outs[1][1:4]):
        assert torch.allclose(a.double(), b.double(), rtol=1e-5, atol=1e-8), float((a - b).abs().max())
    # the first centered-RMSprop update is lr * g / (sqrt(a (1 - a)) |g| + eps): an element
    # whose |g| is near eps moves by up to lr / eps times its gradient's rounding difference
    a, b = outs[0][4], outs[1][4]
    assert torch.allclose(a.double(), b.double(), rtol=1e-5, atol=1e-6), float((a - b).abs().max())


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_actor_q_values_precision_vs_fp32_module(dtype):
    """The GPU actor's batched q-values (reference ``actor.py:160-161``: an fp32
    ``DuellingDQN`` forward) against a torch fp32 forward of the same frames: with the
    fp32 learner the actor runs the split hi / lo kernels (<= 1e-4 relative); the
    bf16-operand actor is a different precision class (~1e-2)."""
    from apex_dqn_amd.actors.gpu_actor import make_gpu_actor_group
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    E = 96
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Actor": {"num_actors": E},
                                "Learner": {"replay_sample_size": 64},
                                "Runtime": {"use_graphs": False, "dtype": dtype}})
    torch.manual_seed(3)
    rp = GpuReplayShard(1000, 1000, 1200, 4, device=DEV)
    L = FusedNatureLearner(cfg, DEV, rp)
    assert L.split == (dtype == "fp32")
    grp = make_gpu_actor_group(cfg, L, rp, E)
    assert grp.split == L.split
    rng = np.random.default_rng(5)
    seqs = rp.append_frames(rng.integers(0, 255, (E + 8, 84, 84), dtype=np.uint8))
    payload = np.stack([seqs[i:i + 4] for i in range(E)])
    grp.eps.zero_()                                   # greedy: a = argmax q
    q, a = grp.policy(payload)
    slots = torch.from_numpy((payload % rp.F).astype(np.int32)).to(DEV)
    q_ref = L.q_values(rp.gather_frames(slots)).double().cpu()
    rel = float((torch.from_numpy(q).double() - q_ref).norm() / q_ref.norm())
    print(f"{dtype} actor q-values vs fp32 module: {rel:.2e}")
    if dtype == "fp32":
        assert rel < 1e-4, rel
        assert np.array_equal(a, q.argmax(1))
    else:
        assert rel > 1e-4        # the bf16 actor is measurably coarser (the reason for the split path)


def test_pipelined_actor_groups_step_all_envs():
    """Runtime.actor_pipeline: the rank's envs as two groups stepped in turn (one group's
    host env step overlaps the other's inference): every env acts once per step, the
    groups take consecutive env ids and the rank's epsilon-ladder slices, episodes land
    in one list, and the transitions reach the replay."""
    from apex_dqn_amd.actors.gpu_actor import PipelinedActorGroups, ladder_slice, make_gpu_actor_group
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    E = 64
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Actor": {"num_actors": E, "n_step_transition_batch_size": 32},
                                "Learner": {"replay_sample_size": 64},
                                "Runtime": {"use_graphs": False, "env_backend": "fake_ale"}})
    torch.manual_seed(3)
    rp = GpuReplayShard(4000, 4000, 4200, 4, device=DEV)
    L = FusedNatureLearner(cfg, DEV, rp)
    grp = make_gpu_actor_group(cfg, L, rp, E, pipeline=2)
    assert isinstance(grp, PipelinedActorGroups) and grp.E == E and len(grp.groups) == 2
    assert grp.groups[0].stream is not grp.groups[1].stream
    assert [g.global_offset for g in grp.groups] == [0, E // 2]
    np.testing.assert_allclose(grp.eps.cpu().numpy(), np.array(ladder_slice(cfg, E, 0, 1, E), dtype=np.float32))
    n0 = rp.size()
    ins = sum(grp.step() for _ in range(40))
    torch.cuda.synchronize()
    assert all(g.t == 40 for g in grp.groups)
    assert ins == grp.inserted > 0 and rp.size() - n0 == ins
    assert all(g.episodes is grp.episodes for g in grp.groups)
    grp.reset_episodes()
    assert all(g.payload is None for g in grp.groups)
    grp.step()                                        # fresh episodes after an actor restart
    assert all(g.t == 41 for g in grp.groups)


@pytest.mark.gpu
def test_staged_frame_append_matches_copy():
    """GpuReplayShard.stage_frames: frames written straight into the pinned staging
    buffer and appended from it land in the HBM ring exactly as a copied append does,
    across both staging buffers and a ring wrap."""
    import numpy as np
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    a = GpuReplayShard(100, 100, 64, 4, device=dev, seed=1)
    b = GpuReplayShard(100, 100, 64, 4, device=dev, seed=1)
    rng = np.random.default_rng(0)
    for it in range(9):
        f = rng.integers(0, 255, (24, 84, 84), dtype=np.uint8)
        buf = a.stage_frames(24)
        assert buf is not None and buf.shape == (24, 84, 84)
        buf[...] = f
        sa = a.append_frames(buf)
        sb = b.append_frames(f)
        np.testing.assert_array_equal(sa, sb)
    torch.cuda.synchronize()
    assert torch.equal(a.frames, b.frames)


def _get_or_dead(q, p, timeout: float):
    """The child's result, failing at once (instead of after ``timeout``) if it died."""
    import queue
    import time
    t_end = time.time() + timeout
    while time.time() < t_end:
        try:
            return q.get(timeout=2)
        except queue.Empty:
            if not p.is_alive():
                raise AssertionError(f"worker died with exit code {p.exitcode}")
    raise AssertionError("worker timed out")


def _dp_variants_worker(q, port):
    """Forced DP at world 1 (RCCL process group of one rank; captured 4-update graphs):
    the same 8 updates through every DP-step variant -- torch.distributed vs the native
    communicator (whose conv1 bucket is all-reduced inline), factored vs all-reduced fc
    exchange, the sharded fc optimizer on / off (learner/dp_step.py), and a DP graph
    capture that fails (injected) and falls back to the eager DP step."""
    import faulthandler
    import os
    faulthandler.enable()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="1", RANK="0")
    import numpy as np
    import torch
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import Comm
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Comm.from_env(device=dev, force=True)
    variants = {
        "torch_factors": ("torch", "factors", "off", False),
        "native_factors": ("native", "factors", "off", False),
        "native_factors_shard": ("native", "factors", "on", False),
        "torch_factors_shard": ("torch", "factors", "on", False),
        "native_factors_shard_fallback": ("native", "factors", "on", True),
        "torch_allreduce": ("torch", "allreduce", "off", False),
        "torch_allreduce_shard": ("torch", "allreduce", "on", False),
    }
    out = {}
    for name, (cb, ex, sh, inject) in variants.items():
        cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                    "Learner": {"replay_sample_size": 256, "q_target_sync_freq": 6},
                                    "Runtime": {"use_graphs": True, "graph_steps": 4, "presample": True,
                                                "force_dp": True, "comm_backend": cb, "dp_fc_exchange": ex,
                                                "dp_shard_update": sh}})
        rp = GpuReplayShard(4000, 4000, 4100, 4, device=dev, seed=0x5EED)
        rng = np.random.default_rng(9)
        seqs = rp.append_frames(rng.integers(0, 255, (3000, 84, 84), dtype=np.uint8))
        K = 2800
        st = np.stack([seqs[i:i + 4] for i in range(K)])
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K).astype(np.float32),
                       Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
        torch.manual_seed(3)
        L = FusedNatureLearner(cfg, dev, rp, comm=comm)
        assert L._dp and L.coll.name == cb and L._shard == (sh == "on") and L._fc_factors == (ex == "factors")
        L._inject_capture_failure = inject
        L.steps(8)
        torch.cuda.synchronize()
        L.materialize()
        rep = L.comm_report()
        out[name] = dict(p=L.p32.cpu(), v=L.rms_v.cpu(), t=L.t32.cpu(), pb=L._pbf_all.cpu(), leaf=rp.leaf.cpu(),
                         graphs=L._graphs_enabled(), fallback=L.graph_fallback, rep=rep)
    comm._native.check()
    comm.shutdown()
    same = lambda a, b: all(torch.equal(out[a][k], out[b][k]) for k in ("p", "v", "t", "pb", "leaf"))  # noqa: E731
    res = {
        "torch==native": same("torch_factors", "native_factors"),
        "shard==unsharded": same("native_factors", "native_factors_shard"),
        "torch shard==native shard": same("torch_factors_shard", "native_factors_shard"),
        "fallback==graphs": same("native_factors_shard_fallback", "native_factors_shard"),
        "allreduce shard~unsharded": float((out["torch_allreduce"]["p"] - out["torch_allreduce_shard"]["p"]).abs().max()),
        "graphs": {k: v["graphs"] for k, v in out.items()},
        "fallback": {k: v["fallback"] for k, v in out.items()},
        "rep": {k: v["rep"] for k, v in out.items()},
    }
    q.put(res)


@pytest.mark.gpu
def test_dp_step_variants_bit_identical():
    """Every DP-step variant takes the same updates at world 1 (see _dp_variants_worker);
    the sharded all-reduce exchange differs only in the clip norm's summation order.  The
    injected capture failure leaves that learner on the eager DP step (graph_fallback set,
    graphs off) with updates identical to the captured ones; the communicator reports one
    rank and the checked all-reduce of rank + 1 gives 1."""
    import random
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_dp_variants_worker, args=(q, 29600 + random.randint(301, 600)))
    p.start()
    res = _get_or_dead(q, p, 400)
    p.join(timeout=60)
    assert p.exitcode == 0
    for k in ("torch==native", "shard==unsharded", "torch shard==native shard", "fallback==graphs"):
        assert res[k] is True, (k, res)
    assert res["allreduce shard~unsharded"] < 1e-6, res
    for name, g in res["graphs"].items():
        # torch.distributed runs eager DP steps (fused_learner: _dp_graphs)
        assert g == (not name.endswith("fallback") and name.startswith("native")), (name, res)
        assert (res["fallback"][name] is not None) == name.endswith("fallback"), (name, res)
    for name, r in res["rep"].items():
        assert r["comm_world"] == 1 and r["init_allreduce_ok"], (name, r)


@pytest.mark.gpu
def test_emulated_world_step_runs_sharded():
    """bench.py --emulate-world: rank 0's share of an 8-rank global-batch step on one GPU
    (parallel/rccl.py EmulatedCollectives) -- 74-row buffers, the sharded fc update over
    rows [0, 128), captured graphs, finite updates, about 512 / 8 rows drawn per update."""
    import numpy as np
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.parallel.dist import EmulatedComm
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    dev = torch.device("cuda", 0)
    for dtype in ("fp32", "bf16"):
        cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                    "Learner": {"replay_sample_size": 512},
                                    "Runtime": {"use_graphs": True, "graph_steps": 5, "dtype": dtype}})
        rp = GpuReplayShard(8000, 8000, 8100, 4, device=dev, seed=1)
        rng = np.random.default_rng(2)
        seqs = rp.append_frames(rng.integers(0, 255, (7000, 84, 84), dtype=np.uint8))
        K = 6000
        st = np.stack([seqs[i:i + 4] for i in range(K)])
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 4, K), R=rng.normal(size=K).astype(np.float32),
                       Gamma=np.full(K, 0.97, np.float32), priority=rng.random(K).astype(np.float32) + 0.01))
        L = FusedNatureLearner(cfg, dev, rp, comm=EmulatedComm(8, 0, dev))
        assert L._dp and L.B == 74 and L._shard and L._fc_S == 128 and L.coll.name == "emulated"
        assert L.comm_report()["init_allreduce_ok"]
        L.prepare_graphs()         # (its warm replays count rows too: state-preserving otherwise)
        p0 = L.p32.clone()
        L.valid_rows_total.zero_()
        L.steps(10)
        torch.cuda.synchronize()
        assert L._graphs_enabled() and L.graph_captures >= 1
        assert torch.isfinite(L.p32).all() and not torch.equal(L.p32, p0)
        rows = int(L.valid_rows_total.item()) / 10
        assert 40 <= rows <= 74, rows
