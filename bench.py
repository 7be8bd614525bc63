#!/usr/bin/env python
"""Headline benchmark: learner grad-steps/sec at batch 512 on 84x84x4 frames,
dueling NatureCNN (BASELINE.json metric), on N MI355X of one node.

One process per GPU (torchrun env vars).  Each rank owns an HBM replay shard
prefilled with synthetic uint8 frames (no datasets on the box) and a
data-parallel learner replica.  By default (``--batch-scope global``) the N shards
form ONE prioritized replay: every update is one global draw of 512 samples and
each rank computes the rows that landed in its shard (strong scaling; see below).
A timed step is the complete learner update: prioritized sample + frame gather,
online fwd on [S_t;S_t+n] and target fwd on S_t+n, DDQN/Huber/IS loss +
priorities, full backward, the RCCL gradient exchange (N>1; sharded fc optimizer
+ parameter all-gather, learner/dp_step.py), clip + centered RMSprop, priority
write-back, plus the periodic target sync / FIFO eviction at their cadences.

Precision: ``--dtype fp32`` (default) matches the reference learner
(``learner.py:37-38`` computes in fp32): the hand-written kernels run split
hi/lo bf16 operands (three MFMAs per product, fp32 accumulation; see
learner/fused_learner.py).  The JSON's ``value`` is that fp32 number; unless
``--no-bf16-extra``, the same run also times the bf16-operand learner and reports
it as ``value_bf16``.

Timing: ``--warmup`` untimed updates, then every HIP graph the timed region
replays is captured (``learner.prepare_graphs``: state-preserving, no updates) and
replayed ``--prep-warm`` times from a snapshot that is then restored
(``learner.rewarm``: no update is kept; without it a 20-step window after a 5-step
warm-up read 1.5-2 % below a 400-step window, with it they agree within 0.5 %:
``scripts/warm_ab.sh``, ``profiles/r2_prep_warm_ab.txt``), then EXACTLY ``--steps``
updates between barrier + synchronize brackets; the max over ranks is reported.
``graph_captures_in_timed`` must be 0.

``value`` = whole-job batch-512 gradient steps per second.  One rank: steps/s.  With
data parallelism (``--batch-scope``):

* ``global`` (default; ``scaling: "strong"``): every update is ONE global prioritized
  draw of exactly 512 samples over the N replay shards -- the reference learner's update
  (``learner.py:68``, ``replay_sample_size``) -- and each rank computes the rows that
  landed in its shard (ceil(512/N (1 + slack)) + 2 row buffers, ``ApexConfig.dp_batch``).
  ``value`` = updates/s (``value_strong``); ``samples_per_dp_step`` is the mean global
  batch M actually drawn (512 unless a shard held more than its slack of the mass).
* ``per_rank`` (``scaling: "weak"``): every rank draws up to 512 rows, so an update
  averages up to N x 512 samples; ``value`` = (sum of M over the timed steps) / 512 /
  time (``value_weak``), ``value_nominal`` = N x (DP steps/s).

At N > 1 the run also measures the other scope (fp32) and prints both ``value_strong``
and ``value_weak`` with the rows each rank computed (``per_rank_rows``).

N > 1 diagnostics in the JSON: ``comm_world`` (the rank count the communicator itself
reports), ``init_allreduce_ok`` (a checked all-reduce of rank + 1 through the DP step's
collectives, = N (N + 1) / 2), ``dp_graphs`` (the DP step ran as captured HIP graphs;
``graph_fallback`` names why not).  Every phase runs under a watchdog
(``--phase-timeout``): a rank stuck in a collective exits non-zero naming its phase.

Before this process makes any HIP call, each rank at N > 1 captures and replays the DP
step in ONE child process (``runtime/capture_probe.py``: its own RCCL communicator and
rendezvous under a separate store prefix); a child that crashes, hangs or fails on any
rank sends every rank to the eager DP step for that measurement (``dp_capture_probe``:
exit status per rank, verdict per measurement, seconds).  After the timed region the
run checks itself: ``replicas_identical`` (checksums of every rank's fp32 master weights
and RMSprop state agree) and ``graph_matches_eager`` (one captured update equals the same
update run eagerly from the same snapshot, bit for bit, on every rank); ``param_sha256``
fingerprints the final fp32 weights.

``--emulate-world W`` (one GPU): rank 0's share of a W-rank global-batch step -- its
rows, its 1/W fc optimizer slice and fc weight-gradient rows, the sharded replay draw
-- with every collective a device copy of its true size (``parallel/rccl.py
EmulatedCollectives``).  ``value`` is then that per-rank step's rate, the W-GPU update
rate if RCCL's latency hides behind the compute; labelled ``emulated_world``.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
# HIP maps every stream to one of GPU_MAX_HW_QUEUES hardware queues (4 by default); the
# learner's two step streams, the data-parallel collective / fork streams and the actor
# groups' streams exceed four, and a stream that shares a queue runs behind that queue's
# other work (actor inference queued behind the learner's step graphs starved the actors:
# profiles/r4_e2e_actor_streams_ab.txt).  Read when HIP initialises, so set before it.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_STEPS_PER_S = 2.32  # BASELINE.md north-star row (reference learner compute, B=512, 4x84x84, fp32 CPU)
METRIC = "learner grad-steps/sec at batch 512, 84x84x4 dueling DQN"


def make_replay(args, device, rank):
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    cap = args.replay
    frames_cap = cap + 4096
    replay = GpuReplayShard(cap, cap, frames_cap, 4, alpha=0.6, beta=0.4, device=device, seed=rank + 1)
    # synthetic prefill: random frames straight into HBM + random n-step records
    g = torch.Generator(device=device).manual_seed(1000 + rank)
    replay.frames.copy_(torch.randint(0, 256, replay.frames.shape, generator=g, device=device, dtype=torch.uint8))
    replay.frame_head = frames_cap
    rng = np.random.default_rng(rank)
    chunk = 16384
    for s in range(0, cap, chunk):
        K = min(chunk, cap - s)
        base = rng.integers(0, frames_cap - 8, size=K)
        st = base[:, None] + np.arange(4)[None]
        nx = st + 3
        replay.insert(dict(S_t=st, S_tpn=nx, A_t=rng.integers(0, args.actions, K),
                           R=rng.normal(size=K).astype(np.float32), Gamma=np.full(K, 0.99 ** 3, np.float32),
                           priority=rng.random(K).astype(np.float32) + 0.01))
    replay.rebuild()
    return replay


def learner_config(args, dtype, rank, scope=None) -> dict:
    """The learner's config (ApexConfig dict) of one measurement."""
    return {
        "env_conf": {"state_shape": [4, 84, 84], "action_dim": args.actions, "name": "SyntheticPong"},
        "Learner": {"replay_sample_size": args.batch, "q_target_sync_freq": 2500, "remove_old_xp_freq": 100,
                    "min_replay_mem_size": 0},
        "Replay_Memory": {"soft_capacity": args.replay},
        "Runtime": {"use_graphs": not args.no_graphs, "use_hip_kernels": args.backend == "hip",
                    "seed": 1234 + rank, "network": args.network, "dtype": dtype,
                    "presample": not args.no_presample, "force_dp": args.force_dp, "comm_backend": args.comm,
                    "batch_scope": scope or args.batch_scope, "allreduce_dtype": args.allreduce_dtype,
                    "dp_fc_exchange": args.dp_fc_exchange, "dp_shard_update": args.dp_shard_update,
                    **({} if args.graph_steps is None else {"graph_steps": args.graph_steps})},
    }


def measurements(args, world: int):
    """(name, dtype, batch scope) of every learner this run builds, in order."""
    dp = world > 1 or args.force_dp
    scope = args.batch_scope if dp else "global"
    out = [("headline", args.dtype, scope)]
    if world > 1 and not args.no_scope_extra:
        out.append(("other_scope", args.dtype, "per_rank" if scope == "global" else "global"))
    if not args.no_bf16_extra and args.dtype == "fp32":
        out.append(("bf16", "bf16", scope))
    return out


def capture_probe(args, world: int, rank: int, local_rank: int):
    """The DP step's graph capture tried first in a child process per rank
    (runtime/capture_probe.py), before this process makes any HIP call: a native crash
    in capture (or a hang in RCCL's first captured collectives) costs the child, and the
    variants that failed on any rank run the eager DP step here.  Returns the report
    for the JSON (``dp_capture_probe``), or None when not applicable."""
    mode = args.capture_probe
    nature = args.network in ("nature64", "nature32") and args.learner == "fused" and args.backend == "hip"
    graphs = not args.no_graphs and args.comm == "native" and args.dist_backend == "nccl"
    if mode == "off" or args.emulate_world or not (nature and graphs):
        return None
    if not (world > 1 or (args.force_dp and mode == "on")):
        return None
    from apex_dqn_amd.config import RuntimeConf
    from apex_dqn_amd.runtime.capture_probe import run_probe
    variants = [{"name": n, "cfg": learner_config(args, dt, rank, sc), "steps": args.graph_steps or RuntimeConf.graph_steps}
                for (n, dt, sc) in measurements(args, world)]
    log = open(os.path.join(args.capture_probe_log, f"capture_probe_rank{rank}.log"), "wb") \
        if args.capture_probe_log else None
    try:
        return run_probe(variants, rank, world, local_rank, timeout=args.capture_probe_timeout, log=log)
    finally:
        if log is not None:
            log.close()


def make_learner(args, dtype, device, comm, rank, replay, scope=None, probe=None, name=None):
    from apex_dqn_amd.config import ApexConfig
    cfg = ApexConfig.from_dict(learner_config(args, dtype, rank, scope))
    torch.manual_seed(cfg.Runtime.seed)       # random-init weights: reproducible runs (DP: rank 0's broadcast)
    if args.learner == "graph" or (args.network == "impala" and args.graph_impala):
        from apex_dqn_amd.learner.graph_learner import GraphLearner
        return cfg, GraphLearner(cfg, device, replay, comm=comm)
    if args.network in ("nature64", "nature32"):
        from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
        L = FusedNatureLearner(cfg, device, replay, comm=comm, backend=args.backend)
        if probe is not None and not probe["ok"].get(name, False):
            # the out-of-process capture failed on some rank: eager DP step on every rank
            L.graph_fallback = "capture probe: child exit status per rank %s, captures %s" % (probe["rc"], probe["ok"])
        return cfg, L
    from apex_dqn_amd.learner.impala_learner import FusedImpalaLearner
    return cfg, FusedImpalaLearner(cfg, device, replay, comm=comm, backend=args.backend)


def measure(cfg, learner, replay, comm, warmup: int, steps: int, prep_warm: int = 0, wd=None,
            timeout: float = 0.0, tag: str = "") -> dict:
    L = cfg.Learner
    from contextlib import nullcontext

    def phase(name):
        return wd.phase(tag + name, timeout) if wd is not None else nullcontext()

    def run(n):
        """n learner updates; the FIFO eviction + tree rebuild at its cadence runs
        between graph launches (learners with ``steps`` replay multi-step graphs)."""
        f = L.remove_old_xp_freq
        while n > 0:
            k = min(n, f - learner.num_q_updates % f)
            if hasattr(learner, "steps"):
                learner.steps(k)
            else:
                for _ in range(k):
                    learner.step()
            n -= k
            if learner.num_q_updates % f == 0:
                replay.remove_to_fit()
                replay.rebuild()
                if hasattr(learner, "refresh_replay_stats"):
                    learner.refresh_replay_stats()

    with phase("warmup"):
        run(warmup)
        torch.cuda.synchronize()
    # every graph the timed region replays, captured now (no learner updates)
    with phase("graph capture"):
        caps = learner.prepare_graphs() if hasattr(learner, "prepare_graphs") else 0
        if hasattr(learner, "rewarm"):
            learner.rewarm(prep_warm)     # state-preserving: no update is kept
        torch.cuda.synchronize()
    vr = getattr(learner, "valid_rows_total", None)
    if vr is not None:
        vr.zero_()                    # DP: rows each rank actually drew, counted by the head kernel
    with phase("barrier before the timed steps"):
        torch.cuda.synchronize()
        comm.barrier()
        torch.cuda.synchronize()
    with phase("timed steps"):
        t0 = time.perf_counter()
        run(steps)
        torch.cuda.synchronize()
        comm.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    dt = comm.allreduce_scalar(dt, "max") if comm.active else dt
    caps_after = getattr(learner, "graph_captures", 0)
    dp = bool(getattr(learner, "_dp", False)) and vr is not None
    valid = float(vr.item()) if dp else None
    if dp and comm.active:
        valid = comm.allreduce_scalar(valid, "sum")
    return dict(dt=dt, prep_graph_captures=int(caps), graph_captures_in_timed=int(caps_after - caps),
                valid_rows=valid,
                prep_warm_replays=int(prep_warm) if hasattr(learner, "rewarm") else 0,
                metrics=learner.last_metrics())


def main():
    # diagnostics: APEX_TRACEBACK_AFTER=<s> dumps every thread's stack to stderr after s
    # seconds (a hung multi-rank run names its blocking call instead of going silent)
    if os.environ.get("APEX_TRACEBACK_AFTER"):
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["APEX_TRACEBACK_AFTER"]), repeat=True)
    args = parser().parse_args()
    global _RESULT_OUT
    _RESULT_OUT = _claim_stdout()
    run(args)


_RESULT_OUT = sys.stdout


def _claim_stdout():
    """The driver reads ONE JSON line from stdout, but libraries print there too (RCCL
    writes its version banner to stdout when a communicator initialises): point fd 1 at
    stderr for the whole run (child processes inherit that) and keep a private handle on
    the real stdout for the result line."""
    sys.stdout.flush()
    fd = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(fd, "w")


def parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--actions", type=int, default=4)
    ap.add_argument("--replay", type=int, default=100000, help="transitions per shard")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="learner precision of the headline value (fp32 = the reference's)")
    ap.add_argument("--no-bf16-extra", action="store_true",
                    help="skip the extra bf16-operand measurement (value_bf16)")
    ap.add_argument("--learner", default="fused", choices=["fused", "graph"],
                    help="fused = hand-written HIP learner; graph = torch autograd on MIOpen / hipBLASLt "
                         "(the vendor-library baseline)")
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-presample", action="store_true",
                    help="sample at the head of each step instead of inside the previous step's optimizer launch")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 collectives: nccl (= RCCL over xGMI) or gloo (rehearsing several ranks on one GPU)")
    ap.add_argument("--comm", default="native", choices=["torch", "native"],
                    help="DP collectives: the native RCCL communicator (csrc/comm/rccl_comm.cpp; captured "
                         "graphs) or torch.distributed (RCCL process group; eager DP steps)")
    ap.add_argument("--batch-scope", default="global", choices=["global", "per_rank"],
                    help="DP: global = one 512-sample update over all ranks (strong scaling, the reference's "
                         "update); per_rank = 512 rows per rank (weak scaling)")
    ap.add_argument("--no-scope-extra", action="store_true",
                    help="N > 1: skip measuring the other --batch-scope (value_weak / value_strong)")
    ap.add_argument("--dp-fc-exchange", default="auto", choices=["auto", "factors", "allreduce"],
                    help="DP exchange of the fc gradient (Runtime.dp_fc_exchange)")
    ap.add_argument("--allreduce-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="DP gradient all-reduce payload (Runtime.allreduce_dtype)")
    ap.add_argument("--force-dp", action="store_true",
                    help="run the data-parallel step (RCCL collectives captured in the graphs, sharded "
                         "replay) even on one rank: capture check and segmented-step overhead")
    ap.add_argument("--graph-steps", type=int, default=None,
                    help="learner updates per HIP-graph launch (Runtime.graph_steps; 1 = one graph per update)")
    ap.add_argument("--graph-impala", action="store_true",
                    help="IMPALA on the torch-autograd graph learner (MIOpen) instead of the HIP kernels")
    ap.add_argument("--prep-warm", type=int, default=4,
                    help="untimed, state-preserving replays of the multi-step graph right before the timed "
                         "window (learner.rewarm: no update is kept; reported as prep_warm_replays)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="one GPU: run rank 0's share of a W-rank global-batch DP step, collectives as device "
                         "copies of their true sizes (reported as emulated_world)")
    ap.add_argument("--dp-shard-update", default="auto", choices=["auto", "on", "off"],
                    help="DP: shard the fc optimizer by output rows (Runtime.dp_shard_update)")
    ap.add_argument("--phase-timeout", type=float, default=600.0,
                    help="watchdog: seconds any bench phase may take before the rank exits non-zero")
    ap.add_argument("--capture-probe", default="auto", choices=["auto", "on", "off"],
                    help="DP graphs: capture + replay the DP step first in one child process per rank, before "
                         "this process touches the GPU (auto: at world > 1; on: also --force-dp at world 1)")
    ap.add_argument("--capture-probe-timeout", type=float, default=150.0,
                    help="seconds the capture probe's child may take")
    ap.add_argument("--capture-probe-log", default=None,
                    help="directory for the probe children's output (capture_probe_rank<r>.log)")
    ap.add_argument("--network", default="nature64", choices=["nature64", "nature32", "impala"],
                    help="nature64 = the headline fused-HIP learner; nature32 runs on it zero-padded; impala on csrc/impala_split.hip (fp32) / csrc/impala.hip (bf16)")
    return ap


def run(args) -> None:

    from apex_dqn_amd.ops.switches import SW
    from apex_dqn_amd.parallel.dist import Comm, EmulatedComm
    from apex_dqn_amd.runtime.watchdog import PhaseWatchdog

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    emu = int(args.emulate_world)
    if emu and world > 1:
        raise SystemExit("--emulate-world runs on one process")
    wd = PhaseWatchdog(rank)
    to = float(args.phase_timeout)
    if args.force_dp and world == 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
    # before ANY HIP call of this process (torch.cuda.is_available() initialises HIP)
    with wd.phase("capture probe", args.capture_probe_timeout + 60.0):
        probe = capture_probe(args, world, rank, local_rank)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a GPU")
    # one rank per GPU; the modulo only matters when rehearsing several ranks on
    # fewer GPUs (device_count() does not initialise the GPU)
    dev_idx = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev_idx)
    device = torch.device("cuda", dev_idx)
    with wd.phase("process group init", to):
        if emu:
            comm = EmulatedComm(emu, 0, device)
            args.force_dp = True
        else:
            comm = Comm.from_env(backend=args.dist_backend, device=device, force=args.force_dp)
    wd.comm = comm
    with wd.phase("replay prefill", to):
        replay = make_replay(args, device, rank)
    dp = world > 1 or args.force_dp
    scope = args.batch_scope if dp else "global"

    def value_of(r, sc):
        """whole-job batch-512 grad-steps/s of a measurement at scope ``sc``: updates/s
        (global: every update is one 512-sample draw over all shards), or the drawn
        samples in units of 512 per second (per_rank: an update averages M <= N 512)."""
        if r["valid_rows"] is None:
            return args.steps / r["dt"] * world
        if sc == "global":
            return args.steps / r["dt"]
        return r["valid_rows"] / args.batch / r["dt"]

    with wd.phase("learner init (comm init, parameter broadcast)", to):
        cfg, learner = make_learner(args, args.dtype, device, comm, rank, replay, scope, probe, "headline")
    rows = learner.B
    diag = {}
    if dp and hasattr(learner, "comm_report"):
        with wd.phase("checked init all-reduce", to):
            diag = learner.comm_report()
    res = measure(cfg, learner, replay, comm, args.warmup, args.steps, args.prep_warm, wd, to)
    dp_graphs = bool(getattr(learner, "_dp", False)) and learner._graphs_enabled() if dp else None
    fallback = getattr(learner, "graph_fallback", None)
    shard = bool(getattr(learner, "_shard", False))
    if dp:
        # after the timed region: did the replicas stay bit-identical, and does the
        # captured update equal the eager one from the same state (both collectives)
        diag["dp_capture_probe"] = probe if probe is not None else "not run (%s)" % (
            "emulated world" if emu else "eager DP step" if not dp_graphs else "off" if args.capture_probe == "off"
            else "world 1")
        with wd.phase("replica check", to):
            diag["replicas_identical"] = bool(learner.check_replicas()) if hasattr(learner, "check_replicas") \
                else None
        with wd.phase("graph vs eager check", to):
            diag["graph_matches_eager"] = learner.graph_matches_eager() \
                if hasattr(learner, "graph_matches_eager") else None
    if hasattr(learner, "p32") and not emu:
        if hasattr(learner, "materialize"):
            learner.materialize()      # (sharded update: every rank's fc rows; a collective)
        import hashlib
        diag["param_sha256"] = hashlib.sha256(learner.p32.detach().cpu().numpy().tobytes()).hexdigest()[:16]
    other = None
    if world > 1 and not args.no_scope_extra:
        # the other batch scope, fp32: both scalings from one run
        osc = "per_rank" if scope == "global" else "global"
        del learner
        torch.cuda.empty_cache()
        cfg_o, learner_o = make_learner(args, args.dtype, device, comm, rank, replay, osc, probe, "other_scope")
        other = dict(measure(cfg_o, learner_o, replay, comm, args.warmup, args.steps, args.prep_warm, wd, to,
                             "other scope: "),
                     scope=osc, rows=learner_o.B)
        learner = learner_o
    extra = None
    if not args.no_bf16_extra and args.dtype == "fp32":
        del learner
        torch.cuda.empty_cache()
        cfg_b, learner_b = make_learner(args, "bf16", device, comm, rank, replay, scope, probe, "bf16")
        extra = measure(cfg_b, learner_b, replay, comm, args.warmup, args.steps, args.prep_warm, wd, to, "bf16: ")
        learner = learner_b
    dt = res["dt"]
    ms = 1e3 * dt / args.steps
    value = value_of(res, scope)
    # DP: a step's global batch is M = the rows the W ranks drew from their shards
    # (global scope: 512 unless a shard outgrew its slack; per_rank: <= W (B - 2))
    samples_per_step = res["valid_rows"] / args.steps if res["valid_rows"] is not None else None
    m = res["metrics"]
    if rank == 0:
        kind = getattr(learner, "kind", "fused")
        ops = getattr(learner, "ops", None)
        out = {
            "metric": METRIC,
            "value": round(value, 2), "unit": "grad-steps/s (batch 512)", "n_gpus": 1 if emu else world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 4),
            "higher_is_better": True, "scaling": "strong" if scope == "global" else "weak",
            "vs_baseline": round(value / BASELINE_STEPS_PER_S, 2), "dtype": args.dtype, "data": "synthetic",
            "config": {"model": ("dueling NatureCNN (reference DuellingDQN, conv1=64), 4x84x84, A=%d" % args.actions
                                  if args.network == "nature64" else
                                  "dueling %s, 4x84x84, A=%d" % (args.network, args.actions)),
                       "global_batch": args.batch * (world if scope == "per_rank" else 1), "seq_len": 1,
                       "parallelism": ("dp%d-emulated-rank0" % emu) if emu else
                       ("dp%d" % world + ("-dp-step" if args.force_dp and world == 1 else "")),
                       "batch_scope": scope,
                       "per_gpu_batch": args.batch if scope == "per_rank" else round(args.batch / (emu or world), 2),
                       "per_rank_rows": rows,
                       "allreduce_dtype": args.allreduce_dtype if dp else None,
                       "dp_fc_exchange": ("factors" if getattr(learner, "_fc_factors", False) else "allreduce")
                       if dp else None,
                       "replay_per_gpu": args.replay,
                       "learner": kind + ("/" + ops.name if ops is not None and args.learner == "fused" else
                                          "/torch-autograd"),
                       "dp_collectives": getattr(getattr(learner, "coll", None), "name", None)
                       if (world > 1 or args.force_dp) else None,
                       "dp_shard_update": shard if dp else None,
                       "hip_graphs": not args.no_graphs},
            "math": ("fp32 master weights, gradients and optimizer; GEMM operands as bf16 hi + lo "
                     "(hi*hi + lo*hi + hi*lo MFMAs, fp32 accumulation)" if args.dtype == "fp32"
                     and args.learner == "fused" else
                     ("torch fp32 (MIOpen / hipBLASLt)" if args.learner == "graph" and args.dtype == "fp32" else
                      "bf16 operands, fp32 accumulation / master weights / optimizer")),
            "switches": SW.non_default(),      # kernel-path switches off their defaults (ops/switches.py)
            "prep_graph_captures": res["prep_graph_captures"],
            "graph_captures_in_timed": res["graph_captures_in_timed"],
            "prep_warm_replays": res["prep_warm_replays"],
            "loss": round(m["loss"], 5), "grad_norm": round(m["grad_norm"], 5),
            "is_weight_mean": round(m.get("is_weight_mean", float("nan")), 5),
        }
        if dp:
            out["dp_graphs"] = dp_graphs
            out["graph_fallback"] = fallback
        out.update(diag)
        if emu:
            out["emulated_world"] = emu
            out["emulation"] = ("rank 0 of a %d-rank global-batch step on one GPU; collectives are device copies "
                                "of their true sizes (RCCL latency / xGMI time not included)" % emu)
        if samples_per_step is not None and emu:
            out["rank0_rows_drawn_per_step"] = round(samples_per_step, 2)
        elif samples_per_step is not None:
            out["samples_per_dp_step"] = round(samples_per_step, 2)
            out["value_nominal"] = round(args.steps / dt * world, 2)
            out["value_" + ("strong" if scope == "global" else "weak")] = round(value, 2)
        if other is not None:
            k = "strong" if other["scope"] == "global" else "weak"
            out["value_" + k] = round(value_of(other, other["scope"]), 2)
            out["ms_per_step_" + k] = round(1e3 * other["dt"] / args.steps, 4)
            out["samples_per_dp_step_" + k] = round(other["valid_rows"] / args.steps, 2)
            out["per_rank_rows_" + k] = other["rows"]
            out["graph_captures_in_timed_" + k] = other["graph_captures_in_timed"]
        if extra is not None:
            out["value_bf16"] = round(value_of(extra, scope), 2)
            out["ms_per_step_bf16"] = round(1e3 * extra["dt"] / args.steps, 4)
            out["graph_captures_in_timed_bf16"] = extra["graph_captures_in_timed"]
        print(json.dumps(out), file=_RESULT_OUT, flush=True)
    with wd.phase("shutdown", to):
        comm.shutdown()
    wd.close()


if __name__ == "__main__":
    main()
