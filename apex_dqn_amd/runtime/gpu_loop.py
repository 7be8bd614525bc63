"""Per-rank Ape-X loop for image configs: actor group + HBM replay shard +
fused learner on one device (GPU rank, or CPU for tests with the torch backend).

One process per GPU; with torchrun the ranks form a data-parallel learner
over RCCL and each owns a replay shard fed by its own actor group.
Reference parity: ``main.py:28-61`` (launch) + ``Learner.learn``
(``learner.py:63-80``): wait for ``min_replay_mem_size``, then sample /
update / priority write-back every step, ``remove_to_fit`` every
``remove_old_xp_freq`` steps; plus what the reference lacks -- periodic
checkpoints, JSONL metrics, synchronized start across ranks.
"""
from __future__ import annotations

import collections
import contextlib
import os
import sys
import time
from typing import Any, Deque, Dict, Optional

import numpy as np
import torch

from ..actors.gpu_actor import make_gpu_actor_group
from ..config import ApexConfig
from ..learner.fused_learner import FusedNatureLearner
from ..replay.gpu_replay import GpuReplayShard
from ..utils.metrics import MetricsLogger


FILL_CHECK_EVERY = 16      # fill phase: group steps between readiness all-reduces (DP)
WATCHDOG_EXIT_CODE = 75    # a multi-rank watchdog timeout exits the process with this code


def _chunk_cap(graph_steps: int) -> int:
    """Learner updates per loop chunk with an actor thread: whole multi-update graphs,
    about 20 updates (two chunks in flight bound how long an actor insert waits behind
    the learner)."""
    g = max(1, graph_steps)
    return g * max(1, 20 // g)


def build_replay(cfg: ApexConfig, device, num_envs: int, seed: int = 0, world: int = 1) -> GpuReplayShard:
    """This rank's shard of the global replay: ``soft_capacity / world`` transitions
    (the learners turn the shards into one prioritized replay, replay/gpu_replay.py)."""
    rm = cfg.Replay_Memory
    soft, cap = cfg.shard_capacity(world)
    n, C = cfg.Actor.num_steps, cfg.frame_stack
    frame_cap = int(cap * 1.25) + (n + C + 4) * num_envs + 64
    return GpuReplayShard(cap, soft, frame_cap, C, alpha=rm.priority_exponent,
                          beta=rm.importance_sampling_exponent, eps=cfg.Runtime.priority_eps, device=device,
                          seed=seed)


def _start_torch_profiler(device):
    """torch.profiler with CPU + GPU (roctracer on ROCm) activities."""
    acts = [torch.profiler.ProfilerActivity.CPU]
    if device.type == "cuda":
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    p = torch.profiler.profile(activities=acts, record_shapes=False)
    p.start()
    return p


def train_frames(cfg: ApexConfig, device, learner_steps: int, comm=None,
                 metrics: Optional[MetricsLogger] = None, num_envs: Optional[int] = None,
                 actor_steps_per_update: int = 1, max_actor_steps: Optional[int] = None,
                 backend: Optional[str] = None, async_actors: Optional[bool] = None) -> Dict[str, Any]:
    """See :func:`_train_frames`.  With asynchronous actors on a GPU the learner (and
    the compute stream the actors' inserts ride on) runs on a HIGH-priority HIP stream:
    the actor thread's inference kernels (its own, default-priority stream) fill the gaps
    between learner kernels instead of delaying them (Runtime.learner_stream_priority)."""
    device = torch.device(device)
    if async_actors is None:
        async_actors = bool(cfg.Runtime.async_actors) and device.type == "cuda"
    if not (async_actors and device.type == "cuda" and cfg.Runtime.learner_stream_priority):
        return _train_frames(cfg, device, learner_steps, comm, metrics, num_envs, actor_steps_per_update,
                             max_actor_steps, backend, async_actors)
    prev = torch.cuda.current_stream(device)
    hi = torch.cuda.Stream(device, priority=torch.cuda.Stream.priority_range()[1])
    hi.wait_stream(prev)
    torch.cuda.set_stream(hi)
    try:
        return _train_frames(cfg, device, learner_steps, comm, metrics, num_envs, actor_steps_per_update,
                             max_actor_steps, backend, async_actors)
    finally:
        prev.wait_stream(hi)
        torch.cuda.set_stream(prev)


def _train_frames(cfg: ApexConfig, device, learner_steps: int, comm=None,
                  metrics: Optional[MetricsLogger] = None, num_envs: Optional[int] = None,
                  actor_steps_per_update: int = 1, max_actor_steps: Optional[int] = None,
                  backend: Optional[str] = None, async_actors: Optional[bool] = None) -> Dict[str, Any]:
    """Train for ``learner_steps`` updates.  Actors stop after ``max_actor_steps``
    group steps (default ``Actor.T``: every env takes T steps, ``actor.py:159``); the
    learner keeps going on the replay, as the reference's learner process does.

    ``async_actors`` (default ``Runtime.async_actors``): the actor group steps on its
    own host thread (runtime/actor_thread.py) once the replay holds
    ``min_replay_mem_size``; otherwise actor and learner alternate
    (``actor_steps_per_update`` group steps per update; deterministic, for tests)."""
    device = torch.device(device)
    rank = comm.rank if comm is not None else 0
    world = comm.world_size if comm is not None else 1
    rt, L = cfg.Runtime, cfg.Learner
    E = num_envs or cfg.Runtime.actors_per_rank or max(1, cfg.Actor.num_actors // world)
    torch.manual_seed(rt.seed)
    replay = build_replay(cfg, device, E, seed=rt.seed + rank, world=world)
    if cfg.network in ("nature64", "nature32") and (cfg.Runtime.use_hip_kernels or device.type != "cuda"):
        learner = FusedNatureLearner(cfg, device, replay, comm=comm, backend=backend)
    elif cfg.network == "impala" and cfg.Runtime.use_hip_kernels:
        # hand-written IMPALA learner: csrc/impala_split.hip (Runtime.dtype fp32: split
        # hi / lo operands) or csrc/impala.hip (bf16 operands), fp32 accumulation / master weights
        from ..learner.impala_learner import FusedImpalaLearner
        learner = FusedImpalaLearner(cfg, device, replay, comm=comm, backend=backend)
    else:
        # graph-captured torch-autograd learner on the same HBM replay (use_hip_kernels off)
        from ..learner.graph_learner import GraphLearner
        learner = GraphLearner(cfg, device, replay, comm=comm)
    ckpt_path = os.path.join(rt.ckpt_dir, "checkpoint.pt") if rt.ckpt_dir else None
    # restart after a learner-rank failure (torchrun --max-restarts / run_elastic):
    # every rank resumes the same checkpoint, so the DP replicas stay identical.
    # Loaded before the actor group is built: its parameter slot copies the learner's.
    if ckpt_path and rt.resume and os.path.exists(ckpt_path):
        learner.load(ckpt_path)
        if metrics is not None:
            metrics.log("resume", step=learner.num_q_updates, path=ckpt_path)
    if async_actors is None:
        async_actors = bool(rt.async_actors) and device.type == "cuda"
    # async actors: the envs as Runtime.actor_pipeline groups stepped in turn (the host's env
    # work of one group hides another's inference); the lock-step loop keeps one group
    if async_actors and int(rt.actor_pipeline) > 2 and device.type == "cuda":
        # measured on MI355X: 4 groups starve (each group's finish waits ~1.2 ms for its
        # inference, 10-17k env frames/s, profiles/r4_diag_e2e_actor_pipeline4_starved.txt) --
        # the groups' streams likely share the process's few hardware queues
        # (GPU_MAX_HW_QUEUES) with the learner's step graphs
        sys.stderr.write(f"warning: Runtime.actor_pipeline={rt.actor_pipeline} > 2 measured far slower on "
                         f"MI355X (actor streams share hardware queues with the learner); 2 is the default\n")
    group = make_gpu_actor_group(cfg, learner, replay, E, rank, world, seed=rt.seed,
                                 pipeline=int(rt.actor_pipeline) if async_actors else 1)
    if ckpt_path and rt.resume and os.path.exists(ckpt_path):
        _restore_actor_rng(group, ckpt_path)
    min_local = max(L.min_replay_mem_size // world, L.replay_sample_size)
    max_actor_steps = int(max_actor_steps if max_actor_steps is not None else cfg.Actor.T)
    t0 = time.time()
    st = _LoopState(t0, learner.num_q_updates)
    # ---- fill: the actors alone until every shard holds min_replay_mem_size / world.
    # With several ranks readiness is agreed on every FILL_CHECK_EVERY group steps (a
    # host-blocking all-reduce per step would serialise the fill); every rank steps its
    # group once per iteration, so all ranks reach the checks together.
    it = 0
    while True:
        if st.actor_steps < max_actor_steps:
            group.step()
            st.actor_steps += 1
        it += 1
        ready = float(replay.size() > min_local or st.actor_steps >= max_actor_steps)
        if comm is not None and comm.active:
            if it % FILL_CHECK_EVERY:
                continue
            ready = comm.allreduce_scalar(ready, "min")
        if ready >= 1.0:
            break
    learner.refresh_replay_stats()
    # multi-rank: host calls that can block on peers (graph warm-up / first replays with
    # their collectives, learner chunks) run under a deadline that aborts the
    # communicators and exits non-zero naming the phase (learner/fused_learner.py
    # prepare_graphs: those phases are not recoverable in process)
    wd = None
    if world > 1 and device.type == "cuda":
        from .watchdog import PhaseWatchdog
        wd = PhaseWatchdog(rank, comm)

    def guard(name):
        return wd.phase(name, rt.step_timeout) if wd is not None else contextlib.nullcontext()

    runner = None
    if async_actors:
        from .actor_thread import ActorRunner
        # every graph the loop replays is captured before the actor thread starts
        # launching work (a capture must not see other threads' launches)
        if hasattr(learner, "prepare_graphs"):
            with guard("graph capture"):
                learner.prepare_graphs()
        runner = ActorRunner(group, max_actor_steps - st.actor_steps, timeout=rt.heartbeat_timeout,
                             on_event=(lambda kind, **kw: metrics.log(kind, **kw)) if metrics is not None else None)
        st.actor_base = st.actor_steps
        st.runner = runner
        old_switch = sys.getswitchinterval()
        sys.setswitchinterval(5e-4)      # the learner thread only needs the GIL briefly per chunk
        runner.start()
    prof = None
    inflight: Deque = collections.deque()
    on_cuda = device.type == "cuda"
    try:
        while learner.num_q_updates < learner_steps:
            n = learner.num_q_updates
            if runner is not None:
                runner.check()
                st.actor_steps = st.actor_base + runner.steps
                # chunk: up to the next eviction / log / checkpoint / profiler boundary
                k = min(learner_steps - n, _to_boundary(n, L.remove_old_xp_freq),
                        _to_boundary(n, rt.log_every) if rt.log_every else learner_steps,
                        _to_boundary(n, rt.ckpt_freq) if (ckpt_path and rt.ckpt_freq) else learner_steps,
                        _to_boundary(n, rt.replica_check_every) if (world > 1 and rt.replica_check_every)
                        else learner_steps,
                        _chunk_cap(int(getattr(rt, "graph_steps", 1) or 1)))
                if rt.torch_profile_dir and prof is None and n < rt.torch_profile_start:
                    k = min(k, rt.torch_profile_start - n)
            else:
                for _ in range(actor_steps_per_update):
                    if st.actor_steps < max_actor_steps:
                        group.step()
                        st.actor_steps += 1
                k = 1
            if rt.torch_profile_dir and learner.num_q_updates == rt.torch_profile_start and prof is None:
                prof = _start_torch_profiler(device)
            if runner is not None and not on_cuda:
                with replay.lock:       # CPU tensors: no stream ordering between the threads
                    _learn(learner, k)
            else:
                with guard("learner chunk"):
                    _learn(learner, k)
            if on_cuda:
                # at most two chunks queued (the actor's inserts never wait long behind
                # them); the wait is the step watchdog in both actor modes
                ev = torch.cuda.Event()
                ev.record()
                inflight.append(ev)
                while len(inflight) > 2:
                    _wait_event(inflight.popleft(), rt.step_timeout, comm)
            n = learner.num_q_updates
            if prof is not None and n >= rt.torch_profile_start + rt.torch_profile_steps:
                prof.stop()
                os.makedirs(rt.torch_profile_dir, exist_ok=True)
                prof.export_chrome_trace(os.path.join(rt.torch_profile_dir, f"trace_rank{rank}.json"))
                prof, rt.torch_profile_dir = None, None
            if world > 1 and rt.replica_check_every and n % rt.replica_check_every == 0 and \
                    hasattr(learner, "check_replicas") and not learner.check_replicas() and metrics is not None:
                metrics.log("replica_divergence", step=n, action="re-broadcast from rank 0")
            if n % L.remove_old_xp_freq == 0:
                replay.remove_to_fit()
                replay.rebuild()
                if learner.refresh_replay_stats():
                    # the per-rank rows grew (DP global batch): the step graphs were
                    # dropped.  Recapture them now with the actor thread quiesced -- a
                    # capture must not see another thread's launches -- on every rank
                    # (the same gathered statistics: every rank grew alike)
                    if runner is not None:
                        runner.pause()
                    if hasattr(learner, "prepare_graphs"):
                        with guard("graph recapture after a row resize"):
                            learner.prepare_graphs()
                    if runner is not None:
                        runner.resume()
                    if metrics is not None:
                        metrics.log("rows_resized", step=n, rows=int(learner.B))
            if rt.log_every and n % rt.log_every == 0:
                if runner is not None:
                    st.actor_steps = st.actor_base + runner.steps
                _log(metrics, learner, group, replay, st, rt, world, device)
            if ckpt_path and rt.ckpt_freq and n % rt.ckpt_freq == 0:
                if hasattr(learner, "materialize"):
                    learner.materialize()      # sharded DP update: a collective, every rank
                if rank == 0:
                    learner.save(ckpt_path, extra=_actor_rng(group))
    finally:
        if runner is not None:
            runner.stop()
            st.actor_steps = st.actor_base + runner.steps
            sys.setswitchinterval(old_switch)
        if wd is not None:
            wd.close()
    if on_cuda:
        torch.cuda.synchronize(device)
    rets = [r for (_, _, r) in group.episodes]
    return {"learner": learner, "replay": replay, "actors": group, "losses": st.losses,
            "episodes": group.episodes, "actor_steps": st.actor_steps,
            "actor_restarts": runner.restarts if runner is not None else 0,
            "mean_return_last": float(np.mean(rets[-20:])) if rets else float("nan"),
            "wall_s": time.time() - t0}


class _LoopState:
    def __init__(self, t0: float, n0: int):
        self.t0 = t0
        self.actor_steps = 0
        self.actor_base = 0
        self.runner = None
        self.losses = []
        self.n_ep_seen = 0
        self.t_last, self.n_last, self.ins_last, self.steps_last = t0, n0, 0, 0


def _rng_groups(group) -> list:
    """The actor groups whose device RNG counters drive the epsilon-greedy draws (every
    group of a pipelined actor, ``Runtime.actor_pipeline``)."""
    gs = getattr(group, "groups", None) or [group]
    return [g for g in gs if getattr(g, "ctr", None) is not None]


def _actor_rng(group) -> Dict[str, Any]:
    """Every actor group's device RNG counter for the checkpoint (``ctrs``, one per
    pipelined group; ``ctr`` = group 0's, the older single-counter format)."""
    ctrs = [int(g.ctr.item()) for g in _rng_groups(group)]
    return {"actor_rng": {"ctr": ctrs[0], "ctrs": ctrs}} if ctrs else {}


def _restore_actor_rng(group, path: str) -> None:
    """Restore every group's counter (a checkpoint with one counter restores group 0's
    and leaves the others at their fresh state)."""
    from ..utils.checkpoint import load_checkpoint
    ck = load_checkpoint(path) or {}
    a = ck.get("actor_rng")
    if not isinstance(a, dict):
        return
    gs = _rng_groups(group)
    ctrs = a.get("ctrs") or [a["ctr"]]
    for g, c in zip(gs, ctrs):
        g.ctr.fill_(int(c))


def _wait_event(ev, timeout: float, comm=None) -> None:
    """Wait for a queued learner chunk, at most ``timeout`` seconds (watchdog: a hung
    kernel or collective fails the rank -- the communicators are aborted first -- so
    torchrun's elastic restart resumes the group from the last checkpoint).  With
    several ranks the process exits at once (``os._exit``): a rank blocked in a hung
    collective would otherwise hang again in the teardown."""
    deadline = time.time() + float(timeout)
    while not ev.query():
        if time.time() > deadline:
            msg = f"learner step watchdog: queued GPU work did not finish in {timeout:.0f} s"
            if comm is not None and hasattr(comm, "abort"):
                comm.abort()
            if comm is not None and getattr(comm, "active", False):
                sys.stderr.write(f"[rank {comm.rank}] {msg}; exiting for an elastic restart\n")
                sys.stderr.flush()
                os._exit(WATCHDOG_EXIT_CODE)
            raise RuntimeError(msg)
        time.sleep(2e-4)


def _to_boundary(n: int, every: int) -> int:
    return every - n % every if every and every > 0 else 1 << 62


def _learn(learner, k: int) -> None:
    if k > 1 and hasattr(learner, "steps"):
        learner.steps(k)
    else:
        for _ in range(k):
            learner.step()


def _log(metrics, learner, group, replay, st: "_LoopState", rt, world: int, device) -> None:
    m = learner.last_metrics()
    st.losses.append(m["loss"])
    if metrics is None:
        return
    n = learner.num_q_updates
    now = time.time()
    dt = max(now - st.t_last, 1e-9)
    eps_ = group.eps.float()
    eps_list = list(group.episodes)
    new_eps = eps_list[st.n_ep_seen:]
    rets = [r for (_, _, r) in eps_list[-50:]]
    lens = [ln for (_, ln, _) in eps_list[-50:]]
    metrics.log("learner", step=n, loss=m["loss"], td_abs=m["td_abs_mean"], grad_norm=m["grad_norm"],
                is_weight_mean=m.get("is_weight_mean", float(learner.S["weights"].mean())),
                valid_rows=m.get("valid_rows", learner.B),
                learner_kind=getattr(learner, "kind", "fused"),
                replay=replay.size(), actor_steps=st.actor_steps, inserted=group.inserted,
                episodes=len(eps_list),
                mean_return=float(np.mean(rets)) if rets else float("nan"),
                mean_ep_len=float(np.mean(lens)) if lens else float("nan"),
                eps_min=float(eps_.min()), eps_max=float(eps_.max()),
                grad_steps_per_s=(n - st.n_last) / dt,
                env_frames_per_s=(st.actor_steps - st.steps_last) * group.E * world / dt,
                inserts_per_s=(group.inserted - st.ins_last) * world / dt,
                steps_per_s=n / max(now - st.t0, 1e-9),
                actor_thread=st.runner is not None,
                actor_restarts=st.runner.restarts if st.runner is not None else 0)
    for (env_id, ep_len, ep_ret) in new_eps[:rt.episode_lines_per_log]:
        metrics.episode(env_id, st.actor_steps, ep_len, ep_ret)
    st.n_ep_seen = len(eps_list)
    if rt.profile_phases and device.type == "cuda":
        metrics.log("phases_ms", step=n, **learner.profile_step())
    st.t_last, st.n_last, st.ins_last, st.steps_last = time.time(), n, group.inserted, st.actor_steps
