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

import os
import time
from typing import Any, Dict, Optional

import numpy as np
import torch

from ..actors.gpu_actor import make_gpu_actor_group
from ..config import ApexConfig
from ..learner.fused_learner import FusedNatureLearner
from ..replay.gpu_replay import GpuReplayShard
from ..utils.metrics import MetricsLogger


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
                 backend: Optional[str] = None) -> Dict[str, Any]:
    device = torch.device(device)
    rank = comm.rank if comm is not None else 0
    world = comm.world_size if comm is not None else 1
    rt, L = cfg.Runtime, cfg.Learner
    E = num_envs or cfg.Runtime.actors_per_rank or max(1, cfg.Actor.num_actors // world)
    torch.manual_seed(rt.seed)
    replay = build_replay(cfg, device, E, seed=rt.seed + rank, world=world)
    if cfg.network in ("nature64", "nature32"):
        learner = FusedNatureLearner(cfg, device, replay, comm=comm, backend=backend)
    elif cfg.network == "impala" and cfg.Runtime.use_hip_kernels:   # csrc/impala.hip learner
        from ..learner.impala_learner import FusedImpalaLearner
        learner = FusedImpalaLearner(cfg, device, replay, comm=comm, backend=backend)
    else:   # graph-captured torch-autograd learner on the same HBM replay
        from ..learner.graph_learner import GraphLearner
        learner = GraphLearner(cfg, device, replay, comm=comm)
    group = make_gpu_actor_group(cfg, learner, replay, E, rank, world, seed=rt.seed)
    min_local = max(L.min_replay_mem_size // world, L.replay_sample_size)
    started = False
    t0 = time.time()
    actor_steps = 0
    max_actor_steps = max_actor_steps or 10 ** 12
    losses = []
    ckpt_path = os.path.join(rt.ckpt_dir, "checkpoint.pt") if rt.ckpt_dir else None
    # restart after a learner-rank failure (torchrun --max-restarts / run_elastic):
    # every rank resumes the same checkpoint, so the DP replicas stay identical
    if ckpt_path and rt.resume and os.path.exists(ckpt_path):
        learner.load(ckpt_path)
        if metrics is not None:
            metrics.log("resume", step=learner.num_q_updates, path=ckpt_path)
    prof = None
    n_ep_seen = 0
    t_last, n_last, ins_last, steps_last = t0, learner.num_q_updates, 0, 0
    while learner.num_q_updates < learner_steps and actor_steps < max_actor_steps:
        for _ in range(actor_steps_per_update):
            group.step()
            actor_steps += 1
        if not started:
            ready = float(replay.size() > min_local)
            if comm is not None and comm.active:
                ready = comm.allreduce_scalar(ready, "min")
            if ready < 1.0:
                continue
            started = True
            learner.refresh_replay_stats()
        if rt.torch_profile_dir and learner.num_q_updates == rt.torch_profile_start and prof is None:
            prof = _start_torch_profiler(device)
        learner.step()
        n = learner.num_q_updates
        if prof is not None and n >= rt.torch_profile_start + rt.torch_profile_steps:
            prof.stop()
            os.makedirs(rt.torch_profile_dir, exist_ok=True)
            prof.export_chrome_trace(os.path.join(rt.torch_profile_dir, f"trace_rank{rank}.json"))
            prof, rt.torch_profile_dir = None, None
        if n % L.remove_old_xp_freq == 0:
            replay.remove_to_fit()
            replay.rebuild()
            learner.refresh_replay_stats()
        if rt.log_every and n % rt.log_every == 0:
            m = learner.last_metrics()
            losses.append(m["loss"])
            if metrics is not None:
                now = time.time()
                dt = max(now - t_last, 1e-9)
                eps_ = group.eps.float()
                new_eps = group.episodes[n_ep_seen:]
                rets = [r for (_, _, r) in group.episodes[-50:]]
                lens = [ln for (_, ln, _) in group.episodes[-50:]]
                metrics.log("learner", step=n, loss=m["loss"], td_abs=m["td_abs_mean"], grad_norm=m["grad_norm"],
                            is_weight_mean=float(learner.S["weights"].mean()),
                            learner_kind=getattr(learner, "kind", "fused"),
                            replay=replay.size(), actor_steps=actor_steps, inserted=group.inserted,
                            episodes=len(group.episodes),
                            mean_return=float(np.mean(rets)) if rets else float("nan"),
                            mean_ep_len=float(np.mean(lens)) if lens else float("nan"),
                            eps_min=float(eps_.min()), eps_max=float(eps_.max()),
                            grad_steps_per_s=(n - n_last) / dt,
                            env_frames_per_s=(actor_steps - steps_last) * group.E * world / dt,
                            inserts_per_s=(group.inserted - ins_last) * world / dt,
                            steps_per_s=n / max(now - t0, 1e-9))
                for (env_id, ep_len, ep_ret) in new_eps[:rt.episode_lines_per_log]:
                    metrics.episode(env_id, actor_steps, ep_len, ep_ret)
                n_ep_seen = len(group.episodes)
                if rt.profile_phases and device.type == "cuda":
                    metrics.log("phases_ms", step=n, **learner.profile_step())
                t_last, n_last, ins_last, steps_last = time.time(), learner.num_q_updates, group.inserted, actor_steps
        if ckpt_path and rt.ckpt_freq and n % rt.ckpt_freq == 0 and rank == 0:
            learner.save(ckpt_path)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    rets = [r for (_, _, r) in group.episodes]
    return {"learner": learner, "replay": replay, "actors": group, "losses": losses,
            "episodes": group.episodes, "actor_steps": actor_steps,
            "mean_return_last": float(np.mean(rets[-20:])) if rets else float("nan"),
            "wall_s": time.time() - t0}
