"""Training orchestration for the CPU/generic path.

``train_inline``      -- actors, replay and learner in one process (tests,
                         quick runs).
``train_multiprocess`` -- the reference's process topology done right
                         (``main.py:37-61``): N actor processes feed the
                         learner process through a queue; the learner owns
                         the replay (no manager server, no inserter busy-spin
                         ``main.py:21-25``, no unlocked concurrent replay access
                         A24); parameters go back through ``SharedParams``;
                         a supervisor restarts actors whose heartbeat stops
                         (fault tolerance absent from the reference).

The MI355X path (``runtime/gpu_loop.py``) keeps the same structure but owns
an HBM replay shard and the fused learner per GPU rank.
"""
from __future__ import annotations

import copy
import multiprocessing as mp
import os
import queue
import time
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from ..actors.actor_group import ActorGroup, HostFrameStore
from ..config import ApexConfig
from ..envs.vector_envs import make_vec_env
from ..learner.torch_learner import TorchLearner
from ..models.dueling import build_network
from ..replay.host_replay import PrioritizedReplay
from ..utils.metrics import MetricsLogger
from .shared_params import SharedParams


def _make_group(cfg: ApexConfig, num_envs: int, offset: int, total: int, seed: int) -> ActorGroup:
    env = make_vec_env(cfg.env_backend, cfg.env_conf.name, num_envs, cfg.env_conf.action_dim,
                       seed=seed + offset)
    a = cfg.Actor
    return ActorGroup(env, num_envs, a.num_steps, a.gamma, cfg.frame_stack, a.epsilon, a.alpha,
                      global_actor_offset=offset, total_actors=total, seed=seed, materialize=True)


def _make_policy(net: torch.nn.Module, device):
    def policy(obs):
        with torch.no_grad():
            return net(torch.as_tensor(obs).to(device))[2].float().cpu().numpy()
    return policy


def train_inline(cfg: ApexConfig, learner_steps: int, device="cpu",
                 metrics: Optional[MetricsLogger] = None, actor_steps_per_update: int = 1,
                 max_actor_steps: Optional[int] = None) -> Dict[str, Any]:
    torch.manual_seed(cfg.Runtime.seed)
    device = torch.device(device)
    a, L = cfg.Actor, cfg.Learner
    group = _make_group(cfg, a.num_actors, 0, a.num_actors, cfg.Runtime.seed)
    replay = PrioritizedReplay(cfg.Replay_Memory.soft_capacity, cfg.Replay_Memory.priority_exponent,
                               cfg.Replay_Memory.importance_sampling_exponent,
                               capacity=cfg.replay_capacity, priority_eps=cfg.Runtime.priority_eps,
                               seed=cfg.Runtime.seed, is_normalise=cfg.Runtime.is_normalise)
    learner = TorchLearner(cfg, device)
    actor_net = copy.deepcopy(learner.Q).eval()
    policy = _make_policy(actor_net, device)
    losses: List[float] = []
    t_actor = 0
    max_actor_steps = max_actor_steps or (10 ** 12)
    while learner.num_q_updates < learner_steps and t_actor < max_actor_steps:
        for _ in range(actor_steps_per_update):
            group.step(policy)
            t_actor += 1
            if t_actor % a.Q_network_sync_freq == 0:
                actor_net.load_state_dict(learner.Q.state_dict())
        b = group.drain()
        if b is not None:
            replay.add(b)
        if replay.size() > L.min_replay_mem_size:
            batch = replay.sample(L.replay_sample_size)
            out = learner.step(batch)
            replay.set_priorities(batch["idx"], out["td_abs"])
            losses.append(out["loss"])
            if learner.num_q_updates % L.remove_old_xp_freq == 0:
                replay.remove_to_fit()
            if metrics is not None and learner.num_q_updates % cfg.Runtime.log_every == 0:
                metrics.log("learner", step=learner.num_q_updates, loss=out["loss"],
                            replay=replay.size(), grad_norm=out["grad_norm"])
            ck = cfg.Runtime
            if ck.ckpt_dir and ck.ckpt_freq and learner.num_q_updates % ck.ckpt_freq == 0:
                learner.save(os.path.join(ck.ckpt_dir, "checkpoint.pt"))
    returns = [r for (_, _, r) in group.episodes]
    return {"learner": learner, "replay": replay, "losses": losses, "episodes": group.episodes,
            "mean_return_last": float(np.mean(returns[-20:])) if returns else float("nan"),
            "actor_steps": t_actor}


# ----------------------------------------------------------------------- multiprocess
def _actor_proc(rank_id: int, cfg_dict: Dict[str, Any], num_envs: int, offset: int, total: int,
                shared: SharedParams, out_q, heartbeat, stop_evt, max_steps: int):
    torch.set_num_threads(1)
    cfg = ApexConfig.from_dict(cfg_dict)
    group = _make_group(cfg, num_envs, offset, total, cfg.Runtime.seed)
    net = build_network(cfg.network, cfg.env_conf.state_shape, cfg.env_conf.action_dim,
                        obs_scale=cfg.Runtime.obs_scale).eval()
    ver, sd = shared.read(-1)
    if sd is not None:
        net.load_state_dict(sd)
    policy = _make_policy(net, "cpu")
    flush = max(1, cfg.Actor.n_step_transition_batch_size)
    t = 0
    while not stop_evt.is_set() and t < max_steps:
        group.step(policy)
        t += 1
        heartbeat[rank_id] = time.time()
        if group.builder.size >= flush:
            b = group.drain()
            if b is not None:
                b["episodes"] = np.array(group.episodes, dtype=np.float64).reshape(-1, 3)
                group.episodes.clear()
                out_q.put(b)
        if t % cfg.Actor.Q_network_sync_freq == 0:
            ver2, sd = shared.read(ver)
            if sd is not None:
                net.load_state_dict(sd)
                ver = ver2


def train_multiprocess(cfg: ApexConfig, learner_steps: int, num_procs: Optional[int] = None,
                       device="cpu", metrics: Optional[MetricsLogger] = None,
                       max_wall_s: float = 3600.0, kill_actor_at: Optional[int] = None) -> Dict[str, Any]:
    """Reference topology (learner + N actor processes), correct and zero-copy."""
    ctx = mp.get_context("spawn")
    a, L = cfg.Actor, cfg.Learner
    nprocs = num_procs or a.num_actors
    per = [a.num_actors // nprocs + (1 if i < a.num_actors % nprocs else 0) for i in range(nprocs)]
    offsets = np.concatenate([[0], np.cumsum(per)[:-1]]).astype(int)
    learner = TorchLearner(cfg, torch.device(device))
    shared = SharedParams({k: v.cpu() for k, v in learner.Q.state_dict().items()}, ctx)
    out_q = ctx.Queue(maxsize=1024)
    heartbeat = ctx.Array("d", [time.time()] * nprocs, lock=False)
    stop_evt = ctx.Event()
    cfg_dict = cfg.to_dict()

    def spawn(i):
        p = ctx.Process(target=_actor_proc, args=(i, cfg_dict, per[i], int(offsets[i]), a.num_actors,
                                                  shared, out_q, heartbeat, stop_evt, a.T),
                        daemon=True)
        p.start()
        return p

    procs = [spawn(i) for i in range(nprocs)]
    replay = PrioritizedReplay(cfg.Replay_Memory.soft_capacity, cfg.Replay_Memory.priority_exponent,
                               cfg.Replay_Memory.importance_sampling_exponent,
                               capacity=cfg.replay_capacity, priority_eps=cfg.Runtime.priority_eps,
                               seed=cfg.Runtime.seed, is_normalise=cfg.Runtime.is_normalise)
    episodes, losses, restarts = [], [], 0
    t0 = time.time()
    try:
        while learner.num_q_updates < learner_steps and time.time() - t0 < max_wall_s:
            got = 0
            while True:
                try:
                    b = out_q.get(timeout=0.05 if replay.size() <= L.min_replay_mem_size else 0.0005)
                except queue.Empty:
                    break
                for e in b.pop("episodes"):
                    episodes.append(tuple(e))
                replay.add(b)
                got += 1
                if got > 64:
                    break
            # supervisor: restart dead / stalled actor processes
            if kill_actor_at is not None and learner.num_q_updates == kill_actor_at and restarts == 0:
                procs[0].kill()
                kill_actor_at = None
            for i, p in enumerate(procs):
                stalled = time.time() - heartbeat[i] > cfg.Runtime.heartbeat_timeout
                if not p.is_alive() or stalled:
                    if p.is_alive():
                        p.kill()
                    p.join(timeout=5)
                    if p.exitcode not in (0, None) or stalled:
                        heartbeat[i] = time.time()
                        procs[i] = spawn(i)
                        restarts += 1
            if replay.size() <= L.min_replay_mem_size:
                continue
            batch = replay.sample(L.replay_sample_size)
            out = learner.step(batch)
            replay.set_priorities(batch["idx"], out["td_abs"])
            losses.append(out["loss"])
            if learner.num_q_updates % cfg.Runtime.param_publish_freq == 0:
                shared.publish(learner.Q.state_dict())
            if learner.num_q_updates % L.remove_old_xp_freq == 0:
                replay.remove_to_fit()
            if metrics is not None and learner.num_q_updates % cfg.Runtime.log_every == 0:
                metrics.log("learner", step=learner.num_q_updates, loss=out["loss"],
                            replay=replay.size(), restarts=restarts)
    finally:
        stop_evt.set()
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
    returns = [r for (_, _, r) in episodes]
    return {"learner": learner, "replay": replay, "losses": losses, "episodes": episodes,
            "restarts": restarts,
            "mean_return_last": float(np.mean(returns[-20:])) if returns else float("nan")}
