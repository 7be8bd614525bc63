"""Vectorised actor group: E environments acting with one batched forward.

Replaces the reference's one-process-per-actor loop (``Actor.run``,
``actor.py:146-191``, batch-1 CPU inference per env step, a ``\\r`` print per
step, pickled 5-transition messages through a Manager queue) with:

* one batched network forward for all E envs of the group (GPU when the
  learner is on GPU);
* a per-env epsilon vector from the Ape-X ladder eps_i = eps^(1+alpha*i/(N-1))
  over the *global* actor index (``actor.py:111-114``; N=1 safe);
* the sliding-window n-step builder with actor-side initial priorities
  (``actor.py:127-143`` semantics, defects fixed);
* frame stacking by reference: for frame-based envs each new 84x84 frame is
  stored once (in the replay's frame ring) and observations/transitions carry
  the C frame sequence numbers of their stack -- the HBM-sizing trick of
  SURVEY Appendix C (7 KB instead of 56 KB per transition);
* periodic parameter refresh every ``Q_network_sync_freq`` steps
  (``actor.py:189-191``).
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

import numpy as np
import torch

from ..config import epsilon_ladder
from .nstep import make_nstep_builder


class HostFrameStore:
    """Frame ring in host memory (CPU path / tests): seq -> 84x84 frame."""

    def __init__(self, capacity: int, frame_shape):
        self.capacity = int(capacity)
        self.frames = np.zeros((self.capacity,) + tuple(frame_shape), np.uint8)
        self.head = 0  # next sequence number

    def append(self, frames: np.ndarray) -> np.ndarray:
        n = len(frames)
        seqs = self.head + np.arange(n, dtype=np.int64)
        self.frames[seqs % self.capacity] = frames
        self.head += n
        return seqs

    def gather(self, seqs: np.ndarray) -> np.ndarray:
        return self.frames[np.asarray(seqs) % self.capacity]


class ActorGroup:
    """E envs + batched policy.  ``policy(obs_batch) -> q (E, A)`` numpy or tensor."""

    def __init__(self, env, num_envs: int, n: int, gamma: float, frame_stack: int,
                 eps_base: float = 0.4, eps_alpha: float = 7.0, global_actor_offset: int = 0,
                 total_actors: Optional[int] = None, seed: int = 0,
                 frame_store=None, materialize: bool = True,
                 obs_builder: Optional[Callable] = None):
        self.env = env
        self.E = int(num_envs)
        self.C = int(frame_stack)
        self.frame_based = bool(getattr(env, "frame_based", False))
        total = total_actors or self.E
        ladder = epsilon_ladder(total, eps_base, eps_alpha)
        self.eps = np.array(ladder[global_actor_offset:global_actor_offset + self.E], np.float64)
        self.rng = np.random.default_rng(seed + 7919 * global_actor_offset)
        self.frame_store = frame_store
        # payload: frame seqs (frame-based + store) | stacked frames | state vector
        if self.frame_based and frame_store is not None and not materialize:
            self.mode = "refs"
            obs_shape, obs_dtype = (self.C,), np.int64
        elif self.frame_based:
            self.mode = "stack"
            obs_shape, obs_dtype = (self.C,) + tuple(env.obs_shape), np.uint8
        else:
            self.mode = "state"
            obs_shape, obs_dtype = tuple(env.obs_shape), np.float32
        self.obs_builder = obs_builder
        self.builder = make_nstep_builder(self.E, n, gamma, obs_shape, obs_dtype,
                                    env_id_offset=global_actor_offset)
        self.t = 0
        self.episodes = []   # (env_id, ep_len, ep_return)
        self._cur = None

    # ------------------------------------------------------------------
    def _ingest(self, obs: np.ndarray, reset_mask: np.ndarray) -> np.ndarray:
        """Update the per-env stacks with a new observation; return payload."""
        if self.mode == "state":
            self._cur = obs.astype(np.float32)
            return self._cur.copy()
        if self.mode == "stack":
            if self._cur is None:
                self._cur = np.repeat(obs[:, None], self.C, axis=1)
            else:
                self._cur = np.concatenate([self._cur[:, 1:], obs[:, None]], axis=1)
                r = np.nonzero(reset_mask)[0]
                if len(r):
                    self._cur[r] = np.repeat(obs[r][:, None], self.C, axis=1)
            return self._cur.copy()
        seqs = self.frame_store.append(obs)
        if self._cur is None:
            self._cur = np.repeat(seqs[:, None], self.C, axis=1)
        else:
            self._cur = np.concatenate([self._cur[:, 1:], seqs[:, None]], axis=1)
            r = np.nonzero(reset_mask)[0]
            if len(r):
                self._cur[r] = seqs[r][:, None]
        return self._cur.copy()

    def observation(self, payload: np.ndarray):
        """Network input for the current payload."""
        if self.obs_builder is not None:
            return self.obs_builder(payload)
        if self.mode == "refs":
            return self.frame_store.gather(payload)
        return payload

    def reset(self) -> None:
        obs = self.env.reset()
        self._cur = None
        self.payload = self._ingest(obs, np.ones(self.E, bool))

    def select_actions(self, q: np.ndarray) -> np.ndarray:
        greedy = q.argmax(axis=1)
        rand = self.rng.integers(0, q.shape[1], size=self.E)
        explore = self.rng.random(self.E) < self.eps
        return np.where(explore, rand, greedy)

    def step(self, policy: Callable) -> None:
        if self._cur is None:
            self.reset()
        q = policy(self.observation(self.payload))
        if isinstance(q, torch.Tensor):
            q = q.float().cpu().numpy()
        actions = self.select_actions(q)
        obs, rew, done, info = self.env.step(actions)
        prev = self.payload
        self.payload = self._ingest(obs, done)
        self.builder.step(prev, q, actions, rew, done, self.payload)
        # real game overs only (episodic-life terminals carry NaN / -1 episode info)
        d = np.nonzero(info.get("real_done", done))[0]
        for e in d:
            self.episodes.append((int(self.builder.env_ids[e]), int(info["episode_length"][e]),
                                  float(info["episode_return"][e])))
        self.t += 1

    def drain(self, max_items: Optional[int] = None) -> Optional[Dict[str, np.ndarray]]:
        return self.builder.get(max_items)
