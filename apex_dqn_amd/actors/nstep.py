"""Vectorised sliding-window n-step transition builder.

Replaces the reference ``ExperienceBuffer`` (``actor.py:15-93``) with the
intended Ape-X semantics:

* one n-step transition is emitted **every** env step (sliding window), not
  one per n+1 steps (defect A9);
* ``R = sum_{k<n} gamma^k r_{t+k}`` exactly once (defect A7 double counts);
* ``Gamma = gamma^n`` (defect A8 uses gamma^(n-1)), and 0 when the episode
  terminated inside the window (defect A10 never masks terminals);
* on episode end the partial windows are flushed as terminal transitions;
* keys are unique int64 ``(global_env_id << 40) | seq`` (defect A11: string
  concatenation collides);
* gamma comes from the config (defect A12 hard-codes 0.99).

The actor's initial priority ``|R + Gamma*max_a q(S_{t+n}) - q(S_t, A_t)|``
(``actor.py:127-143``, A1 fixed: one priority per transition) needs
``q(S_{t+n})``, which the actor only computes on its next step, so a full
window transition waits one step in a per-env "pending" slot.

Everything is vectorised over E environments (one actor group); the
observation payload per step is an arbitrary fixed-shape array (the frame
sequence numbers of the stacked frames for Atari, the state vector for
CartPole).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np


class NStepBuilder:
    def __init__(self, num_envs: int, n: int, gamma: float, obs_shape, obs_dtype,
                 env_id_offset: int = 0):
        self.E = int(num_envs)
        self.n = int(n)
        self.gamma = float(gamma)
        self.obs_shape = tuple(obs_shape)
        self.obs_dtype = np.dtype(obs_dtype)
        E, n_ = self.E, self.n
        self.w_obs = np.zeros((E, n_) + self.obs_shape, self.obs_dtype)
        self.w_act = np.zeros((E, n_), np.int64)
        self.w_rew = np.zeros((E, n_), np.float64)
        self.w_qsa = np.zeros((E, n_), np.float64)
        self.cnt = np.zeros(E, np.int64)
        # one pending (full-window, non-terminal) transition per env awaiting q(S_{t+n})
        self.p_valid = np.zeros(E, bool)
        self.p_obs = np.zeros((E,) + self.obs_shape, self.obs_dtype)
        self.p_next = np.zeros((E,) + self.obs_shape, self.obs_dtype)
        self.p_act = np.zeros(E, np.int64)
        self.p_R = np.zeros(E, np.float64)
        self.p_qsa = np.zeros(E, np.float64)
        self.p_key = np.zeros(E, np.int64)
        self.seq = np.zeros(E, np.int64)
        self.env_ids = np.arange(E, dtype=np.int64) + int(env_id_offset)
        self.disc = self.gamma ** np.arange(n_, dtype=np.float64)
        self._out: List[Dict[str, np.ndarray]] = []

    # ------------------------------------------------------------------
    def _keys(self, idx: np.ndarray) -> np.ndarray:
        k = (self.env_ids[idx] << 40) | (self.seq[idx] & ((1 << 40) - 1))
        self.seq[idx] += 1
        return k

    def _emit(self, obs, nxt, act, R, gamma_n, prio, key, env):
        if len(act) == 0:
            return
        self._out.append(dict(S_t=obs, S_tpn=nxt, A_t=act.astype(np.int64),
                              R=R.astype(np.float32), Gamma=gamma_n.astype(np.float32),
                              priority=prio.astype(np.float32), key=key.astype(np.int64),
                              env=env.astype(np.int64)))

    def step(self, obs: np.ndarray, q: np.ndarray, actions: np.ndarray,
             rewards: np.ndarray, dones: np.ndarray, next_obs: np.ndarray) -> None:
        """Record one vectorised env step.

        obs:      (E, *obs_shape) payload of S_t (the state acted on)
        q:        (E, A) q-values of S_t from the actor's network
        actions:  (E,) actions taken
        rewards:  (E,) rewards received
        dones:    (E,) episode terminated after this step
        next_obs: (E, *obs_shape) payload of S_{t+1} (ignored where done)
        """
        E = self.E
        q = np.asarray(q, np.float64)
        actions = np.asarray(actions, np.int64)
        rewards = np.asarray(rewards, np.float64)
        dones = np.asarray(dones, bool)
        qmax = q.max(axis=1)
        # 1) finish pending transitions: their bootstrap state is S_t
        pv = np.nonzero(self.p_valid)[0]
        if len(pv):
            gn = self.gamma ** self.n
            target = self.p_R[pv] + gn * qmax[pv]
            prio = np.abs(target - self.p_qsa[pv])
            self._emit(self.p_obs[pv].copy(), self.p_next[pv].copy(), self.p_act[pv],
                       self.p_R[pv], np.full(len(pv), gn), prio, self.p_key[pv], self.env_ids[pv])
            self.p_valid[pv] = False
        # 2) append step t to every window
        ar = np.arange(E)
        c = self.cnt
        self.w_obs[ar, c] = obs
        self.w_act[ar, c] = actions
        self.w_rew[ar, c] = rewards
        self.w_qsa[ar, c] = q[ar, actions]
        self.cnt = c + 1
        # 3) terminal envs: flush every window entry as a terminal transition
        d_idx = np.nonzero(dones)[0]
        if len(d_idx):
            for e in d_idx:
                m = int(self.cnt[e])
                rw = self.w_rew[e, :m]
                # R_j = sum_{k>=j} gamma^(k-j) r_k over the remaining window
                R = np.array([np.dot(self.disc[:m - j], rw[j:]) for j in range(m)])
                prio = np.abs(R - self.w_qsa[e, :m])
                keys = np.array([self._keys(np.array([e]))[0] for _ in range(m)], np.int64)
                self._emit(self.w_obs[e, :m].copy(), np.repeat(obs[e:e + 1], m, axis=0),
                           self.w_act[e, :m].copy(), R, np.zeros(m), prio, keys,
                           np.full(m, self.env_ids[e]))
            self.cnt[d_idx] = 0
        # 4) full windows (non-terminal): move the oldest entry into the pending slot
        f_idx = np.nonzero((self.cnt == self.n) & ~dones)[0]
        if len(f_idx):
            R = self.w_rew[f_idx] @ self.disc
            self.p_valid[f_idx] = True
            self.p_obs[f_idx] = self.w_obs[f_idx, 0]
            self.p_next[f_idx] = next_obs[f_idx]
            self.p_act[f_idx] = self.w_act[f_idx, 0]
            self.p_R[f_idx] = R
            self.p_qsa[f_idx] = self.w_qsa[f_idx, 0]
            self.p_key[f_idx] = self._keys(f_idx)
            # slide the window by one
            self.w_obs[f_idx, :-1] = self.w_obs[f_idx, 1:]
            self.w_act[f_idx, :-1] = self.w_act[f_idx, 1:]
            self.w_rew[f_idx, :-1] = self.w_rew[f_idx, 1:]
            self.w_qsa[f_idx, :-1] = self.w_qsa[f_idx, 1:]
            self.cnt[f_idx] -= 1

    # ------------------------------------------------------------------
    @property
    def size(self) -> int:
        return int(sum(len(o["A_t"]) for o in self._out))

    def get(self, max_items: Optional[int] = None) -> Optional[Dict[str, np.ndarray]]:
        """Pop up to ``max_items`` emitted transitions (all if None) as one batch."""
        if not self._out:
            return None
        out = {k: np.concatenate([o[k] for o in self._out]) for k in self._out[0]}
        self._out = []
        if max_items is not None and len(out["A_t"]) > max_items:
            rest = {k: v[max_items:] for k, v in out.items()}
            out = {k: v[:max_items] for k, v in out.items()}
            self._out = [rest]
        return out


def make_nstep_builder(num_envs: int, n: int, gamma: float, obs_shape, obs_dtype, env_id_offset: int = 0):
    """The native builder (csrc/runtime/nstep.cpp) when the host runtime library is
    available, else this numpy one (its test oracle).  APEX_NUMPY_NSTEP=1 forces numpy."""
    import os
    if os.environ.get("APEX_NUMPY_NSTEP", "0") != "1":
        from ..runtime import native
        if native.available():
            return native.NativeNStepBuilder(num_envs, n, gamma, obs_shape, obs_dtype, env_id_offset)
    return NStepBuilder(num_envs, n, gamma, obs_shape, obs_dtype, env_id_offset)


def nstep_returns_reference(rewards, dones, gamma: float, n: int):
    """Slow scalar oracle for a single env trajectory (used by tests).

    Returns a list of (t, R, Gamma) for every start index t.
    """
    T = len(rewards)
    out = []
    # episode boundaries
    for t in range(T):
        R, g, term = 0.0, 1.0, False
        k = 0
        while k < n and t + k < T:
            R += g * rewards[t + k]
            g *= gamma
            if dones[t + k]:
                term = True
                k += 1
                break
            k += 1
        if term:
            out.append((t, R, 0.0))
        elif k == n:
            out.append((t, R, gamma ** n))
        # else: trajectory truncated by T, transition not yet complete
    return out
