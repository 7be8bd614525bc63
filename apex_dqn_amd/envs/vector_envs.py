"""Vectorised environments.

The reference builds a single ``gym.make(name)`` per actor with no wrappers
(``env.py:3-4``) and preprocesses frames with a broken truncating reshape
(``actor.py:117-119``, defect A14).  gym / ALE are not installed in this
image (nor on the offline GPU box), so the engine ships:

* ``CartPoleVec``   -- numpy CartPole-v1 dynamics for E envs (BASELINE config 1);
* ``SyntheticAtariVec`` -- Atari-shaped (84x84 uint8 frame per step) env with
  learnable dynamics, for the GPU configs on synthetic frames;
* ``AtariPreprocess`` + ``ALEVec`` -- correct Atari preprocessing (gray,
  area-resize to 84x84, frame-skip with max-pool, no-op starts, reward clip)
  around ``ale_py`` when it is importable.

All envs auto-reset: ``step`` returns the first observation of the next
episode for envs that finished.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import numpy as np


class CartPoleVec:
    """CartPole-v1 (Barto, Sutton & Anderson) physics, vectorised."""

    gravity = 9.8
    masscart = 1.0
    masspole = 0.1
    total_mass = masscart + masspole
    length = 0.5
    polemass_length = masspole * length
    force_mag = 10.0
    tau = 0.02
    theta_threshold = 12 * 2 * math.pi / 360
    x_threshold = 2.4
    max_steps = 500

    obs_shape = (4,)
    obs_dtype = np.float32
    action_dim = 2
    frame_based = False

    def __init__(self, num_envs: int, seed: int = 0):
        self.E = int(num_envs)
        self.rng = np.random.default_rng(seed)
        self.state = np.zeros((self.E, 4), np.float64)
        self.t = np.zeros(self.E, np.int64)
        self.ep_ret = np.zeros(self.E, np.float64)

    def _reset_idx(self, idx):
        self.state[idx] = self.rng.uniform(-0.05, 0.05, size=(len(idx), 4))
        self.t[idx] = 0
        self.ep_ret[idx] = 0.0

    def reset(self) -> np.ndarray:
        self._reset_idx(np.arange(self.E))
        return self.state.astype(np.float32)

    def step(self, actions: np.ndarray):
        x, x_dot, th, th_dot = self.state.T
        force = np.where(np.asarray(actions) == 1, self.force_mag, -self.force_mag)
        cos, sin = np.cos(th), np.sin(th)
        temp = (force + self.polemass_length * th_dot ** 2 * sin) / self.total_mass
        th_acc = (self.gravity * sin - cos * temp) / (
            self.length * (4.0 / 3.0 - self.masspole * cos ** 2 / self.total_mass))
        x_acc = temp - self.polemass_length * th_acc * cos / self.total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * x_acc
        th = th + self.tau * th_dot
        th_dot = th_dot + self.tau * th_acc
        self.state = np.stack([x, x_dot, th, th_dot], axis=1)
        self.t += 1
        term = (np.abs(x) > self.x_threshold) | (np.abs(th) > self.theta_threshold)
        trunc = self.t >= self.max_steps
        done = term | trunc
        rew = np.ones(self.E, np.float32)
        self.ep_ret += rew
        info = {"episode_return": np.where(done, self.ep_ret, np.nan),
                "episode_length": np.where(done, self.t, -1), "truncated": trunc & ~term}
        idx = np.nonzero(done)[0]
        if len(idx):
            self._reset_idx(idx)
        return self.state.astype(np.float32), rew, done, info


class SyntheticAtariVec:
    """Atari-shaped synthetic env: one 84x84 uint8 frame per step.

    Hidden state s in [0, S); the frame is a fixed random "sprite sheet" image
    for s plus a moving bar, so a conv net can infer s.  Reward 1 when the
    action equals s mod A.  Episodes end with probability ``p_end`` per step
    or at ``max_len``.
    """

    obs_dtype = np.uint8
    frame_based = True
    frame_out = True          # step(actions, out=...) writes the frames into ``out``

    def __init__(self, num_envs: int, action_dim: int = 6, seed: int = 0,
                 num_states: int = 32, p_end: float = 0.01, max_len: int = 1000,
                 frame_hw=(84, 84)):
        self.E = int(num_envs)
        self.action_dim = int(action_dim)
        self.S = int(num_states)
        self.rng = np.random.default_rng(seed)
        h, w = frame_hw
        self.obs_shape = (h, w)
        bank_rng = np.random.default_rng(1234)
        self.bank = bank_rng.integers(0, 64, size=(self.S, h, w), dtype=np.uint8)
        for s in range(self.S):   # a bright block whose position encodes s
            r0 = (s * 5) % (h - 12)
            c0 = (s * 11) % (w - 12)
            self.bank[s, r0:r0 + 12, c0:c0 + 12] = 200
        self.p_end = float(p_end)
        self.max_len = int(max_len)
        self.s = np.zeros(self.E, np.int64)
        self.t = np.zeros(self.E, np.int64)
        self.ep_ret = np.zeros(self.E, np.float64)

    def _frames(self, out: Optional[np.ndarray] = None) -> np.ndarray:
        # the gather returns a fresh array, or fills ``out`` (e.g. the replay's pinned staging;
        # mode 'clip': numpy buffers ``out`` under the default 'raise')
        f = self.bank[self.s] if out is None else np.take(self.bank, self.s, axis=0, out=out, mode="clip")
        col = (self.t * 3) % self.obs_shape[1]
        f[np.arange(self.E), :, col] = 255
        return f

    def reset(self) -> np.ndarray:
        self.s = self.rng.integers(0, self.S, size=self.E)
        self.t[:] = 0
        self.ep_ret[:] = 0
        return self._frames()

    def step(self, actions: np.ndarray, out: Optional[np.ndarray] = None):
        actions = np.asarray(actions, np.int64)
        rew = (actions == (self.s % self.action_dim)).astype(np.float32)
        self.s = (self.s * 7 + actions + 1 + self.rng.integers(0, 2, size=self.E)) % self.S
        self.t += 1
        self.ep_ret += rew
        done = (self.rng.random(self.E) < self.p_end) | (self.t >= self.max_len)
        info = {"episode_return": np.where(done, self.ep_ret, np.nan),
                "episode_length": np.where(done, self.t, -1)}
        idx = np.nonzero(done)[0]
        if len(idx):
            self.s[idx] = self.rng.integers(0, self.S, size=len(idx))
            self.t[idx] = 0
            self.ep_ret[idx] = 0
        return self._frames(out), rew, done, info


def _area_matrix(n_out: int, n_in: int) -> np.ndarray:
    """Row-stochastic area-interpolation matrix (n_out, n_in)."""
    m = np.zeros((n_out, n_in), np.float64)
    scale = n_in / n_out
    for i in range(n_out):
        a, b = i * scale, (i + 1) * scale
        j0, j1 = int(math.floor(a)), int(math.ceil(b))
        for j in range(j0, min(j1, n_in)):
            lo, hi = max(a, j), min(b, j + 1)
            if hi > lo:
                m[i, j] = (hi - lo) / scale
    return m


class AtariPreprocess:
    """Gray-scale + area resize to 84x84 uint8 (fixes defect A14)."""

    def __init__(self, in_hw=(210, 160), out_hw=(84, 84)):
        self.ry = _area_matrix(out_hw[0], in_hw[0])
        self.rx = _area_matrix(out_hw[1], in_hw[1])
        self.w = np.array([0.299, 0.587, 0.114])
        self.ry32 = self.ry.astype(np.float32)
        self.rxT32 = np.ascontiguousarray(self.rx.T.astype(np.float32))

    def __call__(self, rgb: np.ndarray) -> np.ndarray:
        """rgb: (..., H, W, 3) uint8 -> (..., 84, 84) uint8 (two matmuls, no einsum)."""
        gray = rgb.astype(np.float32) @ self.w.astype(np.float32)
        out = np.matmul(np.matmul(self.ry32, gray), self.rxT32)
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)


class FakeALE:
    """Deterministic stand-in for one ALE emulator (``ale_py.ALEInterface``
    subset: act / getScreenRGB / game_over / reset_game / lives /
    getMinimalActionSet).  A bright block moves with the actions over a
    frame-indexed background; every 7th emulator frame pays a reward of
    ``reward_scale`` (so clipping is observable), a life is lost every
    ``life_frames`` frames and the game ends with the last life.  Lets the DQN
    wrapper stack below run (and be tested) without ROMs."""

    def __init__(self, seed: int = 0, lives: int = 3, life_frames: int = 60, reward_scale: float = 5.0,
                 n_actions: int = 6, target: bool = False):
        self.rng = np.random.default_rng(seed)
        self.max_lives, self.life_frames, self.reward_scale = lives, life_frames, reward_scale
        self.n_actions = n_actions
        # target mode (backend "fake_ale_target"): the 7th-frame reward is paid only while
        # the block is in the right third of the screen -- a policy to learn (move right
        # and stay), observable only through the frames (learning-parity runs)
        self.target = bool(target)
        self.frames_total = 0
        self.reset_game()

    def getMinimalActionSet(self):  # noqa: N802 - ALE naming
        return list(range(self.n_actions))

    def reset_game(self):
        self.t = 0
        self._lives = self.max_lives
        self.x = int(self.rng.integers(10, 140))

    def lives(self) -> int:
        return self._lives

    def game_over(self) -> bool:
        return self._lives <= 0

    def act(self, a: int) -> float:
        if self.game_over():
            return 0.0
        self.t += 1
        self.frames_total += 1
        self.x = int(np.clip(self.x + (int(a) % 3 - 1) * 3, 0, 150))
        if self.t % self.life_frames == 0:
            self._lives -= 1
        if self.target and self.x < 100:
            return 0.0
        return self.reward_scale if self.t % 7 == 0 else 0.0

    def getScreenRGB(self) -> np.ndarray:  # noqa: N802
        img = np.full((210, 160, 3), (self.t * 3) % 256, np.uint8)
        img[100:120, self.x:self.x + 10] = 255
        img[5, :, 0] = self.t % 256  # per-frame marker (distinguishes the pooled frames)
        return img


class AtariWrapperVec:
    """The standard DQN/Ape-X Atari preprocessing over any emulator exposing the
    ALE interface (the reference calls plain ``gym.make`` with none of these,
    ``env.py:3-4``):

    * frame-skip ``k`` with the max over the last two raw frames (flicker);
    * up to ``noop_max`` random no-op actions after every reset;
    * optional FIRE after reset (games that wait for it);
    * episodic life: ``done`` on a lost life (bootstrapping stops), the
      emulator only resets on game over;
    * reward clipping to sign(r);
    * gray + area resize to 84x84 uint8 (``AtariPreprocess``).

    ``info`` carries the UNCLIPPED game-episode return / length when a game
    ends (``real_done``), NaN / -1 otherwise."""

    obs_dtype = np.uint8
    frame_based = True
    obs_shape = (84, 84)
    frame_out = True          # step(actions, out=...) writes the frames into ``out``

    def __init__(self, emulators, frame_skip: int = 4, noop_max: int = 30, clip_rewards: bool = True,
                 episodic_life: bool = True, fire_reset: bool = False, seed: int = 0):
        self.envs = list(emulators)
        self.E = len(self.envs)
        self.actions = list(self.envs[0].getMinimalActionSet())
        self.action_dim = len(self.actions)
        self.pre = AtariPreprocess()
        self.frame_skip, self.noop_max, self.clip = int(frame_skip), int(noop_max), bool(clip_rewards)
        self.episodic_life, self.fire_reset = bool(episodic_life), bool(fire_reset)
        self.rng = np.random.default_rng(seed)
        self.ep_ret = np.zeros(self.E)
        self.ep_len = np.zeros(self.E, np.int64)
        self.lives = np.array([e.lives() for e in self.envs])

    def _reset_one(self, i: int) -> np.ndarray:
        emu = self.envs[i]
        emu.reset_game()
        for _ in range(int(self.rng.integers(0, self.noop_max + 1))):
            emu.act(self.actions[0])
            if emu.game_over():
                emu.reset_game()
        if self.fire_reset and len(self.actions) > 1:
            emu.act(self.actions[1])
        self.lives[i] = emu.lives()
        return self.pre(emu.getScreenRGB())

    def reset(self) -> np.ndarray:
        self.ep_ret[:] = 0
        self.ep_len[:] = 0
        return np.stack([self._reset_one(i) for i in range(self.E)])

    def step(self, actions, out: Optional[np.ndarray] = None):
        obs = np.zeros((self.E, 84, 84), np.uint8) if out is None else out    # every row is written below
        rew = np.zeros(self.E, np.float32)
        done = np.zeros(self.E, bool)
        real_done = np.zeros(self.E, bool)
        ep_r = np.full(self.E, np.nan)
        ep_l = np.full(self.E, -1)
        for i, a in enumerate(actions):
            emu = self.envs[i]
            r, last2 = 0.0, []
            for k in range(self.frame_skip):
                r += emu.act(self.actions[int(a)])
                if k >= self.frame_skip - 2:
                    last2.append(emu.getScreenRGB())
                if emu.game_over():
                    break
            if not last2:
                last2.append(emu.getScreenRGB())
            frame = np.maximum(last2[0], last2[-1])
            self.ep_ret[i] += r
            self.ep_len[i] += 1
            rew[i] = np.sign(r) if self.clip else r
            lives = emu.lives()
            if emu.game_over():
                done[i] = real_done[i] = True
                ep_r[i], ep_l[i] = self.ep_ret[i], self.ep_len[i]
                self.ep_ret[i], self.ep_len[i] = 0, 0
                obs[i] = self._reset_one(i)
                continue
            if self.episodic_life and lives < self.lives[i]:
                done[i] = True          # a lost life ends the transition chain, not the game
            self.lives[i] = lives
            obs[i] = self.pre(frame)
        return obs, rew, done, {"episode_return": ep_r, "episode_length": ep_l, "real_done": real_done}


class ALEVec(AtariWrapperVec):  # pragma: no cover - ale_py is not available in this image
    """``AtariWrapperVec`` over real ALE emulators (``ale_py``), when importable."""

    def __init__(self, game: str, num_envs: int, seed: int = 0, **kw):
        from ale_py import ALEInterface, roms
        name = game.replace("NoFrameskip-v4", "").replace("-v0", "")
        snake = "".join("_" + c.lower() if c.isupper() else c for c in name).lstrip("_")
        emus = []
        for i in range(int(num_envs)):
            ale = ALEInterface()
            ale.setInt("random_seed", seed + i)
            ale.setFloat("repeat_action_probability", 0.0)
            ale.loadROM(roms.get_rom_path(snake))
            emus.append(ale)
        super().__init__(emus, seed=seed, **kw)


def make_vec_env(backend: str, name: str, num_envs: int, action_dim: int,
                 seed: int = 0, frame_hw: Optional[Tuple[int, int]] = None):
    """Factory replacing ``make_local_env`` (``env.py:3-4``)."""
    if backend == "cartpole":
        from ..runtime import native
        return native.NativeCartPoleVec(num_envs, seed=seed) if native.available() else CartPoleVec(num_envs, seed)
    if backend == "synthetic":
        return SyntheticAtariVec(num_envs, action_dim=action_dim, seed=seed,
                                 frame_hw=frame_hw or (84, 84))
    if backend in ("fake_ale", "fake_ale_target"):
        return AtariWrapperVec([FakeALE(seed=seed + i, n_actions=action_dim, target=backend == "fake_ale_target")
                                for i in range(num_envs)], seed=seed)
    if backend == "ale":  # pragma: no cover
        return ALEVec(name, num_envs, seed=seed)
    raise ValueError(f"unknown env backend {backend!r}")
