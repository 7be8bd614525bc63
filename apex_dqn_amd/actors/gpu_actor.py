"""GPU actor group: E environments, one batched forward through the learner's
kernels, device-side epsilon-greedy, frames stored once in the replay ring.

Reference: ``Actor.run`` (``actor.py:146-191``) -- per env step a batch-1 CPU
forward, an epsilon-greedy draw (``:121-125``), an n-step buffer add and a
pickled queue put every 5 transitions, a ``state_dict`` pull every 500 steps.
Here one step of the group:

  1. conv1 reads the group's current frame stacks from the replay ring by slot
     (no stacking copy), conv2/conv3/fc, then ``actor_head`` computes q and the
     epsilon-greedy action per env on the device (one launch, counter RNG);
  2. one small D2H copy of (q, action) per env;
  3. the vectorised envs step; each new frame is appended ONCE to the HBM
     frame ring (uint8), observations are C frame sequence numbers;
  4. the sliding-window n-step builder emits transitions with initial
     priorities, inserted into the local replay shard by one kernel.

The actor keeps its own parameter slot (fp32 master weights + the bf16 compute
copy, with its lo plane when the learner is fp32), refreshed from the learner with
a D2D copy every ``Q_network_sync_freq`` steps (reference ``actor.py:189-191``).

Precision: the reference actor runs the fp32 network (``actor.py:161`` ``.float()``)
and derives the initial priorities from those q-values (``actor.py:127-143``).  With
the fp32 learner (``Runtime.dtype = fp32``, split hi / lo operands) the actor runs the
same split kernels on its batch -- conv1 on the fp32 weights, hi / lo activation
planes through conv2 / conv3 / fc, ``actor_head`` on hi + lo -- so its q-values, the
epsilon-greedy argmax and the initial |delta| priorities carry fp32-class error,
not bf16's 2^-9.

Epsilon ladder over ranks: env i of rank r is actor ``i * world + r`` of the global
ladder eps^(1 + alpha k / (N - 1)) (interleaved), so every rank's replay shard holds a
mix of exploratory and greedy actors -- with contiguous slices rank 0 would hold all
the most exploratory ones and the shards' priority mass would differ systematically,
which shrinks the global batch M of the sharded draw.

Actor and learner overlap (the reference runs them as separate processes): the
group's frame appends, inference and D2H copies run on its own stream, and
``policy`` waits for that stream only, so the env stepping on the host and the
actor's kernels proceed while the learner's step is still executing on the
compute stream.  Transition inserts (records + sum-tree) stay on the compute
stream -- single writer, stream-ordered with the learner's sampling and priority
write-back -- after a wait on the actor stream for the frames they reference.
The compute stream is the one current when the group is built, so the group can
step on its own host thread (runtime/actor_thread.py) while the learner thread
replays its graphs on that stream.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import torch

from ..config import epsilon_ladder
from ..ops.switches import SW
from .nstep import make_nstep_builder


class GpuActorGroup:
    def __init__(self, cfg, learner, replay, env, num_envs: int, global_offset: int = 0,
                 total_actors: Optional[int] = None, seed: int = 0, rank: int = 0, world: int = 1):
        self.cfg = cfg
        self.learner = learner
        self.replay = replay
        self.env = env
        self.E = int(num_envs)
        self.C = learner.C
        self.A = learner.A
        self.ops = learner.ops
        d = learner.device
        self.device = d
        a = cfg.Actor
        self.eps = torch.tensor(ladder_slice(cfg, self.E, rank, world, total_actors), dtype=torch.float32, device=d)
        self.seed = int(seed) * 7919 + global_offset
        self.ctr = torch.zeros(1, dtype=torch.int64, device=d)
        ad = learner.act_dtype
        # fp32 learner (split operands): the actor runs the split kernels too
        # (Runtime.actor_precision = "bf16": the hi planes only -- cheaper inference, bf16-class
        # q-values and initial priorities)
        self.split = bool(getattr(learner, "split", False)) and cfg.Runtime.actor_precision != "bf16"
        self.slots = torch.zeros(self.E, self.C, dtype=torch.int32, device=d)
        self.frames_buf = torch.zeros(self.E, self.C, 84, 84, dtype=torch.uint8, device=d) \
            if self.ops.name != "hip" else torch.zeros(1, self.C, 84, 84, dtype=torch.uint8, device=d)

        def act(*shape):
            return (torch.zeros(*shape, dtype=ad, device=d),
                    torch.zeros(*shape, dtype=ad, device=d) if self.split else None)

        self.y1, self.y1_lo = act(self.E, 20, 20, 64)
        self.y2, self.y2_lo = act(self.E, 9, 9, 64)
        self.y3, self.y3_lo = act(self.E, 7, 7, 64)
        self.h, self.h_lo = act(self.E, 1024)
        self.q = torch.zeros(self.E, self.A, dtype=torch.float32, device=d)
        self.act = torch.zeros(self.E, dtype=torch.int32, device=d)
        self.q_host = torch.zeros(self.E, self.A, dtype=torch.float32).pin_memory() \
            if d.type == "cuda" else torch.zeros(self.E, self.A)
        self.a_host = torch.zeros(self.E, dtype=torch.int32).pin_memory() \
            if d.type == "cuda" else torch.zeros(self.E, dtype=torch.int32)
        # actor parameter slot: fp32 master copy + the bf16 compute copy [hi | lo]
        self.p32 = learner.p32.clone()
        n = self.p32.numel()
        self._pbf_all = (learner._pbf_all if self.split else learner.pbf).clone()
        self.pbf = self._pbf_all[:n]
        self.P = learner.layout.views(self.p32)
        self.Pb = learner.layout.views(self.pbf)
        self.Pl = learner.layout.views(self._pbf_all[n:]) if self.split else None
        self.builder = make_nstep_builder(self.E, a.num_steps, a.gamma, (self.C,), np.int64, env_id_offset=global_offset)
        self.global_offset = global_offset
        self.payload: Optional[np.ndarray] = None
        self.t = 0
        self.episodes: List[tuple] = []
        self.inserted = 0
        self._init_stream()
        # conv1 -> conv2 as the learner's fused kernel (csrc/conv12_fused.hip, y1 kept in LDS)
        # on a backend of the group's own: its weight fragments are the actor slot's, packed
        # at every parameter sync on the actor stream
        self.c12_ops = None
        if getattr(learner, "_c12", False) and self.ops.name == "hip" and self.ops._conv12_native():
            from ..ops.fused_ops import HipBackend
            self.c12_ops = HipBackend()
            with self._on_stream():
                self._pack_c12()

    def _c12_weights(self):
        P, Pb, Pl = self.P, self.Pb, self.Pl
        return ((P["w1"], P["b1"], None, None), (Pb["w2"], Pl["w2"] if self.split else None, P["b2"], None, None, None))

    def _pack_c12(self) -> None:
        c1, c2 = self._c12_weights()
        P, Pb, Pl = self.P, self.Pb, self.Pl
        c3 = (Pb["w3"], Pl["w3"] if self.split else None, P["b3"], None, None, None)
        self.c12_ops.conv12_pack(c1, c2, self.cfg.Runtime.obs_scale, sets=1, c3=c3)

    # ---------------------------------------------------------------- stream
    def _init_stream(self) -> None:
        cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if cuda else None
        # the learner's stream: inserts go there from whichever thread steps the group
        self.compute_stream = torch.cuda.current_stream(self.device) if cuda else None

    def _on_compute(self):
        import contextlib
        return torch.cuda.stream(self.compute_stream) if self.compute_stream is not None \
            else contextlib.nullcontext()

    def _on_stream(self):
        import contextlib
        return torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()

    def _wait_stream(self) -> None:
        """Host waits for the actor stream only (not for the learner's queued step)."""
        if self.stream is not None:
            self.stream.synchronize()

    def _after_learner(self) -> None:
        """Actor stream waits for everything queued on the compute stream so far."""
        if self.stream is not None:
            self.stream.wait_stream(self.compute_stream)

    def _before_insert(self) -> None:
        """Compute stream waits for the actor stream's frame appends."""
        if self.stream is not None:
            self.compute_stream.wait_stream(self.stream)

    # ---------------------------------------------------------------- params
    def sync_params(self) -> None:
        self._after_learner()
        with self._on_stream():
            self._copy_params()

    def _copy_params(self) -> None:
        self.p32.copy_(self.learner.p32)
        self._pbf_all.copy_(self.learner._pbf_all if self.split else self.learner.pbf)
        if getattr(self, "c12_ops", None) is not None:
            self._pack_c12()

    def reset_episodes(self) -> None:
        """Drop the partial n-step windows and start fresh episodes (actor restart)."""
        a = self.cfg.Actor
        self.builder = make_nstep_builder(self.E, a.num_steps, a.gamma, (self.C,), np.int64,
                                          env_id_offset=self.global_offset)
        self.payload = None

    # --------------------------------------------------------------- acting
    def _ingest(self, frames: np.ndarray, reset_mask: np.ndarray) -> np.ndarray:
        with self._on_stream():
            seqs = self.replay.append_frames(frames)
        if self.payload is None:
            cur = np.repeat(seqs[:, None], self.C, axis=1)
        else:
            cur = np.concatenate([self.payload[:, 1:], seqs[:, None]], axis=1)
            r = np.nonzero(reset_mask)[0]
            if len(r):
                cur[r] = seqs[r][:, None]
        return cur

    def reset(self) -> None:
        self.payload = self._ingest(self.env.reset(), np.ones(self.E, bool))

    def policy(self, payload: np.ndarray):
        """Batched q + epsilon-greedy for the given frame-seq payload (E, C) (actor stream)."""
        with self._on_stream():
            self._policy(payload)
        self._wait_stream()
        return self.q_host.numpy().copy(), self.a_host.numpy().astype(np.int64)

    def _policy(self, payload: np.ndarray):
        """Inference for the payload's frame stacks (on the actor stream): slots in, the
        kernels (one HIP graph replay with Runtime.actor_graph: captured once, outside the
        actor thread -- the fill phase's first step), q / actions out to pinned memory."""
        sl = torch.from_numpy((payload % self.replay.F).astype(np.int32))
        if self.device.type == "cuda":
            if getattr(self, "_slots_host", None) is None:
                self._slots_host = torch.zeros(self.E, self.C, dtype=torch.int32).pin_memory()
            self._slots_host.copy_(sl)
            sl = self._slots_host
        self.slots.copy_(sl, non_blocking=True)
        if self._use_graph():
            if getattr(self, "_graph", None) is None:
                self._policy_kernels()            # warm: kernel library, workspaces
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.stream, capture_error_mode="thread_local"):
                    self._policy_kernels()
                self._graph = g
            self._graph.replay()
        else:
            self._policy_kernels()
        self.q_host.copy_(self.q, non_blocking=True)
        self.a_host.copy_(self.act, non_blocking=True)

    def _use_graph(self) -> bool:
        return bool(getattr(self.cfg.Runtime, "actor_graph", False)) and self.stream is not None \
            and type(self)._policy_kernels is GpuActorGroup._policy_kernels

    def _policy_kernels(self) -> None:
        ops, P, Pb, Pl, E = self.ops, self.P, self.Pb, self.Pl, self.E
        c3 = None
        if self.c12_ops is not None:
            c1, c2 = self._c12_weights()
            if 0 < E <= SW.conv123_max_images:      # conv3 in the same launch, from y2 in LDS
                c3 = (Pb["w3"], Pl["w3"] if self.split else None, P["b3"], None, None, None)
            self.c12_ops.conv12_fwd(self.replay.frames, self.slots, self.frames_buf, self.cfg.Runtime.obs_scale,
                                    None, None, self.y2, self.y2_lo, c1, c2, rows_first=E, copy_n=0, pack_sets=0,
                                    c3=c3, y3=self.y3, y3_lo=self.y3_lo if self.split else None)
        elif self.split:   # fp32-class: the learner's split kernels (hi / lo planes throughout)
            ops.conv1_fwd_ring(self.replay.frames, self.slots, self.frames_buf, Pb["w1"], P["b1"],
                               self.cfg.Runtime.obs_scale, self.y1, w32=P["w1"], out_lo=self.y1_lo)
            ops.conv_fwd(self.y1, Pb["w2"], P["b2"], 2, self.y2, x_lo=self.y1_lo, w_lo=Pl["w2"], out_lo=self.y2_lo)
        else:
            ops.conv1_fwd_ring(self.replay.frames, self.slots, self.frames_buf, Pb["w1"], P["b1"],
                               self.cfg.Runtime.obs_scale, self.y1)
            ops.conv_fwd(self.y1, Pb["w2"], P["b2"], 2, self.y2)
        # (SW.actor_fc_ksplit: the actors' fc forward with few K splits -- a throughput job
        # beside the learner, where the chip-filling split's partial planes cost HBM traffic)
        ks = dict(ksplit=SW.actor_fc_ksplit) if SW.actor_fc_ksplit > 0 else {}
        if self.split:
            if c3 is None:
                ops.conv_fwd(self.y2, Pb["w3"], P["b3"], 1, self.y3, x_lo=self.y2_lo, w_lo=Pl["w3"],
                             out_lo=self.y3_lo)
            ops.fc_fwd(self.y3.reshape(E, 3136), Pb["wfc"], P["bfc"], self.h, x_lo=self.y3_lo.reshape(E, 3136),
                       w_lo=Pl["wfc"], out_lo=self.h_lo, **ks)
        else:
            if c3 is None:
                ops.conv_fwd(self.y2, Pb["w3"], P["b3"], 1, self.y3)
            ops.fc_fwd(self.y3.reshape(E, 3136), Pb["wfc"], P["bfc"], self.h, **ks)
        heads = {k: P[k] for k in ("wv", "bv", "wa", "ba")}
        ops.actor_head(self.h, heads, self.eps, self.ctr, self.seed, self.q, self.act, H_lo=self.h_lo)
        self.ctr += 1

    def step(self) -> int:
        """One env step for all E envs; returns the number of transitions inserted."""
        if self.payload is None:
            self.reset()
        q, actions = self.policy(self.payload)
        return self._env_step(q, actions)

    # split step (PipelinedActorGroups): the policy launch returns at once; the finish
    # waits for its q / actions, steps the envs and inserts
    def launch_policy(self) -> None:
        if self.payload is None:
            self.reset()
        with self._on_stream():
            self._policy(self.payload)
        self._pending = torch.cuda.Event() if self.stream is not None else None
        if self._pending is not None:
            self._pending.record(self.stream)

    def finish_step(self) -> int:
        """Wait for the launched inference, step the envs, append the frames, insert."""
        ev = getattr(self, "_pending", None)
        if ev is not None:
            ev.synchronize()
        self._pending = None
        return self._env_step(self.q_host.numpy().copy(), self.a_host.numpy().astype(np.int64))

    def _env_step(self, q: np.ndarray, actions: np.ndarray) -> int:
        # frame-producing envs write straight into the replay's pinned staging buffer (the
        # frame append then starts its H2D copy from it: no staging copy on the host thread)
        stage = getattr(self.replay, "stage_frames", None) if getattr(self.env, "frame_out", False) else None
        buf = stage(self.E) if stage is not None else None
        frames, rew, done, info = self.env.step(actions, out=buf) if buf is not None else self.env.step(actions)
        prev = self.payload
        self.payload = self._ingest(frames, done)
        self.builder.step(prev, q, actions, rew, done, self.payload)
        # an episode ends at a real game over; with episodic-life wrappers a lost
        # life is a terminal for the n-step targets only (its info is NaN / -1)
        for e in np.nonzero(info.get("real_done", done))[0]:
            self.episodes.append((int(self.builder.env_ids[e]), int(info["episode_length"][e]),
                                  float(info["episode_return"][e])))
        self.t += 1
        if self.t % self.cfg.Actor.Q_network_sync_freq == 0:
            self.sync_params()
        n = 0
        if self.builder.size >= self.cfg.Actor.n_step_transition_batch_size:
            b = self.builder.get()
            if b is not None:
                self._before_insert()
                with self._on_compute():
                    self.replay.insert(b)
                n = len(b["A_t"])
                self.inserted += n
        return n


class PipelinedActorGroups:
    """A rank's envs as K actor groups (own envs, HIP stream and buffers each) stepped in
    turn: group k's q / actions are read back, its envs stepped, its frames appended and
    its transitions inserted while the inference of the groups after it runs on the GPU.
    A single group waits for its own inference every step (~0.3 ms of a ~0.6 ms step on
    the Pong-shaped config, the kernels queued behind the learner's: scripts/archive/diag_e2e_actor.py);
    here the host's env work hides it.  Each env still acts on its latest frame stack
    (every group's policy is launched after its previous env step), so the transitions are
    those of one group of K * E envs; the groups take consecutive env ids and slices of
    the rank's epsilon ladder.  Exposes the GpuActorGroup attributes the GPU loop and the
    actor thread use (E, eps, episodes, inserted, ctr, step, reset_episodes).  (The
    reference runs one process per actor, ``main.py:50-54``; here a rank's actors are
    batched rows of these groups.)"""

    def __init__(self, groups: List["GpuActorGroup"]):
        self.groups = list(groups)
        self.E = sum(g.E for g in self.groups)
        self.eps = torch.cat([g.eps for g in self.groups])
        self.episodes = self.groups[0].episodes
        for g in self.groups[1:]:
            g.episodes = self.episodes          # one time-ordered episode list
        self.ctr = self.groups[0].ctr           # checkpointed RNG counter (group k's draws use their own seed)
        self._launched = False

    @property
    def inserted(self) -> int:
        return sum(g.inserted for g in self.groups)

    def step(self) -> int:
        if not self._launched:
            for g in self.groups:
                g.launch_policy()
            self._launched = True
        n = 0
        for g in self.groups:
            n += g.finish_step()
            g.launch_policy()
        return n

    def reset_episodes(self) -> None:
        for g in self.groups:
            ev = getattr(g, "_pending", None)
            if ev is not None:       # a launched inference: let it land, drop its result
                ev.synchronize()
                g._pending = None
            g.reset_episodes()
        self._launched = False


def ladder_slice(cfg, E: int, rank: int, world: int, total_actors: Optional[int] = None) -> List[float]:
    """The epsilons of rank ``rank``'s E envs: actors ``i * world + rank`` of the global
    ladder over ``total_actors`` (default E * world) actors, interleaved across ranks."""
    a = cfg.Actor
    total = max(int(total_actors or E * world), E * world)
    ladder = epsilon_ladder(total, a.epsilon, a.alpha)
    return [ladder[i * world + rank] for i in range(E)]


class GraphActorGroup(GpuActorGroup):
    """Actor group for ``GraphLearner`` networks (IMPALA-deep): the
    frame stacks are gathered from the replay ring on the device, the actor's own
    network copy (refreshed every ``Q_network_sync_freq`` steps) runs in bf16, and
    epsilon-greedy is drawn on the device; one small D2H copy per step."""

    def __init__(self, cfg, learner, replay, env, num_envs: int, global_offset: int = 0,
                 total_actors: Optional[int] = None, seed: int = 0, rank: int = 0, world: int = 1):
        import copy
        self.cfg, self.learner, self.replay, self.env = cfg, learner, replay, env
        self.E, self.C, self.A = int(num_envs), learner.C, learner.A
        d = learner.device
        self.device = d
        a = cfg.Actor
        self.eps = torch.tensor(ladder_slice(cfg, self.E, rank, world, total_actors), dtype=torch.float32, device=d)
        self.gen = torch.Generator(device=d)
        self.gen.manual_seed(int(seed) * 7919 + global_offset)
        self.slots = torch.zeros(self.E, self.C, dtype=torch.int32, device=d)
        self.net = copy.deepcopy(learner.Q)
        for p in self.net.parameters():
            p.requires_grad_(False)
        self.q_host = torch.zeros(self.E, self.A, dtype=torch.float32)
        self.a_host = torch.zeros(self.E, dtype=torch.int64)
        if d.type == "cuda":
            self.q_host, self.a_host = self.q_host.pin_memory(), self.a_host.pin_memory()
        self.builder = make_nstep_builder(self.E, a.num_steps, a.gamma, (self.C,), np.int64, env_id_offset=global_offset)
        self.global_offset = global_offset
        self.payload = None
        self.t = 0
        self.episodes = []
        self.inserted = 0
        self._init_stream()

    def _copy_params(self) -> None:
        with torch.no_grad():
            for dst, src in zip(self.net.parameters(), self.learner.Q.parameters()):
                dst.copy_(src)

    def _policy(self, payload: np.ndarray):
        self.slots.copy_(torch.from_numpy((payload % self.replay.F).astype(np.int32)), non_blocking=True)
        frames = self.replay.gather_frames(self.slots)
        q = self.learner.actor_forward(self.net, frames)
        greedy = q.argmax(dim=1)
        u = torch.rand(self.E, generator=self.gen, device=self.device)
        rand_a = torch.randint(0, self.A, (self.E,), generator=self.gen, device=self.device)
        act = torch.where(u < self.eps, rand_a, greedy)
        self.q_host.copy_(q, non_blocking=True)
        self.a_host.copy_(act, non_blocking=True)


class ImpalaActorGroup(GpuActorGroup):
    """Actor group for the hand-written IMPALA learner (``FusedImpalaLearner``):
    the trunk runs on the learner's csrc/impala.hip kernels over the group's E
    frame stacks (read straight from the replay ring by slot) with the group's
    own parameter slot, then the ``actor_head`` kernel draws epsilon-greedy."""

    def __init__(self, cfg, learner, replay, env, num_envs: int, global_offset: int = 0,
                 total_actors: Optional[int] = None, seed: int = 0, rank: int = 0, world: int = 1):
        self.cfg, self.learner, self.replay, self.env = cfg, learner, replay, env
        self.E, self.C, self.A = int(num_envs), learner.C, learner.A
        self.ops = learner.ops
        d = learner.device
        self.device = d
        a = cfg.Actor
        self.eps = torch.tensor(ladder_slice(cfg, self.E, rank, world, total_actors), dtype=torch.float32, device=d)
        self.h_lo = None
        self.seed = int(seed) * 7919 + global_offset
        self.ctr = torch.zeros(1, dtype=torch.int64, device=d)
        self.slots = torch.zeros(self.E, self.C, dtype=torch.int32, device=d)
        self.ps = learner.actor_param_set()
        self.bufs = learner.alloc_trunk(self.E)
        self.q = torch.zeros(self.E, self.A, dtype=torch.float32, device=d)
        self.act = torch.zeros(self.E, dtype=torch.int32, device=d)
        self.q_host = torch.zeros(self.E, self.A, dtype=torch.float32)
        self.a_host = torch.zeros(self.E, dtype=torch.int32)
        if d.type == "cuda":
            self.q_host, self.a_host = self.q_host.pin_memory(), self.a_host.pin_memory()
        self.builder = make_nstep_builder(self.E, a.num_steps, a.gamma, (self.C,), np.int64, env_id_offset=global_offset)
        self.global_offset = global_offset
        self.payload = None
        self.t = 0
        self.episodes = []
        self.inserted = 0
        self._init_stream()

    def _copy_params(self) -> None:
        self.learner.refresh_param_set(self.ps)

    def _policy(self, payload: np.ndarray):
        self.slots.copy_(torch.from_numpy((payload % self.replay.F).astype(np.int32)), non_blocking=True)
        h = self.learner.trunk_forward(self.slots, self.ps, self.bufs)
        heads = {k: self.ps["V"][k] for k in ("wv", "bv", "wa", "ba")}
        self.ops.actor_head(h, heads, self.eps, self.ctr, self.seed, self.q, self.act, H_lo=self.bufs.get("h_lo"))
        self.ctr += 1
        self.q_host.copy_(self.q, non_blocking=True)
        self.a_host.copy_(self.act, non_blocking=True)


def make_gpu_actor_group(cfg, learner, replay, num_envs: int, rank: int = 0, world: int = 1,
                         seed: int = 0, pipeline: int = 1):
    """The rank's actor group; ``pipeline`` K > 1 (NatureCNN learners on a GPU): K groups
    of num_envs / K envs stepped in turn (PipelinedActorGroups)."""
    from ..envs.vector_envs import make_vec_env
    total = max(cfg.Actor.num_actors, num_envs * world)
    K = int(pipeline)
    if K > 1 and num_envs % K == 0 and num_envs // K >= 1 and getattr(learner, "kind", "") not in ("graph", "impala"):
        h = num_envs // K
        eps_all = ladder_slice(cfg, num_envs, rank, world, total)
        groups = []
        for k in range(K):
            env = make_vec_env(cfg.env_backend, cfg.env_conf.name, h, cfg.env_conf.action_dim,
                               seed=seed + 1000 * rank + 100003 * k)
            g = GpuActorGroup(cfg, learner, replay, env, h, global_offset=rank * num_envs + k * h,
                              total_actors=total, seed=seed + rank, rank=rank, world=world)
            g.eps = torch.tensor(eps_all[k * h:(k + 1) * h], dtype=torch.float32, device=learner.device)
            groups.append(g)
        return PipelinedActorGroups(groups)
    env = make_vec_env(cfg.env_backend, cfg.env_conf.name, num_envs, cfg.env_conf.action_dim,
                       seed=seed + 1000 * rank)
    kind = getattr(learner, "kind", "")
    cls = {"graph": GraphActorGroup, "impala": ImpalaActorGroup}.get(kind, GpuActorGroup)
    return cls(cfg, learner, replay, env, num_envs, global_offset=rank * num_envs,
               total_actors=total, seed=seed + rank, rank=rank, world=world)
