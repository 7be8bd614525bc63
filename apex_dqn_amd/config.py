"""Typed configuration for the Ape-X engine.

Accepts the reference ``parameters.json`` schema verbatim (four sections:
``env_conf``, ``Actor``, ``Learner``, ``Replay_Memory`` --
reference ``parameters.json:1-34``, consumed at ``main.py:29-33``) and adds an
optional ``Runtime`` section for everything the reference hard-codes
(learner T at ``main.py:46``, optimizer at ``learner.py:26``, the
ExperienceBuffer gamma at ``actor.py:25``) or lacks entirely (device, world
size, checkpointing, network variant, env backend).

``--set Section.key=value`` overrides are parsed with JSON semantics
(``--set Learner.replay_sample_size=512``,
``--set env_conf.state_shape=[4,84,84]``).
"""
from __future__ import annotations

import copy
import dataclasses
import json
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np


@dataclass
class EnvConf:
    state_shape: List[int] = field(default_factory=lambda: [1, 84, 84])
    action_dim: int = 4
    name: str = "RiverraidNoFrameskip-v4"


@dataclass
class ActorConf:
    num_actors: int = 5
    T: int = 50000
    num_steps: int = 3
    epsilon: float = 0.4
    alpha: float = 7.0
    gamma: float = 0.99
    n_step_transition_batch_size: int = 5
    Q_network_sync_freq: int = 500


@dataclass
class LearnerConf:
    remove_old_xp_freq: int = 100
    q_target_sync_freq: int = 2500
    min_replay_mem_size: int = 20000
    replay_sample_size: int = 32
    load_saved_state: Any = False


@dataclass
class ReplayConf:
    soft_capacity: int = 100000
    priority_exponent: float = 0.6
    importance_sampling_exponent: float = 0.4


@dataclass
class RuntimeConf:
    """Extension section (not present in the reference; all optional)."""

    device: str = "auto"            # "auto" | "cpu" | "cuda"
    world_size: int = 1
    dtype: str = "fp32"             # GPU learner precision: "fp32" (the reference's; split hi/lo bf16
                                    # operands, 3 MFMAs per product) | "bf16" (bf16 operands)
    seed: int = 0
    learner_T: int = 500000         # reference hard-codes 500000 (main.py:46)
    network: str = "auto"           # "auto" | "nature64" | "nature32" | "mlp" | "impala"
    env_backend: str = "auto"       # "auto" | "synthetic" | "cartpole" | "ale" | "fake_ale" | "fake_ale_target"
    frame_stack: Optional[int] = None  # defaults to state_shape[0]
    actors_per_rank: Optional[int] = None  # defaults to num_actors / world_size
    obs_scale: float = 1.0 / 255.0  # uint8 -> float scale fed to conv nets
    # optimizer: centered RMSprop as in the Ape-X paper (reference passes the
    # decay 0.95 as weight_decay by mistake, learner.py:26).
    lr: float = 0.00025 / 4
    rms_decay: float = 0.95
    rms_eps: float = 1.5e-7
    centered_rmsprop: bool = True
    grad_clip: float = 40.0
    loss: str = "huber"             # "huber" | "mse" (0.5*delta^2, reference learner.py:48)
    huber_delta: float = 1.0
    priority_eps: float = 1e-6      # priority floor: leaves hold (|delta| + priority_eps)^alpha
    use_is_weights: bool = True
    is_normalise: str = "batch_max"  # IS weights (N P(i))^-beta divided by their max over the sampled batch
                                    # ("batch_max", the PER / Ape-X papers' 1 / max_i w_i; with DP the global
                                    # batch) or over the whole replay ("global_min": (p / p_min)^-beta, which
                                    # shrinks every update when a few priorities sit at the floor)
    ckpt_dir: Optional[str] = None
    ckpt_freq: int = 0              # learner steps between checkpoints (0 = off)
    metrics_path: Optional[str] = None
    log_every: int = 100
    param_publish_freq: int = 1     # learner steps between param publishes to actors
    use_hip_kernels: bool = True    # GPU path: hand-written HIP kernels
    use_graphs: bool = True         # GPU path: capture the learner step in a HIP graph
    profile_phases: bool = False    # at every log interval, time one eager step per phase (CUDA events)
    episode_lines_per_log: int = 4  # reference-format episode console lines per log interval (rank 0)
    torch_profile_dir: Optional[str] = None  # torch.profiler (ROCm activities) trace of a few steps
    torch_profile_start: int = 50   # first profiled learner step
    torch_profile_steps: int = 5
    resume: bool = True             # continue from ckpt_dir/checkpoint.pt when it exists (restarts)
    allreduce_dtype: str = "fp32"   # DP gradient all-reduce payload: "fp32" (exact) | "bf16" (half the bytes)
    presample: bool = True          # draw step t+1's batch at the end of step t (fused learner; on the HIP
                                    # backend inside the optimizer launch)
    graph_steps: int = 20           # learner updates per HIP-graph launch in learner.steps(n) (single
                                    # rank and DP alike: the DP step's collectives are captured too;
                                    # divides the default eviction cadence; 20 vs 10: 2,732 / 2,726 vs
                                    # 2,703 / 2,684 steps/s at 20 / 5, 2,729 / 2,744 vs 2,718 / 2,717 at
                                    # 200 / 20, profiles/r6_ab_graph_steps.txt; 10 vs 4: 3505 vs 3472)
    actor_learner_ratio: float = 0.0  # in-process actor steps per learner step (0 = separate)
    replay_capacity: Optional[int] = None  # physical capacity, global over the ranks' shards
                                           # (default: soft_capacity * 1.25 + 1024)
    heartbeat_timeout: float = 60.0
    comm_backend: str = "native"    # DP collectives: "native" (parallel/rccl.py: own RCCL communicator on its
                                    # own comm stream; the step is one captured HIP graph) | "torch"
                                    # (torch.distributed process group; eager DP steps: its watchdog's
                                    # event cache is not capture-safe on this ROCm / torch build)
    force_dp: bool = False          # run the data-parallel step (collectives + sharded replay) even at
                                    # world 1 (needs an initialised process group; checks / overhead)
    batch_scope: str = "global"     # DP: "global" = Learner.replay_sample_size is the batch of ONE update
                                    # summed over all ranks (the reference's / Ape-X's update, learner.py:68:
                                    # strong scaling; each rank computes the rows of the global draw that fall
                                    # in its shard) | "per_rank" = every rank draws up to that many rows (a
                                    # W-rank update averages up to W x the batch: weak scaling)
    dp_batch_slack: float = 0.125   # global scope: rows a rank can hold beyond B/W, as a fraction of B/W (plus
                                    # 2): the draw takes exactly B strata while no shard holds more than
                                    # (rows - 2) / B of the total priority mass, fewer otherwise
    dp_fc_exchange: str = "auto"    # DP exchange of the fc layer's gradient: "allreduce" (the 1024 x 3136 fp32
                                    # gradient) | "factors" (all-gather every rank's dH / fc-input rows -- the
                                    # operands the kernels use -- and form the gradient of the whole global
                                    # batch on each rank: ~(B_total x 4160) values instead of 3.2 M, exact and
                                    # bit-identical across ranks) | "auto" (factors while 1 < W and W x rows
                                    # <= 1024)
    dp_rows_adaptive: bool = True   # global scope: grow the per-rank rows (and recapture the step) when a
                                    # shard's share of the priority mass outgrows them, checked at init and
                                    # at every eviction (learner/dp_step.py _fit_rows), so M stays B
    dp_shard_update: str = "auto"   # DP: the fc layer's optimizer (96 % of the parameters) sharded by output rows
                                    # over the ranks, the updated rows all-gathered (learner/dp_step.py):
                                    # "on" | "off" | "auto" (on at world > 1 when 1024 / (64 W) is whole)
    replica_check_every: int = 5000  # DP: learner steps between replica checksum checks (0 = off)
    step_timeout: float = 300.0     # GPU loop watchdog: seconds a queued learner chunk may take
    async_actors: bool = True       # GPU loop: the actor group steps on its own host thread
    actor_precision: str = "learner"  # GPU actor inference: "learner" (the learner's precision; fp32-class
                                      # split kernels with dtype fp32, as the reference's fp32 actors) |
                                      # "bf16" (hi planes only: faster, bf16-class q-values / priorities)
    actor_graph: bool = True        # GPU actors: the inference launches replayed as one HIP graph per step
                                    # (host launch overhead: ~0.13 ms per step for the eager launches)
    actor_pipeline: int = 2         # async GPU actors: the rank's envs as this many groups stepped in
                                    # turn, so one group's host env step overlaps another's inference
                                    # (actors/gpu_actor.py PipelinedActorGroups; 1 = one group)
    learner_stream_priority: bool = True   # async GPU actors: learner on a high-priority HIP stream
                                    # (runtime/actor_thread.py), concurrent with the learner


@dataclass
class ApexConfig:
    env_conf: EnvConf = field(default_factory=EnvConf)
    Actor: ActorConf = field(default_factory=ActorConf)
    Learner: LearnerConf = field(default_factory=LearnerConf)
    Replay_Memory: ReplayConf = field(default_factory=ReplayConf)
    Runtime: RuntimeConf = field(default_factory=RuntimeConf)

    # ------------------------------------------------------------------ io
    @classmethod
    def from_dict(cls, d: Dict[str, Any], strict: bool = False) -> "ApexConfig":
        sections = {
            "env_conf": EnvConf,
            "Actor": ActorConf,
            "Learner": LearnerConf,
            "Replay_Memory": ReplayConf,
            "Runtime": RuntimeConf,
        }
        kw = {}
        for name, klass in sections.items():
            raw = dict(d.get(name, {}) or {})
            known = {f.name for f in dataclasses.fields(klass)}
            unknown = set(raw) - known
            if unknown and strict:
                raise KeyError(f"unknown keys in section {name}: {sorted(unknown)}")
            kw[name] = klass(**{k: v for k, v in raw.items() if k in known})
        extra = set(d) - set(sections)
        if extra and strict:
            raise KeyError(f"unknown sections: {sorted(extra)}")
        cfg = cls(**kw)
        cfg.validate()
        return cfg

    @classmethod
    def load(cls, path: str, overrides: Sequence[str] = ()) -> "ApexConfig":
        with open(path, "r") as f:
            d = json.load(f)
        d = apply_overrides(d, overrides)
        return cls.from_dict(d)

    def to_dict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)

    def save(self, path: str) -> None:
        with open(path, "w") as f:
            json.dump(self.to_dict(), f, indent=2)

    # ------------------------------------------------------------ derived
    def validate(self) -> None:
        ss = self.env_conf.state_shape
        if not isinstance(ss, (list, tuple)) or len(ss) not in (1, 3):
            raise ValueError(f"env_conf.state_shape must be [C,H,W] or [D], got {ss}")
        if self.env_conf.action_dim < 1:
            raise ValueError("env_conf.action_dim must be >= 1")
        if self.Actor.num_actors < 1:
            raise ValueError("Actor.num_actors must be >= 1")
        if self.Actor.num_steps < 1:
            raise ValueError("Actor.num_steps must be >= 1")
        if not (0.0 <= self.Actor.gamma <= 1.0):
            raise ValueError("Actor.gamma must be in [0,1]")
        if self.Learner.replay_sample_size < 1:
            raise ValueError("Learner.replay_sample_size must be >= 1")
        if self.Runtime.world_size < 1:
            raise ValueError("Runtime.world_size must be >= 1")
        if self.Runtime.comm_backend not in ("torch", "native"):
            raise ValueError("Runtime.comm_backend must be 'torch' or 'native'")
        if int(self.Runtime.actor_pipeline) < 1:
            raise ValueError("Runtime.actor_pipeline must be >= 1")
        if self.Runtime.actor_precision not in ("learner", "bf16"):
            raise ValueError("Runtime.actor_precision must be 'learner' or 'bf16'")
        if self.Runtime.is_normalise not in ("batch_max", "global_min"):
            raise ValueError("Runtime.is_normalise must be 'batch_max' or 'global_min'")
        if self.Runtime.batch_scope not in ("global", "per_rank"):
            raise ValueError("Runtime.batch_scope must be 'global' or 'per_rank'")
        if not self.Runtime.dp_batch_slack >= 0.0:
            raise ValueError("Runtime.dp_batch_slack must be >= 0")
        if self.Runtime.dp_shard_update not in ("auto", "on", "off"):
            raise ValueError("Runtime.dp_shard_update must be 'auto', 'on' or 'off'")
        if self.Runtime.dp_fc_exchange not in ("auto", "factors", "allreduce"):
            raise ValueError("Runtime.dp_fc_exchange must be 'auto', 'factors' or 'allreduce'")
        if self.Runtime.loss not in ("huber", "mse"):
            raise ValueError("Runtime.loss must be 'huber' or 'mse'")
        net = self.network
        if net in ("nature64", "nature32", "impala") and len(ss) != 3:
            raise ValueError(f"network {net} needs an image state_shape [C,H,W], got {ss}")
        if net in ("nature64", "nature32") and tuple(ss[1:]) != (84, 84):
            raise ValueError(f"NatureCNN expects 84x84 frames, got {ss}")

    @property
    def network(self) -> str:
        if self.Runtime.network != "auto":
            return self.Runtime.network
        return "nature64" if len(self.env_conf.state_shape) == 3 else "mlp"

    @property
    def env_backend(self) -> str:
        if self.Runtime.env_backend != "auto":
            return self.Runtime.env_backend
        name = self.env_conf.name.lower()
        if "cartpole" in name:
            return "cartpole"
        if "synthetic" in name:
            return "synthetic"
        # Atari ids: use ALE when importable, otherwise a synthetic env of the same shape
        try:  # pragma: no cover - ale_py is not installed in this image
            import ale_py  # noqa: F401
            return "ale"
        except Exception:
            return "synthetic"

    @property
    def frame_stack(self) -> int:
        if self.Runtime.frame_stack is not None:
            return int(self.Runtime.frame_stack)
        ss = self.env_conf.state_shape
        return int(ss[0]) if len(ss) == 3 else 1

    @property
    def replay_capacity(self) -> int:
        if self.Runtime.replay_capacity is not None:
            return int(self.Runtime.replay_capacity)
        return int(self.Replay_Memory.soft_capacity * 1.25) + 1024

    def shard_capacity(self, world: int) -> Tuple[int, int]:
        """(soft, physical) transitions held by ONE of ``world`` replay shards: the
        global FIFO bound ``Replay_Memory.soft_capacity`` (``replay.py:71-80``) split
        evenly, ceil-rounded; the physical ring keeps the configured headroom."""
        w = max(int(world), 1)
        soft = -(-int(self.Replay_Memory.soft_capacity) // w)
        if self.Runtime.replay_capacity is not None:
            phys = -(-int(self.Runtime.replay_capacity) // w)
        else:
            phys = int(soft * 1.25) + 1024
        return soft, max(phys, soft)

    def dp_batch(self, world: int, dp: bool = True) -> Tuple[int, int]:
        """(rows per rank, cap on the global batch M) of a learner update on ``world``
        data-parallel ranks (``dp``: the sharded DP step runs, world > 1 or forced).

        * no DP: (B, B);
        * ``batch_scope = "per_rank"``: (B, W B) -- every rank draws up to B rows;
        * ``batch_scope = "global"``: one update takes B = ``replay_sample_size`` draws
          over all shards, as the reference's single learner (``learner.py:68``); rank r
          holds ceil(B / W (1 + dp_batch_slack)) + 2 rows (B at W = 1), enough for its
          share of the global draw while its shard carries at most (rows - 2) / B of
          the total mass (replay/gpu_replay.py ``enable_sharding``)."""
        B = int(self.Learner.replay_sample_size)
        W = max(int(world), 1)
        if not dp:
            return B, B
        if self.Runtime.batch_scope == "per_rank":
            return B, W * B
        if W == 1:
            return B, B
        rows = int(np.ceil(B / W * (1.0 + float(self.Runtime.dp_batch_slack)) - 1e-9)) + 2
        return min(rows, B + 2), B

    def copy(self) -> "ApexConfig":
        return copy.deepcopy(self)


def _parse_value(v: str) -> Any:
    try:
        return json.loads(v)
    except (json.JSONDecodeError, ValueError):
        low = v.lower()
        if low in ("true", "false"):
            return low == "true"
        return v


def apply_overrides(d: Dict[str, Any], overrides: Sequence[str]) -> Dict[str, Any]:
    """Apply ``Section.key=value`` overrides to a raw config dict."""
    d = copy.deepcopy(d)
    for ov in overrides or ():
        if "=" not in ov:
            raise ValueError(f"override must be Section.key=value, got {ov!r}")
        path, val = ov.split("=", 1)
        parts = path.split(".")
        if len(parts) != 2:
            raise ValueError(f"override path must be Section.key, got {path!r}")
        sec, key = parts
        d.setdefault(sec, {})[key] = _parse_value(val)
    return d


def epsilon_ladder(num_actors: int, epsilon: float = 0.4, alpha: float = 7.0) -> List[float]:
    """Per-actor exploration rates eps_i = eps^(1 + alpha*i/(N-1)).

    Reference ``actor.py:111-114`` divides by zero for N=1 (defect A13); a
    single actor gets the base epsilon here.
    """
    denom = max(num_actors - 1, 1)
    return [float(epsilon ** (1.0 + alpha * i / denom)) for i in range(num_actors)]
