"""Dueling Q-networks (PyTorch reference implementations).

These modules are the *semantic* definition of every network family and the
CPU / oracle path.  The MI355X training paths (``learner/fused_learner.py``
for the NatureCNN, ``learner/impala_learner.py`` for IMPALA-deep) run the same
math through hand-written HIP kernels on a flat parameter buffer
(``models/flat_params.py``) and convert to/from these modules' ``state_dict``
so checkpoints stay interchangeable.

``DuellingDQN`` keeps the reference key names exactly
(``duelling_network.py:8-19``: ``layer1.0.weight`` ... ``advantage.bias``)
so ``torch.load(p)['Q_state']`` checkpoints load unchanged, and keeps the
``forward -> (value, advantage, q)`` contract (``duelling_network.py:28``).

Deliberate deviation: the advantage mean is taken per
sample (``adv.mean(1)``), not over the whole batch tensor as in
``duelling_network.py:27``.
"""
from __future__ import annotations

from typing import Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F


def dueling_combine(value: torch.Tensor, adv: torch.Tensor) -> torch.Tensor:
    """q = v + a - mean_a(a), per sample."""
    return value + adv - adv.mean(dim=1, keepdim=True)


class _ObsScale(nn.Module):
    def __init__(self, scale: float):
        super().__init__()
        self.scale = float(scale)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if x.dtype == torch.uint8:
            return x.float() * self.scale
        return x.float() if not x.is_floating_point() else x


class DuellingDQN(nn.Module):
    """Dueling NatureCNN: 3 conv + two 512-wide streams + value/advantage heads.

    ``conv1_channels`` = 64 matches the reference checkpoint layout
    (``duelling_network.py:8``); 32 gives the Nature/dueling-paper variant.
    uint8 input is scaled by ``obs_scale`` (1/255 by default); float input is
    used as given (the reference feeds raw 0..255 floats).
    """

    def __init__(self, state_shape: Sequence[int], action_dim: int,
                 conv1_channels: int = 64, obs_scale: float = 1.0 / 255.0):
        super().__init__()
        self.input_shape = tuple(state_shape)
        self.action_dim = int(action_dim)
        c = int(state_shape[0])
        c1 = int(conv1_channels)
        self.pre = _ObsScale(obs_scale)
        self.layer1 = nn.Sequential(nn.Conv2d(c, c1, 8, stride=4), nn.ReLU())
        self.layer2 = nn.Sequential(nn.Conv2d(c1, 64, 4, stride=2), nn.ReLU())
        self.layer3 = nn.Sequential(nn.Conv2d(64, 64, 3, stride=1), nn.ReLU())
        self.value_stream_layer = nn.Sequential(nn.Linear(64 * 7 * 7, 512), nn.ReLU())
        self.advantage_stream_layer = nn.Sequential(nn.Linear(64 * 7 * 7, 512), nn.ReLU())
        self.value = nn.Linear(512, 1)
        self.advantage = nn.Linear(512, self.action_dim)

    def features(self, x: torch.Tensor) -> torch.Tensor:
        x = self.pre(x)
        x = self.layer3(self.layer2(self.layer1(x)))
        return x.reshape(x.shape[0], -1)

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        h = self.features(x)
        value = self.value(self.value_stream_layer(h))
        advantage = self.advantage(self.advantage_stream_layer(h))
        return value, advantage, dueling_combine(value, advantage)


class MLPDuellingDQN(nn.Module):
    """Dueling MLP for low-dimensional states (CartPole config)."""

    def __init__(self, state_shape: Sequence[int], action_dim: int, hidden: int = 128):
        super().__init__()
        d = int(state_shape[0]) if len(state_shape) == 1 else int(torch.tensor(state_shape).prod())
        self.input_shape = tuple(state_shape)
        self.action_dim = int(action_dim)
        self.layer1 = nn.Sequential(nn.Linear(d, hidden), nn.ReLU())
        self.value_stream_layer = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU())
        self.advantage_stream_layer = nn.Sequential(nn.Linear(hidden, hidden), nn.ReLU())
        self.value = nn.Linear(hidden, 1)
        self.advantage = nn.Linear(hidden, self.action_dim)

    def forward(self, x: torch.Tensor):
        h = self.layer1(x.float().reshape(x.shape[0], -1))
        value = self.value(self.value_stream_layer(h))
        advantage = self.advantage(self.advantage_stream_layer(h))
        return value, advantage, dueling_combine(value, advantage)


class _ResBlock(nn.Module):
    def __init__(self, ch: int):
        super().__init__()
        self.conv0 = nn.Conv2d(ch, ch, 3, padding=1)
        self.conv1 = nn.Conv2d(ch, ch, 3, padding=1)

    def forward(self, x):
        y = self.conv0(F.relu(x))
        y = self.conv1(F.relu(y))
        return x + y


class _ImpalaStack(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, 3, padding=1)
        self.res0 = _ResBlock(cout)
        self.res1 = _ResBlock(cout)

    def forward(self, x):
        x = self.conv(x)
        x = F.max_pool2d(x, 3, stride=2, padding=1)
        return self.res1(self.res0(x))


class ImpalaDuellingDQN(nn.Module):
    """IMPALA-deep ResNet trunk (16/32/32 channels) with dueling heads.

    BASELINE.json config 5 ("IMPALA-deep ResNet dueling Q-net on Atari"); not
    present in the reference.
    """

    def __init__(self, state_shape: Sequence[int], action_dim: int,
                 channels: Sequence[int] = (16, 32, 32), hidden: int = 256,
                 obs_scale: float = 1.0 / 255.0):
        super().__init__()
        c, h, w = (int(s) for s in state_shape)
        self.input_shape = (c, h, w)
        self.action_dim = int(action_dim)
        self.pre = _ObsScale(obs_scale)
        stacks = []
        cin = c
        for ch in channels:
            stacks.append(_ImpalaStack(cin, ch))
            cin = ch
            h, w = (h + 1) // 2, (w + 1) // 2
        self.stacks = nn.ModuleList(stacks)
        flat = cin * h * w
        self.value_stream_layer = nn.Sequential(nn.Linear(flat, hidden), nn.ReLU())
        self.advantage_stream_layer = nn.Sequential(nn.Linear(flat, hidden), nn.ReLU())
        self.value = nn.Linear(hidden, 1)
        self.advantage = nn.Linear(hidden, self.action_dim)

    def forward(self, x):
        x = self.pre(x)
        for s in self.stacks:
            x = s(x)
        hcat = F.relu(x).reshape(x.shape[0], -1)
        value = self.value(self.value_stream_layer(hcat))
        advantage = self.advantage(self.advantage_stream_layer(hcat))
        return value, advantage, dueling_combine(value, advantage)


def build_network(kind: str, state_shape: Sequence[int], action_dim: int,
                  obs_scale: float = 1.0 / 255.0) -> nn.Module:
    if kind == "nature64":
        return DuellingDQN(state_shape, action_dim, conv1_channels=64, obs_scale=obs_scale)
    if kind == "nature32":
        return DuellingDQN(state_shape, action_dim, conv1_channels=32, obs_scale=obs_scale)
    if kind == "mlp":
        return MLPDuellingDQN(state_shape, action_dim)
    if kind == "impala":
        return ImpalaDuellingDQN(state_shape, action_dim, obs_scale=obs_scale)
    raise ValueError(f"unknown network kind {kind!r}")


REFERENCE_KEYS = (
    "layer1.0.weight", "layer1.0.bias", "layer2.0.weight", "layer2.0.bias",
    "layer3.0.weight", "layer3.0.bias",
    "value_stream_layer.0.weight", "value_stream_layer.0.bias",
    "advantage_stream_layer.0.weight", "advantage_stream_layer.0.bias",
    "value.weight", "value.bias", "advantage.weight", "advantage.bias",
)
