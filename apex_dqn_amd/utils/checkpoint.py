"""Checkpoint save / load.

Format preserved from the reference (``learner.py:18-23``):
``torch.load(path)['Q_state']`` is a ``DuellingDQN`` state_dict with the
reference key names.  The reference never saves (defect A28); here rank 0
saves that dict plus optional extras (``Q_target_state``,
``optimizer_state``, ``num_q_updates``, ``rng``, ``config``) that old loaders
ignore.  Loading always uses ``weights_only=True`` (no pickle execution).
"""
from __future__ import annotations

import os
from typing import Any, Dict, Optional

import torch


def save_checkpoint(path: str, q_state: Dict[str, torch.Tensor], **extras: Any) -> None:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    payload = {"Q_state": {k: v.detach().cpu().contiguous() for k, v in q_state.items()}}
    for k, v in extras.items():
        if v is not None:
            payload[k] = v
    tmp = path + ".tmp"
    torch.save(payload, tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint


def load_checkpoint(path: str) -> Optional[Dict[str, Any]]:
    """Return the checkpoint dict, or None (with the reference's warning)."""
    try:
        return torch.load(path, map_location="cpu", weights_only=True)
    except FileNotFoundError:
        print("WARNING: No trained model found. Training from scratch")
        return None
