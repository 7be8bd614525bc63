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
from typing import Any, Dict, List, Optional, Sequence, Tuple

import torch

# (segment name, flat offset, element count) of a learner's flat parameter buffer
Segments = Sequence[Tuple[str, int, int]]


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


def pack_flat_state(segments: Segments, **flats: torch.Tensor) -> Dict[str, Any]:
    """Per-parameter state kept in a flat buffer (RMSprop's ``rms_v`` / ``rms_m``), saved
    per named segment with the layout it came from: a later engine whose flat layout
    orders or pads the segments differently still restores every value to its parameter
    (:func:`unpack_flat_state`)."""
    out: Dict[str, Any] = {"layout": [[str(n), int(o), int(k)] for n, o, k in segments]}
    for key, flat in flats.items():
        f = flat.detach().cpu()
        out[key] = {n: f[o:o + k].clone() for n, o, k in segments}
    return out


def unpack_flat_state(opt: Any, segments: Segments, untagged_network: Optional[str] = None,
                      network: Optional[str] = None, **dsts: torch.Tensor) -> bool:
    """Restore :func:`pack_flat_state` output into the flat buffers ``dsts`` of the current
    layout ``segments``.  State whose segments do not match by name and size is refused
    (returns False, with a warning, buffers untouched): the caller then starts the optimizer
    state fresh rather than misaligned.

    Untagged state -- an older checkpoint's raw flat vectors, written before the tag
    existed -- is accepted when it was saved by the same network (``untagged_network``,
    from the checkpoint's config, equals ``network``) and every vector has exactly the
    current flat buffer's length: this engine's flat layout (``models/flat_params.py``
    nature segments and their padding) has not changed since, so the vector is the buffer.
    Dropping it instead would restart centered RMSprop at v = m = 0 -- a several-times
    larger step on every parameter in mid-training."""
    if not isinstance(opt, dict) or not dsts:
        return False
    if "layout" not in opt:
        raw = all(isinstance(opt.get(key), torch.Tensor) and opt[key].numel() == dst.numel()
                  for key, dst in dsts.items())
        if raw and network is not None and untagged_network == network:
            for key, dst in dsts.items():
                dst.copy_(opt[key].reshape(-1).to(dst.dtype))
            print("WARNING: checkpoint optimizer state has no layout tag (an older flat vector); restored by "
                  "length (same network, %d values)" % next(iter(dsts.values())).numel())
            return True
        print("WARNING: checkpoint optimizer state has no layout tag (an older flat vector) and does not match "
              "this network's flat buffer; RMSprop state not restored (starts fresh)")
        return False
    saved = {str(n): int(k) for n, _, k in opt["layout"]}
    cur = {n: int(k) for n, _, k in segments}
    if saved != cur or any(not isinstance(opt.get(key), dict) for key in dsts):
        print("WARNING: checkpoint optimizer state layout does not match this network; "
              "RMSprop state not restored (starts fresh)")
        return False
    for key, dst in dsts.items():
        src = opt[key]
        for n, o, k in segments:
            dst[o:o + k].copy_(src[n].reshape(-1).to(dst.dtype))
    return True


def checkpoint_network(ck: Dict[str, Any]) -> Optional[str]:
    """The network a checkpoint was saved by (its ``config``), or None."""
    c = ck.get("config") if isinstance(ck, dict) else None
    if not isinstance(c, dict):
        return None
    rt = c.get("Runtime") or {}
    net = rt.get("network", "auto")
    if net == "auto":
        shape = (c.get("env_conf") or {}).get("state_shape") or []
        net = "nature64" if len(shape) == 3 else "mlp"
    return str(net)


def layout_segments(layout) -> List[Tuple[str, int, int]]:
    """Segments of a ``models.flat_params.FlatLayout``."""
    out = []
    for name, shape in layout.segments:
        n = 1
        for d in shape:
            n *= d
        out.append((name, layout.offsets[name], n))
    return out


REFERENCE_OBS_SCALE = 1.0   # the reference feeds raw 0..255 floats (actor.py:117-119,161, learner.py:37)


def checkpoint_obs_scale(ck: Dict[str, Any]) -> float:
    """Input scale the checkpoint's weights were trained with: ``config`` holds it
    for checkpoints written here; a checkpoint without ``config`` comes from the
    reference, whose networks see raw 0..255 pixels."""
    cfg = ck.get("config")
    if isinstance(cfg, dict):
        rt = cfg.get("Runtime") or {}
        if "obs_scale" in rt:
            return float(rt["obs_scale"])
    return REFERENCE_OBS_SCALE


def adopt_obs_scale(ck: Dict[str, Any], runtime_conf) -> bool:
    """Set ``runtime_conf.obs_scale`` to the checkpoint's input scale (with a loud
    warning when it changes); returns True if it changed."""
    new = checkpoint_obs_scale(ck)
    old = float(runtime_conf.obs_scale)
    if abs(new - old) <= 1e-12 * max(abs(old), 1.0):
        return False
    origin = "reference-format checkpoint (no config): raw 0..255 pixel input" if "config" not in ck \
        else "checkpoint config"
    print(f"WARNING: Runtime.obs_scale {old:g} -> {new:g} from the {origin}; the loaded weights expect it")
    runtime_conf.obs_scale = new
    return True

