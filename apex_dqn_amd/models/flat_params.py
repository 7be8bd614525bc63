"""Flat parameter buffer for the fused NatureCNN dueling network.

All parameters of the online network live in ONE contiguous fp32 buffer (in
the kernels' layouts), with a bf16 "compute copy" of the same layout that the
MFMA kernels read and the fused RMSprop kernel rewrites in the same pass.  The
gradient buffer has the identical layout, so the data-parallel all-reduce is
one flat collective and the optimizer is one multi-tensor kernel.

Conversion to/from the reference ``DuellingDQN`` ``state_dict``
(``duelling_network.py:8-19`` key names and shapes) is exact, so checkpoints
written by either side load on the other.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

ALIGN = 64  # elements (256 B): every segment starts 16-B aligned for dwordx4 access


def nature_segments(C: int, A: int, c1: int = 64) -> List[Tuple[str, Tuple[int, ...]]]:
    """Flat order: the small tensors (convs, heads) first, the 3.2 M-parameter fc layer
    last, so the fc weights are one contiguous suffix: the data-parallel exchange treats
    [0, wfc) and [wfc, end) as its two buckets and the single-rank step updates the fc
    suffix early (learner/fused_learner.py)."""
    return [
        ("w1", (c1, C, 8, 8)), ("b1", (c1,)),
        ("w2", (64, 4, 4, c1)), ("b2", (64,)),
        ("w3", (64, 3, 3, 64)), ("b3", (64,)),
        ("wv", (512,)), ("bv", (1,)),
        ("wa", (A, 512)), ("ba", (A,)),
        ("wfc", (1024, 3136)), ("bfc", (1024,)),
    ]


class FlatLayout:
    def __init__(self, segments):
        self.segments = list(segments)
        self.offsets: Dict[str, int] = {}
        self.shapes: Dict[str, Tuple[int, ...]] = {}
        off = 0
        for name, shape in self.segments:
            off = (off + ALIGN - 1) // ALIGN * ALIGN
            self.offsets[name] = off
            self.shapes[name] = tuple(shape)
            n = 1
            for s in shape:
                n *= s
            off += n
        self.numel = (off + ALIGN - 1) // ALIGN * ALIGN

    def views(self, flat: torch.Tensor) -> Dict[str, torch.Tensor]:
        out = {}
        for name, shape in self.segments:
            n = 1
            for s in shape:
                n *= s
            o = self.offsets[name]
            out[name] = flat[o:o + n].view(shape)
        return out


def flat_to_reference_state(v: Dict[str, torch.Tensor], c1: int = 64) -> "OrderedDict[str, torch.Tensor]":
    """Engine layout -> reference DuellingDQN state_dict (fp32, CPU).

    ``c1`` < 64: the engine keeps conv1 zero-padded to 64 filters (see
    ``reference_state_to_flat``); only the first ``c1`` filters are exported."""
    def fc_cols_to_chw(w):  # (512, 3136[h,w,c]) -> (512, 3136[c,h,w])
        return w.reshape(-1, 7, 7, 64).permute(0, 3, 1, 2).reshape(w.shape[0], 3136)

    sd = OrderedDict()
    sd["layer1.0.weight"] = v["w1"][:c1].clone()
    sd["layer1.0.bias"] = v["b1"][:c1].clone()
    sd["layer2.0.weight"] = v["w2"][..., :c1].permute(0, 3, 1, 2).contiguous()
    sd["layer2.0.bias"] = v["b2"].clone()
    sd["layer3.0.weight"] = v["w3"].permute(0, 3, 1, 2).contiguous()
    sd["layer3.0.bias"] = v["b3"].clone()
    sd["value_stream_layer.0.weight"] = fc_cols_to_chw(v["wfc"][:512]).contiguous()
    sd["value_stream_layer.0.bias"] = v["bfc"][:512].clone()
    sd["advantage_stream_layer.0.weight"] = fc_cols_to_chw(v["wfc"][512:]).contiguous()
    sd["advantage_stream_layer.0.bias"] = v["bfc"][512:].clone()
    sd["value.weight"] = v["wv"].view(1, 512).clone()
    sd["value.bias"] = v["bv"].clone()
    sd["advantage.weight"] = v["wa"].clone()
    sd["advantage.bias"] = v["ba"].clone()
    return OrderedDict((k, t.detach().float().cpu()) for k, t in sd.items())


def reference_state_to_flat(sd: Dict[str, torch.Tensor], v: Dict[str, torch.Tensor]) -> None:
    """Reference state_dict -> engine layout (in place into the views ``v``).

    A 32-filter conv1 (Nature DQN, ``network = "nature32"``) is stored
    zero-padded to the engine's 64 filters: padded filters and the matching
    conv2 input channels are exact zeros, so the padded activations are
    ReLU(0) = 0, their gradients are exactly 0, and RMSprop (update ~ g) keeps
    them at 0 -- the same math as the 32-filter net, run by the 64-filter kernels."""
    def fc_cols_to_hwc(w):
        return w.reshape(-1, 64, 7, 7).permute(0, 2, 3, 1).reshape(w.shape[0], 3136)

    with torch.no_grad():
        c1 = sd["layer1.0.weight"].shape[0]
        if c1 != v["w1"].shape[0]:
            for k in ("w1", "b1", "w2"):
                v[k].zero_()
        v["w1"][:c1].copy_(sd["layer1.0.weight"])
        v["b1"][:c1].copy_(sd["layer1.0.bias"])
        v["w2"][..., :c1].copy_(sd["layer2.0.weight"].permute(0, 2, 3, 1))
        v["b2"].copy_(sd["layer2.0.bias"])
        v["w3"].copy_(sd["layer3.0.weight"].permute(0, 2, 3, 1))
        v["b3"].copy_(sd["layer3.0.bias"])
        v["wfc"][:512].copy_(fc_cols_to_hwc(sd["value_stream_layer.0.weight"]))
        v["bfc"][:512].copy_(sd["value_stream_layer.0.bias"])
        v["wfc"][512:].copy_(fc_cols_to_hwc(sd["advantage_stream_layer.0.weight"]))
        v["bfc"][512:].copy_(sd["advantage_stream_layer.0.bias"])
        v["wv"].copy_(sd["value.weight"].reshape(512))
        v["bv"].copy_(sd["value.bias"])
        v["wa"].copy_(sd["advantage.weight"])
        v["ba"].copy_(sd["advantage.bias"])
