"""Kernel-path switches: ONE registry.

Every alternative kernel path that survived as an A/B knob lives here with its
measured winner as the default (the measurements are cited per field; the history is
in docs/PERF_NOTES.md).  Production code reads ``SW.<name>``; tests flip a path with
``monkeypatch.setattr(SW, name, value)``; experiments override from the environment
with ONE variable::

    APEX_SWITCHES="conv2_img=0,wg_rows3=384" python bench.py

``bench.py`` prints every non-default value in its JSON (``switches``), so a number
measured off the defaults is labelled as such.
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass
from typing import Any, Dict


@dataclass
class Switches:
    # conv2 forward on the image-resident kernel (csrc/conv2_img.hip) instead of the generic
    # implicit GEMM (bf16 learner without the fused conv1 -> conv2 kernel, actors)
    conv2_img: bool = True
    # split conv2 forward: weights packed into per-lane fragment order by the launcher
    # (76.2 -> 71.0 us at 1536 images, profiles/r2_split_conv2_packed_fwd.jsonl)
    c2f_pack: bool = True
    # conv1 -> conv2 forward fused with y1 in LDS (csrc/conv12_fused.hip), split mode
    conv12_fused: bool = True
    # conv3 fused into the conv1 -> conv2 kernel (y2 read from LDS; csrc/conv12_fused.hip) for
    # launches of at most this many images (0: never).  With its weights in coalesced C3F
    # fragments (written by the optimizer) and its biases loaded ahead, the fused conv3 takes
    # ~3.7 k cycles per image and wins at every size: 512 rows 2,733-2,740 vs 2,678-2,692
    # fp32 updates/s (bf16 4,523-4,529 vs 4,433-4,451), emulated W = 8 157.1-157.3 vs
    # 163.1-169.7 us, W = 4 192.7-193.5 vs 198.1-202.9 us (profiles/r6_ab_conv123_fused_c3f.txt;
    # with the weights read from OHWI rows it lost at 512 rows, r6_ab_conv123_fused.txt)
    conv123_max_images: int = 1 << 20
    # the fused forward's one-plane variant for the bf16 learner (4,105 vs 3,790 steps/s,
    # profiles/r3_ab_conv12_bf16_fused_4105_vs_3790.txt)
    conv12_bf16: bool = True
    # image-resident conv3 / conv2 data gradients (csrc/conv2_img.hip)
    conv3_dgrad_img: bool = True
    conv2_dgrad_img: bool = True
    # split conv2 data gradient: one workgroup per (image, stride-parity class) up to this
    # many images (0: never), per image above it
    conv2_dgrad_cls_max: int = 256
    # the optimizer + sample launch stores the fused forward's online weight fragments
    # (+0.5-1 %, profiles/r3_ab_optimizer_frag_stores_*.txt)
    opt_frags: bool = True
    # the fc layer's split-K epilogue runs inside the DDQN head launch
    fc_epi_in_head: bool = True
    # single-rank step: the weight gradients (fc + heads + priority write-back, conv3,
    # conv2) on a second stream beside the data-gradient chain (graph branches)
    bwd_branches: bool = True
    # the GPU actors' fc forward: this K split (0: the chip-filling split of the learner)
    actor_fc_ksplit: int = 4
    # single-rank branched backward: the fc weight gradient (+ head wgrad + priorities) on
    # the main stream right after the fc dgrad, the branch forking after it ("on"), on the
    # branch beside the dgrad chain ("off"), "auto": main for fp32-class at >= 256 rows
    fc_wgrad_main: str = "auto"
    # cap on the fc forward's K splits (0: fill the chip, ops/fused_ops.py fc_fwd); the DDQN
    # head sums the splits' partials (the deferred epilogue)
    fc_ksplit_max: int = 0
    # device-side image work queues in the persistent kernels: "auto" = only where RCCL's
    # kernels may hold CUs (the DP conv backward at world > 1), "on" / "off" force them
    work_queue: str = "auto"
    # split-K reduction rows per workgroup of the conv3 / conv2 weight gradients (0: the
    # tuned defaults in ops/conv.py)
    wg_rows3: int = 0
    wg_rows2: int = 0
    # IMPALA weight gradients: workgroups per conv and the partial-slab cap (floats)
    impala_wg_target: int = 512
    impala_slab_cap: int = 8 << 20
    # IMPALA bf16 fused residual block rows per band at 16 ch x 42 (swept: 21 777, 14 786, 11 778)
    resblock_r16: int = 14
    # IMPALA stack 1: the max-pool backward inside the ring conv's weight-gradient staging
    impala_pool_wgrad: bool = True
    # IMPALA split kernels' launch shapes "key=value;..." ('' = the defaults of
    # ops/impala.py _split_bands): rb<C>x<H>=R (residual block rows), sc<cin>x<cout>x<H>p<pool>=R
    # (conv rows), wg<cin>x<cout>x<H>=R/threads (weight-gradient variant), wt<cin>x<cout>x<H>=N
    # (weight-gradient workgroup target)
    isplit_bands: str = ""
    # DP step (learner/dp_step.py): the sharded update's fc weight gradient on the branch
    # right behind the factor exchange (True) or on main after conv1's weight gradient
    # (False: emulated W = 8 160.5-162.1 vs 178.6-180.7 us, W = 4 201.5-202.0 vs
    # 199.7-203.6 -- the branch becomes the critical chain; profiles/r6_ab_dp_switches.txt)
    dp_fc_shard_branch: bool = False
    # DP step: one main-stream event for the branch's conv3 + conv2 weight gradients (one
    # cross-queue edge fewer on the critical path; with the fused conv3: emulated W = 4
    # 195.0 / 195.1 vs 197.2 / 197.6 us, W = 8 164.1 / 163.2 vs 170.0 / 166.2,
    # profiles/r6_ab_misc.txt)
    dp_branch_one_wait: bool = True
    # DP step, sharded update with the factored exchange: this rank's fc weight-gradient rows
    # as split-K partials of this many reduction rows each, reduced in conv1's finalize
    # launch (0: one launch over all rows writing the gradient itself; -1: 256 at 8+ ranks,
    # else 128 -- emulated W = 8 157.3 vs 159.0 us, W = 4 193.9 vs 190.5 at 256,
    # profiles/r6_ab_dp_fc_split_rows.txt)
    dp_fc_split_rows: int = -1
    # DP step, sharded update: the [w2, wfc) bucket's clip-norm partials on the branch and
    # conv1's bucket summed inside the optimizer launch (no norm launch on main; emulated W =
    # 8 with the fc gradient on main: 160.5-162.1 us vs 166-169 before)
    dp_norm_split: bool = True

    @classmethod
    def from_env(cls, spec: str = None) -> "Switches":
        sw = cls()
        spec = os.environ.get("APEX_SWITCHES", "") if spec is None else spec
        for item in spec.split(","):
            item = item.strip()
            if not item:
                continue
            if "=" not in item:
                raise ValueError(f"APEX_SWITCHES item must be name=value, got {item!r}")
            k, v = item.split("=", 1)
            f = {f.name: f for f in dataclasses.fields(cls)}.get(k)
            if f is None:
                raise ValueError(f"unknown kernel switch {k!r}")
            setattr(sw, k, _parse(f.type, v))
        return sw

    def non_default(self) -> Dict[str, Any]:
        d = Switches()
        return {f.name: getattr(self, f.name) for f in dataclasses.fields(self)
                if getattr(self, f.name) != getattr(d, f.name)}


def _parse(typ, v: str):
    t = typ if isinstance(typ, str) else typ.__name__
    if t == "bool":
        return v.lower() not in ("0", "false", "off", "no")
    if t == "int":
        return int(v)
    return v


SW = Switches.from_env()
