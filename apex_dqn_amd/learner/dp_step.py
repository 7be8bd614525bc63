"""The data-parallel learner step of :class:`FusedNatureLearner` (one body for the
GPU -- two streams, captured in the step's HIP graph -- and the CPU gloo tests).

Reference: one learner, one update per sampled batch (``learner.py:54-57``,
``replay_sample_size`` at ``:68``).  Here W ranks take that update together: the
sharded replay draws ONE global batch (``replay/gpu_replay.py``), rank r computes the
rows that fell in its shard, and the gradient of the global batch is exchanged:

  main stream     fwd + head -> fc dgrad -> conv3 dgrad -> conv2 dgrad -> conv1 wgrad
                  -> finalize (conv1) -> [conv1 bucket all-reduce, inline] -> clip-norm
                  partials of the conv + head range -> clip + centered RMSprop + the
                  next batch's draw -> (sharded) all-gather of the updated fc rows
  branch stream   head wgrad + priorities, then
                    factors: pack (dH, X) rows -> all-gather       (1.2 MB / rank at W 8)
                    allreduce: fc wgrad -> all-reduce / reduce-scatter of the fc range
                  shard statistics all-gather; conv3 wgrad; conv2 wgrad; [sharded: the
                  fc weight gradient of this rank's 1024 / W output rows from the
                  gathered rows + its clip-norm partials, all-gathered]; finalize
                  (conv3, conv2, heads); all-reduce of the [w2, wfc) bucket; [factors,
                  unsharded: the whole fc weight gradient]

The collectives run in issue order on one comm stream (``parallel/rccl.py``), so the
last one's join covers the rest.

**Sharded update** (``Runtime.dp_shard_update``; ZeRO-style): the fc layer (96 % of
the parameters) is owned in row slices -- rank r updates wfc rows [r S, (r+1) S) and
the matching bias entries, S = 1024 / W -- while the conv + head range (0.12 M
parameters, all-reduced) is updated on every rank.  One optimizer launch covers both
(``csrc/sumtree.hip RmsSegs``), so each rank streams 1/W of the fc's fp32 state
instead of all of it, and its fc weight gradient is only its own rows (factors: from
the gathered rows; allreduce exchange: a reduce-scatter instead of the all-reduce).
The clip norm is global: each rank's fc-slice squared-norm partials are all-gathered
(on the branch, hidden behind the backward) and summed in a fixed order with the conv
range's by every rank, so every replica applies the same coefficient.  The updated
bf16 hi (/ lo) rows and fp32 biases are all-gathered after the optimizer; the next
update's forward waits for them only at its fc layer (conv weights are never
sharded), so the transfer overlaps that update's conv forward.  Between graph
launches every rank holds the full bf16 copy; the fp32 master rows and RMSprop state
of the other ranks' slices are gathered on demand (:meth:`materialize`: checkpoints,
target sync, replica checks).
"""
from __future__ import annotations

from contextlib import nullcontext
from typing import List, Optional, Tuple

import torch

from ..ops.switches import SW

FC_ROWS, FC_COLS = 1024, 3136


class Streams:
    """The step's main stream and its branch.  On a GPU the branch is a second stream
    joined to the main one by events (graph edges under capture); on the CPU every
    method is a no-op and branch work runs inline, so the one step body serves both."""

    def __init__(self, device, side: Optional["torch.cuda.Stream"]):
        self.cuda = torch.device(device).type == "cuda" and side is not None
        self.device = device
        self.side = side
        # a third stream for the sharded update's parameter all-gathers, so the branch's
        # chain of each update starts at its fork like the single-rank step's
        self.aside_stream = torch.cuda.Stream(device) if self.cuda else None

    @property
    def main(self):
        return torch.cuda.current_stream(self.device) if self.cuda else None

    def mark(self):
        """An event at the main stream's current point (None on the CPU)."""
        if not self.cuda:
            return None
        ev = torch.cuda.Event()
        ev.record()
        return ev

    def branch(self, after=None):
        """Context: enqueue on the branch (after the main-stream point ``after``)."""
        if not self.cuda:
            return nullcontext()
        if after is not None:
            self.side.wait_event(after)
        return torch.cuda.stream(self.side)

    def aside(self, after=None):
        """Context: enqueue on the third stream (after the main-stream point ``after``); the
        main stream joins it through the work handles of what was issued there."""
        if not self.cuda:
            return nullcontext()
        if after is not None:
            self.aside_stream.wait_event(after)
        return torch.cuda.stream(self.aside_stream)

    def join(self) -> None:
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.side)


class DataParallelStep:
    """Mixin: the DP step of the fused NatureCNN learner.  Needs the learner's buffers,
    ``self.coll`` (parallel/rccl.py), ``self.layout`` and ``self.ops``."""

    _fc_split = False       # sharded update: the fc rows' gradient as split-K partials (_dp_setup)
    _fc_split_rows = 128    # their reduction rows per split (SW.dp_fc_split_rows, _dp_setup)
    _fc_cpb = -1

    # ------------------------------------------------------------------ setup
    def _dp_setup(self) -> None:
        """Sharding decision and the buffers of the sharded update (after the fc
        exchange is chosen)."""
        W, rank = self.world, (self.comm.rank if self.comm is not None else 0)
        mode = self.rt.dp_shard_update
        if mode not in ("auto", "on", "off"):
            raise ValueError("Runtime.dp_shard_update must be 'auto', 'on' or 'off'")
        ok = self._dp and not self._comm_bf16 and FC_ROWS % (64 * W) == 0
        self._shard = ok and (mode == "on" or (mode == "auto" and W > 1))
        self._params_pending = None     # the last update's fc-row all-gather (sharded)
        self._defer_params = False      # set while capturing an update that another follows
        self._gather_due = None         # (event,): the optimizer point a deferred gather follows
        hip = self.ops.name == "hip" and getattr(self.ops, "native_conv", False)
        # the fc weight gradient from the gathered factor rows as split-K partials reduced in
        # a grad_finalize launch (one norm partial per finalize block), sharded or not -- the
        # two stay bit-identical
        self._fc_split_rows = int(SW.dp_fc_split_rows) if SW.dp_fc_split_rows >= 0 else (256 if W >= 8 else 128)
        self._fc_split = self._dp and self._fc_factors and self._fc_split_rows > 0
        S = FC_ROWS // W if self._shard else FC_ROWS
        self._fc_cpb = -max(1, S // 128)       # direct finalize: ~393 norm partials at any S
        if not self._shard:
            return
        off = self.layout.offsets
        self._fc_S, self._fc_r0 = S, rank * S
        o0 = self._fc_r0
        self._segs = [(0, off["wfc"]), (off["wfc"] + o0 * FC_COLS, S * FC_COLS), (off["bfc"] + o0, S)]
        # this rank's fc-slice clip-norm partials (sent) and the gathered ones (norm_part[:W
        # nfc]): the fc wgrad kernel writes 4 per workgroup (ops/conv.py wgrad_blocks), the
        # torch backend and the sqnorm kernel's 64-block launch fewer
        if self._fc_factors and hip and self._fc_split:
            # split-K partials reduced in conv1's grad_finalize launch: one norm partial per
            # finalize block of the fc job (ops/conv.py finalize_job_blocks)
            from ..ops.conv import finalize_job_blocks
            nfc = finalize_job_blocks(dict(n=S * FC_COLS, nb=S, cpb=self._fc_cpb))
        elif self._fc_factors and hip:
            from ..ops.conv import wgrad_blocks
            nfc = 4 * wgrad_blocks(S, FC_COLS, 1 if self.split else 0)
        else:
            nfc = 64
        self._nfc_max = nfc
        self.fcn_send = torch.zeros(nfc, dtype=torch.float64, device=self.device)
        if W * nfc + 64 > self.norm_part.numel():
            raise ValueError(f"norm partials: {W} x {nfc} + 64 slots exceed norm_part")

    def _alloc_factors(self) -> None:
        """The factored exchange's row buffer: W x rows of [dH | dH lo | X | X lo]; this rank
        packs into its own block (the all-gather runs in place)."""
        ncol = sum(self._fx_cols)
        self.fx_recv = torch.zeros(self.world * self.B, ncol, dtype=self.act_dtype, device=self.device)
        r = self.comm.rank
        self.fx_send = self.fx_recv[r * self.B:(r + 1) * self.B]

    # ---------------------------------------------------- adaptive row buffer
    def rows_needed(self, stats=None) -> int:
        """Global batch scope: the fewest rows per rank with which the next global draw
        takes all ``mcap`` samples -- the draw's M = min(mcap, floor((rows - 2) sum T / max T))
        (replay/gpu_replay.py ``global_draw``, csrc/sumtree.hip) -- for the gathered shard
        masses T (a host read of the statistics)."""
        from ..replay.gpu_replay import SHARD_STATS
        st = self.replay.shard_stats if stats is None else stats
        T = st.double().reshape(self.world, SHARD_STATS)[:, 0].cpu().numpy()
        sm, tmax = float(T.sum()), float(T.max())
        if not (tmax > 0.0):
            return 0
        import math
        r = int(math.ceil(self.mcap * tmax / sm)) + 2
        while math.floor((r - 2) * sm / tmax) < self.mcap:      # (the kernel's exact rounding)
            r += 1
        return r

    def _fit_rows(self) -> bool:
        """Grow the per-rank row buffer when a shard's share of the priority mass would make
        the global draw shrink below ``replay_sample_size`` (``Runtime.dp_rows_adaptive``;
        the default buffer holds B / W (1 + dp_batch_slack) + 2 rows).  Every rank reads the
        same gathered statistics, so every rank picks the same size; the new size keeps
        the configured slack above the current need.  Buffers are reallocated and the HIP
        graphs recaptured (a rare, host-side event at the eviction cadence).  Returns
        whether the buffer grew."""
        if not (self._dp and self.world > 1 and self.rt.batch_scope == "global" and self.rt.dp_rows_adaptive):
            return False
        need = self.rows_needed()
        if need <= self.B:
            return False
        import math
        grow = int(math.ceil((need - 2) * (1.0 + float(self.rt.dp_batch_slack)))) + 2
        self._resize_rows(max(need, min(grow, self.mcap + 2)))
        return True

    def _resize_rows(self, rows: int) -> None:
        self.B = int(rows)
        self._alloc(self.B)
        if self._fc_factors:
            self._alloc_factors()
        self._graphs = self._multi = None
        self._graphs_warm = False
        self._params_pending = self._gather_due = None
        self._sample_ver = None
        self.rows_resized = getattr(self, "rows_resized", 0) + 1

    def _fc_rows(self, flat: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(whole fc weight range, this rank's rows) of a flat-layout tensor."""
        o = self.layout.offsets["wfc"]
        whole = flat[o:o + FC_ROWS * FC_COLS]
        r0, S = self._fc_r0, self._fc_S
        return whole, whole[r0 * FC_COLS:(r0 + S) * FC_COLS]

    def _fc_bias(self, flat: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        o = self.layout.offsets["bfc"]
        whole = flat[o:o + FC_ROWS]
        return whole, whole[self._fc_r0:self._fc_r0 + self._fc_S]

    # ------------------------------------------------------------------- step
    def _dp_body(self) -> None:
        """One data-parallel update (see the module docstring)."""
        B, rt, ops, G, Pb, Pl, S = self.B, self.rt, self.ops, self.G, self.Pb, self.Pl, self.S
        sp = self.split
        off = self.layout.offsets
        cut, o2 = off["wfc"], off["w2"]
        coll, br = self.coll, self._streams
        factors, shard = self._fc_factors, self._shard
        self._seg1()                      # forward + head (the weight gradients come below)
        jobs, works = [], {}
        fork = br.mark()
        ops.fc_dgrad(self.dH, self.y3[:B], Pb["wfc"], self.dY3,
                     **self._lo(dh_lo=self.dH_lo, w_lo=sp and Pl["wfc"], dx_lo=self.dY3_lo))
        prio = (self.replay, S["idx"], S["gen"], self.td_abs)
        with br.branch(fork):
            if factors:
                # head weight gradient + priority write-back + the factor-row pack, one launch
                segs = [self.dH, self.dH_lo, self.y3[:B].reshape(B, FC_COLS), self.y3_lo[:B].reshape(B, FC_COLS)] \
                    if sp else [self.dH, self.y3[:B].reshape(B, FC_COLS)]
                ops.head_wgrad(self.h, self.dhead, self._head_params(G), prio=prio, pack=(self.fx_send, segs),
                               **self._lo(Hon_lo=self.h_lo))
            else:
                ops.fc_head_wgrad(self.dH, self.y3[:B], G["wfc"], G["bfc"], self.h, self.dhead, G, prio,
                                  **self._lo(dh_lo=self.dH_lo, x_lo=sp and self.y3_lo[:B], Hon_lo=self.h_lo))
                if self._comm_bf16 and not shard:
                    self.gcomm[cut:].copy_(self.g32[cut:])
            # (the HIP priority write-back kernel has left this shard's sum / min in its slot)
            fresh = self.ops.name == "hip" and getattr(self.replay, "use_hip", False)
            with coll.fused():        # (RCCL: one launch for the fc exchange + the statistics)
                if factors:
                    works["fc"] = coll.all_gather_into(self.fx_recv, self.fx_send)
                elif shard:
                    # reduce-scatter: this rank's fc rows (in place) and bias entries
                    w_all, w_own = self._fc_rows(self.g32)
                    b_all, b_own = self._fc_bias(self.g32)
                    coll.reduce_scatter_into(w_own, w_all)
                    works["fc"] = coll.reduce_scatter_into(b_own, b_all)
                else:
                    works["fc"] = coll.all_reduce(self.gcomm[cut:])
                works["stats"] = self.replay.gather_shard_stats(async_op=True, coll=coll, fresh_local=fresh)
            nfc = 0
            fc_on_branch = shard and SW.dp_fc_shard_branch
            if fc_on_branch:
                # this rank's fc rows of the global batch's gradient (+ their clip-norm
                # partials) right behind the exchange, on the branch: no main-stream wait
                # on the branch's exchange (one cross-queue edge fewer on the critical path)
                works["fc"].wait()
                nfc = self._fc_shard_grad_norm()
        # conv3 / conv2 data gradients on main, conv3's weight gradient on the branch
        one_wait = SW.dp_branch_one_wait
        ev3 = None if one_wait else br.mark()
        ops.conv_dgrad(self.dY3, Pb["w3"], 1, self.y2[:B], self.dY2,
                       **self._lo(dy_lo=self.dY3_lo, w_lo=sp and Pl["w3"], dx_lo=self.dY2_lo))
        if not one_wait:
            with br.branch(ev3):
                self._conv3_wgrad(jobs)
        ev2 = br.mark()
        ops.conv_dgrad(self.dY2, Pb["w2"], 2, self.y1[:B], self.dY1,
                       **self._lo(dy_lo=self.dY2_lo, w_lo=sp and Pl["w2"], dx_lo=self.dY1_lo))
        # the branch's conv2 wgrad, then conv1's wgrad on main.  The fc exchange's result
        # reaches the branch by stream order: the collectives were issued from the branch
        # (graphs: the comm stream IS the branch; eager torch: the work handle's wait).
        # The main stream does not wait for the exchange before conv1's wgrad: a main-stream
        # wait there made conv1's wgrad start only after the branch's conv2 wgrad in the
        # replayed graph (trace r5_emu8e: ~28 us idle; 5,025-5,033 vs 5,128-5,158 updates/s
        # emulated at W = 8, profiles/r5_ab_dp_capture_order.txt).
        with br.branch(ev2):
            if one_wait:
                # (one main-stream event for both weight gradients: conv2 dgrad's input is
                # conv3 dgrad's output, so both are ready at this point)
                self._conv3_wgrad(jobs)
            self._conv2_wgrad(jobs)
        jobs1 = []
        ops.conv1_wgrad_ring(self.dY1, self.replay.frames, self.slots[:B], self.frames, rt.obs_scale, G["w1"],
                             G["b1"], jobs=jobs1, **self._lo(dy_lo=self.dY1_lo))
        with br.branch():
            if factors and not shard:
                works["fc"].wait()
                if self._fc_split:
                    # the global batch's whole fc weight gradient as split-K partials,
                    # reduced in the branch's finalize launch below (norm partials first)
                    nfc = self._fc_wgrad_gathered(jobs)
            # conv2 / conv3 / head bucket [w2, wfc): reduced on the branch and all-reduced
            # from it while conv1's weight gradient runs -- only conv1's bucket follows the
            # last backward kernel
            ops.finalize_grads(jobs, None, None)
            if self._comm_bf16:
                self.gcomm[o2:cut].copy_(self.g32[o2:cut])
            works["cv2"] = coll.all_reduce(self.gcomm[o2:cut])
            if factors and not shard and not self._fc_split:
                # the global batch's whole fc weight gradient (identical on every rank)
                nfc = self._fc_wgrad_gathered()
            n_pre = 0
            if SW.dp_norm_split and self._presample and not self._comm_bf16 and (shard or factors):
                # the clip-norm partials of the reduced buckets on the branch, right behind
                # their all-reduces (first in norm_part, after the fc partials of the unsharded
                # factored exchange); conv1's bucket -- reduced last, on main -- is summed inside
                # the optimizer launch (norm_prefix): no norm launch on the critical path
                works["cv2"].wait()
                # (not with the all-reduce exchange: the 3.2 M-float fc bucket's norm on the
                # branch -- the chain that also carries that bucket -- lengthened the forced-DP
                # step at world 1 by 73 us at 64 blocks and still cost 0.7 % at 1,024:
                # 2,636 vs 2,656 updates/s, profiles/r6_ab_forced_dp_norm_split.txt, the 0.7 %
                # being this block's branch wait alone; the optimizer's own norm pass stays there)
                if shard:
                    n_pre = ops.sqnorm_ranges((self.g32[o2:cut],), self.norm_part, 64)
                elif factors:
                    n_pre = nfc + ops.sqnorm_ranges((self.g32[o2:cut],), self.norm_part[nfc:], 64)
        if shard and not fc_on_branch and self._fc_split:
            # this rank's fc rows of the global batch's gradient as split-K partials (the
            # rows fill the chip only when the reduction is split), reduced in conv1's
            # finalize launch with one clip-norm partial per finalize block
            works["fc"].wait()
            nfc = self._fc_shard_grad_norm(jobs1)
        ops.finalize_grads(jobs1, None, None)
        if shard and not fc_on_branch and not self._fc_split:
            # this rank's fc rows of the global batch's gradient (+ their clip-norm partials)
            # on main after conv1's (the exchange finished long before: one edge, no stall)
            works["fc"].wait()
            nfc = self._fc_shard_grad_norm()
        self._npart = 0
        self._mark("conv_backward")
        if self._comm_bf16:
            self.gcomm[:o2].copy_(self.g32[:o2])
        fcn = (self.norm_part[n_pre:n_pre + self.world * nfc], self.fcn_send[:nfc]) if shard else None
        if getattr(coll, "inline", False) and self._ordered_coll:
            # conv1's bucket (+ the fc clip-norm partials) on the main stream itself, one
            # RCCL launch: one join of the branch (in order: covers every collective issued
            # from it), then no fork / join edge on the critical path
            br.join()
            if getattr(coll, "stream", None) is not br.side:
                works["cv2"].wait()      # (issued from the branch itself: the join covers it)
            with coll.fused(inline=True):
                coll.all_reduce_inline(self.gcomm[:o2])
                if fcn is not None:
                    coll.all_gather_inline(*fcn)
        else:
            with coll.fused():
                w_cv = coll.all_reduce(self.gcomm[:o2])
                if fcn is not None:
                    works["cv1"] = w_cv
                    w_cv = coll.all_gather_into(*fcn)
            br.join()
            if self._ordered_coll:
                w_cv.wait()          # the collectives run in issue order: covers the rest
            else:
                for w in works.values():
                    w.wait()
                w_cv.wait()
        self._mark("allreduce_wait")
        if shard:
            if n_pre:
                self._seg3(norm_slots=n_pre + self.world * nfc, segs=self._segs, norm_prefix=self.g32[:o2])
            else:
                n0 = self.world * nfc
                nr = ops.sqnorm_ranges((self.g32[:cut],), self.norm_part[n0:], 64)
                self._seg3(norm_slots=n0 + nr, segs=self._segs)
            if self._defer_params and self._streams.cuda:
                # inside a multi-update capture: issued once the next update's conv12 is
                # enqueued (forward_all -> _issue_params), so conv12 stays the optimizer's
                # first-captured child and keeps the main queue (round-5 trace r5_emu8d)
                self._gather_due = (self._streams.mark(),)
            else:
                self._gather_params()
        elif n_pre:
            self._seg3(norm_slots=n_pre, norm_prefix=self.g32[:o2])
        elif factors:
            nr = ops.sqnorm_ranges((self.g32[:cut],), self.norm_part[nfc:], 64)
            self._seg3(norm_slots=nfc + nr)
        else:
            self._seg3()         # (the optimizer's own clip-norm pass over the reduced gradient)

    def _gathered_cols(self):
        R, c = self.fx_recv, [0]
        for w in self._fx_cols:
            c.append(c[-1] + w)
        cols = [R[:, c[i]:c[i + 1]] for i in range(len(self._fx_cols))]
        return (cols[0], cols[1], cols[2], cols[3]) if self.split else (cols[0], None, cols[1], None)

    def _fc_wgrad_gathered(self, jobs=None) -> int:
        """The fc weight gradient of the global batch from the all-gathered (dH, X) rows
        (identical on every rank), with its clip-norm partials in norm_part[0:].
        Returns the partial slots written.  With ``jobs``: split-K partials reduced by the
        finalize launch of ``jobs`` (``SW.dp_fc_split_rows``)."""
        dy, dy_lo, x, x_lo = self._gathered_cols()
        if jobs is not None:
            return self.ops.fc_wgrad_split(dy, x, self.G["wfc"], self.G["bfc"], jobs, self._fc_split_rows,
                                           self.norm_part, cpb=self._fc_cpb, **self._lo(dh_lo=dy_lo, x_lo=x_lo))
        return self.ops.fc_wgrad(dy, x, self.G["wfc"], self.G["bfc"], norm=(self.norm_part, 0),
                                 **self._lo(dh_lo=dy_lo, x_lo=x_lo)) or 0

    def _fc_shard_grad_norm(self, jobs=None) -> int:
        """Sharded update: this rank's fc rows of the gradient (factors: computed from the
        gathered rows; allreduce exchange: already reduce-scattered) and their squared-norm
        partials in ``fcn_send``.  Returns the partial count (equal on every rank).  With
        ``jobs`` (factors, ``SW.dp_fc_split_rows``): split-K partials, reduced by the
        finalize launch of ``jobs`` that writes the norm partials."""
        _, w_own = self._fc_rows(self.g32)
        _, b_own = self._fc_bias(self.g32)
        if self._fc_factors and jobs is not None:
            dy, dy_lo, x, x_lo = self._gathered_cols()
            r0, S = self._fc_r0, self._fc_S
            n = self.ops.fc_wgrad_split(dy[:, r0:r0 + S], x, w_own.view(S, FC_COLS), b_own, jobs,
                                        self._fc_split_rows, self.fcn_send,
                                        cpb=self._fc_cpb,
                                        **self._lo(dh_lo=None if dy_lo is None else dy_lo[:, r0:r0 + S], x_lo=x_lo))
        elif self._fc_factors:
            dy, dy_lo, x, x_lo = self._gathered_cols()
            r0, S = self._fc_r0, self._fc_S
            n = self.ops.fc_wgrad(dy[:, r0:r0 + S], x, w_own.view(S, FC_COLS), b_own,
                                  norm=(self.fcn_send, 0),
                                  **self._lo(dh_lo=None if dy_lo is None else dy_lo[:, r0:r0 + S],
                                             x_lo=x_lo)) or 0
        else:
            n = self.ops.sqnorm_ranges((w_own, b_own), self.fcn_send, 64)
        assert 0 < n <= self._nfc_max, (n, self._nfc_max)
        return n

    def _gather_params(self) -> None:
        """All-gather every rank's updated fc rows (bf16 hi / lo) and fc biases (fp32), in
        place; the next forward waits for it at its fc layer (:meth:`_wait_params`)."""
        coll = self.coll
        works = []
        with coll.fused():            # (RCCL: one launch)
            w_all, w_own = self._fc_rows(self.pbf)
            works.append(coll.all_gather_into(w_all, w_own))
            if self.split:
                l_all, l_own = self._fc_rows(self.pbf_lo)
                works.append(coll.all_gather_into(l_all, l_own))
            b_all, b_own = self._fc_bias(self.p32)
            works.append(coll.all_gather_into(b_all, b_own))
        self._params_pending = works

    def _issue_params(self) -> None:
        """Issue a deferred fc-row all-gather (see the end of :meth:`_dp_body`) on the third stream,
        after the optimizer point it was deferred from."""
        due = getattr(self, "_gather_due", None)
        if due is not None:
            self._gather_due = None
            with self._streams.aside(due[0]), self.coll.on_stream(self._streams.aside_stream):
                # (RCCL keeps one communicator's kernels in issue order by itself; the
                # next collective, the branch's, forks from main after the fc forward
                # that waits for these)
                self._gather_params()

    def _wait_params(self) -> None:
        """The current stream waits for the last update's fc-row all-gathers, if pending
        (the last first: on an in-order comm stream its join covers the others, which
        then add no edge)."""
        self._issue_params()
        ws = getattr(self, "_params_pending", None)
        if ws:
            for w in reversed(ws):
                w.wait()
        self._params_pending = None

    # ------------------------------------------------------------ full state
    def materialize(self) -> None:
        """Sharded update: gather every rank's fp32 fc rows and RMSprop state, so that
        ``p32`` / ``rms_v`` / ``rms_m`` hold the whole model (a collective: every rank calls
        it at the same update).  Between calls each rank keeps only its own rows current.
        Checkpoints, the target sync and the replica check call it."""
        if not getattr(self, "_shard", False):
            return
        self._wait_params()
        if getattr(self.comm, "emulated", False):
            # (an emulated world has no other ranks: its all-gathers would overwrite the
            # other slices with copies of this rank's rows)
            return
        works = []
        # (t32: every rank's own rows are right -- copies of its p32 rows at the last sync)
        for t in (self.p32, self.t32, self.rms_v, self.rms_m):
            w_all, w_own = self._fc_rows(t)
            works.append(self.coll.all_gather_into(w_all, w_own))
            b_all, b_own = self._fc_bias(t)
            works.append(self.coll.all_gather_into(b_all, b_own))
        for w in works:
            w.wait()
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self._materialized_at = self.num_q_updates

    def _check_materialized(self) -> None:
        """Before reading the whole fp32 state (save): gathered at this update."""
        if not getattr(self, "_shard", False):
            return
        if getattr(self.comm, "emulated", False):
            raise RuntimeError("sharded DP update in an emulated world: only this rank's fc rows exist, "
                               "there is no whole model to save")
        if self.world == 1:
            self.materialize()
        elif getattr(self, "_materialized_at", None) != self.num_q_updates:
            raise RuntimeError("sharded DP update: call learner.materialize() on every rank before save()")

    # ---------------------------------------------------------- diagnostics
    def comm_report(self) -> dict:
        """What the collectives see: the rank count the communicator reports and a checked
        all-reduce of rank + 1 (must be W (W + 1) / 2).  A collective."""
        if not self._dp:
            return {"comm_world": 1, "init_allreduce_ok": True}
        coll = self.coll
        try:
            cw = int(coll.world())
        except Exception as e:  # pragma: no cover - depends on the RCCL build
            cw = f"error: {e!r}"
        rank = self.comm.rank
        t = torch.full((1,), float(rank + 1), dtype=torch.float32, device=self.device)
        coll.all_reduce(t).wait()
        got = float(t.item())
        W = self.world
        emulated = getattr(self.comm, "emulated", False)
        want = float(rank + 1) if emulated else W * (W + 1) / 2.0
        return {"comm_world": cw, "init_allreduce": got, "init_allreduce_ok": got == want}


def shard_layout(world: int) -> List[Tuple[int, int]]:
    """(first fc row, rows) owned by each of ``world`` ranks under the sharded update."""
    S = FC_ROWS // world
    return [(r * S, S) for r in range(world)]
