"""fp32-class ("split") IMPALA-deep kernels (csrc/impala_split.hip) against fp64 PyTorch.

Activations are fp32 planar-16 tensors; the kernels split each value into bf16 hi + lo
planes in LDS and weights into hi + lo fragments, and issue hi*hi + lo*hi + hi*lo
MFMAs with fp32 accumulation.  Tolerance 1e-4 norm-wise relative (the bf16-operand
kernels of csrc/impala.hip sit near 1e-2 on the same data), and the whole learner step
is checked against an fp32 torch step with the bf16-operand step as the contrast.
"""
import numpy as np
import pytest
import torch

from apex_dqn_amd.ops.impala import ConvSpec, TorchImpalaOps, frag_elems

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TOL = 1e-4


def _rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _hops():
    from apex_dqn_amd.ops.impala import HipImpalaOps
    return HipImpalaOps()


def _spec(cin, cout, H, cin_real=None, seed=0):
    """(kernel spec with hi / lo fragments, fp64-oracle spec with the fp32 master weights)"""
    g = torch.Generator().manual_seed(seed)
    cr = cin_real or cin
    w = (torch.randn(cout, cr, 3, 3, generator=g) * 0.2).to(DEV)
    wt = (torch.randn(cout, cr, 3, 3, generator=g) * 0.2).to(DEV)
    b = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    bt = (torch.randn(cout, generator=g) * 0.1).to(DEV)
    cs = ConvSpec("t", cin, cout, cr, H, H, w=w, b=b, wb=w.to(torch.bfloat16))
    cs.extra["wl"] = (w - cs.wb.float()).to(torch.bfloat16)
    cs.extra["w_tgt"] = wt.to(torch.bfloat16)
    cs.extra["w_tgt_lo"] = (wt - cs.extra["w_tgt"].float()).to(torch.bfloat16)
    cs.extra["b_tgt"] = bt
    kind = 2 if cr < cin else 0
    fe, feT = frag_elems(cin, cout), frag_elems(cout, cin)
    z = lambda n: torch.zeros(n, dtype=torch.bfloat16, device=DEV)  # noqa: E731
    cs.frag, cs.frag_lo, cs.frag_tgt, cs.frag_tgt_lo = z(fe), z(fe), z(fe), z(fe)
    cs.fragT, cs.fragT_lo = z(feT), z(feT)
    jobs = [(cs.wb, cs.frag, cin, cout, cr, kind), (cs.extra["wl"], cs.frag_lo, cin, cout, cr, kind),
            (cs.extra["w_tgt"], cs.frag_tgt, cin, cout, cr, kind),
            (cs.extra["w_tgt_lo"], cs.frag_tgt_lo, cin, cout, cr, kind)]
    if cr == cin:
        jobs += [(cs.wb, cs.fragT, cin, cout, cr, 1), (cs.extra["wl"], cs.fragT_lo, cin, cout, cr, 1)]
    _hops().pack(jobs)
    ref = ConvSpec("r", cin, cout, cr, H, H, w=w, b=b, wb=w)
    ref.extra["w_tgt"], ref.extra["b_tgt"] = wt, bt
    return cs, ref


def _t(N, P, H, g, scale=1.0):
    return torch.randn(N, P, H, H, 16, generator=g, device=DEV) * scale


FWD_SHAPES = [(16, 16, 42), (16, 32, 42), (32, 16, 42), (32, 32, 21), (32, 32, 11)]


@pytest.mark.parametrize("cin,cout,H", FWD_SHAPES)
def test_split_sconv_fwd_and_dgrad_vs_fp64(cin, cout, H):
    hops, tops = _hops(), TorchImpalaOps()
    N = 6
    g = torch.Generator(device=DEV).manual_seed(1)
    x = _t(N, cin // 16, H, g)
    add, mask = _t(N, cout // 16, H, g), _t(N, cout // 16, H, g)
    cs, ref = _spec(cin, cout, H)
    for kw in (dict(), dict(relu_in=True, add=add), dict(relu_in=True, relu_out=True, mask=mask),
               dict(second=cs.extra["b_tgt"], n_switch=4, relu_in=True)):
        y = torch.zeros(N, cout // 16, H, H, 16, dtype=torch.float32, device=DEV)
        yr = torch.zeros(y.shape, dtype=torch.float64, device=DEV)
        hops.conv(x, cs, y, **kw)
        kr = dict(kw)
        if "second" in kr:
            kr["second"] = ref.extra["b_tgt"]
        tops.conv(x.double(), ref, yr, **kr)
        assert _rel(y, yr) < TOL, (kw.keys(), _rel(y, yr))
    if cin == cout or (cin, cout) == (16, 32):
        dy = _t(N, cout // 16, H, g)
        m2, a2 = _t(N, cin // 16, H, g), _t(N, cin // 16, H, g)
        dx = torch.zeros(N, cin // 16, H, H, 16, dtype=torch.float32, device=DEV)
        dxr = torch.zeros(dx.shape, dtype=torch.float64, device=DEV)
        hops.conv(dy, cs, dx, transpose=True, mask=m2, add=a2)
        tops.conv(dy.double(), ref, dxr, transpose=True, mask=m2.double(), add=a2.double())
        assert _rel(dx, dxr) < TOL, _rel(dx, dxr)


@pytest.mark.parametrize("cin,cout,H", [(16, 32, 42), (32, 32, 21)])
def test_split_sconv_pool_vs_fp64(cin, cout, H):
    hops, tops = _hops(), TorchImpalaOps()
    N = 5
    g = torch.Generator(device=DEV).manual_seed(2)
    x = _t(N, cin // 16, H, g)
    cs, ref = _spec(cin, cout, H, seed=5)
    Ho = (H + 1) // 2
    p = torch.zeros(N, cout // 16, Ho, Ho, 16, dtype=torch.float32, device=DEV)
    a = torch.zeros(N, cout // 16, Ho, Ho, 16, dtype=torch.uint8, device=DEV)
    hops.conv_pool(x, cs, p, a, second=cs.extra["b_tgt"], n_switch=2)
    y = torch.zeros(N, cout // 16, H, H, 16, dtype=torch.float64, device=DEV)
    tops.conv(x.double(), ref, y, second=ref.extra["b_tgt"], n_switch=2)
    pr = torch.zeros(p.shape, dtype=torch.float64, device=DEV)
    ar = torch.zeros_like(a)
    tops.maxpool(y, pr, ar)
    assert _rel(p, pr) < TOL
    assert (a == ar).float().mean().item() > 0.999


def _ring(g, F=80):
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    raw = torch.randint(0, 256, (F, 84, 84), generator=g, dtype=torch.uint8, device=DEV)
    return to_s2d(raw)


def test_split_ring_conv_pool_and_wgrad_vs_fp64():
    """Stack 1's entry conv on the uint8 frame ring (exact pixels x hi + lo weights),
    fused with the max pool, and its weight gradient from the ring."""
    hops, tops = _hops(), TorchImpalaOps()
    g = torch.Generator(device=DEV).manual_seed(3)
    ring = _ring(g)
    N = 5
    slots = torch.randint(0, 80, (N, 4), generator=g, dtype=torch.int32, device=DEV)
    cs, ref = _spec(16, 16, 84, cin_real=4, seed=7)
    kw = dict(ring=ring, slots=slots, scale=1.0 / 255)
    p = torch.zeros(N, 1, 42, 42, 16, dtype=torch.float32, device=DEV)
    a = torch.zeros(N, 1, 42, 42, 16, dtype=torch.uint8, device=DEV)
    hops.conv_pool(None, cs, p, a, second=cs.extra["b_tgt"], n_switch=3, **kw)
    y = torch.zeros(N, 1, 84, 84, 16, dtype=torch.float64, device=DEV)
    tops.conv(None, ref, y, second=ref.extra["b_tgt"], n_switch=3, **kw)
    pr, ar = torch.zeros(p.shape, dtype=torch.float64, device=DEV), torch.zeros_like(a)
    tops.maxpool(y, pr, ar)
    assert _rel(p, pr) < TOL
    assert (a == ar).float().mean().item() > 0.999
    dy = _t(N, 1, 84, g)
    gw, gb = torch.zeros(16, 4, 3, 3, device=DEV), torch.zeros(16, device=DEV)
    gwr, gbr = torch.zeros(16, 4, 3, 3, dtype=torch.float64, device=DEV), torch.zeros(16, dtype=torch.float64,
                                                                                       device=DEV)
    jobs = []
    hops.wgrad(dy, None, cs, gw, gb, jobs, ring=ring, slots=slots, scale=1.0 / 255)
    hops.finalize(jobs)
    tops.wgrad(dy.double(), None, ref, gwr, gbr, [], ring=ring, slots=slots, scale=1.0 / 255)
    assert _rel(gw, gwr) < TOL and _rel(gb, gbr) < TOL


@pytest.mark.parametrize("N,groups", [(5, 0), (37, 0), (37, 6)])
def test_ring_wgrad_fused_pool_backward_bit_identical(N, groups):
    """The ring conv's weight gradient straight from the pooled gradient + argmax codes
    (max-pool backward inside its staging) equals max-pool backward then weight gradient
    bit for bit, and the fp64 oracle within tolerance."""
    hops, tops = _hops(), TorchImpalaOps()
    g = torch.Generator(device=DEV).manual_seed(8)
    ring = _ring(g)
    slots = torch.randint(0, 80, (N, 4), generator=g, dtype=torch.int32, device=DEV)
    cs, ref = _spec(16, 16, 84, cin_real=4, seed=9)
    # argmax codes from a real max pool (ties make some pixels take several windows)
    x = torch.randn(N, 1, 84, 84, 16, generator=g, device=DEV).round()
    p = torch.zeros(N, 1, 42, 42, 16, dtype=torch.float32, device=DEV)
    a = torch.zeros(N, 1, 42, 42, 16, dtype=torch.uint8, device=DEV)
    tops.maxpool(x, p, a)
    dp = _t(N, 1, 42, g)
    kw = dict(ring=ring, slots=slots, scale=1.0 / 255, groups=groups)
    outs = []
    for fused in (True, False):
        gw, gb = torch.zeros(16, 4, 3, 3, device=DEV), torch.zeros(16, device=DEV)
        jobs = []
        if fused:
            hops.wgrad(dp, None, cs, gw, gb, jobs, pool_amax=a, **kw)
        else:
            dc = torch.zeros(N, 1, 84, 84, 16, device=DEV)
            hops.maxpool_bwd(dp, a, dc)
            hops.wgrad(dc, None, cs, gw, gb, jobs, **kw)
        hops.finalize(jobs)
        outs.append((gw, gb))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    gwr = torch.zeros(16, 4, 3, 3, dtype=torch.float64, device=DEV)
    gbr = torch.zeros(16, dtype=torch.float64, device=DEV)
    tops.wgrad(dp.double(), None, ref, gwr, gbr, [], pool_amax=a, ring=ring, slots=slots, scale=1.0 / 255)
    assert _rel(outs[0][0], gwr) < TOL and _rel(outs[0][1], gbr) < TOL


WG_SHAPES = [(16, 16, 42), (16, 32, 42), (32, 32, 21), (32, 32, 11)]


@pytest.mark.parametrize("cin,cout,H", WG_SHAPES)
def test_split_sconv_wgrad_vs_fp64(cin, cout, H):
    hops, tops = _hops(), TorchImpalaOps()
    N = 37
    g = torch.Generator(device=DEV).manual_seed(4)
    x, dy = _t(N, cin // 16, H, g), _t(N, cout // 16, H, g)
    cs, ref = _spec(cin, cout, H)
    for relu in (False, True):
        gw, gb = torch.zeros(cout, cin, 3, 3, device=DEV), torch.zeros(cout, device=DEV)
        gwr = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, device=DEV)
        gbr = torch.zeros(cout, dtype=torch.float64, device=DEV)
        jobs = []
        hops.wgrad(dy, x, cs, gw, gb, jobs, relu_in=relu)
        hops.finalize(jobs)
        tops.wgrad(dy.double(), x.double(), ref, gwr, gbr, [], relu_in=relu)
        assert _rel(gw, gwr) < TOL and _rel(gb, gbr) < TOL, (relu, _rel(gw, gwr), _rel(gb, gbr))


# every (rows, threads) instantiation of the split weight gradient (SCONV_WG_S_SHAPES)
WG_VARIANTS = [(16, 16, 42, 11, 512), (16, 32, 42, 7, 256), (32, 32, 21, 11, 512), (32, 32, 11, 11, 256)]


@pytest.mark.parametrize("cin,cout,H,R,nthr", WG_VARIANTS)
def test_split_sconv_wgrad_variants_vs_fp64(cin, cout, H, R, nthr, monkeypatch):
    from apex_dqn_amd.ops import impala as impala_mod
    hops, tops = _hops(), TorchImpalaOps()
    assert hops.lib.apex_sconv_wgrad_split_rows(cin, cout, H, H, 0, R, nthr) == R
    monkeypatch.setitem(impala_mod.SPLIT_BANDS, ("wg", cin, cout, H), (R, nthr))
    N = 19
    g = torch.Generator(device=DEV).manual_seed(6)
    x, dy = _t(N, cin // 16, H, g), _t(N, cout // 16, H, g)
    cs, ref = _spec(cin, cout, H)
    gw, gb = torch.zeros(cout, cin, 3, 3, device=DEV), torch.zeros(cout, device=DEV)
    gwr = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, device=DEV)
    gbr = torch.zeros(cout, dtype=torch.float64, device=DEV)
    for groups in (0, 5):
        gw.zero_(), gb.zero_()
        jobs = []
        hops.wgrad(dy, x, cs, gw, gb, jobs, relu_in=True, groups=groups)
        hops.finalize(jobs)
        if groups == 0:
            tops.wgrad(dy.double(), x.double(), ref, gwr, gbr, [], relu_in=True)
        assert _rel(gw, gwr) < TOL and _rel(gb, gbr) < TOL, (groups, _rel(gw, gwr), _rel(gb, gbr))


@pytest.mark.parametrize("C,H", [(16, 42), (32, 21), (32, 11)])
def test_split_resblock_vs_fp64(C, H):
    hops, tops = _hops(), TorchImpalaOps()
    N = 7
    g = torch.Generator(device=DEV).manual_seed(5)
    x = _t(N, C // 16, H, g)
    (c0, r0), (c1, r1) = _spec(C, C, H, seed=3), _spec(C, C, H, seed=4)
    for relu_out in (False, True):
        out = torch.zeros(N, C // 16, H, H, 16, dtype=torch.float32, device=DEV)
        ys = torch.zeros_like(out)
        outr = torch.zeros(out.shape, dtype=torch.float64, device=DEV)
        ysr = torch.zeros_like(outr)
        kw = dict(n_save=4, target=True, n_switch=5, relu_out=relu_out)
        hops.resblock(x, c0, c1, out, ysave=ys, **kw)
        tops.resblock(x.double(), r0, r1, outr, ysave=ysr, **kw)
        assert _rel(out, outr) < TOL, _rel(out, outr)
        assert _rel(ys[:4], ysr[:4]) < TOL
        assert torch.count_nonzero(ys[4:]) == 0
    # output as bf16 hi / lo planes (the last block writing the fc operand rows)
    oh = torch.zeros(N, C // 16, H, H, 16, dtype=torch.bfloat16, device=DEV)
    ol = torch.zeros_like(oh)
    hops.resblock(x, c0, c1, oh, out_lo=ol, target=True, n_switch=5, relu_out=True)
    assert _rel(oh.double() + ol.double(), outr) < TOL


def test_split_maxpool_bwd_and_merge():
    hops, tops = _hops(), TorchImpalaOps()
    g = torch.Generator(device=DEV).manual_seed(6)
    for (P, H) in ((1, 84), (2, 42), (2, 21)):
        x = _t(3, P, H, g)
        Ho = (H + 1) // 2
        y = torch.zeros(3, P, Ho, Ho, 16, device=DEV)
        a = torch.zeros(3, P, Ho, Ho, 16, dtype=torch.uint8, device=DEV)
        tops.maxpool(x, y, a)
        dy = _t(3, P, Ho, g)
        dx = torch.zeros(3, P, H, H, 16, device=DEV)
        dxr = torch.zeros(dx.shape, dtype=torch.float64, device=DEV)
        hops.maxpool_bwd(dy, a, dx)
        tops.maxpool_bwd(dy.double(), a, dxr)
        assert _rel(dx, dxr) < 1e-6
    v = torch.randn(9, 3904, generator=g, device=DEV)
    hi = v.to(torch.bfloat16)
    lo = (v - hi.float()).to(torch.bfloat16)
    out = torch.zeros_like(v)
    hops.merge(hi, lo, out)
    torch.testing.assert_close(out, hi.float() + lo.float(), rtol=0, atol=0)


def _learner(dtype, backend, B=64):
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.impala_learner import FusedImpalaLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    torch.manual_seed(0)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": B},
                                "Runtime": {"grad_clip": 40.0, "network": "impala", "use_graphs": False,
                                            "dtype": dtype}})
    rp = GpuReplayShard(256, 256, 400, 4, device=DEV)
    rng = np.random.default_rng(0)
    seqs = rp.append_frames(rng.integers(0, 255, (200, 84, 84), dtype=np.uint8))
    K = 150
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    nx = np.stack([seqs[i + 3:i + 7] for i in range(K)])
    gam = np.full(K, 0.97)
    gam[::5] = 0.0
    rp.insert(dict(S_t=st, S_tpn=nx, A_t=rng.integers(0, 6, K), R=rng.normal(size=K) * 3, Gamma=gam,
                   priority=rng.random(K)))
    return FusedImpalaLearner(cfg, DEV, rp, backend=backend)


def test_split_impala_step_matches_fp32_torch_step():
    """Whole split step (HIP, Runtime.dtype fp32) vs the fp32 torch step on the same
    parameters and batch.  Every backward data-gradient op of the HIP step, re-run in
    fp64 on the HIP step's own inputs, is within 2e-5 (measured ~4e-6; torch fp32 ~3e-7).
    End to end, |delta| and the fc / head gradients match at fp32 class (< 1e-4); the
    trunk weight gradients differ by up to ~5e-3 because ReLU masks and max-pool winners
    flip where an activation lies within the two forwards' ~1e-6 difference of a tie (a
    handful of units per layer, each moving one O(1) term of a sum over ~1e5;
    scripts/archive/diag_impala_split.py) -- the bf16-operand HIP step on the same data is the
    contrast (>= 10x worse)."""
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    cudnn_was = torch.backends.cudnn.enabled
    torch.backends.cudnn.enabled = False      # oracle convs: torch's native fp32 path
    try:
        _step_vs_torch()
    finally:
        torch.backends.cudnn.enabled = cudnn_was


def _step_vs_torch():
    tops = TorchImpalaOps()
    Lt = _learner("fp32", "torch")
    errs = {}
    for dt in ("fp32", "bf16"):
        Lh = _learner(dt, "hip")
        Lh.p32.copy_(Lt.p32)
        Lh._refresh_bf16()
        Lh.sync_target()
        Lh._seg1()
        Lh._seg2()
        if dt == "fp32":
            Lt._seg1()
            for s in range(3):     # the oracle backward routes through the kernels' pool winners
                Lt.fw[s]["amax"].copy_(Lh.fw[s]["amax"])
            Lt._seg2()
        torch.cuda.synchronize()
        assert torch.equal(Lh.slots, Lt.slots)
        gh, gt = Lh.module_state(Lh.G), Lt.module_state(Lt.G)
        e = {k: float((gh[k] - gt[k]).norm() / (gt[k].norm() + 1e-12)) for k in gh}
        e["td_abs"] = _rel(Lh.td_abs, Lt.td_abs)
        errs[dt] = e
        if dt == "fp32":
            # per-op: each data-gradient kernel of the step in fp64 on its own HIP inputs
            B = Lh.B
            dO = Lh.dfeat32[:, :3872].view(B, 2, 11, 11, 16)
            for s in (2, 1, 0):
                f, b = Lh.fw[s], Lh.bw[s]
                c0, r0a, r0b, r1a, r1b = Lh.specs[s]
                for name, cs, dy, mask, add in (("d_yb", r1b, dO, f["yb"][:B], None),
                                                ("d_ra", r1a, b["d_yb"], f["ra"][:B], dO),
                                                ("d_ya", r0b, b["d_ra"], f["ya"][:B], None),
                                                ("d_p", r0a, b["d_ya"], f["p"][:B], b["d_ra"])):
                    ref = ConvSpec(cs.name, cs.cin, cs.cout, cs.cin_real, cs.H, cs.W, w=cs.w, b=cs.b,
                                   wb=cs.w.double())
                    y = torch.zeros(b[name].shape, dtype=torch.float64, device=DEV)
                    tops.conv(dy.double(), ref, y, transpose=True, mask=mask.double(),
                              add=None if add is None else add.double())
                    assert _rel(b[name], y) < 2e-5, (s, name, _rel(b[name], y))
                if s > 0:
                    dO = Lh.bw[s - 1]["d_o"]
        Lh._seg3()
        torch.cuda.synchronize()
        assert torch.isfinite(Lh.p32).all()
    e32 = errs["fp32"]
    print({k: f"{v:.2e}" for k, v in e32.items()})
    print("bf16 worst", max(errs["bf16"].values()))
    head = {k: v for k, v in e32.items() if not k.startswith("stacks.")}
    assert max(head.values()) < 1e-4, head
    assert max(e32.values()) < 1e-2, e32
    assert max(e32.values()) < 0.1 * max(errs["bf16"].values()), errs


@pytest.mark.parametrize("kind,key,R", [("rb", (16, 42), 10), ("rb", (16, 42), 7), ("rb", (32, 21), 11),
                                        ("rb", (32, 21), 7), ("rb", (32, 11), 6),
                                        ("sc", (16, 16, 42, 0), 21), ("sc", (16, 16, 42, 0), 14),
                                        ("sc", (32, 16, 42, 0), 11), ("sc", (32, 32, 21, 0), 11),
                                        ("sc", (32, 32, 21, 0), 7), ("sc", (16, 32, 42, 1), 6),
                                        ("sc", (32, 32, 21, 1), 8)])
def test_split_band_variants_vs_fp64(kind, key, R, monkeypatch):
    """The row-band variants of the split kernels (ops/impala.py SPLIT_BANDS: fewer staged
    rows per workgroup, more workgroups per CU) compute the same convolutions."""
    from apex_dqn_amd.ops import impala as I
    hops, tops = _hops(), TorchImpalaOps()
    monkeypatch.setattr(I, "SPLIT_BANDS", {(kind,) + key: R})
    g = torch.Generator(device=DEV).manual_seed(R)
    N = 5
    if kind == "rb":
        C, H = key
        x = _t(N, C // 16, H, g)
        (c0, r0), (c1, r1) = _spec(C, C, H, seed=3), _spec(C, C, H, seed=4)
        out = torch.zeros(N, C // 16, H, H, 16, device=DEV)
        ys = torch.zeros_like(out)
        outr = torch.zeros(out.shape, dtype=torch.float64, device=DEV)
        ysr = torch.zeros_like(outr)
        kw = dict(n_save=3, target=True, n_switch=4, relu_out=True)
        hops.resblock(x, c0, c1, out, ysave=ys, **kw)
        tops.resblock(x.double(), r0, r1, outr, ysave=ysr, **kw)
        assert _rel(out, outr) < TOL and _rel(ys[:3], ysr[:3]) < TOL
        return
    cin, cout, H, pool = key
    cs, ref = _spec(cin, cout, H, seed=6)
    x = _t(N, cin // 16, H, g)
    if pool:
        Ho = (H + 1) // 2
        p = torch.zeros(N, cout // 16, Ho, Ho, 16, device=DEV)
        a = torch.zeros(N, cout // 16, Ho, Ho, 16, dtype=torch.uint8, device=DEV)
        hops.conv_pool(x, cs, p, a, second=cs.extra["b_tgt"], n_switch=2)
        y = torch.zeros(N, cout // 16, H, H, 16, dtype=torch.float64, device=DEV)
        tops.conv(x.double(), ref, y, second=ref.extra["b_tgt"], n_switch=2)
        pr, ar = torch.zeros(p.shape, dtype=torch.float64, device=DEV), torch.zeros_like(a)
        tops.maxpool(y, pr, ar)
        assert _rel(p, pr) < TOL and (a == ar).float().mean().item() > 0.999
        return
    # the data-gradient use: (cin, cout) is the transposed conv's (spec cout, spec cin)
    cs, ref = _spec(cout, cin, H, seed=6)
    dy = _t(N, cin // 16, H, g)
    m2, a2 = _t(N, cout // 16, H, g), _t(N, cout // 16, H, g)
    dx = torch.zeros(N, cout // 16, H, H, 16, device=DEV)
    dxr = torch.zeros(dx.shape, dtype=torch.float64, device=DEV)
    hops.conv(dy, cs, dx, transpose=True, mask=m2, add=a2)
    tops.conv(dy.double(), ref, dxr, transpose=True, mask=m2.double(), add=a2.double())
    assert _rel(dx, dxr) < TOL, _rel(dx, dxr)
