"""fp32-accurate ("split") mode of every learner kernel vs fp64 PyTorch references.

Operands are fp32 tensors passed as hi + lo bf16 planes (value = hi + lo); the
kernels run hi.hi + lo.hi + hi.lo bf16 MFMAs with fp32 accumulation (conv1: exact
uint8 pixels x f16 hi + scaled-lo weights) and write fp32-accurate outputs as hi / lo
planes again.  Tolerance 1e-4 relative (norm-wise) -- plain bf16 operands sit at
~3e-3 on the same data, so these tests separate the two paths by > 10x.
"""
import numpy as np
import pytest
import torch

from apex_dqn_amd.ops.switches import SW

from apex_dqn_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)
TOL = 1e-4


def _lib():
    from apex_dqn_amd.ops import _lib as L
    return L.require_kernels()


def _split(x32):
    """fp32 (any device) -> (hi, lo) bf16 planes on the GPU."""
    x32 = x32.to(DEV, torch.float32)
    hi = x32.to(torch.bfloat16)
    lo = (x32 - hi.float()).to(torch.bfloat16)
    return hi, lo


def _join(hi, lo):
    return hi.double() + lo.double()


def _rel(a, b):
    """norm-wise relative error, computed in fp64 on the CPU"""
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def _c(t):
    """fp64 CPU copy for the reference computations"""
    return t.detach().double().cpu()


def _empty2(*shape):
    return (torch.empty(*shape, dtype=torch.bfloat16, device=DEV),
            torch.empty(*shape, dtype=torch.bfloat16, device=DEV))


def test_split_planes_represent_fp32():
    x = torch.randn(1 << 16) * 3
    hi, lo = _split(x)
    assert _rel(_join(hi, lo).cpu(), x.double()) < 5e-6      # ~2^-17 per element (measured 2.4e-6)
    assert _rel(hi.double().cpu(), x.double()) > 1e-3         # bf16 alone: ~2^-9


@pytest.mark.parametrize("N,switch", [(64, 0), (200, 128)])
def test_conv1_split_fwd(N, switch):
    from apex_dqn_amd.ops import conv as C
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    g = torch.Generator(device="cpu").manual_seed(N)
    raw = torch.randint(0, 256, (60, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    ring = to_s2d(raw)
    slots = torch.randint(0, 60, (N, 4), generator=g, dtype=torch.int32).to(DEV)
    wa32 = (torch.randn(64, 4, 8, 8, generator=g) * 0.05).to(DEV)
    wb32 = (torch.randn(64, 4, 8, 8, generator=g) * 0.05).to(DEV)
    wa32[0, 0, 0, :4] = torch.tensor([1e-5, -3e-7, 2e-9, 0.0])   # tiny weights (f16 subnormal range)
    ba = (torch.randn(64, generator=g) * 0.1).to(DEV)
    bb = (torch.randn(64, generator=g) * 0.1).to(DEV)
    hi, lo = _empty2(N, 20, 20, 64)
    two = dict(w2=wb32.to(torch.bfloat16), b2=bb, rows_first=switch, w2_32=wb32) if switch else {}
    C.conv1_s2d_fwd(_lib(), C.Workspace(), ring, slots, wa32.to(torch.bfloat16), ba, 1 / 255.0, hi,
                    w32=wa32, out_lo=lo, **two)
    frames = _c(raw[slots.long()])
    if switch:
        ref = torch.cat([R.conv1_fwd(frames[:switch], _c(wa32), _c(ba), 1 / 255.0, torch.float64),
                         R.conv1_fwd(frames[switch:], _c(wb32), _c(bb), 1 / 255.0, torch.float64)])
    else:
        ref = R.conv1_fwd(frames, _c(wa32), _c(ba), 1 / 255.0, torch.float64)
    assert _rel(_join(hi, lo), ref) < TOL


@pytest.mark.parametrize("layer", [2, 3])
def test_conv_split_fwd_with_weight_switch(layer):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(layer)
    N1, N2 = 128, 64
    if layer == 2:
        x = torch.relu(torch.randn(N1 + N2, 20, 20, 64, generator=g))
        wa, wb = torch.randn(64, 4, 4, 64, generator=g) * 0.03, torch.randn(64, 4, 4, 64, generator=g) * 0.03
        stride, oh = 2, 9
    else:
        x = torch.relu(torch.randn(N1 + N2, 9, 9, 64, generator=g))
        wa, wb = torch.randn(64, 3, 3, 64, generator=g) * 0.04, torch.randn(64, 3, 3, 64, generator=g) * 0.04
        stride, oh = 1, 7
    ba, bb = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    xh, xl = _split(x)
    wah, wal = _split(wa)
    wbh, wbl = _split(wb)
    hi, lo = _empty2(N1 + N2, oh, oh, 64)
    C.conv_fwd(_lib(), xh, wah, ba, stride, hi, wbh, bb, N1, x_lo=xl, w_lo=wal, w2_lo=wbl, out_lo=lo)
    xd = _c(x)
    ref = torch.cat([R.conv_fwd(xd[:N1], _c(wa), _c(ba), stride, torch.float64),
                     R.conv_fwd(xd[N1:], _c(wb), _c(bb), stride, torch.float64)])
    assert _rel(_join(hi, lo), ref) < TOL
    # ReLU applied in fp32 before the split: no negative hi + lo anywhere
    assert float(_join(hi, lo).min()) >= 0.0


@pytest.mark.parametrize("M", [200, 1536])
def test_dense_split_fwd_dgrad_wgrad(M):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(M)
    lib = _lib()
    x = torch.relu(torch.randn(M, 3136, generator=g))
    w = torch.randn(1024, 3136, generator=g) * 0.02
    b = (torch.randn(1024, generator=g) * 0.1).to(DEV)
    xh, xl = _split(x)
    wh, wl = _split(w)
    hi, lo = _empty2(M, 1024)
    C.dense_fwd(lib, xh, wh, b, hi, relu=True, x_lo=xl, w_lo=wl, out_lo=lo)
    ref = R.fc_fwd(_c(x), _c(w), _c(b), torch.float64)
    assert _rel(_join(hi, lo), ref) < TOL
    # data gradient: (dh @ w) * (mask > 0), the natural weight read K-major
    dh = torch.randn(M, 1024, generator=g) * 0.01
    dhh, dhl = _split(dh)
    mask = torch.randn(M, 3136, generator=g).to(DEV, torch.bfloat16)
    gh, gl = _empty2(M, 3136)
    C.dense_dgrad(lib, dhh, wh, gh, mask, dh_lo=dhl, w_lo=wl, out_lo=gl)
    ref2 = (_c(dh) @ _c(w)) * (_c(mask) > 0)
    assert _rel(_join(gh, gl), ref2) < TOL
    # weight gradient
    dw = torch.empty(1024, 3136, device=DEV)
    db = torch.empty(1024, device=DEV)
    C.dense_wgrad(lib, dhh, xh, dw, db, dy_lo=dhl, x_lo=xl)
    assert _rel(dw, _c(dh).t() @ _c(x)) < TOL
    assert _rel(db, _c(dh).sum(0)) < TOL


@pytest.mark.parametrize("N", [3, 64])
def test_conv_split_dgrad(N):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 7)
    lib = _lib()
    w3, w2 = torch.randn(64, 3, 3, 64, generator=g) * 0.04, torch.randn(64, 4, 4, 64, generator=g) * 0.03
    dy3, dy2 = torch.randn(N, 7, 7, 64, generator=g), torch.randn(N, 9, 9, 64, generator=g)
    y2 = torch.randn(N, 9, 9, 64, generator=g).to(DEV, torch.bfloat16)
    y1 = torch.randn(N, 20, 20, 64, generator=g).to(DEV, torch.bfloat16)
    (w3h, w3l), (w2h, w2l), (d3h, d3l), (d2h, d2l) = _split(w3), _split(w2), _split(dy3), _split(dy2)
    h3, l3 = _empty2(N, 9, 9, 64)
    C.conv3_dgrad(lib, d3h, w3h, y2, h3, dy_lo=d3l, w_lo=w3l, out_lo=l3)
    ref3 = R.conv_dgrad(_c(dy3), _c(w3), (N, 9, 9, 64), 1, _c(y2), torch.float64)
    assert _rel(_join(h3, l3), ref3) < TOL
    h1, l1 = _empty2(N, 20, 20, 64)
    C.conv2_dgrad(lib, d2h, w2h, y1, h1, dy_lo=d2l, w_lo=w2l, out_lo=l1)
    ref1 = R.conv_dgrad(_c(dy2), _c(w2), (N, 20, 20, 64), 2, _c(y1), torch.float64)
    assert _rel(_join(h1, l1), ref1) < TOL


@pytest.mark.parametrize("N", [3, 64])
def test_conv_split_wgrad(N):
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N + 11)
    lib = _lib()
    ws = C.Workspace()
    for KH, stride, hin, hout in ((3, 1, 9, 7), (4, 2, 20, 9)):
        dy = torch.randn(N, hout, hout, 64, generator=g)
        x = torch.relu(torch.randn(N, hin, hin, 64, generator=g))
        (dyh, dyl), (xh, xl) = _split(dy), _split(x)
        dw = torch.empty(64, KH, KH, 64, device=DEV)
        db = torch.empty(64, device=DEV)
        jobs = []
        C.conv_wgrad(lib, ws, dyh, xh, KH, stride, dw, db, jobs=jobs, dy_lo=dyl, x_lo=xl)
        C.finalize_grads(lib, jobs)
        rdw = torch.nn.grad.conv2d_weight(_c(x).permute(0, 3, 1, 2), (64, 64, KH, KH), _c(dy).permute(0, 3, 1, 2),
                                          stride=stride).permute(0, 2, 3, 1)
        rdb = _c(dy).sum((0, 1, 2))
        assert _rel(dw, rdw) < TOL, (KH, _rel(dw, rdw))
        assert _rel(db, rdb) < TOL


@pytest.mark.parametrize("N,grid", [(3, 0), (64, 0), (37, 5)])
def test_conv1_split_wgrad(N, grid):
    from apex_dqn_amd.ops import conv as C
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    g = torch.Generator(device="cpu").manual_seed(N + 5)
    raw = torch.randint(0, 256, (40, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    ring = to_s2d(raw)
    slots = torch.randint(0, 40, (N, 4), generator=g, dtype=torch.int32).to(DEV)
    dy = torch.randn(N, 20, 20, 64, generator=g)
    dyh, dyl = _split(dy)
    dw = torch.empty(64, 4, 8, 8, device=DEV)
    db = torch.empty(64, device=DEV)
    C.conv1_wgrad_ring(_lib(), C.Workspace(), dyh, ring, slots, 1 / 255.0, dw, db, grid=grid, dy_lo=dyl)
    x = _c(raw[slots.long()]) / 255.0
    rdw = torch.nn.grad.conv2d_weight(x, (64, 4, 8, 8), _c(dy).permute(0, 3, 1, 2), stride=4)
    assert _rel(dw, rdw) < TOL
    assert _rel(db, _c(dy).sum((0, 1, 2))) < TOL


def test_head_split_matches_fp32_torch():
    """ddqn_head / head_wgrad with lo planes == the torch backend on the joined fp32
    activations (the split-mode head contract)."""
    from apex_dqn_amd.ops.fused_ops import HipBackend, TorchBackend
    B, A = 64, 6
    g = torch.Generator(device="cpu").manual_seed(2)
    H = torch.relu(torch.randn(3 * B, 1024, generator=g))
    Hh, Hl = _split(H)
    P = {"wv": (torch.randn(512, generator=g) * 0.05).to(DEV), "bv": torch.zeros(1, device=DEV),
         "wa": (torch.randn(A, 512, generator=g) * 0.05).to(DEV), "ba": (torch.randn(A, generator=g) * 0.1).to(DEV)}
    Pt = {k: (v * 0.9).contiguous() for k, v in P.items()}
    act = torch.randint(0, A, (B,), generator=g, dtype=torch.int32).to(DEV)
    rew = torch.randn(B, generator=g).to(DEV)
    gam = torch.full((B,), 0.97, device=DEV)
    isw = torch.rand(B, generator=g).to(DEV)
    res = {}
    for name, be in (("hip", HipBackend()), ("torch", TorchBackend(torch.float32))):
        td, loss = torch.zeros(B, device=DEV), torch.zeros(B, device=DEV)
        dHh, dHl = _empty2(B, 1024)
        dhead = torch.zeros(B, A + 1, device=DEV)
        be.head(Hh[:2 * B], Hh[2 * B:], P, Pt, act, rew, gam, isw, True, 1.0, 1.0 / B, td, loss, dHh, dhead,
                lo=(Hl[:2 * B], Hl[2 * B:], dHl))
        gr = {"wv": torch.zeros(512, device=DEV), "bv": torch.zeros(1, device=DEV),
              "wa": torch.zeros(A, 512, device=DEV), "ba": torch.zeros(A, device=DEV)}
        be.head_wgrad(Hh, dhead, gr, Hon_lo=Hl)
        torch.cuda.synchronize()
        res[name] = (td, loss, _join(dHh, dHl), dhead, gr)
    a, b = res["hip"], res["torch"]
    for x, y in zip(a[:4], b[:4]):
        assert _rel(x, y) < 1e-5
    for k in a[4]:
        assert _rel(a[4][k], b[4][k]) < 1e-5, k


def test_rmsprop_writes_split_copy():
    from apex_dqn_amd.ops.fused_ops import HipBackend
    n = 100_003
    g = torch.Generator(device="cpu").manual_seed(1)
    p = torch.randn(n, generator=g).to(DEV)
    gr = (torch.randn(n, generator=g) * 0.1).to(DEV)
    v, m = torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
    hi, lo = _empty2(n)
    parts, norm = torch.zeros(1024, dtype=torch.float64, device=DEV), torch.zeros(1, device=DEV)
    HipBackend().optimizer(p, gr, v, m, hi, 2.5e-4, 0.95, 1.5e-7, 40.0, True, parts, norm, pb_lo=lo)
    torch.cuda.synchronize()
    assert _rel(_join(hi, lo), p.double()) < 5e-6     # ~2^-17 per element (measured 2.4e-6)
    assert torch.equal(hi, p.to(torch.bfloat16))


def _fp64_reference_grads(L):
    """Gradients of the learner's batch under fp64 CPU autograd of the dueling network
    (weights = the learner's fp32 master copy, target = its target copy), evaluated in
    the learner's ReLU activation region: the S_t rows use the learner's own ReLU masks,
    so the oracle is the exact gradient of the same piecewise-linear function.  (A
    pre-activation within ~1e-6 of zero can flip its ReLU under any finite precision; one
    flipped element moves a norm-wise layer gradient by ~1e-3.)  Returns (grads keyed like
    the reference state_dict, |delta|, number of mask flips vs an fp64 forward)."""
    import torch.nn.functional as F
    from apex_dqn_amd.models.dueling import DuellingDQN
    from apex_dqn_amd.models.flat_params import flat_to_reference_state
    B, S, rt = L.B, L.S, L.rt
    sd = {k: v.double().requires_grad_(True) for k, v in L.reference_state_dict().items()}
    Qt = DuellingDQN((4, 84, 84), L.A).double()
    Qt.load_state_dict({k: v.double() for k, v in flat_to_reference_state(L.T).items()})
    Qn = DuellingDQN((4, 84, 84), L.A).double()
    Qn.load_state_dict({k: v.detach() for k, v in sd.items()})
    fr = lambda slots: _c(L.replay.gather_frames(slots)) * rt.obs_scale      # noqa: E731
    s_t, s_n = fr(S["obs"]), fr(S["nxt"])
    nchw = lambda t: (_c(t[:B]) > 0).double().permute(0, 3, 1, 2)            # noqa: E731
    m1, m2, m3 = nchw(L.y1), nchw(L.y2), nchw(L.y3)
    mh = (_c(L.h[:B]) > 0).double()
    p1 = F.conv2d(s_t, sd["layer1.0.weight"], sd["layer1.0.bias"], stride=4)
    p2 = F.conv2d(p1 * m1, sd["layer2.0.weight"], sd["layer2.0.bias"], stride=2)
    p3 = F.conv2d(p2 * m2, sd["layer3.0.weight"], sd["layer3.0.bias"])
    flat = (p3 * m3).reshape(B, 3136)
    hv = F.linear(flat, sd["value_stream_layer.0.weight"], sd["value_stream_layer.0.bias"]) * mh[:, :512]
    ha = F.linear(flat, sd["advantage_stream_layer.0.weight"], sd["advantage_stream_layer.0.bias"]) * mh[:, 512:]
    v = F.linear(hv, sd["value.weight"], sd["value.bias"])
    adv = F.linear(ha, sd["advantage.weight"], sd["advantage.bias"])
    q = v + adv - adv.mean(1, keepdim=True)
    with torch.no_grad():
        a_star = Qn(s_n)[2].argmax(1, keepdim=True)
        G = _c(S["rew"]) + _c(S["gam"]) * Qt(s_n)[2].gather(1, a_star).squeeze(1)
        # ReLU decisions of a plain fp64 forward that differ from the learner's (informational)
        f1 = F.relu(p1)
        f2 = F.relu(F.conv2d(f1, sd["layer2.0.weight"], sd["layer2.0.bias"], stride=2))
        flips = int(((p1 > 0).double() != m1).sum()) + int(((f2 > 0).double() != m2).sum())
    q_sa = q.gather(1, S["act"].long().cpu().view(-1, 1)).squeeze(1)
    delta = G - q_sa
    a = delta.abs()
    per = torch.where(a <= 1.0, 0.5 * delta * delta, a - 0.5)
    loss = (per * _c(S["weights"])).mean()
    loss.backward()
    return {k: t.grad for k, t in sd.items()}, a.detach(), flips


@pytest.mark.parametrize("B", [128, 74, 36])
def test_whole_step_fp32_split_matches_fp64_oracle(B):
    """The whole fused learner step in its default fp32 (split) mode: every gradient
    segment within 1e-3 relative (norm-wise; measured ~1e-5) of fp64 CPU autograd on the
    same batch in the same ReLU region; the bf16-operand mode and the torch fp32 backend
    (MIOpen / hipBLASLt) are measured against the same oracle and printed.  B = 74 / 36:
    the per-rank row counts of a global-batch DP step (ApexConfig.dp_batch), whose
    online / target switch is not on a 128-row tile (two launches per weight set)."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.models.flat_params import flat_to_reference_state
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    errs_all = {}
    for mode, be, dtype in (("fp32_split", "hip", "fp32"), ("bf16", "hip", "bf16"), ("torch_fp32", "torch", "fp32")):
        cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                    "Learner": {"replay_sample_size": B},
                                    "Runtime": {"use_graphs": False, "presample": False, "dtype": dtype}})
        torch.manual_seed(0)
        rp = GpuReplayShard(2000, 2000, 2100, 4, device=DEV, seed=7)
        rng = np.random.default_rng(11)
        seqs = rp.append_frames(rng.integers(0, 255, (1800, 84, 84), dtype=np.uint8))
        K = 1500
        st = np.stack([seqs[i:i + 4] for i in range(K)])
        rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K) * 2,
                       Gamma=np.where(rng.random(K) < 0.1, 0.0, 0.97), priority=rng.random(K)))
        L = FusedNatureLearner(cfg, DEV, rp, backend=be)
        assert L.split == (mode == "fp32_split")
        L._seg1()
        L._seg2()
        torch.cuda.synchronize()
        ref, td_ref, flips = _fp64_reference_grads(L)
        g = flat_to_reference_state(L.G)
        errs_all[mode] = {k: _rel(g[k], ref[k]) for k in ref}
        errs_all[mode]["td_abs"] = _rel(L.td_abs, td_ref)
        print(f"{mode}: {flips} conv ReLU decisions differ from a plain fp64 forward")
    for mode, e in errs_all.items():
        print(f"per-segment relative grad error vs fp64 ({mode}):", {k: f"{v:.2e}" for k, v in e.items()})
    e = errs_all["fp32_split"]
    assert max(e.values()) < 1e-3, e
    # the split path is a different precision class from the bf16-operand path
    assert max(e.values()) < 0.2 * max(errs_all["bf16"].values())


@pytest.mark.parametrize("grid", [0, 5])
def test_conv2_image_resident_split_kernels_vs_generic(monkeypatch, grid):
    """The image-resident conv2 forward / data-gradient kernels in split mode (LDS-DMA
    double-buffered planes; four-wave class-owning dgrad) match fp64 and the generic
    implicit-GEMM split path; small grids walk several images per workgroup across
    the online / target switch."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(grid + 3)
    lib = _lib()
    N1, N2 = 23, 14
    x = torch.relu(torch.randn(N1 + N2, 20, 20, 64, generator=g))
    wa, wb = torch.randn(64, 4, 4, 64, generator=g) * 0.03, torch.randn(64, 4, 4, 64, generator=g) * 0.03
    ba, bb = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    (xh, xl), (wah, wal), (wbh, wbl) = _split(x), _split(wa), _split(wb)
    hi, lo = _empty2(N1 + N2, 9, 9, 64)
    C.conv2_img_fwd(lib, xh, wah, ba, hi, wbh, bb, N1, grid=grid, x_lo=xl, w_lo=wal, w2_lo=wbl, out_lo=lo)
    xd = _c(x)
    ref = torch.cat([R.conv_fwd(xd[:N1], _c(wa), _c(ba), 2, torch.float64),
                     R.conv_fwd(xd[N1:], _c(wb), _c(bb), 2, torch.float64)])
    assert _rel(_join(hi, lo), ref) < TOL
    monkeypatch.setattr(SW, "conv2_img", False)
    gh, gl = _empty2(N1 + N2, 9, 9, 64)
    C.conv_fwd(lib, xh, wah, ba, 2, gh, wbh, bb, N1, x_lo=xl, w_lo=wal, w2_lo=wbl, out_lo=gl)
    assert _rel(_join(hi, lo), _join(gh, gl)) < TOL
    # data gradient
    N = N1 + N2
    dy = torch.randn(N, 9, 9, 64, generator=g)
    y1 = torch.randn(N, 20, 20, 64, generator=g).to(DEV, torch.bfloat16)
    dh, dl = _split(dy)
    h1, l1 = _empty2(N, 20, 20, 64)
    C.conv2_dgrad_img(lib, dh, wah, y1, h1, grid=grid, dy_lo=dl, w_lo=wal, out_lo=l1)
    ref1 = R.conv_dgrad(_c(dy), _c(wa), (N, 20, 20, 64), 2, _c(y1), torch.float64)
    assert _rel(_join(h1, l1), ref1) < TOL
    monkeypatch.setattr(SW, "conv2_dgrad_img", False)
    g1h, g1l = _empty2(N, 20, 20, 64)
    C.conv2_dgrad(lib, dh, wah, y1, g1h, dy_lo=dl, w_lo=wal, out_lo=g1l)
    assert _rel(_join(h1, l1), _join(g1h, g1l)) < TOL


@pytest.mark.parametrize("N,grid", [(74, 0), (146, 0), (37, 5)])
def test_conv2_dgrad_class_split_bit_identical(monkeypatch, N, grid):
    """The small-batch split conv2 data gradient (one workgroup per (image, stride-parity
    class), csrc/conv2_img.hip conv2_dgrad_img_split_cls_kernel) writes exactly the bytes of
    the per-image kernel: same fragments, K order and accumulation; several images per
    workgroup when the grid is small."""
    from apex_dqn_amd.ops import conv as C
    g = torch.Generator(device="cpu").manual_seed(N)
    lib = _lib()
    w = torch.randn(64, 4, 4, 64, generator=g) * 0.03
    dy = torch.randn(N, 9, 9, 64, generator=g)
    y1 = torch.randn(N, 20, 20, 64, generator=g).to(DEV, torch.bfloat16)
    (wh, wl), (dh, dl) = _split(w), _split(dy)
    outs = {}
    for cmax in (0, 4096):
        monkeypatch.setattr(SW, "conv2_dgrad_cls_max", cmax)
        h1, l1 = _empty2(N, 20, 20, 64)
        C.conv2_dgrad_img(lib, dh, wh, y1, h1, grid=grid, dy_lo=dl, w_lo=wl, out_lo=l1)
        torch.cuda.synchronize()
        outs[cmax] = (h1, l1)
    assert torch.equal(outs[0][0].view(torch.int16), outs[4096][0].view(torch.int16))
    assert torch.equal(outs[0][1].view(torch.int16), outs[4096][1].view(torch.int16))
    ref = R.conv_dgrad(_c(dy), _c(w), (N, 20, 20, 64), 2, _c(y1), torch.float64)
    assert _rel(_join(*outs[4096]), ref) < TOL


@pytest.mark.parametrize("split", [True, False])
@pytest.mark.parametrize("grid_images", [64, 600])
def test_conv2_fwd_weights_packed_in_conv1_launch(grid_images, split):
    """The split conv2 forward's weight-fragment pack that rides on the conv1 launch
    (csrc/conv2_wfrag.h c2f_pack_range; fewer and more conv1 workgroups than fragment
    blocks) gives bit-identical conv2 outputs to the conv2 launcher's own pack."""
    from apex_dqn_amd.ops import conv as C
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    g = torch.Generator(device="cpu").manual_seed(21)
    raw = torch.randint(0, 256, (60, 84, 84), generator=g, dtype=torch.uint8).to(DEV)
    ring = to_s2d(raw)
    N = grid_images
    slots = torch.randint(0, 60, (N, 4), generator=g, dtype=torch.int32).to(DEV)
    w1 = (torch.randn(64, 4, 8, 8, generator=g) * 0.05).to(DEV)
    b1 = (torch.randn(64, generator=g) * 0.1).to(DEV)
    y1, y1l = _empty2(N, 20, 20, 64)
    (wh, wl), (w2h, w2l) = _split((torch.randn(64, 4, 4, 64, generator=g) * 0.03).to(DEV)), \
        _split((torch.randn(64, 4, 4, 64, generator=g) * 0.03).to(DEV))
    b2a, b2b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    sw = 2 * N // 3
    outs = [_empty2(N, 9, 9, 64) for _ in range(2)]
    c1lo = dict(w32=w1, out_lo=y1l) if split else {}
    c2lo = (lambda o: dict(x_lo=y1l, w_lo=wl, w2_lo=w2l, out_lo=o)) if split else (lambda o: {})
    C.conv1_s2d_fwd(_lib(), C.Workspace(), ring, slots, w1.to(torch.bfloat16), b1, 1 / 255.0, y1, **c1lo)
    C.conv2_img_fwd(_lib(), y1, wh, b2a, outs[0][0], w2h, b2b, sw, **c2lo(outs[0][1]))
    C.c2f_wfrag_fwd_buffer(DEV).fill_(3.0)    # stale contents: the conv1 launch must overwrite them
    C.conv1_s2d_fwd(_lib(), C.Workspace(), ring, slots, w1.to(torch.bfloat16), b1, 1 / 255.0, y1,
                    c2f=(wh, wl, w2h, w2l) if split else (wh, None, w2h, None), **c1lo)
    C.conv2_img_fwd(_lib(), y1, wh, b2a, outs[1][0], w2h, b2b, sw, packed=True, **c2lo(outs[1][1]))
    torch.cuda.synchronize()
    assert torch.equal(outs[0][0], outs[1][0])
    if split:
        assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("N,switch,copy_n,C,grid", [(1536, 1024, 512, 4, 0), (96, 64, 32, 4, 0), (37, 20, 9, 4, 5),
                                                    (50, 50, 50, 1, 0), (40, 24, 0, 2, 7)])
def test_conv12_fused_split_vs_fp64_and_separate_kernels(N, switch, copy_n, C, grid):
    """conv1 -> conv2 fused (csrc/conv12_fused.hip: y1 kept in LDS, conv2 weights streamed
    from L2 in fragment order) against fp64 and against the two separate split kernels:
    the online / target switch inside a workgroup's range (small grids), the S_t rows'
    y1 written out (copy_n), C in {1, 2, 4}."""
    from apex_dqn_amd.ops import conv as C_
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    g = torch.Generator(device="cpu").manual_seed(N + C)
    raw = torch.randint(0, 256, (80, 84, 84), generator=g, dtype=torch.uint8)
    ring = to_s2d(raw.to(DEV))
    slots = torch.randint(0, 80, (N, C), generator=g, dtype=torch.int32).to(DEV)
    w1a, w1b = (torch.randn(64, C, 8, 8, generator=g) * 0.05).to(DEV), (torch.randn(64, C, 8, 8, generator=g) * 0.05).to(DEV)
    b1a, b1b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    w2a, w2b = torch.randn(64, 4, 4, 64, generator=g) * 0.03, torch.randn(64, 4, 4, 64, generator=g) * 0.03
    b2a, b2b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    (w2ah, w2al), (w2bh, w2bl) = _split(w2a), _split(w2b)
    scale = 1 / 255.0
    ws = C_.Workspace()
    y2h, y2l = _empty2(N, 9, 9, 64)
    y1h, y1l = _empty2(max(copy_n, 1), 20, 20, 64)
    two = switch < N
    kw2 = dict(w1b=w1b, b1b=b1b, w2b=w2bh, w2b_lo=w2bl, b2b=b2b, rows_first=switch) if two else {}
    C_.conv12_fused_fwd(_lib(), ws, ring, slots, w1a, b1a, w2ah, w2al, b2a, scale, y2h, y2l, y1=y1h, y1_lo=y1l,
                        copy_n=copy_n, grid=grid, **kw2)
    torch.cuda.synchronize()
    # fp64 reference
    fr = torch.stack([raw[slots[i].long().cpu()] for i in range(N)]).double() * scale
    ref1 = torch.empty(N, 64, 20, 20, dtype=torch.float64)
    for lo, hi, w, b in ((0, switch, w1a, b1a), (switch, N, w1b, b1b)):
        if hi > lo:
            ref1[lo:hi] = torch.relu(torch.nn.functional.conv2d(fr[lo:hi], _c(w), _c(b), stride=4))
    x1 = ref1.permute(0, 2, 3, 1)      # NHWC
    ref2 = torch.cat([R.conv_fwd(x1[:switch], _c(w2a), _c(b2a), 2, torch.float64)] +
                     ([R.conv_fwd(x1[switch:], _c(w2b), _c(b2b), 2, torch.float64)] if two else []))
    assert _rel(_join(y2h, y2l), ref2) < TOL, _rel(_join(y2h, y2l), ref2)
    if copy_n:
        assert _rel(_join(y1h, y1l)[:copy_n], x1[:copy_n]) < TOL
    # the separate split kernels on the same data (conv1 -> HBM -> conv2)
    s1h, s1l = _empty2(N, 20, 20, 64)
    s2h, s2l = _empty2(N, 9, 9, 64)
    C_.conv1_s2d_fwd(_lib(), ws, ring, slots, w1a.to(torch.bfloat16), b1a, scale, s1h,
                     w1b.to(torch.bfloat16) if two else None, b1b if two else None, switch if two else 0,
                     w32=w1a, w2_32=w1b if two else None, out_lo=s1l)
    C_.conv2_img_fwd(_lib(), s1h, w2ah, b2a, s2h, w2bh if two else None, b2b if two else None, switch if two else 0,
                     x_lo=s1l, w_lo=w2al, w2_lo=w2bl if two else None, out_lo=s2l)
    torch.cuda.synchronize()
    assert _rel(_join(y2h, y2l), _join(s2h, s2l)) < TOL
    if copy_n:
        assert _rel(_join(y1h, y1l)[:copy_n], _join(s1h, s1l)[:copy_n]) < 1e-5


@pytest.mark.parametrize("N,switch,copy_n,C,grid", [(1536, 1024, 512, 4, 0), (37, 20, 9, 4, 5), (50, 50, 50, 1, 0),
                                                    (40, 24, 0, 2, 7)])
def test_conv12_fused_bf16_vs_fp64_and_separate_kernels(N, switch, copy_n, C, grid):
    """The bf16 learner's fused conv1 -> conv2 forward (one plane: f16 conv1 operands, bf16
    y1 in LDS, bf16 conv2 weights) against fp64 at bf16-class tolerance and against the
    two separate bf16 kernels (conv1 -> HBM -> conv2)."""
    from apex_dqn_amd.ops import conv as C_
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    g = torch.Generator(device="cpu").manual_seed(N + C + 100)
    raw = torch.randint(0, 256, (80, 84, 84), generator=g, dtype=torch.uint8)
    ring = to_s2d(raw.to(DEV))
    slots = torch.randint(0, 80, (N, C), generator=g, dtype=torch.int32).to(DEV)
    w1a, w1b = (torch.randn(64, C, 8, 8, generator=g) * 0.05).to(DEV), (torch.randn(64, C, 8, 8, generator=g) * 0.05).to(DEV)
    b1a, b1b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    w2a = (torch.randn(64, 4, 4, 64, generator=g) * 0.03).to(DEV, torch.bfloat16)
    w2b = (torch.randn(64, 4, 4, 64, generator=g) * 0.03).to(DEV, torch.bfloat16)
    b2a, b2b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    scale = 1 / 255.0
    ws = C_.Workspace()
    y2 = torch.full((N, 9, 9, 64), float("nan"), device=DEV, dtype=torch.bfloat16)
    y1 = torch.full((max(copy_n, 1), 20, 20, 64), float("nan"), device=DEV, dtype=torch.bfloat16)
    two = switch < N
    kw2 = dict(w1b=w1b, b1b=b1b, w2b=w2b, w2b_lo=None, b2b=b2b, rows_first=switch) if two else {}
    C_.conv12_fused_fwd(_lib(), ws, ring, slots, w1a, b1a, w2a, None, b2a, scale, y2, None, y1=y1, y1_lo=None,
                        copy_n=copy_n, grid=grid, **kw2)
    torch.cuda.synchronize()
    assert not torch.isnan(y2).any()
    fr = torch.stack([raw[slots[i].long().cpu()] for i in range(N)]).double() * scale
    ref1 = torch.empty(N, 64, 20, 20, dtype=torch.float64)
    for lo, hi, w, b in ((0, switch, w1a, b1a), (switch, N, w1b, b1b)):
        if hi > lo:
            ref1[lo:hi] = torch.relu(torch.nn.functional.conv2d(fr[lo:hi], _c(w), _c(b), stride=4))
    x1 = ref1.permute(0, 2, 3, 1)
    ref2 = torch.cat([R.conv_fwd(x1[:switch], _c(w2a), _c(b2a), 2, torch.float64)] +
                     ([R.conv_fwd(x1[switch:], _c(w2b), _c(b2b), 2, torch.float64)] if two else []))
    e2 = _rel(_c(y2), ref2)
    assert e2 < 1e-2, e2                      # bf16 y1 and y2 roundings (2^-9 each)
    if copy_n:
        e1 = _rel(_c(y1)[:copy_n], x1[:copy_n])
        assert e1 < 5e-3, e1
    s1 = torch.empty(N, 20, 20, 64, device=DEV, dtype=torch.bfloat16)
    s2 = torch.empty(N, 9, 9, 64, device=DEV, dtype=torch.bfloat16)
    C_.conv1_s2d_fwd(_lib(), ws, ring, slots, w1a.to(torch.bfloat16), b1a, scale, s1,
                     w1b.to(torch.bfloat16) if two else None, b1b if two else None, switch if two else 0)
    C_.conv2_img_fwd(_lib(), s1, w2a, b2a, s2, w2b if two else None, b2b if two else None, switch if two else 0)
    torch.cuda.synchronize()
    es = _rel(_c(s2), ref2)
    print(f"bf16 conv2 output vs fp64: fused {e2:.2e}, separate kernels {es:.2e}")
    assert e2 < 1.5 * es + 1e-4               # f16 conv1 operands: no worse than the bf16 kernels


@pytest.mark.parametrize("N,grid", [(1536, 0), (37, 5)])
def test_work_queue_outputs_bit_identical_to_static_order(N, grid, monkeypatch):
    """The persistent kernels' image work queue (csrc/mfma_common.h wq_next, enabled by the
    data-parallel learner) computes every image whole in one workgroup: the fused conv1 ->
    conv2 forward and the split conv2 data gradient give bit-identical outputs with the
    queue on or off, as does the conv1 weight gradient (items = image groups, one partial
    slot per item), and three queued launches in a row (one never-reset counter, read
    modulo items + workgroups) agree too."""
    from apex_dqn_amd.ops import conv as C_
    from apex_dqn_amd.replay.gpu_replay import to_s2d
    g = torch.Generator(device="cpu").manual_seed(N + 11)
    raw = torch.randint(0, 256, (80, 84, 84), generator=g, dtype=torch.uint8)
    ring = to_s2d(raw.to(DEV))
    slots = torch.randint(0, 80, (N, 4), generator=g, dtype=torch.int32).to(DEV)
    w1 = (torch.randn(64, 4, 8, 8, generator=g) * 0.05).to(DEV)
    b1, b2 = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    w2h, w2l = _split(torch.randn(64, 4, 4, 64, generator=g) * 0.03)
    copy_n = N // 3
    dy = torch.randn(N, 9, 9, 64, generator=g)
    dh, dl = _split(dy)
    mask = torch.randn(N, 20, 20, 64, generator=g).to(DEV, torch.bfloat16)
    d1h, d1l = _split(torch.randn(N, 20, 20, 64, generator=g) * 0.1)
    outs = []
    # (the per-image data-gradient kernel: the small-batch (image, class) variant has no queue)
    monkeypatch.setattr(SW, "conv2_dgrad_cls_max", 0)
    for wq, reps in ((False, 1), (True, 3)):
        ws = C_.Workspace()
        monkeypatch.setattr(SW, "work_queue", "on" if wq else "off")   # (the forward's queue is switch-only)
        for _ in range(reps):
            y2h, y2l = _empty2(N, 9, 9, 64)
            y1h, y1l = _empty2(copy_n, 20, 20, 64)
            C_.conv12_fused_fwd(_lib(), ws, ring, slots, w1, b1, w2h, w2l, b2, 1 / 255.0, y2h, y2l, y1=y1h,
                                y1_lo=y1l, copy_n=copy_n, grid=grid)
            dxh, dxl = _empty2(N, 20, 20, 64)
            C_.conv2_dgrad_img(_lib(), dh, w2h, mask, dxh, grid=grid, dy_lo=dl, w_lo=w2l, out_lo=dxl, ws=ws)
            # conv1 weight gradient: items = image groups with per-item partial slots
            dw1, db1 = torch.zeros(64, 4, 8, 8, device=DEV), torch.zeros(64, device=DEV)
            C_.conv1_wgrad_ring(_lib(), ws, d1h, ring, slots, 1 / 255.0, dw1, db1, grid=grid, dy_lo=d1l)
            torch.cuda.synchronize()
            outs.append((y2h, y2l, y1h, y1l, dxh, dxl, dw1, db1))
        if wq:   # each launch consumed exactly items + workgroups values of its counter
            c = [int(t.item()) for k, t in ws.bufs.items() if k[0][0] in ("cf_wq", "c2d_wq", "c1w_wq")]
            assert len(c) == 3 and all(v > 0 and v % 3 == 0 for v in c), c
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)


def _presample_learner(monkeypatch, opt_frags: bool, dtype: str = "fp32"):
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    monkeypatch.setattr(SW, "opt_frags", opt_frags)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 128},
                                "Runtime": {"use_graphs": False, "presample": True, "dtype": dtype}})
    torch.manual_seed(0)
    rp = GpuReplayShard(2000, 2000, 2100, 4, device=DEV, seed=7)
    rng = np.random.default_rng(11)
    seqs = rp.append_frames(rng.integers(0, 255, (1800, 84, 84), dtype=np.uint8))
    K = 1500
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K) * 2,
                   Gamma=np.where(rng.random(K) < 0.1, 0.0, 0.97), priority=rng.random(K)))
    return FusedNatureLearner(cfg, DEV, rp, backend="hip")


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_optimizer_stores_conv12_fragments_bit_identical_to_pack(monkeypatch, dtype):
    """The optimizer + sample launch stores the updated w1 / w2 in the fused forward's
    fragment order (csrc/cf_pack.h cf_frag_store): after real steps the online fragments
    are byte-identical to a fresh pack launch, and the run's weights are bit-identical to
    the pack-launch variant's (SW.opt_frags = False)."""
    from apex_dqn_amd.ops import conv as C
    out = {}
    for opt in (True, False):
        L = _presample_learner(monkeypatch, opt, dtype)
        assert L._c12 and (L._frag_out is not None) == opt
        for _ in range(3):
            L.step()
        torch.cuda.synchronize()
        out[opt] = L.p32.clone()
        if opt:
            ws, dev = L.ops.ws, L.device
            w1f = ws.get(("cf_w1frag",), C.CF_W1FRAG_BYTES, dev, torch.uint8)
            c2f = ws.get(("cf_c2f_wfrag",), 4 * 8192 * 16, dev, torch.uint8)
            half = C.CF_W1FRAG_BYTES // 2          # set 0 (online) of w1; hi + lo planes of set 0 of w2
            planes = 2 if dtype == "fp32" else 1   # (bf16: the hi plane only is read)
            got = (w1f[:half].clone(), c2f[:planes * 8192 * 16].clone())
            c1, c2 = L._conv12_weights()
            L.ops.conv12_pack(c1, c2, L.rt.obs_scale, sets=1)
            torch.cuda.synchronize()
            assert torch.equal(got[0], w1f[:half]), "conv1 fragments differ from the pack launch"
            assert torch.equal(got[1], c2f[:planes * 8192 * 16]), "conv2 C2F fragments differ from the pack launch"
        del L
    assert torch.equal(out[True], out[False])


@pytest.mark.parametrize("N,switch,C,grid,split", [(1536, 1024, 4, 0, True), (222, 148, 4, 0, True),
                                                   (37, 20, 4, 5, True), (50, 50, 1, 0, True),
                                                   (1536, 1024, 4, 0, False), (37, 20, 2, 5, False)])
def test_conv123_fused_vs_fp64_and_separate_conv3(N, switch, C, grid, split):
    """conv3 fused into the conv1 -> conv2 kernel (csrc/conv12_fused.hip conv3_image: y2 from
    LDS, weights straight from OHWI, two K halves summed in fixed order) against fp64 on
    the kernel's own y2, and against the separate implicit-GEMM conv3 on that y2 (split:
    fp32-class tolerance; bf16: one plane).  y2 itself is unchanged by the fusion."""
    from apex_dqn_amd.ops import conv as C_
    from apex_dqn_amd.replay.gpu_replay import to_s2d

    def _j3(hi, lo):
        return hi.double() + (lo.double() if lo is not None else 0.0)
    g = torch.Generator(device="cpu").manual_seed(N + C + 7)
    raw = torch.randint(0, 256, (80, 84, 84), generator=g, dtype=torch.uint8)
    ring = to_s2d(raw.to(DEV))
    slots = torch.randint(0, 80, (N, C), generator=g, dtype=torch.int32).to(DEV)
    w1a, w1b = (torch.randn(64, C, 8, 8, generator=g) * 0.05).to(DEV), (torch.randn(64, C, 8, 8, generator=g) * 0.05).to(DEV)
    b1a, b1b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    w2a, w2b = torch.randn(64, 4, 4, 64, generator=g) * 0.03, torch.randn(64, 4, 4, 64, generator=g) * 0.03
    b2a, b2b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    w3a, w3b = torch.randn(64, 3, 3, 64, generator=g) * 0.04, torch.randn(64, 3, 3, 64, generator=g) * 0.04
    b3a, b3b = (torch.randn(64, generator=g) * 0.1).to(DEV), (torch.randn(64, generator=g) * 0.1).to(DEV)
    if split:
        (w2ah, w2al), (w2bh, w2bl) = _split(w2a), _split(w2b)
        (w3ah, w3al), (w3bh, w3bl) = _split(w3a), _split(w3b)
    else:
        w2ah, w2bh = w2a.to(DEV).to(torch.bfloat16), w2b.to(DEV).to(torch.bfloat16)
        w3ah, w3bh = w3a.to(DEV).to(torch.bfloat16), w3b.to(DEV).to(torch.bfloat16)
        w2al = w2bl = w3al = w3bl = None
    ws = C_.Workspace()
    y2h, y2l = _empty2(N, 9, 9, 64)
    y3h, y3l = _empty2(N, 7, 7, 64)
    y1h, y1l = _empty2(N, 20, 20, 64)
    kw2 = dict(w1b=w1b, b1b=b1b, w2b=w2bh, w2b_lo=w2bl, b2b=b2b, rows_first=switch) if switch < N else {}
    c3 = (w3ah, w3al, b3a, w3bh, w3bl, b3b)
    C_.conv12_fused_fwd(_lib(), ws, ring, slots, w1a, b1a, w2ah, w2al, b2a, 1 / 255.0, y2h, y2l if split else None,
                        y1=y1h, y1_lo=y1l if split else None, copy_n=N // 3, grid=grid, c3=c3, y3=y3h,
                        y3_lo=y3l if split else None, **kw2)
    # the same launch without conv3: y2 must be bit-identical
    z2h, z2l = _empty2(N, 9, 9, 64)
    C_.conv12_fused_fwd(_lib(), ws, ring, slots, w1a, b1a, w2ah, w2al, b2a, 1 / 255.0, z2h, z2l if split else None,
                        y1=y1h, y1_lo=y1l if split else None, copy_n=N // 3, grid=grid, **kw2)
    torch.cuda.synchronize()
    assert torch.equal(y2h, z2h) and (not split or torch.equal(y2l, z2l))
    x2 = _j3(y2h, y2l if split else None).double().cpu()
    w3s = (_j3(w3ah, w3al) if split else w3ah.float()).double().cpu()
    w3t = (_j3(w3bh, w3bl) if split else w3bh.float()).double().cpu()
    ref3 = torch.cat([R.conv_fwd(x2[:switch], w3s, _c(b3a), 1, torch.float64)] +
                     ([R.conv_fwd(x2[switch:], w3t, _c(b3b), 1, torch.float64)] if switch < N else []))
    got = _j3(y3h, y3l if split else None)
    tol = TOL if split else 1e-2
    assert _rel(got, ref3) < tol, _rel(got, ref3)
    # the separate conv3 kernel on the same y2
    s3h, s3l = _empty2(N, 7, 7, 64)
    C_.conv_fwd(_lib(), y2h, w3ah, b3a, 1, s3h, w3bh if switch < N else None, b3b if switch < N else None,
                switch if switch < N else 0, **(dict(x_lo=y2l, w_lo=w3al, w2_lo=w3bl if switch < N else None,
                                                     out_lo=s3l) if split else {}))
    torch.cuda.synchronize()
    sep = _j3(s3h, s3l if split else None)
    assert _rel(got, sep) < (TOL if split else 1e-2), _rel(got, sep)
