"""IMPALA-deep learner: the hand-written step against autograd (CPU, torch ops)
and every csrc/impala.hip kernel against the torch oracle (GPU)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from apex_dqn_amd.config import ApexConfig
from apex_dqn_amd.learner.impala_learner import FEAT_LD, FusedImpalaLearner, fc_column_perm
from apex_dqn_amd.learner.torch_learner import TorchLearner
from apex_dqn_amd.ops.impala import ConvSpec, TorchImpalaOps, from_planar, to_planar
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard


def _setup(B=4, A=6, device="cpu", loss="huber", dtype="fp32"):
    torch.manual_seed(0)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": A, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": B},
                                "Runtime": {"grad_clip": 40.0, "loss": loss, "network": "impala",
                                            "use_graphs": False, "dtype": dtype}})
    rp = GpuReplayShard(256, 256, 400, 4, device=device)
    rng = np.random.default_rng(0)
    seqs = rp.append_frames(rng.integers(0, 255, (200, 84, 84), dtype=np.uint8))
    K = 150
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    nx = np.stack([seqs[i + 3:i + 7] for i in range(K)])
    g = np.full(K, 0.97)
    g[::5] = 0.0
    rp.insert(dict(S_t=st, S_tpn=nx, A_t=rng.integers(0, A, K), R=rng.normal(size=K) * 3, Gamma=g,
                   priority=rng.random(K)))
    return cfg, rp


def test_planar_roundtrip_and_fc_permutation():
    x = torch.randn(3, 32, 11, 11)
    p = to_planar(x)
    assert p.shape == (3, 2, 11, 11, 16)
    torch.testing.assert_close(from_planar(p), x)
    perm = fc_column_perm()
    flat_planar = p.reshape(3, -1)
    torch.testing.assert_close(flat_planar[:, perm], x.reshape(3, -1))


def test_impala_module_state_roundtrip():
    cfg, rp = _setup()
    L = FusedImpalaLearner(cfg, "cpu", rp)
    sd = L.module_state()
    L2 = FusedImpalaLearner(cfg, "cpu", rp)
    L2.load_module_state(sd)
    torch.testing.assert_close(L2.p32, L.p32)
    assert torch.count_nonzero(L.P["wfc"][:, 3872:]) == 0


def test_maxpool_oracle_backward_matches_autograd():
    ops = TorchImpalaOps()
    x = torch.randn(2, 1, 42, 42, 16)
    y = torch.zeros(2, 1, 21, 21, 16)
    amax = torch.zeros(2, 1, 21, 21, 16, dtype=torch.uint8)
    ops.maxpool(x, y, amax)
    xn = from_planar(x).requires_grad_(True)
    yn = F.max_pool2d(xn, 3, 2, 1)
    torch.testing.assert_close(from_planar(y), yn.detach())
    g = torch.randn_like(yn)
    yn.backward(g)
    dx = torch.zeros_like(x)
    ops.maxpool_bwd(to_planar(g), amax, dx)
    torch.testing.assert_close(from_planar(dx), xn.grad)


def _check_vs_autograd(loss):
    cfg, rp = _setup(loss=loss)
    L = FusedImpalaLearner(cfg, "cpu", rp)
    T = TorchLearner(cfg, "cpu")
    T.Q.load_state_dict(L.module_state())
    T.Q_target.load_state_dict(L.module_state(L.T))
    L._seg1()
    L._seg2()
    B = L.B
    S = L.S
    batch = dict(S_t=rp.gather_frames(L.slots[:B]), S_tpn=rp.gather_frames(L.slots[B:2 * B]), A_t=S["act"],
                 R=S["rew"], Gamma=S["gam"], weights=S["weights"])
    lref, td = T.compute_loss_and_priorities(batch)
    T.optimizer.zero_grad()
    lref.backward()
    assert abs(float(lref) - float(L.loss_b.mean())) < 1e-4 * max(1.0, abs(float(lref)))
    torch.testing.assert_close(td, L.td_abs, rtol=1e-4, atol=1e-5)
    gf = L.module_state(L.G)
    for k, p in T.Q.named_parameters():
        torch.testing.assert_close(gf[k], p.grad, rtol=2e-3, atol=1e-6, msg=lambda m: f"{k}: {m}")


def test_impala_fused_backward_matches_autograd_huber():
    _check_vs_autograd("huber")


def test_impala_fused_backward_matches_autograd_mse():
    _check_vs_autograd("mse")


def test_impala_step_updates_and_checkpoint_roundtrip(tmp_path):
    cfg, rp = _setup()
    L = FusedImpalaLearner(cfg, "cpu", rp)
    p0 = L.p32.clone()
    L.step()
    assert not torch.equal(p0, L.p32)
    assert torch.count_nonzero(L.P["wfc"][:, 3872:]) == 0   # pad columns never move
    path = str(tmp_path / "ck.pt")
    L.save(path)
    L2 = FusedImpalaLearner(cfg, "cpu", rp)
    assert L2.load(path)
    torch.testing.assert_close(L2.p32, L.p32)
    torch.testing.assert_close(L2.rms_v, L.rms_v)
    assert L2.num_q_updates == 1


# ------------------------------------------------------------------ GPU kernels
def _spec(cin, cout, H, dev, cin_real=None, seed=0):
    g = torch.Generator().manual_seed(seed)
    cr = cin_real or cin
    cs = ConvSpec("t", cin, cout, cr, H, H)
    cs.w = (torch.randn(cout, cr, 3, 3, generator=g) * 0.2).to(dev)
    cs.b = (torch.randn(cout, generator=g) * 0.1).to(dev)
    cs.wb = cs.w.to(torch.bfloat16)
    wt = (torch.randn(cout, cr, 3, 3, generator=g) * 0.2).to(dev).to(torch.bfloat16)
    cs.extra["w_tgt"], cs.extra["b_tgt"] = wt, (torch.randn(cout, generator=g) * 0.1).to(dev)
    return cs


def _hip_pack(hops, cs, dev):
    from apex_dqn_amd.ops.impala import frag_elems
    cs.frag = torch.zeros(frag_elems(cs.cin, cs.cout), dtype=torch.bfloat16, device=dev)
    cs.fragT = torch.zeros(frag_elems(cs.cout, cs.cin), dtype=torch.bfloat16, device=dev)
    cs.frag_tgt = torch.zeros_like(cs.frag)
    kind = 2 if cs.cin_real < cs.cin else 0
    jobs = [(cs.wb, cs.frag, cs.cin, cs.cout, cs.cin_real, kind), (cs.extra["w_tgt"], cs.frag_tgt, cs.cin, cs.cout,
                                                                    cs.cin_real, kind)]
    if cs.cin_real == cs.cin:
        jobs.append((cs.wb, cs.fragT, cs.cin, cs.cout, cs.cin_real, 1))
    hops.pack(jobs)


FWD_SHAPES = [(16, 16, 42), (16, 32, 42), (32, 16, 42), (32, 32, 21), (32, 32, 11)]


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,H", FWD_SHAPES)
def test_gpu_sconv_fwd_and_dgrad(cin, cout, H):
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    N = 6
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(N, cin // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
    add = torch.randn(N, cout // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
    mask = torch.randn(N, cout // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
    cs = _spec(cin, cout, H, dev)
    _hip_pack(hops, cs, dev)
    for kw in (dict(), dict(relu_in=True, add=add), dict(relu_in=True, relu_out=True, mask=mask),
               dict(second=cs.extra["b_tgt"], n_switch=4, relu_in=True)):
        y = torch.zeros(N, cout // 16, H, H, 16, dtype=torch.bfloat16, device=dev)
        yr = torch.zeros_like(y)
        hops.conv(x, cs, y, **kw)
        tops.conv(x, cs, yr, **kw)
        torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=3e-2, msg=lambda m: f"{kw.keys()}: {m}")
    # data gradient: transposed + flipped weights, (mask > 0), + add
    if cin == cout or (cin, cout) in ((16, 32),):
        dy = torch.randn(N, cout // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
        m2 = torch.randn(N, cin // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
        a2 = torch.randn(N, cin // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
        dx = torch.zeros(N, cin // 16, H, H, 16, dtype=torch.bfloat16, device=dev)
        dxr = torch.zeros_like(dx)
        hops.conv(dy, cs, dx, transpose=True, mask=m2, add=a2)
        tops.conv(dy, cs, dxr, transpose=True, mask=m2, add=a2)
        torch.testing.assert_close(dx.float(), dxr.float(), rtol=2e-2, atol=3e-2)
        # and against autograd's conv2d_input
        ref = torch.nn.grad.conv2d_input((N, cin, H, H), cs.wb.float(), from_planar(dy.float()), padding=1)
        dx2 = torch.zeros_like(dx)
        hops.conv(dy, cs, dx2, transpose=True)
        torch.testing.assert_close(from_planar(dx2.float()), ref, rtol=2e-2, atol=3e-2)


@pytest.mark.gpu
def test_gpu_sconv_ring_input():
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    cfg, rp = _setup(device=dev)
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    cs = _spec(16, 16, 84, dev, cin_real=4)
    _hip_pack(hops, cs, dev)
    slots = torch.randint(0, 150, (5, 4), dtype=torch.int32, device=dev)
    y = torch.zeros(5, 1, 84, 84, 16, dtype=torch.bfloat16, device=dev)
    yr = torch.zeros_like(y)
    kw = dict(ring=rp.frames, slots=slots, scale=1.0 / 255, second=cs.extra["b_tgt"], n_switch=3)
    hops.conv(None, cs, y, **kw)
    tops.conv(None, cs, yr, **kw)
    torch.testing.assert_close(y.float(), yr.float(), rtol=2e-2, atol=3e-2)
    # fused conv + max pool (+ argmax): same pooled values, codes consistent with the values
    p, pr = (torch.zeros(5, 1, 42, 42, 16, dtype=torch.bfloat16, device=dev) for _ in range(2))
    a, ar = (torch.zeros(5, 1, 42, 42, 16, dtype=torch.uint8, device=dev) for _ in range(2))
    hops.conv_pool(None, cs, p, a, **kw)
    tops.maxpool(y, pr, ar)
    torch.testing.assert_close(p.float(), pr.float(), rtol=0, atol=0)
    agree = (a == ar).float().mean().item()
    assert agree > 0.999, agree
    # weight gradient from the ring (x scale)
    dy = torch.randn(5, 1, 84, 84, 16, device=dev).to(torch.bfloat16)
    gw, gb = torch.zeros(16, 4, 3, 3, device=dev), torch.zeros(16, device=dev)
    gwr, gbr = torch.zeros_like(gw), torch.zeros_like(gb)
    jobs = []
    hops.wgrad(dy, None, cs, gw, gb, jobs, ring=rp.frames, slots=slots, scale=1.0 / 255)
    hops.finalize(jobs)
    tops.wgrad(dy, None, cs, gwr, gbr, [], ring=rp.frames, slots=slots, scale=1.0 / 255)
    torch.testing.assert_close(gw, gwr, rtol=1e-2, atol=1e-2)
    torch.testing.assert_close(gb, gbr, rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_gpu_ring_wgrad_fused_pool_backward_bit_identical():
    """bf16: the ring conv's weight gradient straight from the pooled gradient + argmax
    codes equals max-pool backward then weight gradient bit for bit."""
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    cfg, rp = _setup(device=dev)
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    cs = _spec(16, 16, 84, dev, cin_real=4)
    _hip_pack(hops, cs, dev)
    N = 9
    slots = torch.randint(0, 150, (N, 4), dtype=torch.int32, device=dev)
    x = torch.randn(N, 1, 84, 84, 16, device=dev).round().to(torch.bfloat16)   # ties: multi-window pixels
    p = torch.zeros(N, 1, 42, 42, 16, dtype=torch.bfloat16, device=dev)
    a = torch.zeros(N, 1, 42, 42, 16, dtype=torch.uint8, device=dev)
    tops.maxpool(x, p, a)
    dp = torch.randn(N, 1, 42, 42, 16, device=dev).to(torch.bfloat16)
    outs = []
    for fused in (True, False):
        gw, gb = torch.zeros(16, 4, 3, 3, device=dev), torch.zeros(16, device=dev)
        jobs = []
        if fused:
            hops.wgrad(dp, None, cs, gw, gb, jobs, ring=rp.frames, slots=slots, scale=1.0 / 255, pool_amax=a)
        else:
            dc = torch.zeros(N, 1, 84, 84, 16, dtype=torch.bfloat16, device=dev)
            hops.maxpool_bwd(dp, a, dc)
            hops.wgrad(dc, None, cs, gw, gb, jobs, ring=rp.frames, slots=slots, scale=1.0 / 255)
        hops.finalize(jobs)
        outs.append((gw, gb))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


WG_SHAPES = [(16, 16, 42), (16, 32, 42), (32, 32, 21), (32, 32, 11)]


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,H", WG_SHAPES)
def test_gpu_sconv_wgrad(cin, cout, H):
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    N = 37
    g = torch.Generator(device=dev).manual_seed(2)
    x = torch.randn(N, cin // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, cout // 16, H, H, 16, generator=g, device=dev).to(torch.bfloat16)
    cs = _spec(cin, cout, H, dev)
    for relu in (False, True):
        gw, gb = torch.zeros(cout, cin, 3, 3, device=dev), torch.zeros(cout, device=dev)
        gwr, gbr = torch.zeros_like(gw), torch.zeros_like(gb)
        jobs = []
        hops.wgrad(dy, x, cs, gw, gb, jobs, relu_in=relu)
        hops.finalize(jobs)
        tops.wgrad(dy, x, cs, gwr, gbr, [], relu_in=relu)
        scale = gwr.abs().max().item()
        torch.testing.assert_close(gw / scale, gwr / scale, rtol=0, atol=2e-3)
        torch.testing.assert_close(gb, gbr, rtol=1e-3, atol=1e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,H", [(16, 32, 42), (32, 32, 21)])
def test_gpu_sconv_pool_fused(cin, cout, H):
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    N = 5
    x = torch.randn(N, cin // 16, H, H, 16, device=dev).to(torch.bfloat16)
    cs = _spec(cin, cout, H, dev)
    _hip_pack(hops, cs, dev)
    Ho = (H + 1) // 2
    kw = dict(second=cs.extra["b_tgt"], n_switch=2)
    y = torch.zeros(N, cout // 16, H, H, 16, dtype=torch.bfloat16, device=dev)
    hops.conv(x, cs, y, **kw)
    p, pr = (torch.zeros(N, cout // 16, Ho, Ho, 16, dtype=torch.bfloat16, device=dev) for _ in range(2))
    a, ar = (torch.zeros(N, cout // 16, Ho, Ho, 16, dtype=torch.uint8, device=dev) for _ in range(2))
    hops.conv_pool(x, cs, p, a, **kw)
    tops.maxpool(y, pr, ar)          # pool of the (identically computed) unfused conv
    torch.testing.assert_close(p.float(), pr.float(), rtol=0, atol=0)
    assert (a == ar).float().mean().item() > 0.999


@pytest.mark.gpu
@pytest.mark.parametrize("C,H", [(16, 42), (32, 21), (32, 11)])
def test_gpu_resblock_fused(C, H):
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    N = 7
    x = torch.randn(N, C // 16, H, H, 16, device=dev).to(torch.bfloat16)
    c0, c1 = _spec(C, C, H, dev, seed=3), _spec(C, C, H, dev, seed=4)
    _hip_pack(hops, c0, dev)
    _hip_pack(hops, c1, dev)
    for relu_out in (False, True):
        out, outr = (torch.zeros(N, C // 16, H, H, 16, dtype=torch.bfloat16, device=dev) for _ in range(2))
        ys, ysr = (torch.zeros(N, C // 16, H, H, 16, dtype=torch.bfloat16, device=dev) for _ in range(2))
        kw = dict(n_save=4, target=True, n_switch=5, relu_out=relu_out)
        hops.resblock(x, c0, c1, out, ysave=ys, **kw)
        tops.resblock(x, c0, c1, outr, ysave=ysr, **kw)
        torch.testing.assert_close(out.float(), outr.float(), rtol=3e-2, atol=5e-2)
        torch.testing.assert_close(ys[:4].float(), ysr[:4].float(), rtol=2e-2, atol=3e-2)
        assert torch.count_nonzero(ys[4:]) == 0          # rows past n_save are not written


@pytest.mark.gpu
def test_gpu_maxpool():
    from apex_dqn_amd.ops.impala import HipImpalaOps
    dev = torch.device("cuda")
    hops, tops = HipImpalaOps(), TorchImpalaOps()
    for (P, H) in ((1, 84), (2, 42), (2, 21)):
        x = torch.randn(3, P, H, H, 16, device=dev).to(torch.bfloat16)
        Ho = (H + 1) // 2
        y, yr = (torch.zeros(3, P, Ho, Ho, 16, dtype=torch.bfloat16, device=dev) for _ in range(2))
        a, ar = (torch.zeros(3, P, Ho, Ho, 16, dtype=torch.uint8, device=dev) for _ in range(2))
        hops.maxpool(x, y, a)
        tops.maxpool(x, yr, ar)
        assert torch.equal(y, yr) and torch.equal(a, ar)
        dy = torch.randn(3, P, Ho, Ho, 16, device=dev).to(torch.bfloat16)
        dx, dxr = (torch.zeros(3, P, H, H, 16, dtype=torch.bfloat16, device=dev) for _ in range(2))
        hops.maxpool_bwd(dy, a, dx)
        tops.maxpool_bwd(dy, a, dxr)
        torch.testing.assert_close(dx.float(), dxr.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_gpu_impala_learner_matches_torch_backend():
    """Whole hand-written step (HIP) vs the same step on the torch ops (both bf16
    activations on the GPU): loss, priorities and gradients."""
    dev = torch.device("cuda")
    cfg, rp = _setup(B=64, device=dev, dtype="bf16")
    Lh = FusedImpalaLearner(cfg, dev, rp, backend="hip")
    cfg2, rp2 = _setup(B=64, device=dev, dtype="bf16")
    Lt = FusedImpalaLearner(cfg2, dev, rp2, backend="torch")
    Lt.p32.copy_(Lh.p32)
    Lt.pbf.copy_(Lh.pbf)
    Lt.sync_target()
    Lh._seg1()
    Lh._seg2()
    Lt._seg1()
    Lt._seg2()
    torch.cuda.synchronize()
    assert torch.equal(Lh.slots, Lt.slots)
    torch.testing.assert_close(Lh.td_abs, Lt.td_abs, rtol=5e-2, atol=5e-2)
    gh, gt = Lh.module_state(Lh.G), Lt.module_state(Lt.G)
    errs = {k: float((gh[k] - gt[k]).norm() / (gt[k].norm() + 1e-12)) for k in gh}
    # both sides carry bf16 activations; the torch oracle's fc also rounds the bias add
    # in bf16, so the fc-stream gradients (sums over samples with cancellation) differ
    # most (~7 % measured) -- a layout / index bug shows as O(1) error
    bad = {k: e for k, e in errs.items() if not e < (0.12 if "stream" in k else 0.05)}
    assert not bad, bad
    Lh._seg3()
    torch.cuda.synchronize()
    assert torch.isfinite(Lh.p32).all() and float(Lh.gnorm[0]) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_gpu_impala_graph_step_runs(dtype):
    dev = torch.device("cuda")
    cfg, rp = _setup(B=64, device=dev, dtype=dtype)
    cfg.Runtime.use_graphs = True
    L = FusedImpalaLearner(cfg, dev, rp, backend="hip")
    for _ in range(3):
        L.step()
    torch.cuda.synchronize()
    m = L.last_metrics()
    assert np.isfinite(m["loss"]) and np.isfinite(m["grad_norm"])


@pytest.mark.gpu
def test_gpu_impala_multi_step_graph_matches_single_step_graphs():
    """steps(n) replaying 4-update graphs (with a target sync inside the run and a
    host-side replay mutation between calls) == n one-update graph replays (fp32)."""
    dev = torch.device("cuda")
    res = {}
    for k in (1, 4):
        cfg, rp = _setup(B=64, device=dev, dtype="fp32")
        cfg.Runtime.use_graphs = True
        cfg.Runtime.graph_steps = k
        cfg.Learner.q_target_sync_freq = 6
        L = FusedImpalaLearner(cfg, dev, rp, backend="hip")
        L.prepare_graphs()
        assert (L._multi is not None) == (k > 1)
        L.steps(9)
        rp.remove_to_fit()
        rp.rebuild()
        L.steps(8)
        torch.cuda.synchronize()
        assert L.num_q_updates == 17
        res[k] = (L.p32.clone(), L.t32.clone(), rp.leaf.clone(), L.S["idx"].clone())
    # same draws; parameters equal up to the order of the fp32 head-wgrad atomics
    assert torch.equal(res[1][3], res[4][3])
    for a, b in zip(res[1][:3], res[4][:3]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)
