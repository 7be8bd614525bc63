"""The fused learner's hand-written backward (the contract every HIP kernel
implements) against PyTorch autograd through the reference module."""
import numpy as np
import torch

from apex_dqn_amd.config import ApexConfig
from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
from apex_dqn_amd.learner.torch_learner import TorchLearner
from apex_dqn_amd.models.flat_params import flat_to_reference_state
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard


def _setup(loss="huber", A=6, network="nature64"):
    torch.manual_seed(0)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": A, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 8},
                                "Runtime": {"grad_clip": 40.0, "loss": loss, "network": network,
                                            "presample": False}})
    rp = GpuReplayShard(400, 400, 600, 4, device="cpu")
    rng = np.random.default_rng(0)
    seqs = rp.append_frames(rng.integers(0, 255, (300, 84, 84), dtype=np.uint8))
    K = 200
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    nx = np.stack([seqs[i + 3:i + 7] for i in range(K)])
    g = np.full(K, 0.97)
    g[::5] = 0.0
    rp.insert(dict(S_t=st, S_tpn=nx, A_t=rng.integers(0, A, K), R=rng.normal(size=K) * 3, Gamma=g,
                   priority=rng.random(K)))
    return cfg, rp


def _check(loss, network="nature64"):
    cfg, rp = _setup(loss, network=network)
    L = FusedNatureLearner(cfg, "cpu", rp)
    T = TorchLearner(cfg, "cpu")
    T.Q.load_state_dict(L.reference_state_dict())
    T.Q_target.load_state_dict(L.reference_state_dict())
    L._seg1()
    L._seg2()
    B = L.B
    S = L.S
    batch = dict(S_t=L.frames[:B], S_tpn=L.frames[B:2 * B], A_t=S["act"], R=S["rew"], Gamma=S["gam"],
                 weights=S["weights"])
    lref, td = T.compute_loss_and_priorities(batch)
    T.optimizer.zero_grad()
    lref.backward()
    assert abs(float(lref) - float(L.loss_b.mean())) < 1e-5 * max(1.0, abs(float(lref)))
    torch.testing.assert_close(td, L.td_abs, rtol=1e-5, atol=1e-5)
    gf = flat_to_reference_state(L.G, L.c1)
    for k, p in T.Q.named_parameters():
        torch.testing.assert_close(gf[k], p.grad, rtol=1e-4, atol=1e-7)
    return L


def test_fused_backward_matches_autograd_huber():
    _check("huber")


def test_fused_backward_matches_autograd_mse():
    _check("mse")


def test_nature32_runs_zero_padded_on_the_64_filter_path():
    """Nature DQN's 32-filter conv1 is stored padded to 64 filters: the padded
    gradients are exactly zero, so RMSprop keeps the padding at zero."""
    L = _check("huber", network="nature32")
    assert L.c1 == 32
    assert torch.count_nonzero(L.G["w1"][32:]) == 0 and torch.count_nonzero(L.G["b1"][32:]) == 0
    assert torch.count_nonzero(L.G["w2"][..., 32:]) == 0
    L._seg3()
    assert torch.count_nonzero(L.P["w1"][32:]) == 0 and torch.count_nonzero(L.P["w2"][..., 32:]) == 0
    sd = L.reference_state_dict()
    assert sd["layer1.0.weight"].shape[0] == 32 and sd["layer2.0.weight"].shape[1] == 32


def test_fused_step_updates_params_and_priorities():
    cfg, rp = _setup()
    L = FusedNatureLearner(cfg, "cpu", rp)
    p0 = L.p32.clone()
    leaf0 = rp.leaf.clone()
    L.step()
    assert not torch.equal(p0, L.p32)
    assert torch.equal(L.pbf, L.p32)  # fp32 compute copy on CPU
    idx = L.S["idx"]
    assert not torch.equal(leaf0[idx], rp.leaf[idx])
    assert L.num_q_updates == 1


def test_presample_draws_the_same_batches():
    """Drawing step t+1's batch inside step t (beside the optimizer) yields exactly the
    batches of sampling at the head of each step, and host-side replay mutations in
    between force a redraw."""
    import copy
    runs = {}
    for pre in (False, True):
        cfg, rp = _setup()
        cfg = copy.deepcopy(cfg)
        cfg.Runtime.presample = pre
        torch.manual_seed(0)
        L = FusedNatureLearner(cfg, "cpu", rp)
        seen = []
        for t in range(4):
            if t == 2:                      # host-side mutation between steps
                rp.remove_to_fit()
                rp.rebuild()
            L._seg1()
            seen.append(L.S["idx"].clone())
            L._seg2()
            L._seg3()
        runs[pre] = (seen, L.p32.clone())
    for a, b in zip(runs[False][0], runs[True][0]):
        assert torch.equal(a, b)
    torch.testing.assert_close(runs[False][1], runs[True][1], rtol=0, atol=0)


def test_split_mode_plumbing_matches_fp32_autograd():
    """fp32-accurate split mode (hi + lo bf16 planes for every weight copy, activation
    and gradient; the torch backend emulates the HIP kernels' contract on the CPU):
    the whole-step gradients match fp32 autograd to <= 1e-4 relative per segment, so
    every lo plane is routed to the right op."""
    cfg, rp = _setup("huber")
    L = FusedNatureLearner(cfg, "cpu", rp, split=True)
    assert L.split and L.pbf.dtype == torch.bfloat16 and L.y1_lo is not None
    # hi + lo reproduce the fp32 master weights far better than bf16 alone
    err_hi = (L.pbf.float() - L.p32).abs().max()
    err_split = (L.pbf.float() + L.pbf_lo.float() - L.p32).abs().max()
    assert err_split < err_hi / 100
    T = TorchLearner(cfg, "cpu")
    T.Q.load_state_dict(L.reference_state_dict())
    T.Q_target.load_state_dict(L.reference_state_dict())
    L._seg1()
    L._seg2()
    B, S = L.B, L.S
    batch = dict(S_t=L.frames[:B], S_tpn=L.frames[B:2 * B], A_t=S["act"], R=S["rew"], Gamma=S["gam"],
                 weights=S["weights"])
    lref, td = T.compute_loss_and_priorities(batch)
    T.optimizer.zero_grad()
    lref.backward()
    torch.testing.assert_close(td, L.td_abs, rtol=1e-4, atol=1e-4)
    gf = flat_to_reference_state(L.G, L.c1)
    for k, p in T.Q.named_parameters():
        rel = float((gf[k] - p.grad).norm() / (p.grad.norm() + 1e-30))
        assert rel < 1e-4, (k, rel)
    # the optimizer rewrites both planes: hi + lo == fp32 master to ~2^-17 relative
    L._seg3()
    torch.testing.assert_close(L.pbf.float() + L.pbf_lo.float(), L.p32, rtol=2e-5, atol=1e-9)


def test_batch_max_is_normalisation_matches_autograd_on_normalised_weights():
    """Runtime.is_normalise = batch_max (learner/is_norm.py): the fused step keeps the
    sampler's global-min weights in the loss and divides the gradient by the batch's
    largest weight inside the optimizer.  The update must equal centered RMSprop + clip
    applied to the autograd gradient of the loss with weights w / max_batch(w)."""
    import copy
    from apex_dqn_amd.models.flat_params import reference_state_to_flat
    from apex_dqn_amd.ops.fused_ops import TorchBackend
    cfg, rp = _setup("huber")
    rp.leaf[3] = 1e-6 ** 0.6          # a leaf at the priority floor: global-min weights are tiny
    rp._torch_rebuild()
    cfg = copy.deepcopy(cfg)
    cfg.Runtime.is_normalise = "batch_max"
    L = FusedNatureLearner(cfg, "cpu", rp)
    T = TorchLearner(cfg, "cpu")
    T.Q.load_state_dict(L.reference_state_dict())
    T.Q_target.load_state_dict(L.reference_state_dict())
    p0, v0, m0 = L.p32.clone(), L.rms_v.clone(), L.rms_m.clone()
    L._seg1()
    L._seg2()
    B, S = L.B, L.S
    w = S["weights"].clone()
    assert float(w.max()) < 0.1                       # the floor leaf shrinks the global-min weights
    batch = dict(S_t=L.frames[:B], S_tpn=L.frames[B:2 * B], A_t=S["act"], R=S["rew"], Gamma=S["gam"],
                 weights=w / w.max())
    lref, _ = T.compute_loss_and_priorities(batch)
    T.optimizer.zero_grad()
    lref.backward()
    g_ref = torch.zeros_like(L.g32)
    reference_state_to_flat({k: p.grad for k, p in T.Q.named_parameters()}, L.layout.views(g_ref))
    L._seg3()
    assert abs(L.is_scale() - 1.0 / float(w.max())) < 1e-6 / float(w.max())
    rt = cfg.Runtime
    p, v, m = p0.clone(), v0.clone(), m0.clone()
    nrm = torch.zeros(1)
    TorchBackend()._optimizer(p, g_ref, v, m, p.clone(), rt.lr, rt.rms_decay, rt.rms_eps, rt.grad_clip,
                              rt.centered_rmsprop, nrm)
    # the clip norm is the norm of the batch-max gradient (20x+ the global-min one here:
    # the scale is visible there -- a centered RMSprop step itself is nearly invariant
    # to a constant gradient scale, up to eps)
    torch.testing.assert_close(L.gnorm, nrm, rtol=1e-4, atol=1e-9)
    assert float(L.gnorm) > 10 * float(L.g32.double().norm())
    # updates agree to 0.1 % of the per-step move lr / sqrt(alpha (1 - alpha))
    step = rt.lr / (rt.rms_decay * (1 - rt.rms_decay)) ** 0.5
    torch.testing.assert_close(L.p32 - p0, p - p0, rtol=0, atol=1e-3 * step)
    met = L.last_metrics()
    assert abs(met["is_weight_mean"] - float((w / w.max()).mean())) < 1e-5
