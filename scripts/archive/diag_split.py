"""Diagnose the fp32 split learner stage by stage against fp64 recomputations of each
stage from the learner's OWN inputs (so a broken stage shows its own error, not an
inherited one).  Prints one JSON line per stage."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from apex_dqn_amd.config import ApexConfig  # noqa: E402
from apex_dqn_amd.learner.fused_learner import FusedNatureLearner  # noqa: E402
from apex_dqn_amd.ops import reference as R  # noqa: E402
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard  # noqa: E402

DEV = torch.device("cuda", 0)


def j(h, lo):
    return h.double().cpu() + (lo.double().cpu() if lo is not None else 0)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / (b.norm() + 1e-30))


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": B},
                                "Runtime": {"use_graphs": False, "presample": False, "dtype": "fp32"}})
    torch.manual_seed(0)
    rp = GpuReplayShard(2000, 2000, 2100, 4, device=DEV, seed=7)
    rng = np.random.default_rng(11)
    seqs = rp.append_frames(rng.integers(0, 255, (1800, 84, 84), dtype=np.uint8))
    K = 1500
    st = np.stack([seqs[i:i + 4] for i in range(K)])
    rp.insert(dict(S_t=st, S_tpn=st + 3, A_t=rng.integers(0, 6, K), R=rng.normal(size=K) * 2,
                   Gamma=np.where(rng.random(K) < 0.1, 0.0, 0.97), priority=rng.random(K)))
    L = FusedNatureLearner(cfg, DEV, rp, backend="hip")
    L._seg1()
    L._seg2()
    torch.cuda.synchronize()
    P = {k: v.double().cpu() for k, v in L.P.items()}
    S = L.S
    frames = L.replay.gather_frames(L.slots).double().cpu()
    out = {}
    # forward, each layer from the learner's own (joined) input
    y1 = j(L.y1, L.y1_lo)
    out["conv1_fwd"] = rel(y1[:B], R.conv1_fwd(frames[:B], P["w1"], P["b1"], L.rt.obs_scale, torch.float64))
    y2 = j(L.y2, L.y2_lo)
    out["conv2_fwd"] = rel(y2[:2 * B], R.conv_fwd(y1[:2 * B], P["w2"], P["b2"], 2, torch.float64))
    y3 = j(L.y3, L.y3_lo)
    out["conv3_fwd"] = rel(y3[:2 * B], R.conv_fwd(y2[:2 * B], P["w3"], P["b3"], 1, torch.float64))
    h = j(L.h, L.h_lo)
    hr = R.fc_fwd(y3[:2 * B].reshape(2 * B, 3136), P["wfc"], P["bfc"], torch.float64)
    out["fc_fwd_value"] = rel(h[:2 * B, :512], hr[:, :512])
    out["fc_fwd_adv"] = rel(h[:2 * B, 512:], hr[:, 512:])
    # head backward from the learner's h
    dH = j(L.dH, L.dH_lo)
    dq = L.dhead[:, 0].double().cpu().clone()
    dv_ref = dq[:, None] * P["wv"][None, :] * (h[:B, :512] > 0)
    out["dH_value"] = rel(dH[:, :512], dv_ref)
    dadv = L.dhead[:, 1:].double().cpu()
    da_ref = (dadv @ P["wa"]) * (h[:B, 512:] > 0)
    out["dH_adv"] = rel(dH[:, 512:], da_ref)
    # fc weight gradient from the learner's dH and y3
    G = {k: v.double().cpu() for k, v in L.G.items()}
    gw = dH.t() @ y3[:B].reshape(B, 3136)
    out["fc_wgrad_value"] = rel(G["wfc"][:512], gw[:512])
    out["fc_wgrad_adv"] = rel(G["wfc"][512:], gw[512:])
    out["fc_bgrad_value"] = rel(G["bfc"][:512], dH.sum(0)[:512])
    out["fc_bgrad_adv"] = rel(G["bfc"][512:], dH.sum(0)[512:])
    # fc dgrad
    dY3 = j(L.dY3, L.dY3_lo)
    ref = (dH @ P["wfc"]).reshape(B, 7, 7, 64) * (y3[:B] > 0)
    out["fc_dgrad"] = rel(dY3, ref)
    dY2 = j(L.dY2, L.dY2_lo)
    out["conv3_dgrad"] = rel(dY2, R.conv_dgrad(dY3, P["w3"], (B, 9, 9, 64), 1, y2[:B], torch.float64))
    dY1 = j(L.dY1, L.dY1_lo)
    out["conv2_dgrad"] = rel(dY1, R.conv_dgrad(dY2, P["w2"], (B, 20, 20, 64), 2, y1[:B], torch.float64))
    rw3 = torch.nn.grad.conv2d_weight(y2[:B].permute(0, 3, 1, 2), (64, 64, 3, 3), dY3.permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    out["conv3_wgrad"] = rel(G["w3"], rw3)
    rw2 = torch.nn.grad.conv2d_weight(y1[:B].permute(0, 3, 1, 2), (64, 64, 4, 4), dY2.permute(0, 3, 1, 2),
                                      stride=2).permute(0, 2, 3, 1)
    out["conv2_wgrad"] = rel(G["w2"], rw2)
    rw1 = torch.nn.grad.conv2d_weight(frames[:B] * L.rt.obs_scale, (64, 4, 8, 8), dY1.permute(0, 3, 1, 2), stride=4)
    out["conv1_wgrad"] = rel(G["w1"], rw1)
    out["conv1_bgrad"] = rel(G["b1"], dY1.sum((0, 1, 2)))
    # the fp64 module oracle of the whole step on the same batch (as tests/test_gpu_split.py)
    from apex_dqn_amd.models.dueling import DuellingDQN
    Q = DuellingDQN((4, 84, 84), L.A).double()
    Q.load_state_dict({k: v.double() for k, v in L.reference_state_dict().items()})
    keep = {}
    Q.value_stream_layer.register_forward_hook(lambda m, i, o: keep.__setitem__("hv", o))
    Q.advantage_stream_layer.register_forward_hook(lambda m, i, o: keep.__setitem__("ha", o))
    s_t = frames[:B] * L.rt.obs_scale
    v, a, q = Q(s_t)
    hv, ha = keep["hv"], keep["ha"]
    hv.retain_grad()
    ha.retain_grad()
    out["oracle_hv_vs_learner"] = rel(h[:B, :512], hv.detach())
    out["oracle_ha_vs_learner"] = rel(h[:B, 512:], ha.detach())
    act = S["act"].long().cpu()
    q_sa = q.gather(1, act.view(-1, 1)).squeeze(1)
    # the learner's own dq as the upstream gradient: isolates the module's backward
    (q_sa * dq).sum().backward()
    out["oracle_dHv_given_dq"] = rel(dH[:, :512], hv.grad)
    out["oracle_dHa_given_dq"] = rel(dH[:, 512:], ha.grad)
    out["oracle_value_stream_bias"] = rel(G["bfc"][:512], Q.value_stream_layer[0].bias.grad)
    out["oracle_adv_stream_bias"] = rel(G["bfc"][512:], Q.advantage_stream_layer[0].bias.grad)
    out["n_hv_mask_diff"] = float(((h[:B, :512] > 0) != (hv.detach() > 0)).sum())
    out["n_ha_mask_diff"] = float(((h[:B, 512:] > 0) != (ha.detach() > 0)).sum())
    for k, v in out.items():
        print(json.dumps({"stage": k, "rel_err": v}), flush=True)


if __name__ == "__main__":
    main()
