"""Config surface, network definitions and checkpoint format (CPU)."""
import json
import os

import pytest
import torch

from apex_dqn_amd.config import ApexConfig, apply_overrides, epsilon_ladder
from apex_dqn_amd.models.dueling import REFERENCE_KEYS, DuellingDQN, MLPDuellingDQN, ImpalaDuellingDQN, build_network
from apex_dqn_amd.models.flat_params import (FlatLayout, flat_to_reference_state, nature_segments,
                                             reference_state_to_flat)
from apex_dqn_amd.utils.checkpoint import load_checkpoint, save_checkpoint

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_PARAMS = os.path.join(ROOT, "configs", "reference_parameters.json")


def test_reference_parameters_json_loads_verbatim():
    cfg = ApexConfig.load(REF_PARAMS)
    assert cfg.env_conf.state_shape == [1, 84, 84]
    assert cfg.env_conf.action_dim == 4
    assert cfg.Actor.num_actors == 5 and cfg.Actor.num_steps == 3
    assert cfg.Learner.replay_sample_size == 32 and cfg.Learner.q_target_sync_freq == 2500
    assert cfg.Replay_Memory.importance_sampling_exponent == 0.4
    assert cfg.Runtime.learner_T == 500000  # reference main.py:46 hard-codes it
    assert cfg.network == "nature64" and cfg.frame_stack == 1


def test_all_shipped_configs_validate():
    for f in os.listdir(os.path.join(ROOT, "configs")):
        if f.endswith(".json"):
            ApexConfig.load(os.path.join(ROOT, "configs", f))
    ApexConfig.load(os.path.join(ROOT, "parameters.json"))


def test_overrides_and_validation(tmp_path):
    cfg = ApexConfig.load(REF_PARAMS, ["Learner.replay_sample_size=512", "env_conf.state_shape=[4,84,84]",
                                       "Runtime.use_graphs=false"])
    assert cfg.Learner.replay_sample_size == 512 and cfg.env_conf.state_shape == [4, 84, 84]
    assert cfg.Runtime.use_graphs is False
    with pytest.raises(ValueError):
        apply_overrides({}, ["nodot=1"])
    with pytest.raises(ValueError):
        ApexConfig.from_dict({"env_conf": {"state_shape": [4, 64, 64]}})
    with pytest.raises(ValueError):
        ApexConfig.from_dict({"Actor": {"num_actors": 0}})
    p = tmp_path / "c.json"
    cfg.save(str(p))
    assert ApexConfig.load(str(p)).Learner.replay_sample_size == 512


def test_epsilon_ladder_matches_apex_and_single_actor():
    e = epsilon_ladder(5, 0.4, 7)
    assert e[0] == pytest.approx(0.4) and e[-1] == pytest.approx(0.4 ** 8)
    assert all(a > b for a, b in zip(e, e[1:]))
    assert epsilon_ladder(1, 0.4, 7) == [pytest.approx(0.4)]  # reference divides by zero (A13)


@pytest.mark.parametrize("C,A,n", [(1, 4, 3321541), (4, 4, 3333829), (4, 18, 3341011)])
def test_dueling_param_counts_match_reference(C, A, n):
    net = DuellingDQN((C, 84, 84), A)
    assert sum(p.numel() for p in net.parameters()) == n
    assert tuple(net.state_dict().keys()) == REFERENCE_KEYS


def test_dueling_combine_is_per_sample():
    torch.manual_seed(0)
    net = DuellingDQN((4, 84, 84), 6)
    x = torch.randint(0, 255, (3, 4, 84, 84), dtype=torch.uint8)
    v, a, q = net(x)
    torch.testing.assert_close(q, v + a - a.mean(1, keepdim=True))
    # same input gives the same q regardless of batch companions (reference A15 couples samples)
    q1 = net(x[:1])[2]
    torch.testing.assert_close(q1, q[:1], rtol=1e-5, atol=1e-5)


def test_other_network_families_forward():
    for kind, shape in (("mlp", [4]), ("impala", [4, 84, 84]), ("nature32", [4, 84, 84])):
        net = build_network(kind, shape, 5)
        x = torch.zeros((2,) + tuple(shape), dtype=torch.uint8 if len(shape) == 3 else torch.float32)
        v, a, q = net(x)
        assert q.shape == (2, 5) and v.shape == (2, 1)
    assert isinstance(build_network("mlp", [4], 2), MLPDuellingDQN)
    assert isinstance(build_network("impala", [4, 84, 84], 2), ImpalaDuellingDQN)


def test_flat_params_roundtrip_and_forward_equivalence():
    torch.manual_seed(1)
    net = DuellingDQN((4, 84, 84), 6)
    lay = FlatLayout(nature_segments(4, 6))
    flat = torch.zeros(lay.numel)
    V = lay.views(flat)
    reference_state_to_flat(net.state_dict(), V)
    sd = flat_to_reference_state(V)
    for k, t in net.state_dict().items():
        assert torch.equal(sd[k], t), k
    assert lay.numel >= sum(p.numel() for p in net.parameters())
    assert all(o % 64 == 0 for o in lay.offsets.values())


def test_checkpoint_format_reference_compatible(tmp_path):
    net = DuellingDQN((1, 84, 84), 4)
    p = str(tmp_path / "ck.pt")
    save_checkpoint(p, net.state_dict(), num_q_updates=7, config={"a": 1})
    ck = torch.load(p, weights_only=True)  # reference learner.py:20-21 access pattern
    net2 = DuellingDQN((1, 84, 84), 4)
    net2.load_state_dict(ck["Q_state"])
    for k in REFERENCE_KEYS:
        assert torch.equal(net2.state_dict()[k], net.state_dict()[k])
    assert ck["num_q_updates"] == 7
    assert load_checkpoint(str(tmp_path / "missing.pt")) is None


def test_params_file_is_json():
    with open(os.path.join(ROOT, "parameters.json")) as f:
        d = json.load(f)
    assert set(d) >= {"env_conf", "Actor", "Learner", "Replay_Memory"}


def _reference_forward_q(sd, x):
    """Plain fp32 functional forward of the reference DuellingDQN (duelling_network.py:21-28)
    on raw float pixels, with the dueling mean taken per row (defect A-mean fixed)."""
    import torch.nn.functional as F
    h = F.relu(F.conv2d(x, sd["layer1.0.weight"], sd["layer1.0.bias"], stride=4))
    h = F.relu(F.conv2d(h, sd["layer2.0.weight"], sd["layer2.0.bias"], stride=2))
    h = F.relu(F.conv2d(h, sd["layer3.0.weight"], sd["layer3.0.bias"], stride=1)).reshape(x.shape[0], -1)
    v = F.linear(F.relu(F.linear(h, sd["value_stream_layer.0.weight"], sd["value_stream_layer.0.bias"])),
                 sd["value.weight"], sd["value.bias"])
    a = F.linear(F.relu(F.linear(h, sd["advantage_stream_layer.0.weight"], sd["advantage_stream_layer.0.bias"])),
                 sd["advantage.weight"], sd["advantage.bias"])
    return v + a - a.mean(1, keepdim=True)


@pytest.mark.parametrize("with_config", [False, True])
def test_reference_checkpoint_q_values_at_raw_pixel_scale(tmp_path, with_config):
    """A reference-format checkpoint ({'Q_state'} only, learner.py:18-23) loads with
    the reference's raw 0..255 input scale and reproduces its Q-values; a checkpoint
    written here keeps the scale recorded in its config."""
    from apex_dqn_amd.config import ApexConfig
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    torch.manual_seed(3)
    sd = {k: v * 0.2 for k, v in DuellingDQN((4, 84, 84), 6).state_dict().items()}
    p = str(tmp_path / "ref.pt")
    if with_config:
        save_checkpoint(p, sd, config={"Runtime": {"obs_scale": 1.0 / 255.0}})
    else:
        torch.save({"Q_state": sd}, p)
    cfg = ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 6, "name": "Synthetic"},
                                "Learner": {"replay_sample_size": 4, "load_saved_state": p},
                                "Runtime": {"use_graphs": False}})
    rp = GpuReplayShard(16, 16, 32, 4, device="cpu")
    L = FusedNatureLearner(cfg, "cpu", rp)
    scale = 1.0 / 255.0 if with_config else 1.0
    assert L.rt.obs_scale == pytest.approx(scale)
    x = torch.randint(0, 256, (5, 4, 84, 84), dtype=torch.uint8)
    q = L.q_values(x)
    q_ref = _reference_forward_q(sd, x.float() * scale)
    torch.testing.assert_close(q, q_ref, rtol=1e-4, atol=1e-4 * float(q_ref.abs().max()))


def test_kernel_switches_and_impala_launch_shape_keys(monkeypatch):
    """APEX_SWITCHES parsing (one registry) and the IMPALA launch-shape keys of
    SW.isplit_bands (rb / sc / wg / wt), defaults included."""
    from apex_dqn_amd.ops import impala
    from apex_dqn_amd.ops.switches import SW, Switches
    sw = Switches.from_env("impala_wg_target=256,isplit_bands=rb16x42=10;wg32x32x21=11/256;wt32x32x11=128;"
                           "sc16x32x42p1=14")
    assert sw.impala_wg_target == 256 and sw.non_default().keys() == {"impala_wg_target", "isplit_bands"}
    with pytest.raises(ValueError):
        Switches.from_env("no_such_switch=1")
    defaults = impala._split_bands()
    assert defaults[("sc", 16, 16, 84, 1)] == 6 and defaults[("wt", 32, 32, 21)] == 256
    monkeypatch.setattr(SW, "isplit_bands", sw.isplit_bands)
    b = impala._split_bands()
    assert b[("rb", 16, 42)] == 10 and b[("sc", 16, 32, 42, 1)] == 14
    assert b[("wg", 32, 32, 21)] == (11, 256) and b[("wt", 32, 32, 11)] == 128
    assert b[("wt", 32, 32, 21)] == 256          # untouched defaults survive an override list
