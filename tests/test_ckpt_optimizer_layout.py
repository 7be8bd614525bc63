"""Checkpointed optimizer state is tagged with the flat layout it came from
(utils/checkpoint.py pack_flat_state / unpack_flat_state): a resume restores every
RMSprop value to its own parameter even when the engine's flat layout changed.  An
untagged flat vector (a checkpoint written before the tag existed) is restored by
length when the same network saved it -- this engine's flat layout is unchanged since --
and refused otherwise: the state then starts fresh instead of silently misaligned."""
import torch

from apex_dqn_amd.config import ApexConfig
from apex_dqn_amd.models.flat_params import FlatLayout
from apex_dqn_amd.utils.checkpoint import layout_segments, pack_flat_state, unpack_flat_state


def _cfg(path=None):
    return ApexConfig.from_dict({"env_conf": {"state_shape": [4, 84, 84], "action_dim": 4, "name": "Synthetic"},
                                 "Learner": {"replay_sample_size": 8, "load_saved_state": path or False},
                                 "Runtime": {"use_graphs": False}})


def _replay():
    from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
    return GpuReplayShard(64, 64, 80, 4, device="cpu", seed=1)


def test_pack_unpack_survives_reordered_layout():
    a = FlatLayout([("x", (3, 5)), ("y", (7,)), ("z", (2, 2))])
    b = FlatLayout([("z", (2, 2)), ("x", (3, 5)), ("y", (7,))])      # same tensors, other order
    va = torch.arange(a.numel, dtype=torch.float32)
    st = pack_flat_state(layout_segments(a), rms_v=va)
    vb = torch.zeros(b.numel)
    assert unpack_flat_state(st, layout_segments(b), rms_v=vb)
    for name in ("x", "y", "z"):
        assert torch.equal(a.views(va)[name], b.views(vb)[name])


def test_mismatched_or_untagged_state_is_refused(capsys):
    a = FlatLayout([("x", (3, 5)), ("y", (7,))])
    c = FlatLayout([("x", (3, 5)), ("y", (8,))])
    st = pack_flat_state(layout_segments(a), rms_v=torch.ones(a.numel))
    dst = torch.full((c.numel,), 5.0)
    assert not unpack_flat_state(st, layout_segments(c), rms_v=dst)
    assert not unpack_flat_state({"rms_v": torch.ones(a.numel)}, layout_segments(a), rms_v=dst)
    # untagged of this buffer's length: only from the same network
    assert not unpack_flat_state({"rms_v": torch.ones(c.numel)}, layout_segments(c), untagged_network="impala",
                                 network="nature64", rms_v=dst)
    assert torch.equal(dst, torch.full((c.numel,), 5.0))
    assert unpack_flat_state({"rms_v": torch.ones(c.numel)}, layout_segments(c), untagged_network="nature64",
                             network="nature64", rms_v=dst)
    assert torch.equal(dst, torch.ones(c.numel))
    assert "not restored" in capsys.readouterr().out


def test_fused_learner_resume_restores_rmsprop_state(tmp_path):
    from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
    torch.manual_seed(0)
    L = FusedNatureLearner(_cfg(), "cpu", _replay())
    pad = torch.ones_like(L.rms_v, dtype=torch.bool)      # alignment padding: never has state
    for _, o, k in layout_segments(L.layout):
        pad[o:o + k] = False
    L.rms_v.copy_(torch.rand_like(L.rms_v).masked_fill(pad, 0.0))
    L.rms_m.copy_(torch.rand_like(L.rms_m).masked_fill(pad, 0.0))
    p = str(tmp_path / "ck.pt")
    L.save(p)
    L2 = FusedNatureLearner(_cfg(p), "cpu", _replay())
    assert torch.equal(L2.rms_v, L.rms_v) and torch.equal(L2.rms_m, L.rms_m)
    # an older checkpoint: raw flat vectors with no layout tag, same network -> restored
    ck = torch.load(p, weights_only=True)
    ck["optimizer_state"] = {"rms_v": L.rms_v.clone(), "rms_m": L.rms_m.clone()}
    torch.save(ck, p)
    L3 = FusedNatureLearner(_cfg(p), "cpu", _replay())
    assert torch.equal(L3.rms_v, L.rms_v) and torch.equal(L3.rms_m, L.rms_m) and torch.equal(L3.p32, L.p32)
    # ... of another length (e.g. another network's buffer): refused, state fresh
    ck["optimizer_state"] = {"rms_v": L.rms_v[:-64].clone(), "rms_m": L.rms_m[:-64].clone()}
    torch.save(ck, p)
    L4 = FusedNatureLearner(_cfg(p), "cpu", _replay())
    assert torch.count_nonzero(L4.rms_v) == 0 and torch.equal(L4.p32, L.p32)
