"""Checkpoints keep the epsilon-greedy RNG counter of EVERY pipelined actor group
(``Runtime.actor_pipeline`` > 1): after a resume no group repeats the exploration
draws it made before the checkpoint."""
import os
import tempfile
from types import SimpleNamespace

import torch

from apex_dqn_amd.runtime.gpu_loop import _actor_rng, _restore_actor_rng
from apex_dqn_amd.utils.checkpoint import save_checkpoint


def _pipelined(ctrs):
    gs = [SimpleNamespace(ctr=torch.tensor([c], dtype=torch.int64)) for c in ctrs]
    return SimpleNamespace(groups=gs, ctr=gs[0].ctr)


def test_every_group_counter_round_trips():
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "ck.pt")
        save_checkpoint(path, {}, **_actor_rng(_pipelined([11, 29, 5])))
        fresh = _pipelined([0, 0, 0])
        _restore_actor_rng(fresh, path)
        assert [int(g.ctr) for g in fresh.groups] == [11, 29, 5]
        # a single (unpipelined) group and the old one-counter format
        one = SimpleNamespace(ctr=torch.zeros(1, dtype=torch.int64))
        _restore_actor_rng(one, path)
        assert int(one.ctr) == 11
        save_checkpoint(path, {}, actor_rng={"ctr": 7})
        fresh = _pipelined([0, 0])
        _restore_actor_rng(fresh, path)
        assert [int(g.ctr) for g in fresh.groups] == [7, 0]
