"""apex_dqn_amd: an MI355X-native Ape-X (distributed prioritized replay DQN) engine.

Capabilities of lefarov/Ape-X-DQN (actor / learner / replay split,
``parameters.json`` config surface, ``{'Q_state': state_dict}`` checkpoints),
re-designed GPU-first: batched actor groups, an HBM-resident 64-ary sum-tree
replay shard per GPU, and a data-parallel learner whose hot path runs on
hand-written CDNA4 (gfx950) HIP kernels, with RCCL over xGMI between ranks.
"""
__version__ = "0.1.0"

from .config import ApexConfig, epsilon_ladder  # noqa: F401
