import torch, numpy as np, time
from apex_dqn_amd.config import ApexConfig
from apex_dqn_amd.replay.gpu_replay import GpuReplayShard
from apex_dqn_amd.learner.fused_learner import FusedNatureLearner
from apex_dqn_amd.learner.torch_learner import TorchLearner
from apex_dqn_amd.learner.losses import ddqn_loss
torch.manual_seed(0)
cfg = ApexConfig.from_dict({"env_conf":{"state_shape":[4,84,84],"action_dim":6,"name":"Synthetic"},
  "Learner":{"replay_sample_size":8}, "Runtime":{"grad_clip":40.0, "presample":False}})
rp = GpuReplayShard(1000, 1000, 2000, 4, device="cpu")
rng = np.random.default_rng(0)
seqs = rp.append_frames(rng.integers(0,255,(300,84,84),dtype=np.uint8))
K=200
st = np.stack([seqs[i:i+4] for i in range(K)]); nx = np.stack([seqs[i+3:i+7] for i in range(K)])
rp.insert(dict(S_t=st,S_tpn=nx,A_t=rng.integers(0,6,K),R=rng.normal(size=K),Gamma=np.full(K,0.97),priority=rng.random(K)))
L = FusedNatureLearner(cfg, "cpu", rp)
# reference: torch autograd learner with the same params
T = TorchLearner(cfg, "cpu")
T.Q.load_state_dict(L.reference_state_dict()); T.Q_target.load_state_dict(L.reference_state_dict())
# run one fused step body manually and compare grads
L._step_body()
S = L.S
B = L.B
frames = L.frames
batch = dict(S_t=frames[:B], S_tpn=frames[B:2*B], A_t=S["act"], R=S["rew"], Gamma=S["gam"], weights=S["weights"])
loss, td = T.compute_loss_and_priorities(batch)
T.optimizer.zero_grad(); loss.backward()
print("loss ref", float(loss), "fused", float(L.loss_b.mean()))
print("td max diff", float((td - L.td_abs).abs().max()))
from apex_dqn_amd.models.flat_params import flat_to_reference_state
gref = {k: p.grad for k,p in T.Q.named_parameters()}
gf = flat_to_reference_state(L.G)
for k in gref:
    a, b = gref[k], gf[k]
    print(k, float((a-b).abs().max()), float(a.abs().max()))
