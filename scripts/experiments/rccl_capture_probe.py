"""Probe: can an RCCL all-reduce be captured in a HIP graph through torch.distributed on
this stack?  World size 1 (one GPU box), so it checks the capture mechanics only, not
multi-rank behaviour.  Prints one JSON line."""
import json
import os

import torch
import torch.distributed as dist

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29561")
torch.cuda.set_device(0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
x = torch.ones(1 << 20, device="cuda")
dist.all_reduce(x)                      # warm the communicator outside capture
torch.cuda.synchronize()
res = {"eager_ok": bool(x[0].item() == 1.0)}
try:
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            x.mul_(2.0)
            dist.all_reduce(x)
            x.add_(1.0)
    torch.cuda.current_stream().wait_stream(s)
    x.fill_(1.0)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    res.update(capture_ok=True, value=float(x[0].item()), expected=15.0)
except Exception as e:  # noqa: BLE001
    res.update(capture_ok=False, error=repr(e)[:300])
print(json.dumps(res), flush=True)
dist.destroy_process_group()
