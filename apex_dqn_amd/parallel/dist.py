"""Process-group plumbing: one process per GPU, RCCL over xGMI.

Replaces the reference's IPC layer -- an ``mp.Manager`` dict/Queue server and
a ``BaseManager`` replay proxy pickling 13.3 MB state_dicts over AF_UNIX every
learner step (``main.py:37-42``, ``learner.py:24,74``, ``actor.py:106,191``;
SURVEY §2.4.1 M1-M11) -- with collectives:

* ``allreduce_grads`` / ``allreduce_flat``: bucketed gradient all-reduce
  (mean) for the data-parallel learner (M-DP, new);
* ``broadcast_flat`` / ``broadcast_module``: parameter broadcast from rank 0
  (replaces M1-M4 weight publish);
* ``allgather_scalars``: small host-side statistics;
* the DP learner step's collectives (bucketed gradient all-reduce, replay-shard
  statistics all-gather) go through ``parallel/rccl.py``: torch.distributed or the
  native RCCL communicator (``Runtime.comm_backend``).

Backend ``nccl`` is RCCL on ROCm; ``gloo`` serves CPU configs and the
multi-process CPU tests.  Rendezvous comes from torchrun's env vars
(RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT) or an explicit init method.
Bucket size defaults to 16 MB: a ring all-reduce over xGMI is per-link bound
(one outgoing link per ring step), so the engine prefers few large buckets
over many small ones; the 13.4 MB NatureCNN gradient is one to two buckets.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class Comm:
    def __init__(self, rank: int = 0, world_size: int = 1, device: Optional[torch.device] = None,
                 group=None, bucket_bytes: int = 16 << 20):
        self.rank = rank
        self.world_size = world_size
        self.device = device
        self.group = group
        self.bucket_bytes = int(bucket_bytes)

    # ------------------------------------------------------------ setup
    @classmethod
    def from_env(cls, backend: Optional[str] = None, device: Optional[torch.device] = None,
                 timeout_s: float = 300.0, force: bool = False) -> "Comm":
        """``force``: initialise the process group even for one rank (the DP step at
        world 1, ``Runtime.force_dp``; needs MASTER_ADDR / MASTER_PORT)."""
        ws = int(os.environ.get("WORLD_SIZE", "1"))
        if ws <= 1 and not force:
            return cls(0, 1, device)
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("MASTER_PORT", "29511")
        rank = int(os.environ["RANK"])
        if backend is None:
            backend = "nccl" if (device is not None and torch.device(device).type == "cuda") else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if not dist.is_initialized():
            kw = {}
            if backend == "nccl" and device is not None:
                kw["device_id"] = torch.device(device)
            dist.init_process_group(backend=backend, rank=rank, world_size=ws,
                                    timeout=datetime.timedelta(seconds=timeout_s), **kw)
        return cls(rank, ws, device)

    @classmethod
    def init(cls, rank: int, world_size: int, init_method: str, backend: str = "gloo",
             device: Optional[torch.device] = None, force: bool = False) -> "Comm":
        if (world_size > 1 or force) and not dist.is_initialized():
            dist.init_process_group(backend=backend, init_method=init_method, rank=rank,
                                    world_size=world_size,
                                    timeout=datetime.timedelta(seconds=300))
        return cls(rank, world_size, device)

    @property
    def active(self) -> bool:
        return self.world_size > 1

    def barrier(self) -> None:
        if self.active:
            if (self.device is not None and torch.device(self.device).type == "cuda"
                    and dist.get_backend(self.group) == "nccl"):
                dist.barrier(device_ids=[torch.device(self.device).index or 0])
            else:
                dist.barrier()

    def shutdown(self) -> None:
        native = getattr(self, "_native", None)
        if native is not None:
            native.close()
            self._native = None
        if dist.is_initialized():
            dist.destroy_process_group()

    def abort(self) -> None:
        """Failure path: abort the native communicator and the torch.distributed
        process group (outstanding collectives are cancelled, ncclCommAbort under
        RCCL) so the process can exit and torchrun restart the group."""
        native = getattr(self, "_native", None)
        if native is not None:
            native.abort()
            self._native = None
        if dist.is_initialized():
            try:
                dist.distributed_c10d._abort_process_group()
            except Exception:  # pragma: no cover - best effort on the failure path
                pass

    # ------------------------------------------------------ collectives
    def allreduce_flat(self, flat: torch.Tensor, average: bool = True, async_op: bool = False):
        """All-reduce a flat buffer in ``bucket_bytes`` chunks (in place)."""
        if not self.active:
            return None
        n = flat.numel()
        per = max(1, self.bucket_bytes // flat.element_size())
        works = []
        for s in range(0, n, per):
            chunk = flat[s:s + per]
            works.append(dist.all_reduce(chunk, op=dist.ReduceOp.SUM, group=self.group,
                                         async_op=True))
        if async_op:
            return _Pending(works, flat if average else None, self.world_size)
        for w in works:
            w.wait()
        if average:
            flat.div_(self.world_size)
        return None

    def allreduce_grads(self, grads: Sequence[torch.Tensor], average: bool = True) -> None:
        if not self.active:
            return
        grads = [g for g in grads if g is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        self.allreduce_flat(flat, average=average)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def broadcast_flat(self, flat: torch.Tensor, src: int = 0) -> None:
        if self.active:
            dist.broadcast(flat, src=src, group=self.group)

    def broadcast_module(self, module: torch.nn.Module, src: int = 0) -> None:
        if not self.active:
            return
        with torch.no_grad():
            for t in list(module.parameters()) + list(module.buffers()):
                dist.broadcast(t.data, src=src, group=self.group)

    def allgather_scalars(self, values: torch.Tensor) -> torch.Tensor:
        """values: (k,) -> (world, k)."""
        if not self.active:
            return values.reshape(1, -1)
        out = [torch.empty_like(values) for _ in range(self.world_size)]
        dist.all_gather(out, values.contiguous(), group=self.group)
        return torch.stack(out)

    def broadcast_int(self, x: int, src: int = 0) -> int:
        """Rank ``src``'s integer on every rank (int64)."""
        if not self.active:
            return int(x)
        dev = self.device if (self.device is not None and dist.get_backend(self.group) == "nccl") \
            else torch.device("cpu")
        t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
        dist.broadcast(t, src=src, group=self.group)
        return int(t.item())

    def allreduce_scalar(self, x: float, op: str = "sum") -> float:
        if not self.active:
            return float(x)
        dev = self.device if self.device is not None else torch.device("cpu")
        t = torch.tensor([float(x)], dtype=torch.float64, device=dev)
        rop = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(t, op=rop, group=self.group)
        return float(t.item())


class EmulatedComm(Comm):
    """Rank ``rank`` of a ``world``-rank data-parallel job, alone on one GPU
    (``bench.py --emulate-world W``): the learner sizes its step for ``world`` ranks
    (rows per rank, fc row slice, sharded replay) and its collectives become device
    copies of their true sizes (``parallel/rccl.py EmulatedCollectives``).  Host-side
    collectives are identities (no process group); ``active`` is False so callers
    never wait for peers that do not exist."""
    emulated = True

    def __init__(self, world_size: int, rank: int = 0, device: Optional[torch.device] = None):
        super().__init__(rank, world_size, device)

    @property
    def active(self) -> bool:
        return False

    def barrier(self) -> None:
        pass

    def shutdown(self) -> None:
        pass

    def broadcast_flat(self, flat: torch.Tensor, src: int = 0) -> None:
        pass

    def broadcast_int(self, x: int, src: int = 0) -> int:
        return int(x)

    def allreduce_scalar(self, x: float, op: str = "sum") -> float:
        return float(x)


class _Pending:
    def __init__(self, works: List, flat: Optional[torch.Tensor], ws: int):
        self.works, self.flat, self.ws = works, flat, ws

    def wait(self) -> None:
        for w in self.works:
            w.wait()
        if self.flat is not None:
            self.flat.div_(self.ws)
