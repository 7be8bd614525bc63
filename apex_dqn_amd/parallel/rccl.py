"""Native RCCL communicator (``csrc/comm/rccl_comm.cpp``) and the collectives
interface of the data-parallel learner step.

SURVEY §5.8 plans the learner's collectives as a thin native communicator over
librccl with explicit HIP streams, the unique id exchanged through the
torch.distributed rendezvous; §5.3 adds a communicator abort for failure
recovery.  ``RcclComm`` is that communicator: ``ncclCommInitRank`` over the same
librccl torch already loaded (one RCCL instance per process), collectives
enqueued on a dedicated comm stream that waits on the compute stream through
events -- inside a HIP-graph capture these waits become graph edges, so the
learner's DP step stays ONE captured graph -- and ``abort()`` /
``check()`` on the communicator's asynchronous error state.

``make_collectives(comm, backend)`` returns the object the learner step uses:
``TorchCollectives`` (torch.distributed: RCCL via the ``nccl`` process group, or
gloo on CPU), ``NativeCollectives`` (this communicator) or ``EmulatedCollectives``
(``bench.py --emulate-world W``: rank 0's share of a W-rank step on one GPU, every
collective a device copy of its true size on a comm stream).  All expose
``all_reduce(t, op)``, ``all_gather_into(out, inp)`` (in place when ``inp`` is this
rank's chunk of ``out``) and ``reduce_scatter_into(out, inp)``, returning a handle
whose ``wait()`` makes the current stream wait for the result; on a GPU the handle
also carries the completion ``event`` (any stream may wait on it: a graph edge under
capture).  ``all_reduce_inline`` (where ``inline`` is True) enqueues on the current
stream itself -- no fork / join edge on the step's critical path.
"""
from __future__ import annotations

import ctypes
import glob
import os
from typing import Optional

import torch

_DTYPES = {torch.float32: 7, torch.float64: 8, torch.bfloat16: 9, torch.float16: 6, torch.int32: 2,
           torch.int64: 4, torch.uint8: 1}
_OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_LIB = None


def _torch_rccl_path() -> Optional[str]:
    cands = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so*"))
    return cands[0] if cands else None


def load_comm_lib() -> ctypes.CDLL:
    """libapex_comm.so with librccl resolved (torch's bundled copy first)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    from ..ops.build import ensure_current
    # content-addressed (ops/build.py): a stale or missing library is rebuilt, never run
    lib = ctypes.CDLL(ensure_current("comm"))
    c_p, c_i, c_sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    sigs = {
        "apex_comm_load": ([ctypes.c_char_p], c_i),
        "apex_comm_version": ([], c_i),
        "apex_comm_error_string": ([c_i], ctypes.c_char_p),
        "apex_comm_unique_id": ([ctypes.c_char_p], c_i),
        "apex_comm_id_bytes": ([], c_i),
        "apex_comm_init": ([ctypes.POINTER(c_p), c_i, ctypes.c_char_p, c_i], c_i),
        "apex_comm_all_reduce": ([c_p, c_p, c_p, c_sz, c_i, c_i, c_p], c_i),
        "apex_comm_all_gather": ([c_p, c_p, c_p, c_sz, c_i, c_p], c_i),
        "apex_comm_broadcast": ([c_p, c_p, c_p, c_sz, c_i, c_i, c_p], c_i),
        "apex_comm_reduce_scatter": ([c_p, c_p, c_p, c_sz, c_i, c_i, c_p], c_i),
        "apex_comm_count": ([c_p, ctypes.POINTER(c_i), ctypes.POINTER(c_i)], c_i),
        "apex_comm_group_start": ([], c_i),
        "apex_comm_group_end": ([], c_i),
        "apex_comm_async_error": ([c_p], c_i),
        "apex_comm_abort": ([c_p], c_i),
        "apex_comm_destroy": ([c_p], c_i),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes, fn.restype = args, res
    path = _torch_rccl_path()
    rc = lib.apex_comm_load(path.encode() if path else None)
    if rc != 0:
        raise RuntimeError(f"apex_comm_load({path}): {lib.apex_comm_error_string(rc).decode()}")
    _LIB = lib
    return lib


class RcclError(RuntimeError):
    pass


class RcclComm:
    """One RCCL communicator for ``rank`` of ``world`` on ``device``.  The unique id
    comes from rank 0 through ``exchange(id_tensor)`` -- by default a broadcast over
    the initialised torch.distributed default group."""

    def __init__(self, rank: int, world: int, device, exchange=None):
        self.lib = load_comm_lib()
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device(device)
        nb = self.lib.apex_comm_id_bytes()
        buf = ctypes.create_string_buffer(nb)
        if self.rank == 0:
            self._check(self.lib.apex_comm_unique_id(buf), "unique_id")
        idt = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
        if self.world > 1:
            if exchange is None:
                import torch.distributed as dist
                dev = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
                t = idt.to(dev)
                dist.broadcast(t, src=0)
                idt = t.cpu()
            else:
                idt = exchange(idt)
        self._id = bytes(idt.numpy().tobytes())
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            self._check(self.lib.apex_comm_init(ctypes.byref(h), self.world, self._id, self.rank), "comm_init")
        self.handle = h
        self.stream = torch.cuda.Stream(self.device)
        self._closed = False

    def _check(self, rc: int, what: str) -> None:
        if rc != 0:
            raise RcclError(f"rccl {what} failed: {self.lib.apex_comm_error_string(rc).decode()} ({rc})")

    @property
    def version(self) -> int:
        return int(self.lib.apex_comm_version())

    # ----------------------------------------------------------- raw enqueue
    def _enqueue(self, fn, what: str, *args) -> None:
        self._check(fn(self.handle, *args), what)

    def all_reduce_(self, t: torch.Tensor, op: str = "sum", stream=None) -> None:
        """In-place all-reduce on ``stream`` (default: the current stream)."""
        s = stream or torch.cuda.current_stream(self.device)
        self._enqueue(self.lib.apex_comm_all_reduce, "all_reduce", t.data_ptr(), t.data_ptr(), t.numel(),
                      _DTYPES[t.dtype], _OPS[op], s.cuda_stream)

    def all_gather_(self, out: torch.Tensor, inp: torch.Tensor, stream=None) -> None:
        assert out.numel() == inp.numel() * self.world and out.dtype == inp.dtype
        s = stream or torch.cuda.current_stream(self.device)
        self._enqueue(self.lib.apex_comm_all_gather, "all_gather", inp.data_ptr(), out.data_ptr(), inp.numel(),
                      _DTYPES[inp.dtype], s.cuda_stream)

    def reduce_scatter_(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", stream=None) -> None:
        """out = this rank's chunk of the reduction of ``inp`` (world x out.numel())."""
        assert inp.numel() == out.numel() * self.world and out.dtype == inp.dtype
        s = stream or torch.cuda.current_stream(self.device)
        self._enqueue(self.lib.apex_comm_reduce_scatter, "reduce_scatter", inp.data_ptr(), out.data_ptr(),
                      out.numel(), _DTYPES[out.dtype], _OPS[op], s.cuda_stream)

    def count(self):
        """(ranks, this rank) as the RCCL communicator itself reports them."""
        n, r = ctypes.c_int(0), ctypes.c_int(-1)
        self._check(self.lib.apex_comm_count(self.handle, ctypes.byref(n), ctypes.byref(r)), "comm_count")
        return int(n.value), int(r.value)

    def broadcast_(self, t: torch.Tensor, src: int = 0, stream=None) -> None:
        s = stream or torch.cuda.current_stream(self.device)
        self._enqueue(self.lib.apex_comm_broadcast, "broadcast", t.data_ptr(), t.data_ptr(), t.numel(),
                      _DTYPES[t.dtype], int(src), s.cuda_stream)

    # ------------------------------------------------------------- health
    def check(self) -> None:
        """Raise if the communicator has an asynchronous error (peer failure)."""
        rc = self.lib.apex_comm_async_error(self.handle)
        if rc != 0:
            raise RcclError(f"rccl async error: {self.lib.apex_comm_error_string(rc).decode()} ({rc})")

    def abort(self) -> None:
        """Cancel outstanding collectives and free the communicator (a rank whose
        peer died must not block in teardown; the elastic restart rebuilds it)."""
        if not self._closed:
            self.lib.apex_comm_abort(self.handle)
            self._closed = True

    def close(self) -> None:
        if not self._closed:
            torch.cuda.synchronize(self.device)
            self.lib.apex_comm_destroy(self.handle)
            self._closed = True


# ------------------------------------------------------------------ collectives
class _Done:
    event = None

    def wait(self) -> None:
        pass


class _TorchWork:
    event = None

    def __init__(self, work, coll=None):
        self.work = work
        self.coll = coll
        if coll is not None:
            coll._seq += 1
            self.seq = coll._seq

    def wait(self) -> None:
        """The current stream waits for the process group's stream (RCCL: in issue order,
        so a wait covers every earlier collective and later waits on those add no edge)."""
        if self.work is None:
            return
        c = self.coll
        if c is None:
            self.work.wait()
            return
        key = torch.cuda.current_stream(c.device).cuda_stream
        if self.seq > c._joined.get(key, 0):
            self.work.wait()
            c._joined[key] = self.seq


class _GroupedWork:
    """A collective issued inside ``NativeCollectives.fused()``: RCCL launches the group's
    operations at the group's end, so the completion event is recorded there (shared by
    every member)."""

    def __init__(self):
        self.work = None

    @property
    def event(self):
        return self.work.event if self.work is not None else None

    def wait(self) -> None:
        self.work.wait()


class _StreamWork:
    """Completion of a collective enqueued on a collectives object's comm stream: ``wait``
    makes the current stream wait for an event recorded right after it (a graph edge
    under capture), so a later collective still in flight is not waited for.  The
    collectives of one object run in order on one stream, so a join covers every op
    enqueued before it: a wait on an op already covered by an earlier join of the same
    stream adds no edge (each cross-queue edge of a captured graph costs several
    microseconds)."""

    def __init__(self, coll):
        self.coll = coll
        coll._seq += 1
        self.seq = coll._seq
        self.stream = coll.stream
        self.event = torch.cuda.Event()
        self.event.record(self.stream)

    def wait(self) -> None:
        c = self.coll
        cur = torch.cuda.current_stream(c.device)
        if cur.cuda_stream == self.stream.cuda_stream:
            return               # issued on this very stream: already in order
        key = (cur.cuda_stream, self.stream.cuda_stream)
        if self.seq > c._joined.get(key, 0):
            cur.wait_event(self.event)
            c._joined[key] = self.seq


class _StreamColl:
    """Shared plumbing: a comm stream that forks from the current stream per op."""
    inline = False

    def fused(self, inline: bool = False):
        """Context: the collectives issued inside leave as ONE launch where the backend
        can fuse them (RCCL group); elsewhere a no-op."""
        from contextlib import nullcontext
        return nullcontext()

    def _init_stream(self, device):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self._seq = 0          # collectives enqueued
        self._joined = {}      # per waiting stream: the last collective a join covers

    def _fork(self):
        cur = torch.cuda.current_stream(self.device)
        if cur.cuda_stream != self.stream.cuda_stream:
            self.stream.wait_stream(cur)
        return self.stream

    def use_stream(self, stream) -> None:
        """Enqueue the collectives on ``stream`` (the learner's branch stream) instead of a
        stream of their own."""
        self.stream = stream
        self._joined = {}

    def on_stream(self, stream):
        """Context: the collectives issued inside go to ``stream`` (already ordered after
        the collectives of the usual stream by the caller's events)."""
        from contextlib import contextmanager

        @contextmanager
        def ctx():
            prev, self.stream = self.stream, stream
            try:
                yield
            finally:
                self.stream = prev
        return ctx()


class TorchCollectives:
    """torch.distributed.  With the RCCL process group the collectives run on the process
    group's own stream, forked from the current stream; their handles are waited for on
    the step's main (capture-origin) stream only -- a forked stream that waits on a
    stream forked from itself crashed HIP graph capture (hipStreamEndCapture segfault,
    round 5, ``scripts/archive/probe_dp_capture.py``), so this backend runs the DP step eagerly
    (learner/fused_learner.py ``_dp_graphs``).  gloo (CPU
    tests, one-GPU rehearsals) keeps the process group's own handles."""
    name = "torch"
    inline = False

    def __init__(self, group=None, device=None):
        import torch.distributed as dist
        self.group = group
        self._nccl = (device is not None and torch.device(device).type == "cuda"
                      and dist.is_initialized() and dist.get_backend(group) == "nccl")
        self.device = torch.device(device) if device is not None else None
        self._seq = 0
        self._joined = {}

    def _sync(self, t: torch.Tensor) -> bool:
        """gloo on device tensors (one-GPU rehearsals): run the collective synchronously.
        Several async gloo collectives on device tensors in flight at once deadlocked
        4 ranks sharing one GPU (scripts/rehearse_dp.sh 4); gloo has nothing to overlap."""
        import torch.distributed as dist
        return t.is_cuda and dist.get_backend(self.group) != "nccl"

    def _on_stream(self, fn):
        return _TorchWork(fn(), self)

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        import torch.distributed as dist
        rop = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
        if self._nccl:
            return self._on_stream(lambda: dist.all_reduce(t, op=rop, group=self.group, async_op=True))
        if self._sync(t):
            dist.all_reduce(t, op=rop, group=self.group)
            return _Done()
        return _TorchWork(dist.all_reduce(t, op=rop, group=self.group, async_op=True))

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor):
        import torch.distributed as dist
        if self._nccl:
            return self._on_stream(lambda: dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True))
        if dist.get_backend(self.group) == "nccl":      # (no device given: the process group's handle)
            return _TorchWork(dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True))
        # gloo (CPU tests, one-GPU rehearsals; its all_gather takes no CUDA tensors): a
        # SUM all-reduce of the rank-placed rows, exact (every other row is zero); ``inp``
        # may be this rank's chunk of ``out`` (in place)
        W, n = dist.get_world_size(self.group), inp.numel()
        r = dist.get_rank(self.group)
        src = inp.reshape(-1).clone()
        out.zero_()
        out.view(W, n)[r].copy_(src)
        return self.all_reduce(out, "sum")

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum"):
        import torch.distributed as dist
        if self._nccl:
            rop = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
            return self._on_stream(lambda: dist.reduce_scatter_tensor(out, inp, op=rop, group=self.group,
                                                                      async_op=True))
        # gloo has no reduce-scatter: all-reduce a copy, keep this rank's chunk
        W, n = dist.get_world_size(self.group), out.numel()
        r = dist.get_rank(self.group)
        tmp = inp.reshape(-1).clone()
        self.all_reduce(tmp, op).wait()
        out.reshape(-1).copy_(tmp.view(W, n)[r])
        return _Done()

    def world(self) -> int:
        import torch.distributed as dist
        return int(dist.get_world_size(self.group))

    def fused(self, inline: bool = False):
        from contextlib import nullcontext
        return nullcontext()


class NativeCollectives(_StreamColl):
    """The DP step's collectives on the native communicator's own stream."""
    name = "native"
    inline = True

    def __init__(self, comm: RcclComm):
        self.comm = comm
        self.device = comm.device
        self.stream = comm.stream
        self._seq = 0
        self._joined = {}

    _grouped = None     # handles of the open RCCL group (fused())

    def _done(self):
        if self._grouped is not None:
            h = _GroupedWork()
            self._grouped.append(h)
            return h
        return _StreamWork(self)

    def fused(self, inline: bool = False):
        """RCCL group: the collectives issued inside launch together at its end (one kernel
        and one latency instead of one per op: the fc factor rows with the shard
        statistics, the updated fc rows with their biases).  ``inline``: a group of
        ``*_inline`` ops on the current stream (no fork)."""
        from contextlib import contextmanager
        lib = self.comm.lib

        @contextmanager
        def ctx():
            assert self._grouped is None, "RCCL groups do not nest here"
            if not inline:
                self._fork()
            self._grouped = []
            self.comm._check(lib.apex_comm_group_start(), "group_start")
            try:
                yield
            finally:
                members, self._grouped = self._grouped, None
                self.comm._check(lib.apex_comm_group_end(), "group_end")
                if members:
                    w = _StreamWork(self)
                    for m in members:
                        m.work = w
        return ctx()

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        s = self._fork()
        self.comm.all_reduce_(t, op, stream=s)
        return self._done()

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor):
        s = self._fork()
        self.comm.all_gather_(out, inp, stream=s)
        return self._done()

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum"):
        s = self._fork()
        self.comm.reduce_scatter_(out, inp, op, stream=s)
        return self._done()

    def all_reduce_inline(self, t: torch.Tensor, op: str = "sum"):
        """All-reduce enqueued on the CURRENT stream (no fork / join): the caller has
        already joined every collective issued before it, so RCCL's issue order holds."""
        self.comm.all_reduce_(t, op)
        return _Done()

    def all_gather_inline(self, out: torch.Tensor, inp: torch.Tensor):
        """All-gather on the CURRENT stream (as :meth:`all_reduce_inline`)."""
        self.comm.all_gather_(out, inp)
        return _Done()

    def world(self) -> int:
        return self.comm.count()[0]


class EmulatedCollectives(_StreamColl):
    """Rank ``rank``'s view of a ``world``-rank step on ONE GPU (``bench.py
    --emulate-world``): every collective is a device copy of its true size -- an
    all-gather writes this rank's chunk into every slot (the gathered rows / statistics /
    parameters stay valid data), an all-reduce copies the buffer once, a reduce-scatter
    copies this rank's chunk.  Launches are modelled on RCCL's: one collective is ONE
    kernel (``csrc/optimizer.hip copy_segments_kernel``, all its copies), and the
    collectives of a ``fused()`` group leave as ONE kernel at the group's end, as an
    ``ncclGroupStart / End`` pair launches them; non-inline ones run on a comm stream
    joined like the real one's.  It measures the per-rank compute, the graph edges and
    the copies; RCCL's own latency and xGMI transfer time are not in it."""
    name = "emulated"
    inline = True

    def __init__(self, device, world: int, rank: int = 0):
        self._init_stream(device)
        self.W, self.rank = int(world), int(rank)
        self._scratch = {}
        self._group = None          # (segments, handles) of the open fused() group

    def _buf(self, t: torch.Tensor) -> torch.Tensor:
        key = (t.dtype, t.numel())
        b = self._scratch.get(key)
        if b is None:
            b = self._scratch[key] = torch.empty(t.numel(), dtype=t.dtype, device=self.device)
        return b

    @staticmethod
    def _seg(dst: torch.Tensor, src: torch.Tensor):
        assert dst.is_contiguous() and src.is_contiguous() and dst.numel() == src.numel()
        return (src.data_ptr(), dst.data_ptr(), src.numel() * src.element_size(), dst, src)

    def _reduce_segs(self, t: torch.Tensor):
        return [self._seg(self._buf(t), t.reshape(-1))]

    def _gather_segs(self, out: torch.Tensor, inp: torch.Tensor):
        W, n, r = self.W, inp.numel(), self.rank
        rows = out.view(W, n)
        src = inp.reshape(-1)
        return [self._seg(rows[j], src) for j in range(W) if j != r or rows[j].data_ptr() != src.data_ptr()]

    def _scatter_segs(self, out: torch.Tensor, inp: torch.Tensor):
        n = out.numel()
        return [self._seg(out.reshape(-1), inp.reshape(-1)[self.rank * n:(self.rank + 1) * n])]

    def _launch(self, segs) -> None:
        """All copies in as few launches as the kernel's 32 segments allow (one, here)."""
        if not segs:
            return
        if self.device.type != "cuda":
            for _, _, _, dst, src in segs:
                dst.copy_(src)
            return
        from ..ops import _lib
        lib = _lib.require_kernels()
        for i in range(0, len(segs), 32):
            part = segs[i:i + 32]
            arr = lambda k: (ctypes.c_int64 * len(part))(*[int(x[k]) for x in part])  # noqa: E731
            _lib.check(lib.apex_copy_segments(len(part), arr(0), arr(1), arr(2), _lib.stream_ptr(self.device)),
                       "copy_segments")

    def _op(self, segs, inline: bool):
        if self._group is not None:
            self._group[0].extend(segs)
            h = _GroupedWork()
            self._group[1].append(h)
            return h
        if inline:
            self._launch(segs)
            return _Done()
        s = self._fork()
        with torch.cuda.stream(s):
            self._launch(segs)
        return _StreamWork(self)

    def fused(self, inline: bool = False):
        """The group's collectives leave as one copy launch at its end (inline: on the
        current stream; else on the comm stream, forked from the current one)."""
        from contextlib import contextmanager

        @contextmanager
        def ctx():
            assert self._group is None, "groups do not nest here"
            self._group = ([], [])
            try:
                yield
            finally:
                segs, handles = self._group
                self._group = None
                if inline:
                    self._launch(segs)
                    w = _Done()
                else:
                    s = self._fork()
                    with torch.cuda.stream(s):
                        self._launch(segs)
                    w = _StreamWork(self)
                for h in handles:
                    h.work = w
        return ctx()

    def all_reduce(self, t: torch.Tensor, op: str = "sum"):
        return self._op(self._reduce_segs(t), False)

    def all_reduce_inline(self, t: torch.Tensor, op: str = "sum"):
        return self._op(self._reduce_segs(t), True)

    def all_gather_inline(self, out: torch.Tensor, inp: torch.Tensor):
        return self._op(self._gather_segs(out, inp), True)

    def all_gather_into(self, out: torch.Tensor, inp: torch.Tensor):
        return self._op(self._gather_segs(out, inp), False)

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum"):
        return self._op(self._scatter_segs(out, inp), False)

    def world(self) -> int:
        return self.W


def make_collectives(comm, backend: str = "torch", device=None):
    """Collectives for the learner's DP step: ``torch`` (torch.distributed) or
    ``native`` (RcclComm; GPU ranks with an initialised process group); an emulated
    communicator (``parallel/dist.py EmulatedComm``) gets ``EmulatedCollectives``."""
    dev = device if device is not None else getattr(comm, "device", None)
    if getattr(comm, "emulated", False):
        return EmulatedCollectives(dev, comm.world_size, comm.rank)
    if backend == "native":
        nc = getattr(comm, "_native", None)
        if nc is None:
            nc = RcclComm(comm.rank, comm.world_size, dev)
            comm._native = nc
        return NativeCollectives(nc)
    if backend != "torch":
        raise ValueError("Runtime.comm_backend must be 'torch' or 'native'")
    return TorchCollectives(getattr(comm, "group", None), dev)
