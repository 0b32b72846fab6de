"""Data parallelism: one process per GPU, minibatch sharded across ranks, RCCL
all-reduce of the flat gradient buffer per step.

The all-reduce is bucketed and overlapped with the backward: the network's flat
gradient buffer is laid out in forward (state_dict) order and the backward
produces it back to front, so as soon as every gradient above an offset is final
the bucket below the previous watermark is handed to RCCL (async, on its own
stream) while the remaining backward kernels run (OverlapReducer).

BatchNorm stays local to each rank by default (each rank's forward equals the
reference's bs-16 forward on its shard); enable_sync_batchnorm / UGPG_SYNC_BN=1 makes it
normalise over the global batch instead (SURVEY §8e's optional SyncBN).  Gradients are summed and the 1/world_size average
is folded into the RMSprop kernel (``RMSprop.grad_scale``).  Everything here is
device-agnostic so the same code path is exercised with the ``gloo`` backend on
CPU in the test-suite.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

from .flat import contiguous_run


def world() -> tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def init_from_env(backend: str | None = None):
    """Initialise the default process group from torchrun's environment."""
    if not dist.is_available() or dist.is_initialized():
        return world()
    if int(os.environ.get("WORLD_SIZE", "1")) <= 1:
        return 0, 1
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return world()


class _SyncBN:
    """The exchange of synchronised BatchNorm (ops._BN_SYNC): SUM all-reduces, in place and
    stream-ordered, through torch.distributed (RCCL under "nccl") or libugpg's communicator
    (UGPG_COMM=native).  At world size 1 (forced) the exchange is the identity.

    Either way the exchange has an RCCL communicator of its own: the statistics exchange of
    a BatchNorm in the backward must not queue behind the overlapped gradient buckets in
    flight on the default group / the process-wide native communicator (RCCL serialises the
    operations of one communicator)."""

    def __init__(self):
        self.rank, self.nranks = world()
        self.group = dist.new_group(list(range(self.nranks))) if self.nranks > 1 else None
        self._comm = None

    def native(self):
        """Under UGPG_COMM=native (data parallel): this exchange's own libugpg Communicator,
        never the one native_comm() hands the gradient buckets.  Built at the first CUDA
        exchange -- the same BatchNorm of the same forward on every rank, so its rendezvous
        is collective."""
        if self.nranks <= 1 or os.environ.get("UGPG_COMM", "torch") != "native":
            return None
        if self._comm is None:
            self._comm = Communicator()
        return self._comm

    def all_reduce(self, t: torch.Tensor) -> torch.Tensor:
        if self.nranks > 1:
            comm = self.native() if t.is_cuda else None
            if comm is not None:
                comm.all_reduce(t)
            else:
                dist.all_reduce(t, group=self.group)
        return t


def enable_sync_batchnorm(flag: bool = True) -> None:
    """Synchronised BatchNorm (SURVEY §8e's optional policy; default off = local BatchNorm):
    every train-mode BatchNorm of every ugpg model normalises over the GLOBAL batch, as the
    reference's single-process BatchNorm2d does over its whole batch (UG_unet_parts.py:11,
    14), at the cost of two small collectives per BatchNorm per step (forward statistics,
    backward sums).  COLLECTIVE: enable it on every rank (UGPG_SYNC_BN=1 makes the trainers
    do so)."""
    from . import ops
    ops._BN_SYNC = _SyncBN() if flag else None


def sync_batchnorm_enabled() -> bool:
    from . import ops
    return ops._BN_SYNC is not None


def sync_batchnorm_from_env() -> None:
    """UGPG_SYNC_BN=1: synchronised BatchNorm under data parallelism (the trainers call
    this at construction); UGPG_SYNC_BN=force also at world size 1 (the kernels run, the
    exchange is the identity: for measuring their cost on one GPU)."""
    v = os.environ.get("UGPG_SYNC_BN", "0")
    if v == "force" or (v == "1" and world()[1] > 1):
        enable_sync_batchnorm(True)


def shard(batch: torch.Tensor, rank: int, world_size: int) -> torch.Tensor:
    """Contiguous equal shard of the global batch for `rank`."""
    n = batch.shape[0]
    if n % world_size:
        raise ValueError(f"global batch {n} is not divisible by world size {world_size}")
    per = n // world_size
    return batch[rank * per:(rank + 1) * per]


class OverlapReducer:
    """Bucketed SUM all-reduce of one flat gradient buffer, issued during the backward.

    begin(flat, views): a new backward starts; `views` are the per-parameter gradient
    views of `flat` (any order).  done(views): these gradients are final.  Whenever all
    gradients at offsets >= w are final (the watermark w), the elements between w and
    the last issued bucket are issued in buckets of `bucket_bytes` (async).  flush()
    issues the rest; wait() makes the current stream wait for every bucket and returns
    the 1/world_size scale.  Buckets are issued in the same order on every rank (the
    backward is identical), as collectives require."""

    def __init__(self, bucket_bytes: int = 16 << 20):
        self.bucket = max(1, bucket_bytes // 4)
        self.flat = None
        self.works = []

    def begin(self, flat, views):
        base = flat.storage_offset()
        self.flat = flat
        self.ranges = sorted(((v.storage_offset() - base, v.numel()) for v in views if v is not None),
                             reverse=True)
        self.final = set()
        self.k = 0                    # ranges[:k] (highest offsets first) are final
        self.hi = flat.numel()        # [hi, end) already issued
        self.works = []

    def _issue(self, lo, hi):
        while hi > lo:
            a = max(lo, hi - self.bucket)
            self.works.append(_all_reduce_async(self.flat[a:hi]))
            hi = a
        return lo

    def done(self, views):
        if self.flat is None:
            return
        base = self.flat.storage_offset()
        for v in views:
            if v is not None:
                self.final.add(v.storage_offset() - base)
        while self.k < len(self.ranges) and self.ranges[self.k][0] in self.final:
            self.k += 1
        mark = self.ranges[self.k - 1][0] if self.k else self.flat.numel()
        if self.hi - mark >= self.bucket:
            # issue whole buckets only; the remainder waits for more gradients
            lo = self.hi - (self.hi - mark) // self.bucket * self.bucket
            self.hi = self._issue(lo, self.hi)

    def flush(self):
        if self.flat is not None and self.hi > 0:
            self.hi = self._issue(0, self.hi)

    def pending_for(self, grads) -> bool:
        return self.flat is not None and bool(grads) and \
            grads[0].untyped_storage().data_ptr() == self.flat.untyped_storage().data_ptr()

    def wait(self) -> float:
        for w in self.works:
            w.wait()
        self.works = []
        self.flat = None
        return 1.0 / world()[1]


_REDUCER: OverlapReducer | None = None
_OVERLAP = False


def enable_overlap(flag: bool = True) -> None:
    """Opt in to overlapped gradient all-reduce: every ugpg backward then feeds the
    process-wide OverlapReducer (gradients are summed over ranks during the backward)
    and the caller must finish the step with allreduce_gradients (the trainers do)."""
    global _OVERLAP
    _OVERLAP = bool(flag)


class overlapped_allreduce:
    """Context manager: backwards run inside it feed the OverlapReducer (see
    enable_overlap); finish with allreduce_gradients after the block."""

    def __enter__(self):
        self.prev = _OVERLAP
        enable_overlap(True)
        return self

    def __exit__(self, *exc):
        enable_overlap(self.prev)
        return False


def overlap_reducer() -> OverlapReducer | None:
    """The reducer the ugpg backward feeds: None unless enabled, data-parallel, and not
    disabled with UGPG_DP_OVERLAP=0."""
    global _REDUCER
    if not _OVERLAP or world()[1] <= 1 or os.environ.get("UGPG_DP_OVERLAP", "1") == "0":
        return None
    if _REDUCER is None:
        _REDUCER = OverlapReducer(int(os.environ.get("UGPG_DP_BUCKET_MB", "16")) << 20)
    return _REDUCER


_DT = {torch.float32: 0, torch.bfloat16: 1, torch.float64: 2, torch.int64: 3}
_OPS = {"sum": 0, "avg": 1, "max": 2}


class Communicator:
    """libugpg's own RCCL communicator (C-ABI ugpg_comm_*, include/ugpg.h) for one process
    per GPU.  Rendezvous: rank 0's unique id travels through the torch.distributed store
    (or is passed in).  Collectives run on the caller's current HIP stream, in place.

    torch.distributed's "nccl" backend is RCCL too; this handle is the same exchange at the
    C-ABI boundary, for callers that bind libugpg without torch.  Select it
    for the trainer's gradient all-reduce with UGPG_COMM=native."""

    def __init__(self, rank=None, world_size=None, device=None, unique_id: bytes | None = None):
        import ctypes
        from ._C import check, lib
        r, ws = world()
        self.rank = r if rank is None else rank
        self.world_size = ws if world_size is None else world_size
        self.device = torch.cuda.current_device() if device is None else int(device)
        n = lib.ugpg_comm_id_bytes()
        if unique_id is None:
            buf = (ctypes.c_ubyte * n)()
            if self.rank == 0:
                check(lib.ugpg_comm_unique_id(buf, n), "comm_unique_id")
            if self.world_size > 1:
                obj = [bytes(buf) if self.rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                unique_id = obj[0]
            else:
                unique_id = bytes(buf)
        idbuf = (ctypes.c_ubyte * n).from_buffer_copy(unique_id[:n])
        self._h = ctypes.c_void_p()
        check(lib.ugpg_comm_init(ctypes.byref(self._h), self.world_size, self.rank, idbuf, n,
                                 self.device), "comm_init")

    def _stream(self):
        return torch.cuda.current_stream().cuda_stream

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        from ._C import check, lib
        if not t.is_cuda or not t.is_contiguous():
            raise RuntimeError("ugpg Communicator: contiguous ROCm tensors only")
        check(lib.ugpg_comm_allreduce(self._h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                      _OPS[op], self._stream()), "comm_allreduce")
        return t

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        from ._C import check, lib
        if not t.is_cuda or not t.is_contiguous():
            raise RuntimeError("ugpg Communicator: contiguous ROCm tensors only")
        check(lib.ugpg_comm_broadcast(self._h, t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype],
                                      root, self._stream()), "comm_broadcast")
        return t

    def close(self):
        from ._C import check, lib
        if self._h:
            check(lib.ugpg_comm_destroy(self._h), "comm_destroy")
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_COMM: Communicator | None = None


def native_comm() -> Communicator | None:
    """The process-wide libugpg communicator when UGPG_COMM=native (data parallel only)."""
    global _COMM
    if os.environ.get("UGPG_COMM", "torch") != "native" or world()[1] <= 1:
        return None
    if _COMM is None:
        _COMM = Communicator()
    return _COMM


class _NativeWork:
    """async handle of a bucket reduced by the native communicator on a side stream"""

    def __init__(self, comm, t, stream):
        cur = torch.cuda.current_stream()
        stream.wait_stream(cur)
        with torch.cuda.stream(stream):
            comm.all_reduce(t)
            self.done = torch.cuda.Event()
            self.done.record(stream)
        t.record_stream(stream)

    def wait(self):
        torch.cuda.current_stream().wait_event(self.done)


_SIDE = None


def grad_bf16() -> bool:
    """Exchange gradient buckets in bf16?  Opt-in only (UGPG_GRAD_BF16=1).  The default is
    fp32 for every arithmetic, as torch's DDP under autocast exchanges the fp32 .grad: the
    bf16 exchange errs by up to 2^-8 * sum_r |g_r| per element, above the config-3 parity
    floor (G4c) of the output heads at any N > 1 (tests/test_dist_gloo.py::
    test_bf16_exchange_error_bound)."""
    return os.environ.get("UGPG_GRAD_BF16", "0") == "1"


class _Bf16Work:
    """async handle of a bucket exchanged in bf16: the sum is cast back into the fp32
    bucket on the current stream at wait()"""

    def __init__(self, t):
        self.t = t
        if t.is_cuda:
            from . import ops
            self.h = torch.empty(t.numel(), dtype=torch.bfloat16, device=t.device)
            ops.cast_f32_bf16(t, self.h)
        else:  # gloo rehearsal on CPU tensors (tests)
            self.h = t.to(torch.bfloat16)
        self.w = _all_reduce_async(self.h, bf16=False)

    def wait(self):
        self.w.wait()
        if self.t.is_cuda:
            from . import ops
            ops.cast_bf16_f32(self.h, self.t)
        else:
            self.t.copy_(self.h.to(torch.float32))


def _all_reduce_async(t, bf16=None):
    """SUM all-reduce of a gradient bucket: RCCL through torch.distributed (async work), or
    libugpg's communicator on a side stream (UGPG_COMM=native); in bf16 when grad_bf16()."""
    global _SIDE
    if (grad_bf16() if bf16 is None else bf16) and t.dtype == torch.float32:
        return _Bf16Work(t)
    comm = native_comm() if t.is_cuda else None
    if comm is None:
        return dist.all_reduce(t, async_op=True)
    if _SIDE is None:
        _SIDE = torch.cuda.Stream(device=t.device)
    return _NativeWork(comm, t, _SIDE)


def _runs(grads):
    """Split `grads` (in order) into maximal back-to-back runs of one storage."""
    runs, cur = [], []
    for g in grads:
        if cur and contiguous_run(cur + [g]) is None:
            runs.append(cur)
            cur = []
        cur.append(g)
    if cur:
        runs.append(cur)
    return runs


def _allreduce_runs(grads, bucket_bytes):
    """One SUM all-reduce per flat run (bucketed); loose tensors (a run of one, e.g.
    the Herlev head's weights) are packed into one staging buffer and reduced together."""
    loose = []
    step = max(1, bucket_bytes // 4)
    for run in _runs(grads):
        flat = contiguous_run(run) if len(run) > 1 else None
        if flat is None:
            loose.extend(run)
            continue
        base, _, n = flat
        for off in range(0, n, step):
            _all_reduce_async(base[off:off + step]).wait()
    if loose:
        # through the same exchange as the flat runs (bf16 when grad_bf16(), the native
        # communicator when selected)
        stage = torch.cat([g.reshape(-1) for g in loose])
        _all_reduce_async(stage).wait()
        off = 0
        for g in loose:
            g.copy_(stage[off:off + g.numel()].view_as(g))
            off += g.numel()


def allreduce_gradients(params, bucket_bytes: int = 64 << 20):
    """Sum gradients over ranks.  Gradients the backward already handed to the
    OverlapReducer are only waited for; the rest go out as one call per flat run
    (the normal ugpg layout is a single run) plus one call for loose tensors.
    Returns the scale (1/world_size) the optimizer must apply."""
    _, ws = world()
    grads = [p.grad for p in params if p.grad is not None]
    if ws <= 1 or not grads:
        return 1.0
    red = _REDUCER
    pending = red is not None and red.flat is not None
    if pending:
        ptr = red.flat.untyped_storage().data_ptr()
        grads = [g for g in grads if g.untyped_storage().data_ptr() != ptr]
        # the overlapped buckets finish first: with UGPG_COMM=native they run on a second
        # communicator, and two communicators' collectives in flight at once can deadlock
        red.wait()
    if grads:
        _allreduce_runs(grads, bucket_bytes)
    return 1.0 / ws


def broadcast_parameters(module: torch.nn.Module, src: int = 0):
    """Make every replica start from rank `src`'s parameters and buffers."""
    _, ws = world()
    if ws <= 1:
        return
    params = list(module.parameters())
    bufs = list(module.buffers())
    for t in params + bufs:
        dist.broadcast(t.data, src)
    from . import ops
    # written behind autograd's back: cached packs / eval BN params are stale
    ops.weights_written(params + bufs)


def broadcast_buffers(module: torch.nn.Module, src: int = 0):
    """BatchNorm running statistics and num_batches_tracked from rank `src` (SURVEY §8e:
    local BN in the step; replicas agree at validation, stage end and checkpoints)."""
    _, ws = world()
    if ws <= 1:
        return
    bufs = list(module.buffers())
    for t in bufs:
        dist.broadcast(t.data, src)
    from . import ops
    ops.weights_written(bufs)  # cached eval-mode BN parameters are stale


def allreduce_metrics(mbuf, ip: int, n_stat: float, avg_mask: int):
    """Turn this rank's device metrics buffer into the global-batch metrics in place:
    per-rank means (bits of avg_mask) are averaged (equal shards), counts summed, and
    the (mean, unbiased std) pair at [ip, ip+1) pooled over all ranks' n_stat values.
    One float64 SUM all-reduce of n+2 values (libugpg metrics_pack/unpack kernels)."""
    _, ws = world()
    if ws <= 1:
        return mbuf
    from . import ops
    sums = ops.metrics_pack(mbuf, ip, n_stat)
    dist.all_reduce(sums)
    return ops.metrics_unpack(sums, mbuf, ip, avg_mask)


def _has_distributed_sampler(loader) -> bool:
    from torch.utils.data.distributed import DistributedSampler
    for attr in ("sampler", "batch_sampler"):
        s = getattr(loader, attr, None)
        if isinstance(s, DistributedSampler) or isinstance(getattr(s, "sampler", None),
                                                           DistributedSampler):
            return True
    return False


def _batch_fingerprint(t: torch.Tensor) -> torch.Tensor:
    """Per-row float64 fingerprint of a batch, shape (rows, 2): each row's sum and its dot
    product with fixed non-constant weights.  Compared row by row across ranks, so rows in
    a different order -- which shard_batch would split into different, overlapping shards
    -- and rows with equal sums but different content both disagree (one
    position-weighted scalar let swapped rows of near-equal sums through)."""
    r = t.detach().double().reshape(t.shape[0] if t.dim() else 1, -1)
    m = r.shape[1]
    w = torch.sin(torch.arange(1, m + 1, dtype=torch.float64, device=r.device) * 0.7548776662466927) + 1.5
    return torch.stack([r.sum(1), r @ w], 1).reshape(-1)


def check_same_batch(*tensors: torch.Tensor):
    """Raise unless every rank holds the same global batch (inputs and targets): the
    per-row fingerprints of every tensor, all-reduced as MAX of (v, -v), must agree
    element by element (after one tiny all-reduce that checks the sizes agree).  Without a
    DistributedSampler the ranks must draw identical batches (same shuffle seed and
    augmentation RNG); a per-rank seed would otherwise train silently on overlapping
    shards.  Two tiny collectives per call."""
    _, ws = world()
    if ws <= 1:
        return
    dev = torch.device("cuda", torch.cuda.current_device()) \
        if dist.get_backend() == "nccl" else torch.device("cpu")
    fp = torch.cat([_batch_fingerprint(t).to(dev) for t in tensors])
    n = torch.tensor([fp.numel(), -fp.numel()], dtype=torch.float64, device=dev)
    dist.all_reduce(n, op=dist.ReduceOp.MAX)
    if int(n[0]) != -int(n[1]):
        raise RuntimeError(
            f"ugpg data parallel: ranks drew batches of different sizes ({-int(n[1])} .. "
            f"{int(n[0])} fingerprint values)")
    v = torch.cat([fp, -fp])
    dist.all_reduce(v, op=dist.ReduceOp.MAX)
    hi, lo = v[:fp.numel()], -v[fp.numel():]
    bad = (hi - lo) > 1e-9 * hi.abs().clamp_min(1.0)
    if bool(bad.any()):
        i = int(bad.nonzero()[0])
        raise RuntimeError(
            "ugpg data parallel: ranks drew different global batches (fingerprint value "
            f"{i}: {float(lo[i])!r} .. {float(hi[i])!r}); seed the DataLoader / augmentation "
            "identically on every rank or use a DistributedSampler")


def shard_batch(loader, *tensors, check=False):
    """This rank's contiguous equal shard of a global batch drawn from `loader`.

    With a DistributedSampler the loader already yields per-rank batches, so they pass
    through.  Otherwise every rank draws the same global batch (same seed) and keeps
    rows [r*b, (r+1)*b), b = len // world_size; a remainder that does not divide is
    dropped (DistributedSampler(drop_last=True) semantics), and a batch smaller than
    the world size yields None on every rank (skipped consistently).  check=True (the
    trainers pass it for the first batch of each epoch) verifies that every rank drew
    the same global batch (check_same_batch)."""
    rank, ws = world()
    if ws <= 1 or _has_distributed_sampler(loader):
        return tensors
    if check:
        check_same_batch(*tensors)
    n = tensors[0].shape[0]
    per = n // ws
    if per == 0:
        return None
    return tuple(t[rank * per:(rank + 1) * per] for t in tensors)


def max_over_ranks(value: float, device=None) -> float:
    _, ws = world()
    if ws <= 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
