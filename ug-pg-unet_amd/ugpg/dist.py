"""Data parallelism: one process per GPU, minibatch sharded across ranks, one
RCCL all-reduce of the flat gradient buffer per step.

BatchNorm stays local to each rank (each rank's forward equals the reference's
bs-16 forward on its shard); gradients are summed and the 1/world_size average
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


def shard(batch: torch.Tensor, rank: int, world_size: int) -> torch.Tensor:
    """Contiguous equal shard of the global batch for `rank`."""
    n = batch.shape[0]
    if n % world_size:
        raise ValueError(f"global batch {n} is not divisible by world size {world_size}")
    per = n // world_size
    return batch[rank * per:(rank + 1) * per]


def allreduce_gradients(params, bucket_bytes: int = 64 << 20):
    """Sum gradients over ranks.  One call when the grads form a single flat run
    (the normal ugpg layout), otherwise per-tensor calls.  Returns the scale
    (1/world_size) the optimizer must apply."""
    _, ws = world()
    grads = [p.grad for p in params if p.grad is not None]
    if ws <= 1 or not grads:
        return 1.0
    run = contiguous_run(grads)
    if run is not None:
        base, _, n = run
        step = max(1, bucket_bytes // 4)
        for off in range(0, n, step):
            dist.all_reduce(base[off:off + step])
    else:
        for g in grads:
            dist.all_reduce(g)
    return 1.0 / ws


def broadcast_parameters(module: torch.nn.Module, src: int = 0):
    """Make every replica start from rank `src`'s parameters and buffers."""
    _, ws = world()
    if ws <= 1:
        return
    for t in list(module.parameters()) + list(module.buffers()):
        dist.broadcast(t.data, src)


def max_over_ranks(value: float, device=None) -> float:
    _, ws = world()
    if ws <= 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
