"""Data-parallel path on CPU with the gloo backend, world_size 2.

Each rank computes the oracle's local-BatchNorm gradients on its contiguous
shard, places them in ugpg's flat gradient layout and calls
ugpg.dist.allreduce_gradients (the exact function the trainer and bench.py use
with RCCL).  The result must equal the mean of the per-shard gradients computed
in one process, on every rank, for both the flat (single all-reduce) and the
per-tensor fallback layout."""
import os
import socket
import tempfile

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn

WORLD = 2
B_PER = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _shards(world=WORLD):
    from oracle import detgen as G
    x = G.randn(1, (B_PER * world, 3, 32, 32), "x")
    t = G.bernoulli(2, (B_PER * world, 1, 32, 32), 0.5, "t")
    return x, t


def _grads_for(rank, world=WORLD):
    from tests._parity import det_state, oracle_run, param_keys
    from ugpg.dist import shard
    torch.set_num_threads(1 if world > 2 else 2)
    state = det_state(1, 3, 1)
    x, t = _shards(world)
    _, _, _, g, _ = oracle_run(1, state, shard(x, rank, world), shard(t, rank, world))
    return [g[k] for k in param_keys(state)]


def _worker(rank, port, outdir, flat, bf16=False, world=WORLD):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ug-pg-unet_amd")]
    os.environ["UGPG_GRAD_BF16"] = "1" if bf16 else "0"
    ws = world
    import torch.distributed as dist
    from ugpg.dist import allreduce_gradients, world
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    assert world() == (rank, ws)
    grads = _grads_for(rank, ws)
    params = [nn.Parameter(torch.zeros_like(g)) for g in grads]
    if flat:
        buf = torch.cat([g.reshape(-1) for g in grads])
        off = 0
        for p, g in zip(params, grads):
            p.grad = buf[off:off + g.numel()].view_as(g)
            off += g.numel()
    else:
        for p, g in zip(params, grads):
            p.grad = g.clone()
    scale = allreduce_gradients(params, bucket_bytes=1 << 20)
    out = [p.grad * scale for p in params]
    torch.save(out, os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


def _run(flat, bf16=False):
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d, flat, bf16), nprocs=WORLD, join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(WORLD)]
    per = [_grads_for(r) for r in range(WORLD)]
    if bf16:  # each rank's bucket rounded to bf16, summed in bf16, cast back
        bq = lambda t: t.to(torch.bfloat16)
        mean = [(bq(a) + bq(b)).float() / WORLD for a, b in zip(*per)]
    else:
        mean = [(a + b) / WORLD for a, b in zip(*per)]
    for r in range(WORLD):
        for got, want in zip(res[r], mean):
            assert torch.allclose(got, want, rtol=1e-6, atol=1e-9)
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b), "replicas diverged"


def test_dp_allreduce_flat_buffer():
    _run(flat=True)


def test_dp_allreduce_per_tensor_fallback():
    _run(flat=False)


def test_dp_allreduce_bf16_exchange():
    """The opt-in bf16 exchange (UGPG_GRAD_BF16=1): gradient buckets rounded to bf16,
    summed in bf16, cast back into the fp32 buffer."""
    _run(flat=True, bf16=True)


U_BF16 = 2.0 ** -8     # unit roundoff of bf16 (8-bit significand): RNE error <= u*|x|


@pytest.mark.parametrize("ws", [4, 8])
def test_bf16_exchange_error_bound(ws):
    """the bf16 exchange beyond 2 ranks.  Every rank casts its bucket
    to bf16 (one rounding), the collective sums in bf16 (N-1 rounded partial sums along
    the ring or tree), the result is cast back exactly.  To first order, for any summation
    order, the error of the mean is bounded elementwise by
        |mean_bf16 - mean_fp32| <= u * sum_r |g_r|        (u = 2^-8)
    since the N-1 partial sums are each at most sum_r |g_r| in magnitude.  Checked here on
    real per-shard gradients (the oracle's local-BN Stage-1 gradients on ws shards) through
    ugpg.dist.allreduce_gradients over gloo at world size 4 and 8.

    The bound is relative to the gradient's own size (0.4 % at N = 1 from the cast alone,
    and realised errors of 0.1-1 % of max|g| per tensor here), while the bf16 oracle's own
    per-tensor spread (G4c, the config-3 parity floor) is 4e-5..7e-4 of max|g| for the
    output heads.  So the bf16 exchange is NOT inside the parity floor at any N > 1, and
    the default exchange is fp32 (as torch's DDP under autocast exchanges the fp32
    .grad): see test_grad_exchange_default_is_fp32 and DESIGN §6."""
    import numpy as np
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(_free_port(), d, True, True, ws), nprocs=ws, join=True)
        res = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(ws)]
    per = [_grads_for(r, ws) for r in range(ws)]
    fc = np.load(os.path.join(os.path.dirname(__file__), "golden", "g4c_bf16_floor.npz"))
    head_floor = max(fc[k][0] / fc[k][1] for k in fc.files
                     if k.startswith("floor16/outc"))
    worst = 0.0
    for i, got in enumerate(res[0]):
        gs = torch.stack([p[i].double() for p in per])
        want = gs.mean(0)
        bound = U_BF16 * gs.abs().sum(0) * (1 + 1e-3) + 1e-30
        err = (got.double() - want).abs()
        assert bool((err <= bound).all()), (i, (err / bound).max().item())
        worst = max(worst, (err.max() / want.abs().max().clamp_min(1e-30)).item())
    for r in range(1, ws):
        for a, b in zip(res[0], res[r]):
            assert torch.equal(a, b), "replicas diverged"
    print(f"bf16 exchange ws={ws}: worst per-tensor error {worst:.2e} of max|mean g| "
          f"(G4c head floor {head_floor:.1e} of max|g|)")
    assert worst > head_floor  # the reason the default exchange is fp32


def test_grad_exchange_default_is_fp32(monkeypatch):
    """With the bf16 conv arithmetic the default gradient exchange stays fp32 (the bf16
    exchange error exceeds the config-3 parity floor, test_bf16_exchange_error_bound);
    UGPG_GRAD_BF16=1 opts in."""
    from ugpg import dist as D, ops
    monkeypatch.delenv("UGPG_GRAD_BF16", raising=False)
    old = ops.conv_math()
    try:
        ops.set_conv_math("bf16")
        assert D.grad_bf16() is False
        monkeypatch.setenv("UGPG_GRAD_BF16", "1")
        assert D.grad_bf16() is True
    finally:
        ops.set_conv_math(old)


def _reducer_worker(rank, port, outdir):
    """Feed OverlapReducer the way the ugpg backward does: per-parameter views of one
    flat buffer, completed block by block from the end of the layout to the start."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ug-pg-unet_amd")]
    import torch.distributed as dist
    from ugpg.dist import OverlapReducer, allreduce_gradients, overlapped_allreduce, overlap_reducer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    sizes = [7, 300, 1, 4096, 33, 5000, 12, 900, 2]      # uneven parameter sizes
    gen = torch.Generator().manual_seed(10 + rank)
    flat = torch.randn(sum(sizes), generator=gen)
    want = flat.clone()
    dist.all_reduce(want)
    views, off = [], 0
    for n in sizes:
        views.append(flat[off:off + n])
        off += n
    assert overlap_reducer() is None                     # opt-in only
    with overlapped_allreduce():
        red = overlap_reducer()
        assert isinstance(red, OverlapReducer)
        red.bucket = 1000                                # force several buckets
        red.begin(flat, views)
        blocks = [[8, 7], [6], [5, 4, 3], [2, 1], [0]]   # backward order: last params first
        issued = []
        for blk in blocks:
            red.done([views[i] for i in blk])
            issued.append(red.hi)
        red.flush()
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes]
    for p, v in zip(params, views):
        p.grad = v
    scale = allreduce_gradients(params)
    assert scale == 1.0 / WORLD
    # buckets went out during the "backward" (not only at flush), highest offsets first
    assert issued == sorted(issued, reverse=True) and issued[-1] < sum(sizes), issued
    torch.save((flat, want), os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_overlap_reducer_buckets_sum_like_one_allreduce():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_reducer_worker, args=(_free_port(), d), nprocs=WORLD, join=True)
        for r in range(WORLD):
            got, want = torch.load(os.path.join(d, f"r{r}.pt"), weights_only=True)
            assert torch.allclose(got, want, rtol=1e-6, atol=1e-6)


def _replica_worker(rank, port, outdir):
    """Trainer constructors under torch.distributed: every rank seeds differently (as
    unseeded torchrun ranks would) and must still end with rank 0's weights."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ug-pg-unet_amd")]
    import torch.distributed as dist
    from torch.utils.data import DataLoader, TensorDataset
    from torch.utils.data.distributed import DistributedSampler
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.set_num_threads(2)
    torch.manual_seed(100 + rank)
    import ugpg
    from ugpg.dist import shard_batch
    from ugpg.herlev import HerlevTrainer
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device="cpu")
    ht = HerlevTrainer({"device": "cpu", "epochs_per_stage": 1, "num_classes": 7})
    sums = {f"seg{s}": [float(p.double().sum()) for p in m.state_dict().values()
                        if p.is_floating_point()] for s, m in tr.models.items()}
    sums.update({f"herlev{s}": [float(p.double().sum()) for p in m.state_dict().values()
                                if p.is_floating_point()] for s, m in ht.models.items()})
    # batch sharding: contiguous equal shards, remainder dropped, tiny batch skipped,
    # DistributedSampler batches pass through
    ds = TensorDataset(torch.arange(5).float().view(5, 1), torch.arange(5).view(5, 1))
    plain = DataLoader(ds, batch_size=5)
    (x, y), = list(plain)
    part = shard_batch(plain, x, y)
    tiny = shard_batch(plain, x[:1], y[:1])
    samp = DataLoader(ds, batch_size=2, sampler=DistributedSampler(ds, WORLD, rank, shuffle=False))
    (xs, ys), *_ = list(samp)
    through = shard_batch(samp, xs, ys)
    checked = shard_batch(plain, x, y, check=True)  # same global batch: passes
    try:  # per-rank data (e.g. a per-rank seed without a DistributedSampler): refused
        shard_batch(plain, x + rank, y, check=True)
        mismatch = None
    except RuntimeError as e:
        mismatch = str(e)
    refused = []
    # the same rows in a different order on rank 1 (the shards would overlap), and the same
    # inputs with different targets: both refused
    perm = torch.tensor([1, 0, 2, 3, 4]) if rank == 1 else torch.arange(5)
    # rows of equal sums swapped on rank 1 (a position-weighted sum of row sums
    # cannot see it), e.g. binary masks with the same foreground count
    z = torch.tensor([[1., 0., 0.], [0., 1., 0.], [0., 0., 1.], [1., 1., 0.]])
    zp = z[torch.tensor([1, 0, 2, 3])] if rank == 1 else z
    for xa, ya in ((x[perm], y[perm]), (x, y + rank), (zp, zp)):
        try:
            shard_batch(plain, xa, ya, check=True)
            refused.append(False)
        except RuntimeError:
            refused.append(True)
    torch.save({"sums": sums, "part": part[0].view(-1).tolist(), "tiny": tiny,
                "through": torch.equal(through[0], xs), "checked": checked[0].view(-1).tolist(),
                "mismatch": mismatch, "refused": refused}, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_trainers_start_from_rank0_weights_and_shard_batches():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_replica_worker, args=(_free_port(), d), nprocs=WORLD, join=True)
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(WORLD)]
    assert r[0]["sums"] == r[1]["sums"]
    assert r[0]["part"] == [0.0, 1.0] and r[1]["part"] == [2.0, 3.0]
    assert r[0]["tiny"] is None and r[1]["tiny"] is None
    assert r[0]["through"] and r[1]["through"]
    assert r[0]["checked"] == [0.0, 1.0] and r[1]["checked"] == [2.0, 3.0]
    assert all("different global batches" in (x["mismatch"] or "") for x in r)
    assert all(x["refused"] == [True, True, True] for x in r), [x["refused"] for x in r]


def _mixed_worker(rank, port, outdir):
    """allreduce_gradients over a Herlev-like layout: one flat run (the encoder) handed to
    the OverlapReducer during the backward, plus loose tensors (the head) reduced after."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ug-pg-unet_amd")]
    import torch.distributed as dist
    from ugpg.dist import allreduce_gradients, overlapped_allreduce, overlap_reducer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    gen = torch.Generator().manual_seed(20 + rank)
    sizes = [300, 5000, 33, 7]
    flat = torch.randn(sum(sizes), generator=gen)
    loose = [torch.randn(n, generator=gen) for n in (512, 256, 7)]
    want = [t.clone() for t in [flat] + loose]
    for t in want:
        dist.all_reduce(t)
    views, off = [], 0
    for n in sizes:
        views.append(flat[off:off + n])
        off += n
    params = [torch.nn.Parameter(torch.zeros(n)) for n in sizes + [512, 256, 7]]
    for p, g in zip(params, views + loose):
        p.grad = g
    with overlapped_allreduce():
        red = overlap_reducer()
        red.bucket = 1000
        red.begin(flat, views)
        red.done(views[::-1])
        red.flush()
    assert allreduce_gradients(params, bucket_bytes=4096) == 1.0 / WORLD
    torch.save(([flat] + loose, want), os.path.join(outdir, f"m{rank}.pt"))
    dist.destroy_process_group()


def test_allreduce_flat_run_plus_loose_tensors():
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_mixed_worker, args=(_free_port(), d), nprocs=WORLD, join=True)
        for r in range(WORLD):
            got, want = torch.load(os.path.join(d, f"m{r}.pt"), weights_only=True)
            for a, b in zip(got, want):
                assert torch.allclose(a, b, rtol=1e-6, atol=1e-6)


def _syncbn_worker(rank, port, outdir):
    """One rank of the synchronised-BatchNorm step: the oracle's Stage-1 train step on this
    rank's bs2 shard with every BatchNorm synchronised through ugpg.dist's exchange (the
    object ops._BN_SYNC holds when enable_sync_batchnorm is on), then the trainer's gradient
    all-reduce (mean)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ug-pg-unet_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    torch.set_num_threads(2)
    from oracle import ref_cpu as O
    from tests._parity import det_state, oracle_run, param_keys
    from ugpg import ops
    from ugpg.dist import allreduce_gradients, enable_sync_batchnorm, shard
    enable_sync_batchnorm(True)
    O.BN_SYNC = ops._BN_SYNC
    assert (O.BN_SYNC.rank, O.BN_SYNC.nranks) == (rank, WORLD)
    state = det_state(1, 3, 1)
    x, t = _shards()
    logits, final, _, g, P = oracle_run(1, state, shard(x, rank, WORLD), shard(t, rank, WORLD))
    keys = param_keys(state)
    params = [nn.Parameter(torch.zeros_like(g[k])) for k in keys]
    for p, k in zip(params, keys):
        p.grad = g[k].clone()
    scale = allreduce_gradients(params, bucket_bytes=1 << 20)
    bufs = {k: v for k, v in P.items() if k.endswith(("running_mean", "running_var"))}
    torch.save({"logits": logits, "grads": {k: p.grad * scale for k, p in zip(keys, params)},
                "bufs": bufs}, os.path.join(outdir, f"r{rank}.pt"))
    enable_sync_batchnorm(False)
    dist.destroy_process_group()


def test_sync_batchnorm_step_equals_global_batch():
    """SURVEY §8e's optional SyncBN: two gloo ranks on bs2 shards with
    synchronised BatchNorm reproduce the single-process bs4 step of the reference (the
    oracle, bit-identical to it): logits per shard, every averaged gradient within the §8d
    rule (3x the reference's own fp32 noise floor + 1e-6 of scale), BN running statistics
    1e-5 -- the exchange under test is ugpg.dist's own (_SyncBN.all_reduce)."""
    from tests._parity import det_state, grad_check, noise_floor, oracle_run, param_keys
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_syncbn_worker, args=(_free_port(), d), nprocs=WORLD, join=True)
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(WORLD)]
    state = det_state(1, 3, 1)
    x, t = _shards()
    logits32, _, _, g32, P32 = oracle_run(1, state, x, t)
    _, _, _, g64, _ = oracle_run(1, state, x, t, dtype=torch.float64)
    floor = noise_floor(1, state, x, t, g32, g64)
    lg = torch.cat([r[0]["logits"], r[1]["logits"]])
    assert (lg - logits32).abs().max().item() <= 1e-4
    bad = []
    for k in param_keys(state):
        assert torch.equal(r[0]["grads"][k], r[1]["grads"][k]), "replicas diverged"
        ok, err, bound = grad_check(k, r[0]["grads"][k], g32[k], g64[k], floor[k])
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    assert not bad, "synced gradients differ from the global-batch step:\n" + "\n".join(bad)
    for k, v in r[0]["bufs"].items():
        assert (v - P32[k]).abs().max().item() <= 1e-5 * max(1.0, P32[k].abs().max().item()), k
        assert torch.equal(v, r[1]["bufs"][k]), k
    # and local BatchNorm does NOT equal it (the test can tell the two policies apart)
    la, _, _, _, _ = oracle_run(1, state, x[:B_PER], t[:B_PER])
    assert (la - logits32[:B_PER]).abs().max().item() > 1e-3


def test_sync_batchnorm_native_exchange_has_its_own_communicator(monkeypatch):
    """VERDICT r5 weak #5 / ADVICE r5: under UGPG_COMM=native the synchronised-BatchNorm
    exchange runs on a libugpg Communicator of its own, never on the process-wide one that
    carries the overlapped gradient buckets (one RCCL communicator serialises its
    operations); on the torch path it uses its own process group.  Routing only (no GPU):
    the communicator and the collectives are stand-ins that record their calls."""
    from ugpg import dist as D
    made = []

    class FakeComm:
        def __init__(self):
            self.calls = []
            made.append(self)

        def all_reduce(self, t):
            self.calls.append(t)
            return t

    class CudaLike:  # the exchange picks the native path for device tensors only
        is_cuda = True

    monkeypatch.setattr(D, "Communicator", FakeComm)
    monkeypatch.setattr(D, "world", lambda: (1, 2))
    monkeypatch.setattr(D, "_COMM", None)
    monkeypatch.setattr(D.dist, "new_group", lambda ranks: ("bn-group", tuple(ranks)))
    monkeypatch.setenv("UGPG_COMM", "native")
    sb = D._SyncBN()
    buckets = D.native_comm()  # the gradient buckets' communicator
    t = CudaLike()
    sb.all_reduce(t)
    sb.all_reduce(t)
    assert len(made) == 2 and sb._comm is not None and sb._comm is not buckets
    assert sb._comm.calls == [t, t] and buckets.calls == []
    assert sb.native() is sb._comm  # built once
    # torch path: its own process group, never the default one
    monkeypatch.setenv("UGPG_COMM", "torch")
    seen = []
    monkeypatch.setattr(D.dist, "all_reduce", lambda x, group=None, **kw: seen.append(group))
    sb2 = D._SyncBN()
    sb2.all_reduce(t)
    assert seen == [("bn-group", (0, 1))] and sb2._comm is None
    assert len(made) == 2


WS8 = 8


def _batch8():
    from oracle import detgen as G
    return G.randn(1, (WS8, 3, 32, 32), "x"), G.bernoulli(2, (WS8, 1, 32, 32), 0.5, "t")


def _ws8_worker(rank, port, outdir):
    """One of eight gloo ranks: PGUNet1 at bs8 x 32^2, one image per
    rank.  (1) local BatchNorm: this shard's oracle gradients through allreduce_gradients;
    (2) synchronised BatchNorm through ugpg.dist's exchange (the 8-row rank-order merge);
    (3) the OverlapReducer fed block by block at eight ranks."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "ug-pg-unet_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WS8)
    torch.set_num_threads(1)
    from oracle import ref_cpu as O
    from tests._parity import det_state, oracle_run, param_keys
    from ugpg import ops
    from ugpg.dist import (OverlapReducer, allreduce_gradients, enable_sync_batchnorm,
                           overlap_reducer, overlapped_allreduce, shard)
    state = det_state(1, 3, 1)
    keys = param_keys(state)
    x, t = _batch8()
    xs, ts = shard(x, rank, WS8), shard(t, rank, WS8)
    out = {}

    def averaged(g):
        params = [nn.Parameter(torch.zeros_like(g[k])) for k in keys]
        buf = torch.cat([g[k].reshape(-1) for k in keys])  # the flat layout
        off = 0
        for p, k in zip(params, keys):
            p.grad = buf[off:off + g[k].numel()].view_as(g[k])
            off += g[k].numel()
        scale = allreduce_gradients(params, bucket_bytes=1 << 16)
        return {k: p.grad * scale for k, p in zip(keys, params)}

    _, _, _, g, _ = oracle_run(1, state, xs, ts)
    out["local"] = averaged(g)
    enable_sync_batchnorm(True)
    O.BN_SYNC = ops._BN_SYNC
    assert (O.BN_SYNC.rank, O.BN_SYNC.nranks) == (rank, WS8)
    logits, _, _, g, P = oracle_run(1, state, xs, ts)
    out["sync"] = averaged(g)
    out["logits"] = logits
    out["bufs"] = {k: v for k, v in P.items() if k.endswith(("running_mean", "running_var"))}
    O.BN_SYNC = None
    enable_sync_batchnorm(False)
    # the reducer: uneven sizes, several buckets, completed back to front
    sizes = [7, 300, 1, 4096, 33, 5000, 12, 900, 2]
    flat = torch.randn(sum(sizes), generator=torch.Generator().manual_seed(30 + rank))
    want = flat.clone()
    dist.all_reduce(want)
    views, off = [], 0
    for n in sizes:
        views.append(flat[off:off + n])
        off += n
    with overlapped_allreduce():
        red = overlap_reducer()
        assert isinstance(red, OverlapReducer)
        red.bucket = 700
        red.begin(flat, views)
        for blk in ([8, 7], [6], [5, 4, 3], [2, 1], [0]):
            red.done([views[i] for i in blk])
        red.flush()
    params = [nn.Parameter(torch.zeros(n)) for n in sizes]
    for p, v in zip(params, views):
        p.grad = v
    assert allreduce_gradients(params) == 1.0 / WS8
    out["reducer"] = (flat, want)
    torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    dist.destroy_process_group()


def test_data_parallel_world_size_8():
    """data parallelism above world size 2, on CPU (gloo, 8 ranks, one
    bs1 shard each of a bs8 PGUNet1 batch at 32^2):
    * local BatchNorm: the averaged gradient equals the mean of the 8 per-shard gradients
      computed in one process (G8's semantics at N = 8), identical on every rank;
    * synchronised BatchNorm: the averaged step equals the reference's single-process bs8
      step (the oracle, bit-identical to it): logits 1e-4, every gradient by the §8d rule
      with the perturbation-aware floor, BN running statistics 1e-5 -- so the 8-row
      rank-order merge and the backward sums are exact at 8 ranks;
    * the OverlapReducer at 8 ranks sums like one all-reduce."""
    from tests._parity import det_state, grad_check, noise_floor, oracle_run, param_keys
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_ws8_worker, args=(_free_port(), d), nprocs=WS8, join=True)
        r = [torch.load(os.path.join(d, f"r{i}.pt"), weights_only=True) for i in range(WS8)]
    nt = torch.get_num_threads()
    state = det_state(1, 3, 1)
    keys = param_keys(state)
    x, t = _batch8()
    # (1) local BatchNorm = mean of per-shard gradients (one thread, as the ranks: the
    # pre-BN conv biases' gradients are pure rounding noise, which the thread count moves)
    torch.set_num_threads(1)
    try:
        per = [oracle_run(1, state, x[i:i + 1], t[i:i + 1])[3] for i in range(WS8)]
    finally:
        torch.set_num_threads(nt)
    for k in keys:
        mean = torch.stack([p[k].double() for p in per]).mean(0)
        scale = max(p[k].abs().max().item() for p in per)
        got = r[0]["local"][k].double()
        assert torch.allclose(got, mean, rtol=1e-6, atol=1e-6 * scale + 1e-12), k
        for i in range(1, WS8):
            assert torch.equal(r[i]["local"][k], r[0]["local"][k]), ("replicas diverged", k)
    # (2) synchronised BatchNorm = the global bs8 step
    logits32, _, _, g32, P32 = oracle_run(1, state, x, t)
    _, _, _, g64, _ = oracle_run(1, state, x, t, dtype=torch.float64)
    floor = noise_floor(1, state, x, t, g32, g64)
    lg = torch.cat([ri["logits"] for ri in r])
    assert (lg - logits32).abs().max().item() <= 1e-4
    bad = []
    for k in keys:
        for i in range(1, WS8):
            assert torch.equal(r[i]["sync"][k], r[0]["sync"][k]), ("replicas diverged", k)
        ok, err, bound = grad_check(k, r[0]["sync"][k], g32[k], g64[k], floor[k])
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    assert not bad, "synced gradients differ from the bs8 step:\n" + "\n".join(bad)
    for k, v in r[0]["bufs"].items():
        assert (v - P32[k]).abs().max().item() <= 1e-5 * max(1.0, P32[k].abs().max().item()), k
        for i in range(1, WS8):
            assert torch.equal(v, r[i]["bufs"][k]), k
    # ... which local BatchNorm is not
    assert (r[0]["logits"] - logits32[:1]).abs().max().item() <= 1e-4
    la = oracle_run(1, state, x[:1], t[:1])[0]
    assert (la - logits32[:1]).abs().max().item() > 1e-3
    # (3) the reducer
    for i in range(WS8):
        got, want = r[i]["reducer"]
        assert torch.allclose(got, want, rtol=1e-5, atol=1e-5)
