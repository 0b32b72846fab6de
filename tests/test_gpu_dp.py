"""Data-parallel training on the HIP path (golden G8): two ranks (fresh child
processes, gloo, both on cuda:0) run ugpg's trainer on the two halves of a bs4 Stage-2
UG batch.  Checked: replicas identical after construction / weight loading / one step;
the all-reduced gradient equals the mean of the per-shard local-BatchNorm gradients of
the reference (G8 checksums) and of the oracle (full tensors, §8d rule); the post-step
parameters; and the epoch tuple is the global-batch one on every rank."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import detgen as G
from oracle import ref_cpu as O
from tests._parity import (FLOOR_PERTURBATIONS, det_state, grad_check, is_prebn_bias,
                           oracle_run, param_keys, perturbed_state)

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_avg(c, dtype, state=None):
    state = det_state(c["stage"], 3, 1, seed=c["w_seed"]) if state is None else state
    prev = det_state(c["stage"] - 1, 3, 1, seed=c["prev_seed"])
    x = G.randn(c["x_seed"], (c["B"], 3, c["res"], c["res"]), "x")
    t = G.bernoulli(c["t_seed"], (c["B"], 1, c["res"], c["res"]), 0.5, "t")
    per = c["B"] // c["shards"]
    acc = None
    for r in range(c["shards"]):
        xs, ts = x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]
        u = O.uncertainty_map(1, prev, xs, 32, 64)
        _, _, _, g, _ = oracle_run(c["stage"], state, xs, ts, umap=u, dtype=dtype)
        acc = g if acc is None else {k: acc[k] + g[k] for k in g}
    return {k: v / c["shards"] for k, v in acc.items()}


def _run_ranks(tmp_path, *args):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_dp_worker.py"),
                               str(tmp_path), *args], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              cwd=ROOT)
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=300) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    return [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]


def test_dp_two_ranks_match_shard_mean(tmp_path):
    from oracle.make_goldens import G8 as c
    res = _run_ranks(tmp_path)
    # replicas: constructor broadcast, load_stage_weights broadcast, identical step
    for k, v in res[0]["ctor_s3_after"].items():
        assert torch.equal(v, res[1]["ctor_s3_after"][k]), k
    for k, v in res[0]["ctor_s3"].items():     # right after the constructor already
        assert torch.equal(v, res[1]["ctor_s3"][k]), k
    for k, v in res[0]["state"].items():
        if not O._is_buffer(k):
            assert torch.equal(v, res[1]["state"][k]), f"replicas diverged: {k}"
    for k, v in res[0]["grads"].items():
        assert torch.equal(v, res[1]["grads"][k]), f"all-reduced gradient differs: {k}"
    assert res[0]["tuple"] == res[1]["tuple"]
    fx = np.load("tests/golden/g8_dp_shards.npz")
    tup, want = np.array(res[0]["tuple"]), fx["epoch_tuple"]
    assert abs(tup[0] - want[0]) <= 1e-5 * abs(want[0]) and abs(tup[1] - want[1]) <= 1e-5 * abs(want[1])
    assert abs(tup[2] - want[2]) <= 1e-3 and abs(tup[3] - want[3]) <= 1e-3
    assert abs(tup[4] - want[4]) <= 1e-5 and abs(tup[5] - want[5]) <= 1e-5, (tup, want)
    # gradient = sum over ranks (the 1/N is folded into RMSprop) -> mean
    state = det_state(c["stage"], 3, 1, seed=c["w_seed"])
    g32, g64 = _oracle_avg(c, torch.float32), _oracle_avg(c, torch.float64)
    floor = {k: (g32[k].double() - g64[k]).abs().max().item() for k in g32}
    for s, rel in FLOOR_PERTURBATIONS[:4]:
        gp = _oracle_avg(c, torch.float32, perturbed_state(state, s, rel))
        for k in floor:
            floor[k] = max(floor[k], (gp[k].double() - g64[k]).abs().max().item())
    bad, worst = [], []
    for k in param_keys(state):
        ok, err, bound = grad_check(k, res[0]["grads"][k] / 2, g32[k], g64[k], floor[k])
        worst.append((err / bound, k))
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
        gs = fx[f"avg_grad/{k}"]
        mine = (res[0]["grads"][k] / 2).double()
        assert abs(mine.norm().item() - gs[0]) <= 1e-3 * gs[0] + 1e-6, k
    print("DP gradient headroom (err/bound), worst 5:", sorted(worst, reverse=True)[:5])
    assert not bad, "\n".join(bad[:20])
    # one RMSprop step on the averaged gradient: parameter checksums
    # (RMSprop's first update is ~10 lr * sign(g): noise-level sign flips move an element
    # by 2e-3, hence the 1e-4 relative norm tolerance; the rule itself is exact elsewhere)
    for k in param_keys(state):
        if is_prebn_bias(k):
            continue  # noise-level gradient (true value 0): its RMSprop signs are arbitrary
        p = res[0]["state"][k].double()
        assert abs(p.norm().item() - fx[f"post/{k}"][0]) <= 1e-4 * fx[f"post/{k}"][0] + 1e-6, k


@pytest.mark.parametrize("exchange", ["fp32", "bf16"])
def test_dp_two_ranks_bf16_exchange(tmp_path, exchange):
    """Config 3's data parallelism on the HIP path: bf16 conv arithmetic in two fresh
    processes (gloo, both on cuda:0) on the halves of the G8 batch, with the default fp32
    gradient exchange (the exchanged gradient must equal g_0 + g_1 in fp32) and the opt-in
    bf16 exchange (dist._Bf16Work: RNE cast kernels around the all-reduce, summed back into
    the fp32 flat buffer; it must equal bf16(bf16(g_0) + bf16(g_1)) bit for bit), on both
    ranks; each rank's own gradient must be the bf16 oracle's for its shard within the
    bf16 floor rule (the oracle's spread under ulp-level weight perturbations, x3)."""
    from oracle.make_goldens import G8 as c
    from tests._parity import FLOOR_PERTURBATIONS
    res = _run_ranks(tmp_path, "bf16", exchange)
    for k, v in res[0]["grads"].items():
        assert torch.equal(v, res[1]["grads"][k]), f"exchanged gradient differs across ranks: {k}"
    for k, v in res[0]["grads"].items():
        if exchange == "bf16":
            q = lambda t: t.to(torch.bfloat16)
            want = (q(res[0]["local"][k]).float() + q(res[1]["local"][k]).float()).to(torch.bfloat16)
        else:
            want = res[0]["local"][k] + res[1]["local"][k]
        assert torch.equal(v, want.float()), f"{exchange} exchange of {k}"
    # each rank's own gradient vs the bf16 oracle on its shard
    state = det_state(c["stage"], 3, 1, seed=c["w_seed"])
    prev = det_state(c["stage"] - 1, 3, 1, seed=c["prev_seed"])
    x = G.randn(c["x_seed"], (c["B"], 3, c["res"], c["res"]), "x")
    t = G.bernoulli(c["t_seed"], (c["B"], 1, c["res"], c["res"]), 0.5, "t")
    per = c["B"] // 2
    O.CONV_MATH = "bf16"
    try:
        for r in range(2):
            xs, ts = x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]
            u = O.uncertainty_map(1, prev, xs, 32, 64)
            _, _, _, g16, _ = oracle_run(c["stage"], state, xs, ts, umap=u)
            floor = {k: 0.0 for k in g16}
            for sd, rel in FLOOR_PERTURBATIONS[:5]:
                _, _, _, gp, _ = oracle_run(c["stage"], perturbed_state(state, sd, rel), xs, ts,
                                            umap=u)
                for k in floor:
                    floor[k] = max(floor[k], (gp[k].double() - g16[k].double()).abs().max().item())
            bad = []
            for k in param_keys(state):
                err = (res[r]["local"][k].double() - g16[k].double()).abs().max().item()
                bound = 1e-5 if is_prebn_bias(k) else 3 * floor[k] + 1e-6 * g16[k].abs().max().item()
                if err > bound:
                    bad.append(f"rank {r} {k}: {err:.3e} > {bound:.3e}")
            assert not bad, "\n".join(bad[:20])
    finally:
        O.CONV_MATH = "f32"


@pytest.mark.parametrize("stage,B,res", [(1, 4, 32), (4, 4, 64)])
def test_sync_batchnorm_two_ranks_equal_global_batch(tmp_path, stage, B, res):
    """SURVEY §8e's optional SyncBN on the HIP path: two GPU ranks on
    bs B/2 shards with every BatchNorm synchronised (forward statistics gathered, backward
    sums all-reduced: ugpg_bn_stats_pack / ugpg_bn_finalize_merged / ugpg_bn_bwd_partials_*)
    reproduce the reference's single-process bs-B step: logits 1e-3, averaged gradients by
    the §8d rule against the oracle's own noise floor, BN running statistics 1e-5."""
    from tests._parity import noise_floor
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_syncbn_worker.py"),
                               str(tmp_path), str(stage), str(B), str(res)],
                              env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), cwd=ROOT)
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=300) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    res_ = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    state = det_state(stage, 3, 1)
    x = G.randn(1, (B, 3, res, res), "x")
    t = G.bernoulli(2, (B, 1, res, res), 0.5, "t")
    logits32, _, _, g32, P32 = oracle_run(stage, state, x, t)
    _, _, _, g64, _ = oracle_run(stage, state, x, t, dtype=torch.float64)
    floor = noise_floor(stage, state, x, t, g32, g64)
    lg = torch.cat([res_[0]["logits"], res_[1]["logits"]])
    assert (lg - logits32).abs().max().item() <= 1e-3
    bad = []
    for k in param_keys(state):
        assert torch.equal(res_[0]["grads"][k], res_[1]["grads"][k]), f"replicas diverged: {k}"
        ok, err, bound = grad_check(k, res_[0]["grads"][k], g32[k], g64[k], floor[k])
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    assert not bad, "synced gradients differ from the global-batch step:\n" + "\n".join(bad[:20])
    for k, v in res_[0]["bufs"].items():
        assert torch.equal(v, res_[1]["bufs"][k]), k
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(P32[k]), k
        else:
            assert (v - P32[k]).abs().max().item() <= 1e-5 * max(1.0, P32[k].abs().max().item()), k
