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


def test_dp_two_ranks_match_shard_mean(tmp_path):
    from oracle.make_goldens import G8 as c
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u", os.path.join(ROOT, "tests", "_dp_worker.py"),
                               str(tmp_path)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              cwd=ROOT)
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=300) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
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
