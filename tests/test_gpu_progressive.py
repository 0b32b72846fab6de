"""Config 5 -- the progressive 1->4 driver with uncertainty-map transfer
(UncertaintyGuidedProgressiveTrainer.train_progressive, uncertainty_guided_trainer.py:
316-398) -- on the HIP path, pinned to the reference itself.

With every stage lr = 0 only the weight transfers and the BatchNorm running statistics
evolve, so the reference's trajectory is deterministic: G12 records the history the
reference's own train_progressive produced (4 train + 2 val images of 256^2, bs2, two
epochs per stage), every stage model's BN buffers at the end and each best checkpoint.
G12b is the same driver under 2-rank data parallelism with local BatchNorm, built from
the reference's trainer methods (oracle/make_goldens.py:g12b).

Tolerances: losses 1e-5 relative, Dice +-1e-3, U statistics 1e-5,
BN running statistics 1e-5 (of max(1, |v|)), num_batches_tracked exact."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from oracle import ref_cpu as O
from tests._parity import det_state

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LOSS_KEYS = ("train_loss", "val_loss", "base_loss")
DICE_KEYS = ("train_dice", "val_dice")
U_KEYS = ("uncertainty_weights_mean", "uncertainty_weights_std")


def check_history(hist, fx):
    assert hist["stage_transitions"] == [int(v) for v in fx["history/stage_transitions"]]
    for k in LOSS_KEYS + DICE_KEYS + U_KEYS:
        mine, want = np.array(hist[k]), fx[f"history/{k}"]
        assert mine.shape == want.shape, k
        if k in LOSS_KEYS:
            tol = 1e-5 * np.abs(want)
        elif k in DICE_KEYS:
            tol = np.full_like(want, 1e-3)
        else:
            tol = np.full_like(want, 1e-5)
        err = np.abs(mine - want)
        assert (err <= tol).all(), (k, mine.tolist(), want.tolist())
        print(f"{k}: max |err| {err.max():.2e}")


def check_buffers(state, fx, stage, prefix="buf"):
    for k, v in state.items():
        if not O._is_buffer(k):
            continue
        want = fx[f"{prefix}{stage}/{k}"]
        if k.endswith("num_batches_tracked"):
            assert int(v) == int(want), (stage, k, int(v), int(want))
        else:
            w = torch.from_numpy(want)
            err = (v.detach().cpu() - w).abs().max().item()
            assert err <= 1e-5 * max(1.0, w.abs().max().item()), (stage, k, err)


def test_train_progressive_matches_reference(dev, tmp_path):
    from torch.utils.data import DataLoader, TensorDataset
    import ugpg
    from oracle.make_goldens import G12, g12_data
    fx = np.load("tests/golden/g12_progressive.npz")
    torch.manual_seed(0)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
    for s in range(1, 5):
        tr.models[s].load_state_dict(det_state(s, 3, 1, seed=G12["w_seeds"][s]))
        tr.stage_configs[s]["lr"] = 0.0
        tr.stage_configs[s]["epochs_per_stage"] = G12["epochs"]
    tr.setup_optimizer(1)
    x, t, vx, vt = g12_data()
    tl = DataLoader(TensorDataset(x, t), batch_size=G12["bs"], shuffle=False)
    vl = DataLoader(TensorDataset(vx, vt), batch_size=G12["bs"], shuffle=False)
    tr.train_progressive(tl, vl, max_stages=4, save_dir=str(tmp_path))
    check_history(tr.history, fx)
    for s in range(1, 5):
        sd = tr.models[s].state_dict()
        check_buffers(sd, fx, s)
        # parameters: what the transfers produced (lr 0 never moves them)
        for k, v in sd.items():
            if not O._is_buffer(k):
                want = float(fx[f"wsum{s}/{k}"])
                assert abs(v.double().sum().item() - want) <= 1e-9 * max(1.0, abs(want)), (s, k)
        # best checkpoints: the reference's decision (epoch) wherever the two epochs' val
        # Dice differ by more than the Dice tolerance, and its val/train Dice
        st, ep, vd, td = fx[f"ckpt/{s}"]
        ck = torch.load(tmp_path / f"ug_pgunet_stage{s}_best.pth", map_location="cpu",
                        weights_only=True)
        vds = fx["history/val_dice"][2 * (s - 1):2 * s]
        assert ck["stage"] == int(st)
        if abs(vds[1] - vds[0]) > 2e-3:
            assert ck["epoch"] == int(ep), (s, ck["epoch"], ep)
        assert abs(ck["val_dice"] - vd) <= 1e-3 and abs(ck["train_dice"] - td) <= 1e-3


def test_train_progressive_two_ranks(tmp_path):
    """The same driver in 2 fresh processes (gloo, both on cuda:0), one image of each bs2
    batch per rank: identical replicas after every stage, the BN-buffer broadcast taking
    effect (rank 1's buffers differ after its own train epoch, equal rank 0's after the
    broadcast), rank-0-only checkpoints, and rank 0's history and BN buffers equal the
    reference's 2-shard trajectory (G12b)."""
    from tests.test_gpu_dp import _free_port
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               WORLD_SIZE="2", HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, "-u",
                               os.path.join(ROOT, "tests", "_progressive_worker.py"),
                               str(tmp_path)], env=dict(env, RANK=str(r), LOCAL_RANK=str(r)),
                              cwd=ROOT)
             for r in range(2)]
    try:
        rcs = [p.wait(timeout=400) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], rcs
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(2)]
    assert res[0]["history"] == res[1]["history"], "ranks disagree on the history"
    # replicas identical after every stage (parameters and buffers)
    for s in range(1, 5):
        a, b = res[0]["at_stage_end"][s], res[1]["at_stage_end"][s]
        for k, v in a.items():
            assert torch.equal(v, b[k]), f"stage {s}: replicas differ at {k}"
    # the broadcast had something to do: after each train epoch rank 1's running stats
    # (its own shard) differ from rank 0's
    differ = 0
    for (s0, a), (s1, b) in zip(res[0]["after_train"], res[1]["after_train"]):
        assert s0 == s1
        differ += any(not torch.equal(v, b[k]) for k, v in a.items()
                      if k.endswith("running_mean"))
    assert differ == len(res[0]["after_train"]) == 8
    # checkpoints only on rank 0
    assert [f for f in res[1]["ckpts"] if f.endswith(".pth")] == []
    assert sorted(f for f in res[0]["ckpts"] if f.endswith(".pth")) == [
        f"ug_pgunet_stage{s}_best.pth" for s in range(1, 5)]
    # rank 0 against the reference's 2-shard trajectory
    fx = np.load("tests/golden/g12b_progressive_dp2.npz")
    check_history(res[0]["history"], fx)
    for s in range(1, 5):
        check_buffers(res[0]["at_stage_end"][s], fx, s)
