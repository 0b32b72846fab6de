"""Config-5 driver diagnostic: the G12 single-process progressive run (stage lrs 0) twice,
then the 2-rank run (tests/_progressive_worker.py, gloo, both ranks on cuda:0) twice,
printing every history entry next to the reference's (G12 / G12b) and the per-stage
difference between the two epochs (the reference's train losses are equal across the
epochs of a stage: lr 0 leaves the weights, and train-mode BatchNorm ignores the
running statistics).

    python tools/prog_probe.py [--single 2] [--dp 2]
"""
import argparse
import os
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

KEYS = ("train_loss", "val_loss", "base_loss", "train_dice", "val_dice",
        "uncertainty_weights_mean", "uncertainty_weights_std")


def show(tag, hist, fx):
    for k in KEYS:
        mine, want = np.array(hist[k]), fx[f"history/{k}"]
        rel = np.abs(mine - want) / np.maximum(np.abs(want), 1e-12)
        print(f"{tag} {k}: max rel {rel.max():.2e} at {int(rel.argmax())}; "
              f"mine {' '.join(f'{v:.9g}' for v in mine)}", flush=True)
    tl = np.array(hist["train_loss"])
    print(f"{tag} epoch1-epoch2 train_loss per stage: "
          f"{' '.join(f'{tl[2 * i] - tl[2 * i + 1]:+.3e}' for i in range(len(tl) // 2))}", flush=True)


def single(dev):
    from torch.utils.data import DataLoader, TensorDataset
    import ugpg
    from oracle.make_goldens import G12, g12_data
    from tests._parity import det_state
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
    with tempfile.TemporaryDirectory() as d:
        tr.train_progressive(tl, vl, max_stages=4, save_dir=d)
    return tr.history


def dp_run():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2",
               HSA_ENABLE_IPC_MODE_LEGACY="0")
    with tempfile.TemporaryDirectory() as d:
        procs = [subprocess.Popen([sys.executable, "-u", str(ROOT / "tests" / "_progressive_worker.py"), d],
                                  env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), cwd=str(ROOT),
                                  stdout=subprocess.DEVNULL)
                 for r in range(2)]
        rcs = [p.wait(timeout=400) for p in procs]
        assert rcs == [0, 0], rcs
        return [torch.load(Path(d) / f"rank{r}.pt", weights_only=True)["history"] for r in range(2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--single", type=int, default=2)
    ap.add_argument("--dp", type=int, default=2)
    a = ap.parse_args()
    fx1 = np.load(ROOT / "tests/golden/g12_progressive.npz")
    fx2 = np.load(ROOT / "tests/golden/g12b_progressive_dp2.npz")
    for k in ("train_loss",):
        print("G12  ref", " ".join(f"{v:.9g}" for v in fx1[f"history/{k}"]))
        print("G12b ref", " ".join(f"{v:.9g}" for v in fx2[f"history/{k}"]))
    for i in range(a.dp):
        h0, h1 = dp_run()
        show(f"dp{i}", h0, fx2)
    if a.single:
        import contextlib
        import io
        dev = torch.device("cuda:0")
        for i in range(a.single):
            with contextlib.redirect_stdout(io.StringIO()):
                h = single(dev)
            show(f"single{i}", h, fx1)


if __name__ == "__main__":
    main()
