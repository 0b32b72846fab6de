"""MoNuSeg augmentation throughput: the GPU pipeline (ugpg.augment.MoNuSegAugmenter,
inputs resident in HBM) vs the reference's PIL path (oracle/augment_ref.py, one host
thread), on synthetic 1000x1000 RGB tiles + masks -> 256x256 with the reference's
random parameters.  Prints one JSON line.

    python tools/bench_augment.py [--batch 16] [--steps 20] [--size 256]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from oracle import augment_ref as R  # noqa: E402
from ugpg.augment import MoNuSegAugmenter  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--orig", type=int, default=1000)
    ap.add_argument("--cpu-samples", type=int, default=16)
    a = ap.parse_args()
    dev = torch.device("cuda")
    rng = np.random.default_rng(0)
    B, H = a.batch, a.orig
    imgs = rng.integers(0, 256, (B, H, H, 3), dtype=np.uint8)
    masks = (rng.random((B, H, H)) < 0.3).astype(np.uint8)
    di, dm = torch.from_numpy(imgs).to(dev), torch.from_numpy(masks).to(dev)
    aug = MoNuSegAugmenter(a.size, dev)
    seeds = rng.integers(0, 2 ** 32, (a.steps + 1, B))
    params = [[R.draw_params(int(s)) for s in row] for row in seeds]
    aug(di, dm, params[0])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(a.steps):
        aug(di, dm, params[k + 1])
    torch.cuda.synchronize()
    gpu = B * a.steps / (time.perf_counter() - t0)
    # host share (parameter draws + packing) of the GPU path, for the record
    t0 = time.perf_counter()
    for k in range(a.steps):
        [R.draw_params(int(s)) for s in seeds[k]]
    host = (time.perf_counter() - t0) / (B * a.steps)
    pil_imgs = [Image.fromarray(imgs[i % B]) for i in range(a.cpu_samples)]
    pil_masks = [Image.fromarray(masks[i % B]) for i in range(a.cpu_samples)]
    t0 = time.perf_counter()
    for i in range(a.cpu_samples):
        R.joint_transform(pil_imgs[i], pil_masks[i], a.size, params[0][i % B])
    cpu = a.cpu_samples / (time.perf_counter() - t0)
    print(json.dumps({"metric": f"MoNuSeg augmentation images/sec ({H}x{H} -> {a.size}x{a.size}, "
                                "resize+flips+rotate+jitter+ToTensor)",
                      "gpu_images_per_sec": round(gpu, 1), "batch": B,
                      "cpu_pil_images_per_sec": round(cpu, 2), "cpu_threads": 1,
                      "speedup": round(gpu / cpu, 1),
                      "host_param_draw_us_per_image": round(host * 1e6, 2)}))


if __name__ == "__main__":
    main()
