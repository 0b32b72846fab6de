"""HIP-event timing of the bf16-storage max-pool and bilinear x2 forwards (the bf16
arithmetic's encoder / decoder resamplers) at the Stage-4 shapes (bs16), per libugpg build.
    python tools/op16_bench.py [--libs a.so,b.so] [--rounds 3]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tools"), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402
from head_bench import load, timeit  # noqa: E402
from ugpg import _C, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B = 16
    cases = {}
    for (h, c) in [(256, 64), (128, 128), (64, 256), (32, 512)]:
        y = torch.randn(B, h, h, c, device=dev).to(torch.bfloat16)
        act = ops.Act(y, torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1)
        cases[f"maxpool2_fwd16 {h}^2 C{c}"] = (lambda act=act, h=h: ops.maxpool2_fwd(act, bf16=True),
                                               y.numel() * 2 * (1 + 1 / 4) + y.numel() / 4)
    for (h, c) in [(16, 512), (32, 256), (64, 128), (128, 64)]:
        y = torch.randn(B, h, h, c, device=dev).to(torch.bfloat16)
        act = ops.Act(y, torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1)
        cases[f"bilinear_fwd16 {h}->{2 * h} C{c}"] = (
            lambda act=act, h=h: ops.bilinear_nhwc_fwd(act, 2 * h, 2 * h, bf16=True), y.numel() * 2 * 5)
    libs = [p for p in a.libs.split(",") if p] or [None]
    handles = {p: (load(p) if p else _C.lib._lib) for p in libs}
    res = {}
    for _ in range(a.rounds):
        for p in libs:
            _C.lib._lib = handles[p]
            for name, (fn, nbytes) in cases.items():
                res.setdefault((p, name), []).append(timeit(fn))
    for (p, name), v in res.items():
        us = sorted(v)[len(v) // 2]
        print(f"{Path(p).name if p else 'in-tree'} {name}: {us:7.1f} us  "
              f"{cases[name][1] / (us * 1e-6) / 1e9:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
