"""HIP-event timing of the image layer's weight gradient (conv3x3_wgrad_img_kernel) at the
Stage-4 inc shape (bs16 x 256^2, 3 real of 8 image channels, 64 outputs): the plain form
(fp32 dy), and the forms that build dy from the following BatchNorm backward (fp32 y, bf16
y).  --libs: compare libugpg builds (build.py -D ... --out) in one process, interleaved.
    python tools/img_bench.py [--libs a.so,b.so] [--rounds 4]
"""
import argparse
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402
from ugpg import _C, ops  # noqa: E402


def load(path):
    L = ctypes.CDLL(str(Path(path).resolve()))
    for name, (res, args) in _C.SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return L


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="")
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, H, W, C = 16, 256, 256, 64
    g = torch.Generator(device=dev).manual_seed(1)
    img = torch.zeros(B, H, W, 8, device=dev)
    img[..., :3] = torch.randn(B, H, W, 3, device=dev, generator=g)
    srcs = [ops.Act(img)]
    y = torch.randn(B, H, W, C, device=dev, generator=g)
    y16 = y.to(torch.bfloat16)
    da = torch.randn(B, H, W, C, device=dev, generator=g)
    mean, invstd = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    scale, shift = torch.ones(C, device=dev), torch.zeros(C, device=dev) + 0.1
    coef = torch.randn(2 * C, device=dev, generator=g) * 1e-3
    dw = torch.empty(C, 3, 3, 3, device=dev)
    cases = {
        "plain dy fp32": lambda: ops.conv3x3_wgrad(srcs, da, dw, None, 3),
        "BN y fp32": lambda: ops.conv3x3_wgrad(
            srcs, ops.BnLazyDy(da, y, mean, invstd, scale, shift, coef, None), dw, None, 3),
        "BN y bf16": lambda: ops.conv3x3_wgrad(
            srcs, ops.BnLazyDy(da, y16, mean, invstd, scale, shift, coef, None), dw, None, 3),
    }
    nbytes = {"plain dy fp32": 4, "BN y fp32": 8, "BN y bf16": 6}
    libs = [p for p in a.libs.split(",") if p] or [None]
    handles = {p: (load(p) if p else _C.lib._lib) for p in libs}
    res = {}
    for _ in range(a.rounds):
        for p in libs:
            _C.lib._lib = handles[p]
            for name, fn in cases.items():
                try:
                    us = timeit(fn)
                except RuntimeError as e:  # (an older build without this form)
                    us = float("nan")
                    print(f"{p} {name}: {e}", flush=True)
                res.setdefault((p, name), []).append(us)
    for (p, name), v in res.items():
        us = sorted(v)[len(v) // 2]
        gbs = (B * H * W * C * nbytes[name] + img.numel() * 4) / (us * 1e-6) / 1e9
        print(f"{Path(p).name if p else 'in-tree'} {name}: {us:7.1f} us  {gbs:6.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
