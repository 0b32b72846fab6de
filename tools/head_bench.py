"""HIP-event timing of the 1x1 deep-supervision head kernels at the Stage-4 shapes (bs16,
1 class): forward (head_fwd_cj) and backward (head_bwd, with the BatchNorm-backward
partials and the deferred route at 256^2 as the engine runs the top decoder block), with
fp32 and bf16 activation storage.  --libs: compare libugpg builds in one process.
    python tools/head_bench.py [--libs a.so,b.so] [--rounds 3]
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
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B = 16
    g = torch.Generator(device=dev).manual_seed(1)
    cases = {}
    for (h, c) in [(256, 64), (128, 64), (64, 128), (32, 256)]:
        y = torch.randn(B, h, h, c, device=dev, generator=g)
        sc, sh = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
        mean, invstd = torch.randn(c, device=dev) * 0.1, torch.rand(c, device=dev) + 0.5
        w, bias = torch.randn(1, c, device=dev) * 0.1, torch.randn(1, device=dev)
        dh = torch.randn(B * h * h, 1, device=dev)
        dw, db = torch.empty(1, c, device=dev), torch.empty(1, device=dev)
        da = torch.empty(B, h, h, c, device=dev)
        for st, t in (("f32", y), ("bf16", y.to(torch.bfloat16))):
            act = ops.Act(t, sc, sh)
            nb = t.element_size()
            cases[f"fwd {h}^2 C{c} {st}"] = (lambda act=act, w=w, bias=bias: ops.head_fwd(act, w, bias),
                                            t.numel() * nb)
            if h == 256:  # the top decoder block: partials only, da recomputed by the apply
                cases[f"bwd {h}^2 C{c} {st} bnb+defer"] = (
                    lambda act=act, w=w, dh=dh, dw=dw, db=db, da=da, mean=mean, invstd=invstd: ops.head_bwd(
                        act, w, dh, dw, db, da, 0, bnb=(mean, invstd), defer=True), t.numel() * nb)
            else:
                cases[f"bwd {h}^2 C{c} {st}"] = (
                    lambda act=act, w=w, dh=dh, dw=dw, db=db, da=da: ops.head_bwd(act, w, dh, dw, db, da, 0),
                    t.numel() * (nb + 4))
    dl = torch.randn(B, 1, 256, 256, device=dev, generator=g)
    for R in (32, 64, 128):
        cases[f"split_bwd 256->{R}"] = (lambda R=R: ops.heads_split_bwd(dl, [R]), dl.numel() * 4)
    cases["split_bwd 256->32,64,128,256 (the Stage-4 heads)"] = (
        lambda: ops.heads_split_bwd(dl, [32, 64, 128, 256]), 4 * dl.numel() * 4)
    img = torch.randn(B, 3, 256, 256, device=dev, generator=g)
    cases["nchw_to_nhwc 3->8 256^2"] = (lambda: ops.nchw_to_nhwc(img, 8), img.numel() * 4 * (1 + 8 / 3))
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
        nbytes = cases[name][1]
        print(f"{Path(p).name if p else 'in-tree'} {name}: {us:7.1f} us  {nbytes / (us * 1e-6) / 1e9:6.0f} GB/s",
              flush=True)


if __name__ == "__main__":
    main()
