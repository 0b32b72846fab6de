"""Per-layer conv kernel micro-benchmark (Stage-4, bs16) -- all variants in one
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

    python tools/conv_bench.py [--rounds 3] [--maths x6,bf16,f32] [--wgrad]
    python tools/conv_bench.py --libs exp/a.so,exp/b.so ...   (A/B of builds, one process)

Kernel variants are A/B'd as separate builds (`build.py -D ... --out`, then --libs): the
library has no runtime tuning knobs.
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402

from ugpg import _C, ops  # noqa: E402
from ugpg._C import lib  # noqa: E402


def load_lib(path):
    import ctypes
    L = ctypes.CDLL(str(Path(path).resolve()))
    for name, (res, args) in _C.SIGNATURES.items():
        fn = getattr(L, name, None)  # an older build may lack newer entries
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return L

B = 16
# name, H, C0, C1, Cout  (forward convs of PGUNet4; C1 = upsampled half of Up's concat)
LAYERS = [("inc.0", 256, 8, 0, 64), ("inc.3", 256, 64, 0, 64),
          ("down1.0", 128, 64, 0, 128), ("down1.3", 128, 128, 0, 128),
          ("down2.0", 64, 128, 0, 256), ("down2.3", 64, 256, 0, 256),
          ("down3.0", 32, 256, 0, 512), ("down3.3", 32, 512, 0, 512),
          ("down4.0", 16, 512, 0, 512), ("down4.3", 16, 512, 0, 512),
          ("up1.0", 32, 512, 512, 256), ("up1.3", 32, 256, 0, 256),
          ("up2.0", 64, 256, 256, 128), ("up2.3", 64, 128, 0, 128),
          ("up3.0", 128, 128, 128, 64), ("up3.3", 128, 64, 0, 64),
          ("up4.0", 256, 64, 64, 64), ("up4.3", 256, 64, 0, 64)]


def timeit(fn, iters=5):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--maths", default="x6,f32")
    ap.add_argument("--wgrad", action="store_true")
    ap.add_argument("--layers", default="", help="comma-separated layer names (default: all)")
    ap.add_argument("--nostats", action="store_true", help="forward without BatchNorm partials")
    ap.add_argument("--libs", default="", help="comma-separated libugpg builds to compare")
    a = ap.parse_args()
    libs = [(Path(p).stem, load_lib(p)) for p in a.libs.split(",")] if a.libs else [("", None)]
    dev = torch.device("cuda:0")
    rows = {}
    sel = set(a.layers.split(",")) if a.layers else None
    for name, H, C0, C1, Cout in LAYERS:
        if sel and name not in sel:
            continue
        cin = C0 + C1
        real_cin = 3 if cin == 8 else cin
        if cin == 8:  # the image layer reads the raw (channel-padded) image
            srcs = [ops.Act(torch.randn(B, H, H, C0, device=dev))]
        else:
            srcs = [ops.Act(torch.randn(B, H, H, C0, device=dev),
                            torch.rand(C0, device=dev) + 0.5, torch.randn(C0, device=dev) * 0.1)]
        if C1:
            srcs.append(ops.Act(torch.randn(B, H, H, C1, device=dev)))
        w = torch.randn(Cout, real_cin, 3, 3, device=dev) * 0.05
        out = torch.empty(B, H, H, Cout, device=dev)
        # the bf16 arithmetic stores conv outputs of images >= 32 wide in bf16 only, and its
        # sources (activations, dy) likewise
        out16 = torch.empty(B, H, H, Cout, device=dev, dtype=torch.bfloat16)
        srcs16 = [ops.Act(s.y.to(torch.bfloat16), s.scale, s.shift) for s in srcs]
        bias = torch.zeros(Cout, device=dev)
        flops = 2.0 * B * H * H * Cout * 9 * real_cin
        fns = {}
        for m in a.maths.split(","):
            ops.set_conv_math(m)
            wpk = ops.pack_conv3x3(w, ops.conv_pack_k(cin), 0)
            wpk1 = ops.pack_conv3x3(w, real_cin, 1) if real_cin % 64 == 0 else None
            nt = 0  # (slot counts may differ between the compared builds: the largest)
            for _, L in libs:
                if L is not None:
                    lib._lib = L
                nt = max(nt, ops.conv_ntiles(B, H, H, cin, Cout, wpk))
            st = torch.empty(3 * Cout * nt, device=dev)

            st16 = m == "bf16" and H >= 32 and cin >= 16

            def f(m=m, wpk=wpk, st=st, st16=st16):
                ops.set_conv_math(m)
                ops.conv3x3_fwd(srcs16 if st16 else srcs, wpk, bias, Cout, [out16 if st16 else out],
                                stats=None if a.nostats else st)
            fns[f"fwd_{m}"] = f
            if wpk1 is not None:
                dy = torch.randn(B, H, H, Cout, device=dev)
                d0 = torch.empty(B, H, H, C0, device=dev)
                d1 = torch.empty(B, H, H, C1, device=dev) if C1 else None

                dy16 = dy.to(torch.bfloat16)

                def g(m=m, wpk1=wpk1, dy=dy, d0=d0, d1=d1, dy16=dy16, st16=st16):
                    ops.set_conv_math(m)
                    ops.conv3x3_fwd([ops.Act(dy16 if st16 else dy)], wpk1, None, real_cin,
                                    [d0, d1] if C1 else [d0], split=C0 if C1 else None)
                fns[f"dgrad_{m}"] = g
        ops.set_conv_math("x6")
        if a.wgrad:
            dy = torch.randn(B, H, H, Cout, device=dev)
            dw = torch.empty_like(w)
            for m in a.maths.split(","):
                def wg(m=m):
                    ops.set_conv_math(m)
                    ops.conv3x3_wgrad(srcs, dy, dw, None, real_cin)
                fns[f"wgrad_{m}"] = wg
        if libs[0][1] is not None:
            def with_lib(f, L):
                def h():
                    lib._lib = L
                    f()
                return h
            fns = {f"{k}@{tag}": with_lib(f, L) for tag, L in libs for k, f in fns.items()}
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                try:
                    res[k].append(timeit(f))
                except RuntimeError as e:
                    res[k].append(float("nan"))
        ops.set_conv_math("x6")
        rows[name] = {k: (min(v), flops / (min(v) * 1e-3) / 1e12) for k, v in res.items()}
        print(name, " ".join(f"{k}={v[0]:.3f}ms/{v[1]:.0f}TF" for k, v in rows[name].items()),
              flush=True)
    tot = {}
    for r in rows.values():
        for k, (ms, _) in r.items():
            tot[k] = tot.get(k, 0.0) + ms
    print("TOTAL", " ".join(f"{k}={v:.2f}ms" for k, v in tot.items()))


if __name__ == "__main__":
    main()
