"""Per-op HIP-event timing of the memory-bound helper kernels at their Stage-4 shapes
(bs16).  python tools/op_bench.py  ->  one line per op: shape, µs/launch, GB/s."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402
from ugpg import ops  # noqa: E402


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
    dev = torch.device("cuda:0")
    B = 16
    for (h, c) in [(16, 512), (32, 256), (64, 128), (128, 64)]:
        y = torch.randn(B, h, h, c, device=dev)
        sc = torch.rand(c, device=dev) + 0.5
        sh = torch.randn(c, device=dev) * 0.1
        a = ops.Act(y, sc, sh)
        us = timeit(lambda: ops.bilinear_nhwc_fwd(a, 2 * h, 2 * h))
        gb = (y.numel() + 4 * y.numel()) * 4 / (us * 1e-6) / 1e9
        print(f"bilinear_fwd {h}->{2 * h} C{c}: {us:7.1f} us  {gb:6.0f} GB/s", flush=True)
        dout = torch.randn(B, 2 * h, 2 * h, c, device=dev)
        din = torch.empty_like(y)
        us = timeit(lambda: ops.bilinear_nhwc_bwd(dout, h, h, din, False))
        gb = (dout.numel() + y.numel()) * 4 / (us * 1e-6) / 1e9
        print(f"bilinear_bwd {2 * h}->{h} C{c}: {us:7.1f} us  {gb:6.0f} GB/s", flush=True)


if __name__ == "__main__" and (len(sys.argv) < 2 or sys.argv[1] not in ("bn", "heads", "pack")):
    main()


def bn_main():
    """BatchNorm+ReLU backward (reduce, finalize, apply) at the 8 Stage-4 layer shapes."""
    dev = torch.device("cuda:0")
    B = 16
    tot = {}
    for (h, c) in [(256, 64), (128, 128), (64, 256), (32, 512), (16, 512), (32, 256), (64, 128),
                   (128, 64)]:
        y = torch.randn(B, h, h, c, device=dev)
        da = torch.randn_like(y)
        dy = torch.empty_like(y)
        mean, invstd = torch.randn(c, device=dev) * 0.1, torch.rand(c, device=dev) + 0.5
        scale, shift = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1
        dg, dbt, dbias = (torch.empty(c, device=dev) for _ in range(3))
        line = []
        for name in ("bn_bwd",):
            us = timeit(lambda: ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, dy, dg, dbt, dbias))
            gb = 5 * y.numel() * 4 / (us * 1e-6) / 1e9
            tot[name] = tot.get(name, 0.0) + 2 * us
            line.append(f"{name} {us:6.1f} us {gb:5.0f} GB/s")
        print(f"bn_bwd {h}^2 C{c}: " + " | ".join(line), flush=True)
    print("bn_bwd per step (x2 per shape): " + " ".join(f"{k}={v:.0f}us" for k, v in tot.items()))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "bn":
    bn_main()


def heads_main():
    """1x1 deep-supervision head forward at the Stage-4 head shapes (bs16, 1 class)."""
    dev = torch.device("cuda:0")
    B = 16
    tot = 0.0
    for (h, c) in [(32, 256), (64, 128), (128, 64), (256, 64)]:
        y = torch.randn(B, h, h, c, device=dev)
        a = ops.Act(y, torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.1)
        w, b = torch.randn(1, c, device=dev), torch.randn(1, device=dev)
        us = timeit(lambda: ops.head_fwd(a, w, b))
        tot += us
        gb = y.numel() * 4 / (us * 1e-6) / 1e9
        print(f"head_fwd {h}^2 C{c}: {us:7.1f} us  {gb:6.0f} GB/s", flush=True)
    print(f"head_fwd S4 total {tot:.1f} us")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "heads":
    heads_main()


def pack_main():
    """The Stage-4 per-step weight pack (every 3x3 conv: forward + data-gradient layouts)
    as the trainer issues it: one ugpg_pack_conv3x3_batch launch."""
    import ugpg
    dev = torch.device("cuda:0")
    m = ugpg.PGUNet4(3, 1).to(dev)
    specs = []
    for mod in m.modules():
        if isinstance(mod, torch.nn.Conv2d) and mod.kernel_size == (3, 3):
            w = mod.weight
            cin = w.shape[1]
            specs.append((w, ops.conv_pack_k(8 if cin == 3 else cin), 0))
            if cin != 3:
                specs.append((w, cin, 1))
    from ugpg._C import lib
    items, outs = [], []
    for w, k, mode in specs:
        cout, cin = w.shape[0], w.shape[1]
        fmt = ops.conv_weight_format(cout, k) if mode == 0 else ops.conv_weight_format(k, cout)
        out = torch.empty(lib.ugpg_pack_conv3x3_bytes(cout, k, fmt), dtype=torch.uint8, device=dev)
        outs.append(out)
        items.append(ops.PackItem(ops.ptr(w.detach()), ops.ptr(out), cout, cin, int(k), int(mode)))
    arr = (ops.PackItem * len(items))(*items)
    fmt = ops._MATH_FMT[ops.conv_math()]
    us = timeit(lambda: lib.ugpg_pack_conv3x3_batch(arr, len(items), fmt, ops.stream()), n=50)
    print(f"pack S4 ({len(specs)} packs, one launch): {us:7.1f} us", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "pack":
    pack_main()
