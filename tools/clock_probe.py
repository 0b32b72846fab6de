"""In-kernel clock of the x6r forward (diagnostic builds with -D X6R_CLOCK=1 only):
runs one layer back-to-back for >= 2 s on random data, then reads the median over
workgroups of core cycles / 100 MHz ticks around the main loop (MI355X_MICROARCH.md
'DVFS give-back' item 6).

    UGPG_LIB=exp/lib_clock.so python tools/clock_probe.py [--layers inc.3,down2.3]
    UGPG_LIB=exp/lib_stamp.so python tools/clock_probe.py --stamps   (-D X6R_STAMP=1 build:
        loader waves' share of the loop spent waiting for global loads / at barriers)
"""
import argparse
import ctypes
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd"), str(ROOT / "tools")]

import torch  # noqa: E402

from conv_bench import B, LAYERS  # noqa: E402
from ugpg import ops  # noqa: E402
from ugpg._C import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layers", default="inc.3,down1.3,down2.3,up4.0")
    ap.add_argument("--out16", action="store_true", help="bf16 output storage (math bf16)")
    ap.add_argument("--seconds", type=float, default=2.0)
    ap.add_argument("--stamps", action="store_true")
    ap.add_argument("--wgrad", action="store_true", help="time the weight gradient instead")
    ap.add_argument("--math", default="x6", help="conv arithmetic (x6 / bf16)")
    a = ap.parse_args()
    ops.set_conv_math(a.math)
    dev = torch.device("cuda:0")
    fn = lib.ugpg_debug_stamps if a.stamps else lib.ugpg_debug_clock
    fn.argtypes = [ctypes.POINTER(ctypes.c_double)]
    for name, H, C0, C1, Cout in LAYERS:
        if name not in a.layers.split(","):
            continue
        dt16 = torch.bfloat16 if a.out16 and a.math == "bf16" and H >= 32 and C0 >= 16 else torch.float32
        srcs = [ops.Act(torch.randn(B, H, H, C0, device=dev).to(dt16),
                        torch.rand(C0, device=dev) + 0.5, torch.randn(C0, device=dev) * 0.1)]
        if C1:
            srcs.append(ops.Act(torch.randn(B, H, H, C1, device=dev).to(dt16)))
        w = torch.randn(Cout, C0 + C1, 3, 3, device=dev) * 0.05
        out = torch.empty(B, H, H, Cout, device=dev,
                          dtype=torch.bfloat16 if a.out16 and a.math == "bf16" and H >= 32 else torch.float32)
        wpk = ops.pack_conv3x3(w, C0 + C1, 0)
        st = torch.empty(3 * Cout * ops.conv_ntiles(B, H, H, C0 + C1, Cout, wpk), device=dev)
        flops = 2.0 * B * H * H * Cout * 9 * (C0 + C1)
        dy = torch.randn(B, H, H, Cout, device=dev).to(dt16)  # bf16 dy under --out16 (the step's form)
        dw = torch.empty_like(w)
        for pipe in ("default",):
            n, t0 = 0, time.perf_counter()
            while time.perf_counter() - t0 < a.seconds:
                for _ in range(20):
                    if a.wgrad:
                        ops.conv3x3_wgrad(srcs, dy, dw, None, C0 + C1)
                    else:
                        ops.conv3x3_fwd(srcs, wpk, torch.zeros(Cout, device=dev), Cout, [out],
                                        stats=st)
                torch.cuda.synchronize()
                n += 20
            dt = (time.perf_counter() - t0) / n
            v = (ctypes.c_double * 14)()
            nwg = fn(v)
            if not a.stamps:
                what = f"clock {v[0]:.0f} MHz"
            elif a.wgrad:
                what = (f"loader vm_wait {v[0]:.1%} barrier {v[3]:.1%} LDS stores (incl. VALU)"
                        f" {v[11]:.1%} loads+cursor {v[12]:.1%}")
            else:
                what = ("loader vm_wait/barrier per phase " + " ".join(
                    f"p{q}:{v[q]:.1%}/{v[3 + q]:.1%}" for q in range(3)) +
                    f" | compute barrier {v[6]:.1%} epilogue {v[7]:.1%}, {v[8]:.0f} cyc/step;"
                    f" last epilogue: stores {v[9]:.0f} stats {v[10]:.0f} cyc;"
                    f" loader work: halo stores {v[11]:.1%} row DMAs {v[12]:.1%}"
                    f" halo loads+cursors {v[13]:.1%}")
            print(f"{name}: {dt*1e3:.3f} ms/launch {flops/dt/1e12:.0f} TF  {what} "
                  f"(median of {nwg} workgroups)", flush=True)


if __name__ == "__main__":
    main()
