"""Timing probe of the split-bf16 forward conv on one layer shape: full kernel vs
the same kernel with the in-loop prefetch and/or LDS staging disabled
(ugpg_set_tuning("x6_probe"); results are garbage in probe modes).
    python tools/x6_probe.py [H C Cout]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]
import torch  # noqa: E402
from ugpg import ops  # noqa: E402
from ugpg._C import lib  # noqa: E402

H, C, Co = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (64, 256, 256)
B = 16
dev = torch.device("cuda:0")
x = ops.Act(torch.randn(B, H, H, C, device=dev), torch.rand(C, device=dev) + .5, torch.randn(C, device=dev))
w = torch.randn(Co, C, 3, 3, device=dev) * .05
wpk = ops.pack_conv3x3(w, C, 0)
out = torch.empty(B, H, H, Co, device=dev)
fl = 2.0 * B * H * H * C * Co * 9
for pipe in (0, 1):
    lib.ugpg_set_tuning(b"x6_pipe", pipe)
    for probe in (0, 1, 2, 3):
        lib.ugpg_set_tuning(b"x6_probe", probe)
        for _ in range(3):
            ops.conv3x3_fwd([x], wpk, None, Co, [out])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            ops.conv3x3_fwd([x], wpk, None, Co, [out])
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        print(f"pipe {pipe} probe {probe}: {ms:.3f} ms  {fl / ms / 1e9:.0f} TF/s", flush=True)
lib.ugpg_set_tuning(b"x6_probe", 0)
lib.ugpg_set_tuning(b"x6_pipe", 2)
