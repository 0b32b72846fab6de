"""Interleaved in-process A/B of whole UG training steps (Stage 4, bs16, 256^2): the
bench's workload, alternating blocks of steps between two settings so that clock drift
(DVFS, temperature) hits both sides alike.

    python tools/ab_step.py --a "lib:exp/a.so" --b "lib:exp/b.so"

A setting is `lib:path` (a libugpg build, e.g. a `build.py -D ... --out` variant) or
`module._NAME=value` (an int-valued attribute of ugpg.<module>, for a local experiment
patch: the shipped Python layer has no A/B switches); several comma-separated.
"""
import argparse
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]


_LIBS = {}


def apply(setting):
    import ctypes
    import importlib
    from ugpg import _C
    for item in filter(None, setting.split(",")):
        if item.startswith("lib:"):  # swap the library every ugpg op calls through
            path = str(Path(item[4:]).resolve())
            if path not in _LIBS:
                L = ctypes.CDLL(path)
                for name, (res, args) in _C.SIGNATURES.items():
                    fn = getattr(L, name, None)
                    if fn is not None:
                        fn.restype, fn.argtypes = res, args
                _LIBS[path] = L
            _C.lib._lib = _LIBS[path]
        else:
            k, v = item.split("=")
            mod, attr = k.split(".")
            m = importlib.import_module(f"ugpg.{mod}")
            assert hasattr(m, attr), item
            setattr(m, attr, type(getattr(m, attr))(int(v)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--a", required=True)
    ap.add_argument("--b", required=True)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--conv-math", default="x6", choices=("x6", "bf16", "f32"))
    a = ap.parse_args()
    import torch
    import ugpg
    from ugpg import ops
    ops.set_conv_math(a.conv_math)
    from ugpg.trainer import MetricsReadback
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
    tr.current_stage = 4
    tr.current_model = tr.models[4]
    tr.setup_optimizer(4)
    g = torch.Generator().manual_seed(100)
    x = torch.randn(16, 3, 256, 256, generator=g).to(dev)
    t = (torch.rand(16, 1, 256, 256, generator=g) < 0.5).float().to(dev)
    tr.current_model.train()
    tr.models[3].eval()

    def run(n):
        pending = None
        for _ in range(n):
            cur = MetricsReadback(tr.train_step(x, t, 4))
            if pending is not None:
                pending.values()
            pending = cur
        pending.values()

    res = {"a": [], "b": []}
    for side in ("a", "b"):
        apply(getattr(a, side))
        run(2)
    for r in range(a.rounds):
        for side in (("a", "b") if r % 2 == 0 else ("b", "a")):
            apply(getattr(a, side))
            run(1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(a.steps)
            torch.cuda.synchronize()
            res[side].append(1000 * (time.perf_counter() - t0) / a.steps)
        print(f"round {r}: a {res['a'][-1]:.3f} ms  b {res['b'][-1]:.3f} ms", flush=True)
    ma, mb = statistics.median(res["a"]), statistics.median(res["b"])
    print(f"median ms/step  a {ma:.3f}  b {mb:.3f}  b/a {mb / ma:.4f}  ({a.a} | {a.b})")


if __name__ == "__main__":
    main()
