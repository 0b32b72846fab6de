"""Host-side cost of the bench's training step: is the step GPU-bound or launch-bound?

Builds the bench's Stage-4 trainer (bench.py main()), then
  1. per step: synchronize; issue train_step (host time); synchronize (issue + drain);
  2. the bench's pipelined loop timed as bench.py times it;
  3. cProfile of the pipelined loop: where the host time goes (top functions by own time).
  python tools/host_probe.py [--conv-math bf16] [--steps 10]
"""
import argparse
import cProfile
import io
import pstats
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "ug-pg-unet_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conv-math", default="x6")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    import torch
    import ugpg
    from ugpg import ops
    from ugpg.trainer import MetricsReadback

    ops.set_conv_math(args.conv_math)
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
    tr.current_stage = 4
    tr.current_model = tr.models[4]
    tr.setup_optimizer(4)
    g = torch.Generator().manual_seed(100)
    x = torch.randn(args.batch, 3, args.res, args.res, generator=g).to(dev)
    t = (torch.rand(args.batch, 1, args.res, args.res, generator=g) < 0.5).float().to(dev)
    tr.current_model.train()
    tr.models[3].eval()

    def run(n):
        pending = None
        for _ in range(n):
            cur = MetricsReadback(tr.train_step(x, t, 4))
            if pending is not None:
                pending.values()
            pending = cur
        if pending is not None:
            pending.values()

    run(5)
    torch.cuda.synchronize()
    issue, total = [], []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.train_step(x, t, 4)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        issue.append(1e3 * (t1 - t0))
        total.append(1e3 * (t2 - t0))
    med = lambda v: sorted(v)[len(v) // 2]
    print(f"serial step: host issue {med(issue):.3f} ms, issue + drain {med(total):.3f} ms "
          f"(median of {args.steps})")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    print(f"pipelined (bench loop): {1e3 * (time.perf_counter() - t0) / args.steps:.3f} ms/step")
    pr = cProfile.Profile()
    torch.cuda.synchronize()
    pr.enable()
    run(args.steps)
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(args.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumtime").print_stats(args.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
