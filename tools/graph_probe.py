"""Does a captured hipGraph of the bench's training step beat the eager pipelined loop?

Builds the bench's Stage-4 trainer, runs eager warm-up steps, times the bench's pipelined
eager loop, then captures ONE train_step with torch.cuda.graph (recording only: the
kernels run at replay) and times replays of it.  Also checks that a replayed step computes
what an eager step computes (same weights in, same metrics and weights out).
    python tools/graph_probe.py [--conv-math bf16] [--steps 20]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "ug-pg-unet_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--conv-math", default="x6")
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    import torch
    import ugpg
    from ugpg import ops
    from ugpg.trainer import MetricsReadback

    ops.set_conv_math(args.conv_math)
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(100)
    x = torch.randn(16, 3, 256, 256, generator=g).to(dev)
    t = (torch.rand(16, 1, 256, 256, generator=g) < 0.5).float().to(dev)

    def make():
        torch.manual_seed(1234)
        tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
        tr.current_stage = 4
        tr.current_model = tr.models[4]
        tr.setup_optimizer(4)
        tr.current_model.train()
        tr.models[3].eval()
        return tr

    def eager(tr, n):
        pending, last = None, None
        for _ in range(n):
            cur = MetricsReadback(tr.train_step(x, t, 4))
            if pending is not None:
                last = pending.values()
            pending = cur
        return pending.values() if pending is not None else last

    A, B = make(), make()
    m_a = eager(A, 6)
    eager(B, 5)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            mbuf = B.train_step(x, t, 4)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    print("captured", flush=True)
    graph.replay()
    torch.cuda.synchronize()
    m_b = mbuf.tolist()
    pa = list(A.current_model.parameters())
    pb = list(B.current_model.parameters())
    same_w = all(torch.equal(u.detach(), v.detach()) for u, v in zip(pa, pb))
    sa, sb = A.current_model.state_dict(), B.current_model.state_dict()
    same_s = all(torch.equal(sa[k], sb[k]) for k in sa)
    print(f"step 6 metrics eager {m_a[:5]}\nstep 6 metrics graph {m_b[:5]}\n"
          f"weights equal: {same_w}, state (BN buffers) equal: {same_s}", flush=True)
    # timing: the bench's pipelined loop, eager (A) and graph replays (B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eager(A, args.steps)
    torch.cuda.synchronize()
    ms_eager = 1e3 * (time.perf_counter() - t0) / args.steps
    for _ in range(3):
        graph.replay()
    torch.cuda.synchronize()
    pending = None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        graph.replay()
        cur = MetricsReadback(mbuf)
        if pending is not None:
            pending.values()
        pending = cur
    pending.values()
    torch.cuda.synchronize()
    ms_graph = 1e3 * (time.perf_counter() - t0) / args.steps
    t0 = time.perf_counter()
    eager(A, args.steps)
    torch.cuda.synchronize()
    ms_eager2 = 1e3 * (time.perf_counter() - t0) / args.steps
    print(f"eager {ms_eager:.3f} / {ms_eager2:.3f} ms/step, graph replay {ms_graph:.3f} ms/step "
          f"(ratio {ms_graph / min(ms_eager, ms_eager2):.4f})")


if __name__ == "__main__":
    main()
