"""Which kernel of the previous stage's eval forward changes its result when it runs on a
second stream concurrently with the current stage's training step? (diagnostic)

The reference is the Stage-3 eval forward alone; then, repeatedly, the same forward on a
side stream while the Stage-4 forward+backward runs on the current stream.  Every block
output (the raw conv output y of each DoubleConv, the lazily-activated tensors the next
kernels read), the logits and the U map are compared bit for bit with the reference.

    python tools/stream_bisect.py [--reps 6] [--batch 4] [--main fwdbwd|fwd|copy|none]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--main", default="fwdbwd")
    a = ap.parse_args()
    import ugpg
    from ugpg import ops
    from oracle import detgen as G
    from tests._parity import det_state
    dev = torch.device("cuda:0")
    m3 = ugpg.PGUNet3(3, 1).to(dev)
    m3.load_state_dict(det_state(3, 3, 1, seed=13))
    m3.eval()
    m4 = ugpg.PGUNet4(3, 1).to(dev)
    m4.load_state_dict(det_state(4, 3, 1, seed=0))
    m4.train()
    B = a.batch
    x = G.randn(5, (B, 3, 256, 256), "x").to(dev)
    xr = ops.resize_nchw(x, 128, 128, ops.RESIZE_BILINEAR)
    m3.prepare_eval()
    g3 = m3.graph()

    def s3():
        with torch.no_grad():
            logits, st = g3.forward(xr, save=False)
            u = ops.resize_nchw(logits.contiguous(), 256, 256, ops.RESIZE_UNCERTAINTY)
        return [o.y.clone() for o in st["outs"]] + [logits.clone(), u.clone()]

    ref = s3()
    torch.cuda.synchronize()
    names = [f"block{i}" for i in range(len(ref) - 2)] + ["logits", "umap"]
    side = torch.cuda.Stream()
    cur = torch.cuda.current_stream()
    big = torch.empty(1 << 28, device=dev)
    for rep in range(a.reps):
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            got = s3()
        if a.main == "fwdbwd":
            out = m4(x)
            out.mean().backward()
        elif a.main == "fwd":
            with torch.no_grad():
                m4(x)
        elif a.main == "copy":
            for _ in range(20):
                big.mul_(1.0)
        cur.wait_stream(side)
        torch.cuda.synchronize()
        diffs = []
        for n, r, g in zip(names, ref, got):
            if not torch.equal(r, g):
                d = (r.float() - g.float()).abs()
                idx = torch.nonzero(d.flatten() > 0)
                diffs.append(f"{n}: {idx.numel()} elements differ, max {d.max().item():.3e}, "
                             f"first flat index {idx[0].item() if idx.numel() else -1} "
                             f"shape {tuple(r.shape)}")
        print(f"rep {rep} main={a.main}: " + ("identical" if not diffs else "; ".join(diffs[:4])),
              flush=True)


if __name__ == "__main__":
    main()
