"""Where does the trainer's side-stream U map differ from the one-stream order? (diagnostic)

Runs UncertaintyGuidedProgressiveTrainer.train_step with the U map on the side stream and
snapshots, on the stream that produced each one: the input the side stream read, the
previous stage's resized input, its logits, the U map, and (on the current stream right
after the join) the U map the loss reads.  After each step everything is recomputed on one
stream from the snapshot of the input and compared bit for bit.

    python tools/umap_trainer_probe.py [--steps 4] [--reps 2]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4)
    a = ap.parse_args()
    import ugpg
    from ugpg import ops
    from oracle import detgen as G
    from tests._parity import det_state
    dev = torch.device("cuda:0")
    for rep in range(a.reps):
        tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev, uncertainty_alpha=1.0)
        tr.models[3].load_state_dict(det_state(3, 3, 1, seed=13))
        tr.models[4].load_state_dict(det_state(4, 3, 1, seed=0))
        tr.current_stage, tr.current_model = 4, tr.models[4]
        tr.setup_optimizer(4)
        tr.umap_side_stream = True
        snaps = {}
        ul = tr.uncertainty_loss
        orig_gen = type(ul).generate_uncertainty_map

        def gen(self, inp, mp, pr, cr):
            snaps["data"] = inp.clone()
            mp.eval()
            with torch.no_grad():
                x = ops.resize_nchw(inp.detach().float().contiguous(), pr, pr, ops.RESIZE_BILINEAR)
                snaps["x"] = x.clone()
                logits = mp(x)
                snaps["logits"] = logits.clone()
                u = ops.resize_nchw(logits.contiguous(), cr, cr, ops.RESIZE_UNCERTAINTY)
                snaps["u"] = u.clone()
            return u.detach()
        ul.generate_uncertainty_map = gen.__get__(ul)
        orig_fd = tr._forward_device

        def fd(data, target, stage, mbuf):
            out = orig_fd(data, target, stage, mbuf)
            snaps["u_loss"] = out[1].clone()  # current stream, after the join
            return out
        tr._forward_device = fd
        x0 = G.randn(5, (a.batch, 3, 256, 256), "x").to(dev)
        t0 = G.bernoulli(6, (a.batch, 1, 256, 256), 0.5, "t").to(dev)
        for s in range(a.steps):
            d, tt = tr._resize_batch(x0 * 1.0, t0, 256)
            row = tr.train_step(d, tt, 4)
            torch.cuda.synchronize()
            # one-stream recomputation from the snapshots
            m3 = tr.models[3]
            with torch.no_grad():
                rx = ops.resize_nchw(snaps["data"], 128, 128, ops.RESIZE_BILINEAR)
                rl = m3(snaps["x"])
                ru = ops.resize_nchw(snaps["logits"].contiguous(), 256, 256, ops.RESIZE_UNCERTAINTY)
            torch.cuda.synchronize()
            chk = [("data==d", snaps["data"], d), ("x", snaps["x"], rx), ("logits", snaps["logits"], rl),
                   ("u", snaps["u"], ru), ("u_loss==u", snaps["u_loss"], snaps["u"])]
            msg = []
            for n, p, q in chk:
                if torch.equal(p, q):
                    msg.append(f"{n} ok")
                else:
                    dd = (p - q).abs()
                    msg.append(f"{n} DIFF({int((dd > 0).sum())} el, max {dd.max().item():.2e})")
            print(f"rep {rep} step {s}: loss {row[0].item():.6f} u {row[5].item():.6f} | " + ", ".join(msg),
                  flush=True)
        ul.generate_uncertainty_map = orig_gen.__get__(ul)


if __name__ == "__main__":
    main()
