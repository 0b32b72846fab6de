"""Which kernel's result changes when another process runs kernels on the same GPU at
the same time?  (diagnostic; the 2-rank config-5 test shares one GPU between its ranks)

N child processes each run the same train-mode forward (no autograd) of one PGUNet stage
in a loop and compare every block output (the raw conv output y of each DoubleConv), the
logits and, per block, the BatchNorm scale/shift with the process's own first result, bit
for bit; the first differing tensor of each repetition is printed.

    python tools/xproc_bisect.py [--procs 2] [--stage 2] [--batch 1] [--iters 60]
"""
import argparse
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]


def child(a):
    import torch
    import ugpg
    from oracle import detgen as G
    from oracle.make_goldens import G12
    from tests._parity import det_state
    dev = torch.device("cuda:0")
    res = {1: 32, 2: 64, 3: 128, 4: 256}[a.stage]
    m = getattr(ugpg, f"PGUNet{a.stage}")(3, 1).to(dev)
    m.load_state_dict(det_state(a.stage, 3, 1, seed=G12["w_seeds"][a.stage]))
    m.train()
    x = G.randn(77, (a.batch, 3, res, res), "x").to(dev)
    g = m.graph()
    from ugpg.flat import ensure_flat
    ensure_flat(m)

    from ugpg import ops
    rec = []
    _hf, _hc = ops.head_fwd, ops.heads_combine

    def head_fwd(a, w, b):  # record every head output (and its input's checksum)
        h = _hf(a, w, b)
        rec.append((f"head{len(rec)}", h.clone()))
        return h

    ops.head_fwd = head_fwd

    def run():
        rec.clear()
        with torch.no_grad():
            logits, st = g.forward(x, save=True)
        outs = []
        for i, o in enumerate(st["outs"]):
            outs.append((f"block{i}.y", o.y.clone()))
            if o.scale is not None:
                outs.append((f"block{i}.scale", o.scale.clone()))
                outs.append((f"block{i}.shift", o.shift.clone()))
        outs.extend(rec)
        outs.append(("logits", logits.clone()))
        return outs

    if a.micro and os.environ.get("XP_RANK") == "0":
        # this process: only the logits combine (and torch's own kernels) on fixed inputs,
        # while the other process runs whole forwards
        with torch.no_grad():
            _, st = g.forward(x, save=False)
        hs = [h.clone() for _, h in rec]
        B_, nc = x.shape[0], 1
        H = x.shape[2]
        big = torch.randn(1 << 24, device=dev)
        ref_l = ops.heads_combine(hs, B_, H, H, nc).clone()
        ref_t = torch.nn.functional.interpolate(hs[0].permute(0, 3, 1, 2), size=(H, H), mode="bilinear",
                                                align_corners=True).clone()
        ref_b = (big * 1.5 + 0.25).clone()
        F = torch.nn.functional
        hsn = [h.permute(0, 3, 1, 2).contiguous() for h in hs]

        def tcomb():  # torch's own kernels doing the combine (4 gathers + adds)
            o = None
            for h in hsn:
                u = h if h.shape[-1] == H else F.interpolate(h, size=(H, H), mode="bilinear",
                                                             align_corners=True)
                o = u if o is None else o + u
            return o

        ref_c = tcomb().clone()
        ref_r = ops.resize_nchw(hsn[0], H, H, ops.RESIZE_BILINEAR).clone()

        def rall():  # ugpg resize of each head tensor heads_combine reads (the same memory)
            return torch.cat([ops.resize_nchw(h.view(h.shape[0], 1, h.shape[1], h.shape[2]), H, H,
                                              ops.RESIZE_BILINEAR).flatten() for h in hs])

        ref_a = rall().clone()
        ref_l2 = ops.heads_combine([h.clone() for h in hs], B_, H, H, nc).clone()
        torch.cuda.synchronize()
        names = ['heads_combine', 'torch interpolate', 'torch axpb', 'torch combine', 'ugpg resize',
                 'ugpg resize of the heads', 'heads_combine on fresh copies']
        nb = [0] * len(names)
        for it in range(a.iters * 20):
            l = ops.heads_combine(hs, B_, H, H, nc)
            t2 = torch.nn.functional.interpolate(hs[0].permute(0, 3, 1, 2), size=(H, H), mode="bilinear",
                                                 align_corners=True)
            b2 = big * 1.5 + 0.25
            c2 = tcomb()
            r2 = ops.resize_nchw(hsn[0], H, H, ops.RESIZE_BILINEAR)
            a2 = rall()
            l2 = ops.heads_combine([h.clone() for h in hs], B_, H, H, nc)
            torch.cuda.synchronize()
            for i, (r, v) in enumerate(((ref_l, l), (ref_t, t2), (ref_b, b2), (ref_c, c2), (ref_r, r2),
                                        (ref_a, a2), (ref_l2, l2))):
                if not torch.equal(r, v):
                    nb[i] += 1
                    if nb[i] <= 3:
                        d = (r - v).abs()
                        print(f"micro {names[i]} iter {it}: "
                              f"{int((d > 0).sum())} elements differ, max {d.max().item():.3e}", flush=True)
                        if i == 0:
                            os.makedirs("gpurun_out", exist_ok=True)
                            torch.save({"ref": r.cpu(), "bad": v.cpu(), "hs": [h.cpu() for h in hs],
                                        "it": it}, f"gpurun_out/micro_bad_{nb[0]}.pt")
        print("micro: differing repetitions " + ", ".join(f"{n} {k}" for n, k in zip(names, nb)) +
              f" of {a.iters * 20}", flush=True)
        return
    ref = run()
    torch.cuda.synchronize()
    bad = 0
    for it in range(a.iters):
        got = run()
        torch.cuda.synchronize()
        for (n, r), (_, v) in zip(ref, got):
            if not torch.equal(r, v):
                d = (r.float() - v.float()).abs()
                nz = torch.nonzero(d.flatten() > 0)
                print(f"proc {os.environ.get('XP_RANK')} iter {it}: first difference {n} shape "
                      f"{tuple(r.shape)}: {nz.numel()} elements, max {d.max().item():.3e}, first "
                      f"flat index {nz[0].item()}", flush=True)
                bad += 1
                break
    print(f"proc {os.environ.get('XP_RANK')}: {bad} of {a.iters} repetitions differ", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--stage", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--micro", action="store_true",
                    help="process 0 loops the logits combine and torch kernels only")
    a = ap.parse_args()
    if a.child:
        child(a)
        return
    args = [sys.executable, "-u", __file__, "--child", "--stage", str(a.stage), "--batch",
            str(a.batch), "--iters", str(a.iters)] + (["--micro"] if a.micro else [])
    procs = [subprocess.Popen(args, env=dict(os.environ, XP_RANK=str(r)), cwd=str(ROOT))
             for r in range(a.procs)]
    rcs = [p.wait(timeout=500) for p in procs]
    sys.exit(max(rcs))


if __name__ == "__main__":
    main()
