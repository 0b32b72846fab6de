"""Layer-by-layer GPU-vs-oracle diagnostic (forward y and backward dy of every 3x3
conv, in execution order).  Usage: python tools/debug_parity.py STAGE RES B"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch
import torch.nn as nn
import torch.nn.functional as F

from oracle import detgen as G
from oracle import ref_cpu as O
from tests._parity import det_state

stage, res, B = (int(a) for a in sys.argv[1:4])
dev = torch.device("cuda:0")
state = det_state(stage, 3, 1)
x = G.randn(1, (B, 3, res, res), "x")
t = G.bernoulli(2, (B, 1, res, res), 0.5, "t")

# ---- oracle fp64 with recorded conv outputs
rec = []
_conv = F.conv2d


def conv_rec(inp, w, b=None, *a, **k):
    y = _conv(inp, w, b, *a, **k)
    if w.shape[-1] == 3:
        y.retain_grad()
        rec.append(y)
    return y


O.F.conv2d = conv_rec
P = {k: (v.clone().double() if v.is_floating_point() else v.clone()) for k, v in state.items()}
for k in P:
    if P[k].is_floating_point() and not O._is_buffer(k):
        P[k].requires_grad_(True)
logits = O.pgunet_forward(stage, P, x.double(), training=True)
final, _ = O.weighted_loss(O.bce_pixel(logits, t.double(), 5.0), None, 1.0)
final.backward()
O.F.conv2d = _conv

# ---- GPU with recorded y (forward) and dy (backward)
import ugpg  # noqa: E402
from ugpg import engine  # noqa: E402

fw, bw = [], []
_dcf = engine.double_conv_forward


fst = []


def dcf(mod, srcs, ctx, save):
    out = _dcf(mod, srcs, ctx, save)
    fw.append(ctx.y1.clone())
    fw.append(ctx.y2.clone())
    fst.append(ctx.st1)
    fst.append(ctx.st2)
    return out


_bw = engine._bn_relu_wgrad


def bnw(conv, bn, y, st, in_srcs, dy, grads):
    _bw(conv, bn, y, st, in_srcs, dy, grads)
    bw.append(dy.clone())


engine.double_conv_forward = dcf
engine._bn_relu_wgrad = bnw
m = getattr(ugpg, f"PGUNet{stage}")(3, 1)
m.load_state_dict(state)
m = m.to(dev).train()
out = m(x.to(dev))
crit = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([5.0], device=dev), reduction="none")
f, _ = ugpg.UncertaintyGuidedLoss(dev).apply_uncertainty_weighted_loss(crit, out, t.to(dev))
f.backward()
torch.cuda.synchronize()

print(f"stage {stage} res {res} B {B}: logits max|d| {(out.detach().cpu().double() - logits.detach()).abs().max():.3e}")
names = []
a = O.ARCH[stage]
for nm in ["inc"] + [e[0] for e in a["enc"]] + [d[0] for d in a["dec"]]:
    names += [nm + ".conv0", nm + ".conv3"]
for i, (y_o, y_g) in enumerate(zip(rec, fw)):
    yg = y_g.permute(0, 3, 1, 2).cpu().double()
    d = (yg - y_o.detach()).abs().max().item() / max(y_o.detach().abs().max().item(), 1e-30)
    print(f"fwd {names[i]:14s} y rel err {d:.2e}")
# backward order: reverse blocks, conv3 then conv0 within a block
order = []
for nm in reversed(names[::2]):
    order += [nm[:-6] + ".conv3", nm[:-6] + ".conv0"]
idx = {n: i for i, n in enumerate(names)}
for j, dy_g in enumerate(bw):
    n = order[j]
    y_o = rec[idx[n]]
    g_o = y_o.grad.double()
    dg = dy_g.permute(0, 3, 1, 2).cpu().double()
    err = (dg - g_o).abs().max().item()
    sc = g_o.abs().max().item()
    l2 = ((dg - g_o).norm() / g_o.norm()).item()
    # ReLU-mask flips of this conv's BN+ReLU between GPU and fp64 oracle
    i = idx[n]
    sc_g, sh_g = fst[i][2].cpu().double(), fst[i][3].cpu().double()
    pre_g = fw[i].cpu().double() * sc_g + sh_g
    wl = (dg - g_o).abs().flatten().argmax().item()
    print(f"bwd {n:14s} dy max-rel {err / max(sc, 1e-30):.2e} L2-rel {l2:.2e} (max|dy| {sc:.2e}) "
          f"worst-elem |pre-act| {pre_g.permute(0, 3, 1, 2).flatten()[wl].abs().item():.2e}")
named = dict(m.named_parameters())
worst = []
for k, p in P.items():
    if p.grad is None:
        continue
    e = (named[k].grad.cpu().double() - p.grad).abs().max().item() / max(p.grad.abs().max().item(), 1e-30)
    worst.append((e, k))
for e, k in sorted(worst)[-12:]:
    if ".conv_op." in k and k.endswith(".bias") and k.split(".")[-2] in ("0", "3"):
        continue
    l2 = ((named[k].grad.cpu().double() - P[k].grad).norm() / P[k].grad.norm()).item()
    print(f"grad max-rel {e:.2e} L2-rel {l2:.2e} {k}")
l2s = sorted(((named[k].grad.cpu().double() - P[k].grad).norm() / P[k].grad.norm()).item()
             for k in P if P[k].grad is not None and not (k.endswith(".bias") and ".conv_op." in k
                                                            and k.split(".")[-2] in ("0", "3")))
print("grad L2-rel: median %.2e  p90 %.2e  max %.2e" % (l2s[len(l2s) // 2], l2s[int(len(l2s) * .9)], l2s[-1]))
