"""CPU oracle for the UG-PG-UNet hot path (TEST INFRASTRUCTURE -- never shipped).

A functional restatement of the reference's Stage-1..4 Progressive U-Net, the
uncertainty-map fusion, the uncertainty-weighted BCE, RMSprop and the trainer
metrics, written against a flat ``{state_dict key: tensor}`` parameter dict so
that the same weights drive the reference modules, this oracle and the HIP path.
Same torch CPU ops in the same order as the reference, so on CPU it is
bit-identical to it (proved by ``oracle/make_goldens.py`` with ``torch.equal``).

Reference anchors (file:line in tridang04022004/UG-PG-UNet):
  DoubleConv          UG_unet_parts.py:5-19   conv3x3(p1,bias)->BN->ReLU, twice
  InConv / Down / Up  UG_unet_parts.py:21-28, 44-54, 70-81
  OutConv             UG_unet_parts.py:84-91
  PGUNet1..4          UG_unet.py:178-304 (deep-supervision head sum :294-303)
  ProgressiveUNet     UG_unet.py:307-426 (transfer_weights :345-411)
  uncertainty map     UG_unet.py:19-59
  weighted loss       UG_unet.py:61-94
  trainer step/metrics uncertainty_guided_trainer.py:81-256
  Herlev model/step   Herlev/train_herlev.py:29-121, 216-296
  eval metrics/masks  MoNuSegImprove/test_monuseg.py:164-297 (parity unpinned: that
                      module imports cv2 at top level, absent here, so it is restated
                      from its source; its torch calls -- sigmoid, >0.5, nearest
                      interpolate -- are the ATen CPU ops themselves)

Parity: pinned against the imported reference (goldens under tests/golden/).
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
import torch.nn.functional as F

BN_EPS = 1e-5
BN_MOMENTUM = 0.1
STAGE_RES = {1: 32, 2: 64, 3: 128, 4: 256}

# ---------------------------------------------------------------------------
# Architecture tables.  Each stage: the InConv width, the encoder (Down) blocks,
# the decoder (Up) blocks and the 1x1 heads.  Names are the state_dict prefixes.
#   encoder entry: (name, cin, cout)
#   decoder entry: (name, cin_total, cout)  -- input is cat([skip, up(prev)])
#   heads: (name, cin, decoder index)       -- summed coarsest -> finest
# ---------------------------------------------------------------------------
ARCH = {
    1: dict(inc=512, enc=[("down4", 512, 512)], dec=[("up1", 1024, 256)],
            heads=[("outc", 256, 0)]),
    2: dict(inc=256, enc=[("down3", 256, 512), ("down4", 512, 512)],
            dec=[("up1", 1024, 256), ("up2", 512, 128)],
            heads=[("outc1", 256, 0), ("outc2", 128, 1)]),
    3: dict(inc=128, enc=[("down2", 128, 256), ("down3", 256, 512), ("down4", 512, 512)],
            dec=[("up1", 1024, 256), ("up2", 512, 128), ("up3", 256, 64)],
            heads=[("outc1", 256, 0), ("outc2", 128, 1), ("outc3", 64, 2)]),
    4: dict(inc=64, enc=[("down1", 64, 128), ("down2", 128, 256), ("down3", 256, 512),
                         ("down4", 512, 512)],
            dec=[("up1", 1024, 256), ("up2", 512, 128), ("up3", 256, 64), ("up4", 128, 64)],
            heads=[("outc1", 256, 0), ("outc2", 128, 1), ("outc3", 64, 2), ("outc4", 64, 3)]),
}


def _double_conv_spec(prefix, cin, cout):
    out = []
    for ci, (conv_i, bn_i) in enumerate(((0, 1), (3, 4))):
        c_in = cin if ci == 0 else cout
        out.append((f"{prefix}.{conv_i}.weight", (cout, c_in, 3, 3), "conv"))
        out.append((f"{prefix}.{conv_i}.bias", (cout,), "bias"))
        for leaf, shp in (("weight", (cout,)), ("bias", (cout,)), ("running_mean", (cout,)),
                          ("running_var", (cout,)), ("num_batches_tracked", ())):
            out.append((f"{prefix}.{bn_i}.{leaf}", shp, "bn"))
    return out


def block_prefix(name: str) -> str:
    if name == "inc":
        return "inc.conv.conv_op"
    if name.startswith("down"):
        return f"{name}.mpconv.1.conv_op"
    return f"{name}.conv.conv_op"


def state_spec(stage: int, in_channels: int, num_classes: int, key_prefix: str = ""):
    """Ordered (key, shape, kind) list, identical to the reference state_dict order."""
    a = ARCH[stage]
    spec = _double_conv_spec(block_prefix("inc"), in_channels, a["inc"])
    for name, cin, cout in a["enc"]:
        spec += _double_conv_spec(block_prefix(name), cin, cout)
    for name, cin, cout in a["dec"]:
        spec += _double_conv_spec(block_prefix(name), cin, cout)
    for name, cin, _ in a["heads"]:
        spec.append((f"{name}.conv.weight", (num_classes, cin, 1, 1), "conv"))
        spec.append((f"{name}.conv.bias", (num_classes,), "bias"))
    return [(key_prefix + k, s, kd) for k, s, kd in spec]


# ---------------------------------------------------------------------------
# Forward building blocks
# ---------------------------------------------------------------------------

# Synchronised BatchNorm over data-parallel ranks (tests only: the CPU restatement of the
# build's optional SyncBN, ugpg.dist.enable_sync_batchnorm): None, or an exchange object
# with rank, nranks and all_reduce(t) (SUM, in place).
BN_SYNC = None


class _SyncBatchNorm(torch.autograd.Function):
    """Train-mode BatchNorm2d over the GLOBAL batch of all ranks (torch SyncBatchNorm's
    semantics; the reference's single-process BatchNorm2d over its whole batch,
    UG_unet_parts.py:11,14).  Forward: per-rank fp64 (n, mean, M2), gathered by a SUM
    all-reduce into rank rows, merged in rank order (Chan); biased variance for the
    normalisation, unbiased for the running variance.  Backward: the local (sum g,
    sum g*xhat) all-reduced, dy = w*invstd*(g - mean_all(g) - xhat*mean_all(g*xhat));
    dgamma / dbeta are local sums (the gradient all-reduce averages them)."""

    @staticmethod
    def forward(ctx, x, w, b, rm, rv, sync):
        C = x.shape[1]
        xd = x.double()
        n = xd.numel() // C
        mu = xd.mean((0, 2, 3))
        q = ((xd - mu.view(1, -1, 1, 1)) ** 2).sum((0, 2, 3))
        g = torch.zeros(sync.nranks, 3, C, dtype=torch.float64)
        g[sync.rank] = torch.stack([torch.full((C,), float(n), dtype=torch.float64), mu, q])
        sync.all_reduce(g)
        N = torch.zeros(C, dtype=torch.float64)
        m = torch.zeros(C, dtype=torch.float64)
        M2 = torch.zeros(C, dtype=torch.float64)
        for r in range(sync.nranks):
            nr, mr, qr = g[r]
            Nt = N + nr
            d = mr - m
            m = m + d * (nr / Nt)
            M2 = M2 + qr + d * d * (N * nr / Nt)
            N = Nt
        var = M2 / N
        invstd = 1.0 / torch.sqrt(var + BN_EPS)
        with torch.no_grad():
            rm.mul_(1 - BN_MOMENTUM).add_((BN_MOMENTUM * m).to(rm.dtype))
            rv.mul_(1 - BN_MOMENTUM).add_((BN_MOMENTUM * M2 / (N - 1)).to(rv.dtype))
        xhat = ((xd - m.view(1, -1, 1, 1)) * invstd.view(1, -1, 1, 1)).to(x.dtype)
        ctx.save_for_backward(xhat, invstd.to(x.dtype), w)
        ctx.sync, ctx.N = sync, N
        return xhat * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)

    @staticmethod
    def backward(ctx, go):
        xhat, invstd, w = ctx.saved_tensors
        sg = go.double().sum((0, 2, 3))
        sgx = (go.double() * xhat.double()).sum((0, 2, 3))
        s = torch.stack([sg, sgx])
        ctx.sync.all_reduce(s)
        mg, mgx = (s[0] / ctx.N).to(go.dtype), (s[1] / ctx.N).to(go.dtype)
        v = lambda t: t.view(1, -1, 1, 1)
        dx = v(w * invstd) * (go - v(mg) - xhat * v(mgx))
        return dx, sgx.to(go.dtype), sg.to(go.dtype), None, None, None


def _bn(P, pre, x, training):
    rm, rv = P[pre + ".running_mean"], P[pre + ".running_var"]
    if training:
        P[pre + ".num_batches_tracked"].add_(1)
        if BN_SYNC is not None:
            return _SyncBatchNorm.apply(x, P[pre + ".weight"], P[pre + ".bias"], rm, rv, BN_SYNC)
    return F.batch_norm(x, rm, rv, P[pre + ".weight"], P[pre + ".bias"],
                        training, BN_MOMENTUM, BN_EPS)


def _bq(t):
    """Round to bf16 (nearest even) and back."""
    return t.to(torch.bfloat16).to(t.dtype)


class _Bf16Conv3x3(torch.autograd.Function):
    """A 3x3 / pad-1 conv in the build's bf16 arithmetic (BASELINE config 3 -- not a
    reference behaviour; the reference is fp32-only): forward conv(bf16(x), bf16(w)),
    data gradient conv_T(bf16(dy), bf16(w)), weight gradient of bf16(dy) and bf16(x),
    all accumulated in fp32 (bf16 x bf16 products are exact in fp32)."""

    @staticmethod
    def forward(ctx, x, w, b):
        xq, wq = _bq(x), _bq(w)
        ctx.save_for_backward(xq, wq)
        return F.conv2d(xq, wq, b, padding=1)

    @staticmethod
    def backward(ctx, dy):
        xq, wq = ctx.saved_tensors
        dyq = _bq(dy)
        dx = torch.nn.grad.conv2d_input(xq.shape, wq, dyq, padding=1)
        dw = torch.nn.grad.conv2d_weight(xq, wq.shape, dyq, padding=1)
        return dx, dw, dy.sum(dim=(0, 2, 3))


# conv arithmetic of double_conv: "f32" (the reference) or "bf16" (the build's
# config-3 arithmetic, applied where the build runs it: 16-channel-multiple inputs)
CONV_MATH = "f32"


def conv3x3(x, w, b):
    if CONV_MATH == "bf16" and x.shape[1] % 16 == 0:
        return _Bf16Conv3x3.apply(x, w, b)
    return F.conv2d(x, w, b, padding=1)


class _Bf16StoreST(torch.autograd.Function):
    """A conv output stored in bf16 (value rounded to nearest even) whose gradient passes
    straight through: the build's bf16 arithmetic keeps conv outputs in bf16 storage and
    differentiates at the stored value, with fp32 gradients."""

    @staticmethod
    def forward(ctx, y):
        return _bq(y)

    @staticmethod
    def backward(ctx, g):
        return g


# The build's bf16 arithmetic (BASELINE config 3) stores every conv output of an image
# >= 32 wide in bf16 (ugpg.engine: torch.autocast's bf16 conv outputs): BatchNorm then sees
# -- and its statistics describe -- the rounded values.  Off only for experiments.
BF16_STORE = True


def _bf16_store(y):
    """Does the build store this conv output in bf16?"""
    return CONV_MATH == "bf16" and BF16_STORE and y.shape[-1] >= 32


class _Bf16GradRound(torch.autograd.Function):
    """Identity forward; the gradient rounded to bf16 (nearest even): the data gradient of
    a conv stored in bf16, as torch.autocast's conv backward returns grad_input."""

    @staticmethod
    def forward(ctx, x):
        return x

    @staticmethod
    def backward(ctx, g):
        return _bq(g)


# The build's bf16 arithmetic also stores the data gradient of each DoubleConv's second
# conv -- dL/d(its input), the first BatchNorm+ReLU's output gradient -- in bf16 for images
# >= 32 wide (the x6r single-piece epilogue writes da1 in bf16 with the BatchNorm-backward
# partials of the rounded values; the BN1 backward reads it).  Not in a block whose input
# is the image (inc: the 3-channel source, zero-padded to 8, is not a 64-channel multiple,
# so BN1's backward there writes an fp32 dy and the build keeps da1 fp32 too --
# ugpg.engine.double_conv_backward `da16`).  Off only for experiments.
BF16_DGRAD_STORE = True


def double_conv(P, prefix, x, training):
    """Two conv -> BN -> ReLU.  Under CONV_MATH "bf16" a conv output of an image >= 32
    wide is stored in bf16 before its BatchNorm (see _bf16_store), and so is the data
    gradient of the second conv (BF16_DGRAD_STORE) unless the block reads the image."""
    src64 = x.shape[1] % 64 == 0
    for conv_i, bn_i in ((0, 1), (3, 4)):
        if conv_i == 3 and BF16_DGRAD_STORE and src64 and _bf16_store(x):
            x = _Bf16GradRound.apply(x)
        y = conv3x3(x, P[f"{prefix}.{conv_i}.weight"], P[f"{prefix}.{conv_i}.bias"])
        if _bf16_store(y):
            y = _Bf16StoreST.apply(y)
        x = F.relu(_bn(P, f"{prefix}.{bn_i}", y, training))
    return x


def down(P, name, x, training):
    return double_conv(P, block_prefix(name), F.max_pool2d(x, 2), training)


def up(P, name, low, skip, training):
    low = F.interpolate(low, scale_factor=2, mode="bilinear", align_corners=True)
    return double_conv(P, block_prefix(name), torch.cat([skip, low], dim=1), training)


def head(P, name, x):
    return F.conv2d(x, P[f"{name}.conv.weight"], P[f"{name}.conv.bias"])


def pgunet_forward(stage: int, P, x, training: bool = True):
    """PGUNet{stage}.forward on a parameter dict (UG_unet.py:178-304)."""
    a = ARCH[stage]
    feats = [double_conv(P, block_prefix("inc"), x, training)]
    for name, _, _ in a["enc"]:
        feats.append(down(P, name, feats[-1], training))
    cur = feats[-1]
    dec_out = []
    for i, (name, _, _) in enumerate(a["dec"]):
        cur = up(P, name, cur, feats[-2 - i], training)
        dec_out.append(cur)
    out = None
    n_dec = len(dec_out)
    for name, _, di in a["heads"]:
        h = head(P, name, dec_out[di])
        factor = 2 ** (n_dec - 1 - di)
        if factor > 1:
            h = F.interpolate(h, scale_factor=factor, mode="bilinear", align_corners=True)
        out = h if out is None else out + h
    return out


def encoder_features(stage: int, P, x, training: bool = True):
    """HerlevClassificationModel._extract_features (train_herlev.py:83-102)."""
    a = ARCH[stage]
    f = double_conv(P, block_prefix("inc"), x, training)
    for name, _, _ in a["enc"][:-1]:  # every Down except down4
        f = down(P, name, f, training)
    return f


def resize_bilinear(x, res):
    return F.interpolate(x, size=(res, res), mode="bilinear", align_corners=True)


def resize_nearest(t, res):
    return F.interpolate(t, size=(res, res), mode="nearest")


# ---------------------------------------------------------------------------
# Uncertainty-guided loss (UG_unet.py:19-94)
# ---------------------------------------------------------------------------

def uncertainty_map(prev_stage: int, P_prev, x, prev_res: int, cur_res: int):
    with torch.no_grad():
        logits = pgunet_forward(prev_stage, P_prev, resize_bilinear(x, prev_res), training=False)
        prob = torch.sigmoid(logits)
        prob = resize_bilinear(prob, cur_res)
        return (1.0 - 2.0 * torch.abs(prob - 0.5)).detach()


def bce_pixel(logits, target, pos_weight):
    pw = None if pos_weight is None else torch.as_tensor([float(pos_weight)], dtype=logits.dtype)
    return F.binary_cross_entropy_with_logits(logits, target, pos_weight=pw, reduction="none")


def weighted_loss(pixel_loss, umap=None, alpha: float = 1.0):
    """Returns (final_loss tensor, base_loss float)."""
    if umap is None:
        final = torch.mean(pixel_loss)
    else:
        final = torch.mean(pixel_loss * (1.0 + alpha * umap).detach())
    return final, torch.mean(pixel_loss).item()


# Criterion variants fed to apply_uncertainty_weighted_loss (golden G3b): every
# reduction of BCEWithLogitsLoss with and without pos_weight / U, a per-channel
# pos_weight and element weight on a 2-channel output (U broadcast over channels).
LOSS_CASES = [(red, pw, use_u, a) for red in ("none", "mean", "sum") for pw in (None, 5.0)
              for use_u, a in ((False, 1.0), (True, 0.5), (True, 2.0))]
LOSS_CASES_C2 = [("none", "vec_pw"), ("mean", "vec_pw"), ("none", "weight"), ("sum", "weight")]


def loss_case_name(red, pw, use_u, alpha):
    return f"red={red},pw={pw},u={int(use_u)},a={alpha}"


def loss_case_criterion(red, pw, device="cpu"):
    import torch.nn as nn
    p = None if pw is None else torch.tensor([float(pw)], device=device)
    return nn.BCEWithLogitsLoss(pos_weight=p, reduction=red)


def loss_case_criterion_c2(red, kind, device="cpu"):
    """2-channel criteria: pos_weight (2,1,1) = [5, 2], or element weight (2,1,1) = [.7, 1.3]."""
    import torch.nn as nn
    v = torch.tensor([5.0, 2.0] if kind == "vec_pw" else [0.7, 1.3], device=device).view(2, 1, 1)
    if kind == "vec_pw":
        return nn.BCEWithLogitsLoss(pos_weight=v, reduction=red)
    return nn.BCEWithLogitsLoss(weight=v, reduction=red)


# ---------------------------------------------------------------------------
# Optimiser and metrics (uncertainty_guided_trainer.py:81-123)
# ---------------------------------------------------------------------------

def rmsprop_step(params, grads, square_avg, lr, alpha=0.99, eps=1e-8, weight_decay=1e-4):
    """torch.optim.RMSprop single-tensor rule (no momentum, not centred)."""
    with torch.no_grad():
        for k in params:
            g = grads[k]
            if weight_decay != 0:
                g = g.add(params[k], alpha=weight_decay)
            sa = square_avg[k]
            sa.mul_(alpha).addcmul_(g, g, value=1 - alpha)
            params[k].addcdiv_(g, sa.sqrt().add_(eps), value=-lr)


def predictions(logits):
    return (torch.sigmoid(logits) > 0.5).float().squeeze(1)


def dice(pred, target, smooth=1.0):
    p = pred.contiguous().float().view(pred.size(0), -1)
    t = target.contiguous().float().view(target.size(0), -1)
    inter = (p * t).sum(dim=1)
    return ((2.0 * inter + smooth) / (p.sum(dim=1) + t.sum(dim=1) + smooth)).mean()


def accuracy(pred, target):
    bs, h, w = pred.size()
    wrong = pred.ne(target).sum().item()
    return 1 - wrong / (bs * h * w)


# ---------------------------------------------------------------------------
# Progressive weight transfer (UG_unet.py:345-411)
# ---------------------------------------------------------------------------

def transfer_weights(prev_sd, cur_sd):
    """Returns (new_state, copied_keys)."""
    new = OrderedDict((k, v.clone()) for k, v in cur_sd.items())
    copied = []
    for k, src in prev_sd.items():
        if k not in cur_sd or not torch.is_tensor(src) or not torch.is_tensor(cur_sd[k]):
            continue
        dst = cur_sd[k]
        if src.shape == dst.shape:
            new[k] = src.clone()
            copied.append(k)
            continue
        if src.dim() != dst.dim() or src.dim() not in (1, 2, 4):
            continue
        t = dst.clone()
        idx = tuple(slice(0, min(a, b)) for a, b in zip(src.shape[:2], dst.shape[:2]))
        try:
            t[idx] = src[idx]
        except RuntimeError:
            continue
        new[k] = t
        copied.append(k)
    return new, copied


# ---------------------------------------------------------------------------
# One uncertainty-guided training step (uncertainty_guided_trainer.py:186-243)
# ---------------------------------------------------------------------------

def ug_train_step(stage, P_cur, P_prev, x, target, sq_avg, lr, alpha=1.0, pos_weight=5.0):
    """Returns dict with loss terms, metrics and the (pre-step) logits; updates P_cur."""
    res = STAGE_RES[stage]
    x = resize_bilinear(x, res)
    target = resize_nearest(target, res)
    params = {k: v for k, v in P_cur.items() if v.is_floating_point() and not _is_buffer(k)}
    for v in params.values():
        v.requires_grad_(True)
        v.grad = None
    logits = pgunet_forward(stage, P_cur, x, training=True)
    umap = None
    if stage > 1:
        umap = uncertainty_map(stage - 1, P_prev, x, STAGE_RES[stage - 1], res)
    final, base = weighted_loss(bce_pixel(logits, target, pos_weight), umap, alpha)
    final.backward()
    grads = {k: v.grad for k, v in params.items()}
    for v in params.values():
        v.requires_grad_(False)
    rmsprop_step(params, grads, sq_avg, lr)
    pred = predictions(logits.detach())
    tsq = target.squeeze(1)
    return dict(final_loss=final.item(), base_loss=base, logits=logits.detach(),
                dice=dice(pred, tsq).item(), acc=accuracy(pred, tsq.long()),
                unc_mean=umap.mean().item() if umap is not None else 0.0,
                unc_std=umap.std().item() if umap is not None else 0.0,
                grads=grads, umap=umap)


def _is_buffer(key: str) -> bool:
    return key.endswith(("running_mean", "running_var", "num_batches_tracked"))


# ---------------------------------------------------------------------------
# Herlev classification model (train_herlev.py:29-121, 216-296)
# ---------------------------------------------------------------------------

def herlev_head_spec(feature_dim: int, num_classes: int):
    return [("classifier.3.weight", (512, feature_dim), "linear"), ("classifier.3.bias", (512,), "bias"),
            ("classifier.6.weight", (256, 512), "linear"), ("classifier.6.bias", (256,), "bias"),
            ("classifier.9.weight", (num_classes, 256), "linear"),
            ("classifier.9.bias", (num_classes,), "bias")]


def herlev_forward(stage, P, x, training=False, dropout_masks=None):
    """unet encoder -> avgpool -> [dropout] -> 512 -> relu -> [dropout] -> 256 -> relu -> [dropout] -> K.

    `dropout_masks` (3 tensors, already scaled by 1/(1-p)) replaces the RNG so
    that train-mode parity is testable; None with training=False = eval."""
    Q = {k[len("unet."):]: v for k, v in P.items() if k.startswith("unet.")}
    f = encoder_features(stage, Q, x, training)
    h = F.adaptive_avg_pool2d(f, 1).flatten(1)
    for i, (li, act) in enumerate(((3, True), (6, True), (9, False))):
        if dropout_masks is not None:
            h = h * dropout_masks[i]
        h = F.linear(h, P[f"classifier.{li}.weight"], P[f"classifier.{li}.bias"])
        if act:
            h = F.relu(h)
    return h


def herlev_ug_loss(logits, target, prev_logits, alpha, num_classes, class_weights=None):
    """Sample-weighted CE of train_herlev.py:253-281; returns (final, base, weights)."""
    base = F.cross_entropy(logits, target, weight=class_weights)
    if prev_logits is None:
        return base, base, None
    if num_classes > 2:
        p = F.softmax(prev_logits, dim=1)
        u = -torch.sum(p * torch.log(p + 1e-8), dim=1, keepdim=True) / math.log(num_classes)
    else:
        p = torch.sigmoid(prev_logits)
        u = 1.0 - 2.0 * torch.abs(p - 0.5)
    w = (1.0 + alpha * u.squeeze())
    if w.dim() == 0:
        w = w.unsqueeze(0)
    final = torch.mean(F.cross_entropy(logits, target, reduction="none") * w.detach())
    return final, base, w


def herlev_train_step(P_cur, P_prev, x, target, opt, alpha=1.0, num_classes=7,
                      class_weights=None, prev_res=128):
    """One HerlevTrainer training step (train_herlev.py:298-325 with the UG forward pass
    :216-296): Stage-4 classifier forward in train mode (dropout 0.5/0.3/0.2 drawn from
    torch's RNG, as nn.Dropout), the Stage-3 classifier in eval mode on the input resized
    to `prev_res`, the uncertainty-weighted CE, backward, and `opt.step()` (the caller's
    torch.optim.Adam over P_cur's parameters).  The CPU-baseline workload of
    bench.py --workload herlev; returns (final, base)."""
    params = [v for k, v in P_cur.items() if v.is_floating_point() and not _is_buffer(k)]
    opt.zero_grad()
    masks = [(torch.rand(x.shape[0], n) >= p).float() / (1 - p)
             for n, p in ((512, 0.5), (512, 0.3), (256, 0.2))]
    logits = herlev_forward(4, P_cur, x, training=True, dropout_masks=masks)
    with torch.no_grad():
        prev = herlev_forward(3, P_prev, resize_bilinear(x, prev_res), training=False)
    final, base, _ = herlev_ug_loss(logits, target, prev, alpha, num_classes, class_weights)
    final.backward()
    opt.step()
    del params
    return final.item(), base.item()


# ---------------------------------------------------------------------------
# Inference / evaluation (MoNuSegImprove/test_monuseg.py)
# ---------------------------------------------------------------------------
def predict_mask(logits, size):
    """test_monuseg.py:188-195: (sigmoid > 0.5).float() then nearest resize to `size`."""
    probs = torch.sigmoid(logits)
    pred = (probs > 0.5).float()
    return F.interpolate(pred, size=size, mode="nearest"), probs


def calculate_metrics(pred_mask, gt_mask):
    """test_monuseg.py:264-297, numpy on float32 arrays (NEP 50: python scalars weak)."""
    import numpy as np
    pred_flat = np.asarray(pred_mask, dtype=np.float32).flatten()
    gt_flat = np.asarray(gt_mask, dtype=np.float32).flatten()
    intersection = np.sum(pred_flat * gt_flat)
    tp = intersection
    fp = np.sum(pred_flat) - tp
    fn = np.sum(gt_flat) - tp
    tn = len(pred_flat) - tp - fp - fn
    eps = 1e-8
    return {
        "iou": (tp + eps) / (tp + fp + fn + eps),
        "dice": (2 * tp + eps) / (2 * tp + fp + fn + eps),
        "accuracy": (tp + tn + eps) / (tp + tn + fp + fn + eps),
        "precision": (tp + eps) / (tp + fp + eps),
        "recall": (tp + eps) / (tp + fn + eps),
        "specificity": (tn + eps) / (tn + fp + eps),
    }


def evaluate_logits(logits, gt):
    """Per-sample calculate_metrics of (sigmoid(logits) > 0.5) vs gt plus the mean
    probability (test_monuseg.py:199, 244-252) -> list of dicts."""
    probs = torch.sigmoid(logits)
    pred = (probs > 0.5).float()
    out = []
    for b in range(logits.shape[0]):
        m = calculate_metrics(pred[b].numpy(), gt[b].float().numpy())
        m["confidence"] = probs[b].mean().item()
        out.append(m)
    return out
