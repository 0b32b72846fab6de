"""U-Net building blocks with the reference's parameter layout (drop-in for
UG_unet_parts.py).  The submodules only hold parameters/buffers so the
state_dict keys match checkpoints of the reference (``conv_op.{0,1,3,4}``,
``mpconv.1.conv_op.*``, ``conv.conv_op.*``, ``conv.{weight,bias}``); all
arithmetic runs in libugpg kernels through ``engine.UNetGraph``.

Reference anchors: DoubleConv UG_unet_parts.py:5-19, InConv :21-28,
Down :44-54, Up :70-81, OutConv :84-91.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import functional as Fn
from . import ops
from .engine import Block, UNetGraph, _grad_like


def _conv_bn_relu_layers(cin: int, cout: int):
    return [nn.Conv2d(cin, cout, kernel_size=3, padding=1), nn.BatchNorm2d(cout), nn.ReLU(inplace=True)]


def _own_params(module):
    return [p for p in module.parameters()]


class DoubleConv(nn.Module):
    """[conv3x3(pad 1, bias) -> BatchNorm2d -> ReLU] x 2 (UG_unet_parts.py:5-19)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        layers = _conv_bn_relu_layers(in_channels, out_channels)
        layers += _conv_bn_relu_layers(out_channels, out_channels)
        self.conv_op = nn.Sequential(*layers)

    def forward(self, x):
        g = UNetGraph([Block(self, "inc")])
        return Fn.run_act(g, x, _own_params(self))


class InConv(nn.Module):
    """First DoubleConv of every stage (UG_unet_parts.py:21-28)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = DoubleConv(in_channels, out_channels)

    def forward(self, x):
        return self.conv(x)


class Down(nn.Module):
    """MaxPool2d(2) then DoubleConv (UG_unet_parts.py:44-54)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.mpconv = nn.Sequential(nn.MaxPool2d(2), DoubleConv(in_channels, out_channels))

    @property
    def double_conv(self):
        return self.mpconv[1]

    def forward(self, x):
        # standalone use: the pool runs on the materialised NCHW input
        return _StandaloneDown.apply(self, x, *_own_params(self))


class Up(nn.Module):
    """bilinear x2 (align_corners=True) of x1, cat([x2, x1]), DoubleConv
    (UG_unet_parts.py:70-81).  `bilinear` is accepted and ignored, as in the reference."""

    def __init__(self, in_channels, out_channels, bilinear=True):
        super().__init__()
        self.conv = DoubleConv(in_channels, out_channels)

    @property
    def double_conv(self):
        return self.conv

    def forward(self, x1, x2):
        return _StandaloneUp.apply(self, x1, x2, *_own_params(self))


class OutConv(nn.Module):
    """1x1 convolution head (UG_unet_parts.py:84-91)."""

    def __init__(self, in_channels, out_channels):
        super().__init__()
        self.conv = nn.Conv2d(in_channels, out_channels, kernel_size=1)

    def forward(self, x):
        return _StandaloneHead.apply(self, x, self.conv.weight, self.conv.bias)


# ---------------------------------------------------------------------------
# Standalone (per-block) autograd paths: used when a user calls a block on NCHW
# tensors directly.  The PGUNet models never go through these; they run the
# whole network as one graph.
# ---------------------------------------------------------------------------

def _nhwc(x):
    return ops.nchw_to_nhwc(x.detach().float().contiguous(), x.shape[1])


def _pad_act(x_nhwc, c):
    return x_nhwc


class _StandaloneDown(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, *params):
        from .engine import BlockCtx, double_conv_forward
        xa = ops.Act(_nhwc(x))
        p, am = ops.maxpool2_fwd(xa)
        bctx = BlockCtx(srcs=[ops.Act(p)])
        out = double_conv_forward(mod.double_conv, bctx.srcs, bctx, save=True)
        y = out.materialize()
        ctx.mod, ctx.bctx, ctx.am, ctx.xshape, ctx.params = mod, bctx, am, x.shape, params
        return ops.nhwc_to_nchw(y, y.shape[-1])

    @staticmethod
    def backward(ctx, dout):
        from .engine import double_conv_backward
        from .functional import _grad_views
        need = ctx.needs_input_grad
        views = _grad_views(ctx.params, need[2:])
        grads = {p: v for p, v in zip(ctx.params, views) if v is not None}
        da = ops.nchw_to_nhwc(dout.contiguous(), dout.shape[1])
        dp = _grad_like(ctx.bctx.srcs[0].y)
        double_conv_backward(ctx.mod.double_conv, ctx.bctx, da, [dp], [0], grads)
        dx = None
        if need[1]:
            B, C, H, W = ctx.xshape
            dxn = torch.empty(B, H, W, C, dtype=torch.float32, device=dout.device)
            ops.maxpool2_bwd(dp, ctx.am, H, W, dxn, 0)
            dx = ops.nhwc_to_nchw(dxn, C)
        return (None, dx, *views)


class _StandaloneUp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x1, x2, *params):
        from .engine import BlockCtx, double_conv_forward
        low = ops.Act(_nhwc(x1))
        skip = ops.Act(_nhwc(x2))
        h, w = x1.shape[2], x1.shape[3]
        u = ops.bilinear_nhwc_fwd(low, 2 * h, 2 * w)
        bctx = BlockCtx(srcs=[skip, ops.Act(u)])
        out = double_conv_forward(mod.double_conv, bctx.srcs, bctx, save=True)
        y = out.materialize()
        ctx.mod, ctx.bctx, ctx.params = mod, bctx, params
        ctx.s1, ctx.s2 = x1.shape, x2.shape
        return ops.nhwc_to_nchw(y, y.shape[-1])

    @staticmethod
    def backward(ctx, dout):
        from .engine import double_conv_backward
        from .functional import _grad_views
        need = ctx.needs_input_grad
        views = _grad_views(ctx.params, need[3:])
        grads = {p: v for p, v in zip(ctx.params, views) if v is not None}
        da = ops.nchw_to_nhwc(dout.contiguous(), dout.shape[1])
        dskip = _grad_like(ctx.bctx.srcs[0].y)
        du = _grad_like(ctx.bctx.srcs[1].y)
        double_conv_backward(ctx.mod.double_conv, ctx.bctx, da, [dskip, du], [0, 0], grads)
        dx1 = dx2 = None
        if need[1]:
            B, C, h, w = ctx.s1
            dl = torch.empty(B, h, w, C, dtype=torch.float32, device=dout.device)
            ops.bilinear_nhwc_bwd(du, h, w, dl, 0)
            dx1 = ops.nhwc_to_nchw(dl, C)
        if need[2]:
            dx2 = ops.nhwc_to_nchw(dskip, ctx.s2[1])
        return (None, dx1, dx2, *views)


class _StandaloneHead(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mod, x, w, b):
        a = ops.Act(_nhwc(x))
        w2 = w.detach().reshape(w.shape[0], -1).contiguous()
        h = ops.head_fwd(a, w2, b.detach())
        ctx.save_for_backward(w)
        ctx.a, ctx.w2 = a, w2
        return ops.nhwc_to_nchw(h, h.shape[-1])

    @staticmethod
    def backward(ctx, dout):
        (w,) = ctx.saved_tensors
        dh = ops.nchw_to_nhwc(dout.contiguous(), dout.shape[1])
        dw = torch.empty_like(ctx.w2)
        db = torch.empty(w.shape[0], dtype=torch.float32, device=dout.device)
        da = _grad_like(ctx.a.y)
        ops.head_bwd(ctx.a, ctx.w2, dh, dw, db, da, 0)
        dx = ops.nhwc_to_nchw(da, da.shape[-1]) if ctx.needs_input_grad[1] else None
        return None, dx, dw.view_as(w), db
