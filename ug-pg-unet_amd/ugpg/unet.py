"""Stage 1-4 Progressive U-Nets and ProgressiveUNet (drop-in for UG_unet.py).

Reference anchors: PGUNet1 UG_unet.py:178-193, PGUNet2 :196-223, PGUNet3
:226-260, PGUNet4 :263-304, ProgressiveUNet :307-426.  Each PGUNet runs its
whole forward/backward as one UNetGraph on libugpg kernels; the constructor
signatures, attribute names and state_dict keys are the reference's.
"""
from __future__ import annotations

from collections import OrderedDict

import torch
import torch.nn as nn

from . import functional as Fn
from . import ops
from .engine import Block, Head, UNetGraph
from .flat import ensure_flat
from .unet_parts import Down, InConv, OutConv, Up

STAGE_RESOLUTIONS = {1: 32, 2: 64, 3: 128, 4: 256}

# Per stage: InConv width; encoder Down blocks (attr, cin, cout); decoder Up
# blocks (attr, cin, cout); heads (attr, cin).  Decoder i consumes the encoder
# feature that mirrors it as the skip; head i reads decoder output i.
_LAYOUT = {
    1: (512, [("down4", 512, 512)], [("up1", 1024, 256)], ["outc"]),
    2: (256, [("down3", 256, 512), ("down4", 512, 512)],
        [("up1", 1024, 256), ("up2", 512, 128)], ["outc1", "outc2"]),
    3: (128, [("down2", 128, 256), ("down3", 256, 512), ("down4", 512, 512)],
        [("up1", 1024, 256), ("up2", 512, 128), ("up3", 256, 64)], ["outc1", "outc2", "outc3"]),
    4: (64, [("down1", 64, 128), ("down2", 128, 256), ("down3", 256, 512), ("down4", 512, 512)],
        [("up1", 1024, 256), ("up2", 512, 128), ("up3", 256, 64), ("up4", 128, 64)],
        ["outc1", "outc2", "outc3", "outc4"]),
}


class _PGUNetBase(nn.Module):
    STAGE = 0

    def __init__(self, in_channels, num_classes):
        super().__init__()
        width, enc, dec, heads = _LAYOUT[self.STAGE]
        self.inc = InConv(in_channels, width)
        for name, cin, cout in enc:
            setattr(self, name, Down(cin, cout))
        for name, cin, cout in dec:
            setattr(self, name, Up(cin, cout))
        for name, (_, _, cout) in zip(heads, dec):
            setattr(self, name, OutConv(cout, num_classes))
        self._graph_cache = None

    def graph(self) -> UNetGraph:
        if self._graph_cache is None:
            _, enc, dec, heads = _LAYOUT[self.STAGE]
            blocks = [Block(self.inc.conv, "inc")]
            for name, _, _ in enc:
                blocks.append(Block(getattr(self, name).double_conv, "down", (len(blocks) - 1,)))
            n_enc = len(blocks)  # inc + downs
            for i, (name, _, _) in enumerate(dec):
                skip = n_enc - 2 - i
                blocks.append(Block(getattr(self, name).double_conv, "up", (skip, len(blocks) - 1)))
            hd = [Head(getattr(self, name), n_enc + i) for i, name in enumerate(heads)]
            self._graph_cache = UNetGraph(blocks, hd)
        return self._graph_cache

    def encoder_graph(self, n_down: int) -> UNetGraph:
        """inc + the first `n_down` Down blocks (Herlev feature extractor)."""
        _, enc, _, _ = _LAYOUT[self.STAGE]
        blocks = [Block(self.inc.conv, "inc")]
        for name, _, _ in enc[:n_down]:
            blocks.append(Block(getattr(self, name).double_conv, "down", (len(blocks) - 1,)))
        return UNetGraph(blocks)

    def forward(self, x):
        ensure_flat(self)
        return Fn.run_logits(self.graph(), x, list(self.parameters()))

    def prepare_eval(self):
        """Build this model's persistent device state for an eval forward -- the flat
        parameter buffer, the forward weight packs and the eval-mode BatchNorm
        coefficients (all cached on the parameters / modules) -- on the current stream.
        A forward issued afterwards on another stream then only reads that state: the
        trainer runs the previous stage's U-map forward on a second stream, and state
        first created there would be allocated from, and on replacement freed to, that
        stream's pool while the other stream may still read it."""
        ensure_flat(self)
        g = self.graph()
        ops.prepack(g._pack_specs(8, False))
        g.prepare_eval_bn()


class PGUNet1(_PGUNetBase):
    """Stage 1 (32x32): inc -> down4 -> up1 -> outc (UG_unet.py:178-193)."""
    STAGE = 1


class PGUNet2(_PGUNetBase):
    """Stage 2 (64x64), two deep-supervision heads (UG_unet.py:196-223)."""
    STAGE = 2


class PGUNet3(_PGUNetBase):
    """Stage 3 (128x128), three heads (UG_unet.py:226-260)."""
    STAGE = 3


class PGUNet4(_PGUNetBase):
    """Stage 4 (256x256), four heads summed after x8/x4/x2 upsampling (UG_unet.py:263-304)."""
    STAGE = 4


STAGE_CLASSES = {1: PGUNet1, 2: PGUNet2, 3: PGUNet3, 4: PGUNet4}


class _ResizeFn(torch.autograd.Function):
    """Bilinear align-corners resize with its gather-form input gradient."""

    @staticmethod
    def forward(ctx, x, res):
        ctx.hw = x.shape[-2:]
        return ops.resize_nchw(x.detach().float().contiguous(), res, res, ops.RESIZE_BILINEAR)

    @staticmethod
    def backward(ctx, dout):
        return ops.resize_nchw_bwd(dout.contiguous(), *ctx.hw), None


def resize_input(x, res):
    """F.interpolate(x, size=(res,res), bilinear, align_corners=True) on the GPU, with
    its gradient when the input requires one (UG_unet.py:418-424)."""
    if x.shape[-2:] == (res, res):
        return x
    if x.requires_grad and torch.is_grad_enabled():
        return _ResizeFn.apply(x, res)
    return ops.resize_nchw(x.detach().float(), res, res, ops.RESIZE_BILINEAR)


def transfer_state(prev_stage_dict, current_stage_dict):
    """Name-matched (partial) copy of a previous stage's tensors (UG_unet.py:345-411).

    Exact shape -> clone; 4-D/2-D -> copy the leading [out, in] block; 1-D ->
    copy the leading entries; anything else keeps the current value."""
    new_state = OrderedDict((k, v.clone()) for k, v in current_stage_dict.items())
    copied = []
    for key, src in prev_stage_dict.items():
        dst = current_stage_dict.get(key)
        if not (torch.is_tensor(src) and torch.is_tensor(dst)):
            continue
        if src.shape == dst.shape:
            new_state[key] = src.clone()
            copied.append(key)
            continue
        if src.ndim != dst.ndim or src.ndim not in (1, 2, 4):
            continue
        lead = tuple(slice(0, min(a, b)) for a, b in zip(src.shape[:2], dst.shape[:2]))
        merged = dst.clone()
        try:
            merged[lead] = src[lead].to(merged.device, merged.dtype)
        except RuntimeError:
            continue
        new_state[key] = merged
        copied.append(key)
    return new_state, copied


class ProgressiveUNet(nn.Module):
    """All four stages with stage switching (UG_unet.py:307-426).

    Also accepts the README spelling ``ProgressiveUNet(in_channels=3,
    out_channels=2, stage=1)``."""

    def __init__(self, in_channels, num_classes=None, *, out_channels=None, stage=1):
        super().__init__()
        if num_classes is None:
            num_classes = out_channels
        if num_classes is None:
            raise TypeError("ProgressiveUNet needs num_classes (or out_channels)")
        self.in_channels = in_channels
        self.num_classes = num_classes
        self.current_stage = 1
        self.stage_resolutions = dict(STAGE_RESOLUTIONS)
        self.stage1 = PGUNet1(in_channels, num_classes)
        self.stage2 = PGUNet2(in_channels, num_classes)
        self.stage3 = PGUNet3(in_channels, num_classes)
        self.stage4 = PGUNet4(in_channels, num_classes)
        self.stages = {1: self.stage1, 2: self.stage2, 3: self.stage3, 4: self.stage4}
        if stage != 1:
            self.set_stage(stage)

    def set_stage(self, stage):
        if stage not in (1, 2, 3, 4):
            raise ValueError("Stage must be 1, 2, 3, or 4")
        self.current_stage = stage

    def get_current_resolution(self):
        return self.stage_resolutions[self.current_stage]

    def transfer_weights(self, prev_stage_dict, current_stage_dict, stage):
        new_state, copied = transfer_state(prev_stage_dict, current_stage_dict)
        print(f"transfer_weights(stage={stage}): copied {len(copied)} keys (examples: {copied[:5]})")
        return new_state

    def forward(self, x, target_resolution=None):
        res = target_resolution if target_resolution is not None else self.get_current_resolution()
        return self.stages[self.current_stage](resize_input(x, res))
