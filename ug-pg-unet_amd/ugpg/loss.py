"""Uncertainty-map fusion and uncertainty-weighted loss (drop-in for
UncertaintyGuidedLoss, reference UG_unet.py:8-94).

generate_uncertainty_map: resize input to the previous stage's resolution,
run the previous model in eval mode, sigmoid, bilinear-resize the
probabilities back, U = 1 - 2|P - 0.5| (the last three fused in one kernel).
apply_uncertainty_weighted_loss: BCE-with-logits(pos_weight) per pixel,
weighted by (1 + alpha*U), mean -- one fused reduction kernel forward and one
elementwise kernel backward.  Criteria other than BCEWithLogitsLoss are
evaluated by the criterion itself and only the weighting/mean runs in ugpg.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import ops


def _pos_weight_tensor(loss_fn, like):
    pw = getattr(loss_fn, "pos_weight", None)
    if pw is None:
        return None
    if pw.device != like.device or pw.dtype != torch.float32:
        pw = pw.to(device=like.device, dtype=torch.float32)
    return pw.contiguous()


def _fusable_bce(loss_fn, output, target, u):
    """The fused kernel computes BCE-with-logits(pos_weight) per element with a
    scalar pos_weight and reduction='none', weighted and averaged in one pass."""
    if not isinstance(loss_fn, nn.BCEWithLogitsLoss) or loss_fn.weight is not None:
        return False
    if loss_fn.reduction != "none" or output.shape != target.shape:
        return False
    pw = getattr(loss_fn, "pos_weight", None)
    if pw is not None and pw.numel() != 1:
        return False
    return _kernel_layout(output, u)


def _kernel_layout(pixel, u):
    """(B, c, *spatial) element map with U either absent or (B, 1|c, *spatial)."""
    if pixel.dim() < 2 or pixel.numel() == 0:
        return False
    if u is None:
        return True
    return (u.dim() == pixel.dim() and u.shape[0] == pixel.shape[0]
            and u.shape[2:] == pixel.shape[2:] and u.shape[1] in (1, pixel.shape[1]))


class _UGBCEFn(torch.autograd.Function):
    """(logits, target, umap, pos_weight) -> (final, base) with d final/d logits."""

    @staticmethod
    def forward(ctx, logits, target, umap, pos_weight, alpha, out):
        logits, target = logits.contiguous(), target.contiguous().float()
        out = ops.ug_loss_fwd(logits, target, umap, pos_weight, alpha, out)
        ctx.save_for_backward(logits, target)
        ctx.umap, ctx.pw, ctx.alpha = umap, pos_weight, alpha
        final, base = out[0], out[1]
        ctx.mark_non_differentiable(base)
        return final, base

    @staticmethod
    def backward(ctx, gfinal, gbase):
        logits, target = ctx.saved_tensors
        g = gfinal.reshape(1).contiguous().float()
        dx = ops.ug_loss_bwd(logits, target, ctx.umap, ctx.pw, ctx.alpha, g)
        return dx, None, None, None, None, None


class _WeightedMeanFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pixel_loss, umap, alpha):
        pixel_loss = pixel_loss.contiguous().float()
        out = ops.weighted_mean_fwd(pixel_loss, umap, alpha)
        ctx.umap, ctx.alpha = umap, alpha
        ctx.save_for_backward(pixel_loss)
        ctx.mark_non_differentiable(out[1])
        return out[0], out[1]

    @staticmethod
    def backward(ctx, gfinal, gbase):
        (pl,) = ctx.saved_tensors
        g = gfinal.reshape(1).contiguous().float()
        return ops.weighted_mean_bwd(pl, ctx.umap, ctx.alpha, g), None, None


def weighted_loss_tensors(loss_fn, output, target, uncertainty_map=None, alpha=1.0, out=None):
    """Device-side (final_loss, base_loss) -- no host synchronisation.  `out`: optional
    2-float device buffer receiving [final, base] on every path (the trainer's metrics
    buffer reads the losses from it)."""
    final, base, filled = _weighted_loss(loss_fn, output, target, uncertainty_map, alpha, out)
    if out is not None and not filled:
        # non-fused criteria: a device-side copy, no host sync
        out[0].copy_(final.detach().reshape(()))
        out[1].copy_(base.detach().reshape(()))
    return final, base


def _weighted_loss(loss_fn, output, target, uncertainty_map, alpha, out):
    """-> (final, base, filled): only the fused BCE path writes `out` itself.

    Semantics are the reference's (UG_unet.py:78-94) for any criterion:
    ``pixel = loss_fn(output, target)``; ``final = mean(pixel * (1 + alpha*U))`` (plain
    ``mean(pixel)`` without U); ``base = mean(pixel)``.  With ``reduction='mean'|'sum'``
    the criterion already returns a scalar s, so final = s * mean(1 + alpha*U)."""
    u = None
    if uncertainty_map is not None:
        u = uncertainty_map.detach().contiguous().float()
        alpha_eff = float(alpha)
    else:
        alpha_eff = 0.0
    if _fusable_bce(loss_fn, output, target, u):
        pw = _pos_weight_tensor(loss_fn, output)
        return (*_UGBCEFn.apply(output, target, u, pw, alpha_eff, out), out is not None)
    pixel_loss = loss_fn(output, target)
    if pixel_loss.dim() == 0:
        # reduced criterion: torch.mean(s * w) == s * mean(w), w = 1 + alpha*U
        base = pixel_loss.detach()
        if u is None:
            return pixel_loss, base, False
        w_mean = 1.0 + alpha_eff * ops.mean_std(u)[0]
        return pixel_loss * w_mean, base, False
    if _kernel_layout(pixel_loss, u):
        return (*_WeightedMeanFn.apply(pixel_loss, u, alpha_eff), False)
    # any other broadcast between the criterion's output and U: the reference's
    # elementwise expression, evaluated by torch on the device
    base = torch.mean(pixel_loss.detach())
    if u is None:
        return torch.mean(pixel_loss), base, False
    return torch.mean(pixel_loss * (1.0 + alpha_eff * u)), base, False


class UncertaintyGuidedLoss:
    """Uncertainty map from the previous stage + uncertainty-weighted loss."""

    def __init__(self, device="cuda"):
        self.device = device

    def generate_uncertainty_map(self, input_current, model_prev, prev_resolution,
                                 current_resolution):
        model_prev.eval()
        with torch.no_grad():
            x = input_current.detach().float().contiguous()
            if x.shape[-2:] != (prev_resolution, prev_resolution):
                x = ops.resize_nchw(x, prev_resolution, prev_resolution, ops.RESIZE_BILINEAR)
            logits = model_prev(x)
            u = ops.resize_nchw(logits.contiguous(), current_resolution, current_resolution,
                                ops.RESIZE_UNCERTAINTY)
        return u.detach()

    def apply_uncertainty_weighted_loss(self, loss_fn, output_current, target_current,
                                        uncertainty_map=None, alpha=1.0):
        final, base = weighted_loss_tensors(loss_fn, output_current, target_current,
                                            uncertainty_map, alpha)
        return final, base.item()
