"""Alias of the reference module name UG_unet (drop-in import path).

Also provides the older helper class that the reference defines in UG_unet.py
under the name UncertaintyGuidedProgressiveTrainer (UG_unet.py:97-175): a
stateless step helper, distinct from the full trainer in
ugpg.uncertainty_guided_trainer.
"""
import torch.nn as nn

from .loss import UncertaintyGuidedLoss, weighted_loss_tensors
from .unet import PGUNet1, PGUNet2, PGUNet3, PGUNet4, ProgressiveUNet  # noqa: F401
from .unet_parts import DoubleConv, Down, InConv, OutConv, Up  # noqa: F401
from . import ops


class UncertaintyGuidedProgressiveTrainer:
    """Step helper of UG_unet.py:97-175."""

    def __init__(self, device="cuda"):
        self.device = device
        self.uncertainty_loss = UncertaintyGuidedLoss(device)
        self.stage_resolutions = {1: 32, 2: 64, 3: 128, 4: 256}

    def create_uncertainty_weighted_loss_fn(self, base_loss_fn):
        if not hasattr(base_loss_fn, "reduction"):
            return base_loss_fn
        if isinstance(base_loss_fn, nn.BCEWithLogitsLoss):
            return nn.BCEWithLogitsLoss(pos_weight=base_loss_fn.pos_weight, reduction="none")
        return type(base_loss_fn)(reduction="none")

    def uncertainty_guided_forward_pass(self, data, target, current_model, prev_model, stage,
                                        loss_fn, alpha=1.0):
        output = current_model(data)
        umap = None
        if stage > 1 and prev_model is not None:
            umap = self.uncertainty_loss.generate_uncertainty_map(
                data, prev_model, self.stage_resolutions[stage - 1], self.stage_resolutions[stage])
        final, base = weighted_loss_tensors(loss_fn, output, target, umap, alpha)
        stats = ops.mean_std(umap).tolist() if umap is not None else [0.0, 0.0]
        metrics = {"final_loss": final.item(), "base_loss": base.item(),
                   "uncertainty_weight_mean": stats[0], "uncertainty_weight_std": stats[1]}
        return final, metrics
