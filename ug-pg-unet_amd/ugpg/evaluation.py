"""Inference / evaluation path on the ugpg kernels.

Mirrors MoNuSegTester of MoNuSegImprove/test_monuseg.py:106-297 without its image
I/O (PIL/cv2 file reading and resizing are host data loading, out of scope):

  load_model          test_monuseg.py:120-162  checkpoint dict or raw state_dict
  predict             test_monuseg.py:164-201  sigmoid > 0.5, nearest resize back,
                                               confidence = mean probability
  evaluate_batches    test_monuseg.py:203-262  per-sample metrics, mean and std
  calculate_metrics   test_monuseg.py:264-297  iou/dice/accuracy/precision/recall/
                                               specificity, eps 1e-8

Batched on the GPU: ugpg_predict_mask (threshold + nearest resize in one pass) and
ugpg_seg_eval (per-sample counts + the float32 metric formulas in the reference's
operation order), one host synchronisation per batch.
"""
from __future__ import annotations

from typing import Dict, Iterable, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .unet import PGUNet1, PGUNet2, PGUNet3, PGUNet4

METRIC_KEYS = ("iou", "dice", "accuracy", "precision", "recall", "specificity")
_STAGE_MODELS = {1: PGUNet1, 2: PGUNet2, 3: PGUNet3, 4: PGUNet4}


def predict_masks(model: nn.Module, images: torch.Tensor, out_size=None):
    """Masks (B,1,Ho,Wo) of (sigmoid(model(images)) > 0.5), nearest-resized to
    `out_size` (default: the logits' size), and the per-sample confidence (B,)."""
    with torch.no_grad():
        logits = model(images)
    size = tuple(out_size) if out_size is not None else tuple(logits.shape[-2:])
    masks = ops.predict_mask(logits, size)
    conf = ops.seg_eval(logits, torch.zeros_like(logits))[:, 6]
    return masks, conf


def evaluate_logits(logits: torch.Tensor, gt: torch.Tensor) -> Dict[str, torch.Tensor]:
    """Per-sample metrics (device tensors of shape (B,)) of single-channel logits against
    ground-truth masks of the same shape; keys METRIC_KEYS + 'confidence'."""
    m = ops.seg_eval(logits, gt.to(logits.device, torch.float32))
    return {k: m[:, i] for i, k in enumerate(ops.EVAL_KEYS) if k != "tp"}


def calculate_metrics(pred_mask, gt_mask) -> Dict[str, float]:
    """Reference API (test_monuseg.py:264-297) on host arrays: the same numpy float32
    arithmetic; for device tensors of a whole batch use evaluate_logits."""
    pred_flat = np.asarray(pred_mask, dtype=np.float32).flatten()
    gt_flat = np.asarray(gt_mask, dtype=np.float32).flatten()
    tp = np.sum(pred_flat * gt_flat)
    fp = np.sum(pred_flat) - tp
    fn = np.sum(gt_flat) - tp
    tn = len(pred_flat) - tp - fp - fn
    eps = 1e-8
    return {"iou": (tp + eps) / (tp + fp + fn + eps),
            "dice": (2 * tp + eps) / (2 * tp + fp + fn + eps),
            "accuracy": (tp + tn + eps) / (tp + tn + fp + fn + eps),
            "precision": (tp + eps) / (tp + fp + eps),
            "recall": (tp + eps) / (tp + fn + eps),
            "specificity": (tn + eps) / (tn + fp + eps)}


class MoNuSegTester:
    """Evaluation driver with the reference's model loading and metric reporting."""

    def __init__(self, model_path: str | None = None, device="cuda", model: nn.Module | None = None):
        self.device = torch.device(device)
        if model is None and model_path is None:
            raise ValueError("MoNuSegTester needs model_path or model")
        self.model = model.to(self.device) if model is not None else self.load_model(model_path)
        self.model.eval()

    def load_model(self, model_path: str) -> nn.Module:
        """test_monuseg.py:120-162: a checkpoint dict ({'model_state_dict', 'stage', ...})
        or a raw state_dict (stage 4); tensors only (weights_only load)."""
        ckpt = torch.load(model_path, map_location="cpu", weights_only=True)
        if isinstance(ckpt, dict) and "model_state_dict" in ckpt:
            stage = int(ckpt.get("stage", 4))
            state = ckpt["model_state_dict"]
        elif isinstance(ckpt, dict) and all(isinstance(v, torch.Tensor) for v in ckpt.values()):
            stage, state = 4, ckpt
        else:
            raise RuntimeError(f"Unrecognized checkpoint format for: {model_path}")
        model = _STAGE_MODELS.get(stage, PGUNet4)(in_channels=3, num_classes=1)
        model.load_state_dict(state)
        self.stage = stage
        return model.to(self.device)

    def predict(self, images: torch.Tensor, out_size=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Batched predict_image: images (B,3,H,W) in [0,1] at the model resolution ->
        (masks (B,1,Ho,Wo) float on the device, confidence (B,))."""
        return predict_masks(self.model, images.to(self.device, torch.float32), out_size)

    def evaluate_batches(self, batches: Iterable) -> Tuple[Dict[str, float], Dict[str, float]]:
        """evaluate_dataset over (images, masks) batches: per-sample metrics, then their
        mean and (population) std, as the reference reports them."""
        per = {k: [] for k in METRIC_KEYS}
        for images, masks in batches:
            with torch.no_grad():
                logits = self.model(images.to(self.device, torch.float32))
            m = evaluate_logits(logits, masks.to(self.device).reshape(logits.shape)).copy()
            host = {k: m[k].cpu().numpy() for k in METRIC_KEYS}
            for k in METRIC_KEYS:
                per[k].extend(host[k].tolist())
        avg = {k: float(np.mean(np.asarray(v, dtype=np.float32))) for k, v in per.items()}
        std = {k: float(np.std(np.asarray(v, dtype=np.float32))) for k, v in per.items()}
        return avg, std

    calculate_metrics = staticmethod(calculate_metrics)
