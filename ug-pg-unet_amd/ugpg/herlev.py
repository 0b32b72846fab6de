"""Herlev cervical-cell classifier on libugpg (BASELINE config 4; drop-in for
HerlevClassificationModel and the uncertainty-guided step of HerlevTrainer,
reference Herlev/train_herlev.py:29-121, 124-296).

Model: the PGUNet{stage} encoder (InConv + every Down except down4) runs as one
UNetGraph whose output is global-average-pooled inside the same autograd node;
the head (Dropout -> Linear 512 -> ReLU -> Dropout -> Linear 256 -> ReLU ->
Dropout -> Linear K) runs on ugpg linear/dropout kernels.  state_dict keys are the
reference's (`unet.*`, `classifier.{3,6,9}.*`).

Difference to the reference, documented in DESIGN.md: the reference constructor
runs a probe forward on a random image only to read the feature width (always
512 for these encoders) -- which also nudges BatchNorm running statistics and
consumes the global RNG.  ugpg sets the width statically and does not probe.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn as nn

from . import functional as Fn
from . import ops
from .flat import ensure_flat
from .loss import UncertaintyGuidedLoss
from .optim import Adam
from .unet import STAGE_CLASSES, _LAYOUT

FEATURE_DIM = 512  # output width of inc (stage 1) / down3 (stages 2-4)


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        y = ops.linear_fwd(x.contiguous(), w.detach(), b.detach(), relu)
        ctx.save_for_backward(x, w, y)
        ctx.relu = relu
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.relu:
            dy = ops.relu_bwd(y, dy)
        dx = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w)
        db = torch.empty(w.shape[0], dtype=torch.float32, device=dy.device)
        ops.linear_bwd(x.contiguous(), w.detach(), dy, dx, dw, db)
        return dx, dw, db, None


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mask):
        ctx.save_for_backward(mask)
        return ops.mul(x.contiguous(), mask)

    @staticmethod
    def backward(ctx, dy):
        (mask,) = ctx.saved_tensors
        return ops.mul(dy.contiguous(), mask), None


class _CEUGFn(torch.autograd.Function):
    """(logits, target, prev_logits, class_weights, out) -> final = out[0]; the kernel
    also fills the caller's metrics buffer out[1:5] = [base, w_mean, w_std, n_correct]."""

    @staticmethod
    def forward(ctx, logits, target, prev, class_weights, alpha, out):
        _, wts = ops.ce_ug_fwd(logits.contiguous(), target, prev, class_weights, alpha, out)
        ctx.save_for_backward(logits, target)
        ctx.wts, ctx.cw = wts, class_weights
        return out[0]

    @staticmethod
    def backward(ctx, gfinal):
        logits, target = ctx.saved_tensors
        g = gfinal.reshape(1).contiguous().float()
        return ops.ce_ug_bwd(logits, target, ctx.wts, ctx.cw, g), None, None, None, None, None


def _dropout(x, p, training):
    if not training or p == 0.0:
        return x
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())  # host RNG draw, device-side mask
    mask = ops.dropout_mask(x.numel(), p, seed, x.device).view_as(x)
    return _DropoutFn.apply(x, mask)


class HerlevClassificationModel(nn.Module):
    def __init__(self, stage: int, num_classes: int, pretrained_unet_path: str = None):
        super().__init__()
        self.stage = stage
        self.num_classes = num_classes
        self.unet = STAGE_CLASSES[stage](in_channels=3, num_classes=1)
        if pretrained_unet_path and os.path.exists(pretrained_unet_path):
            print(f"Loading pretrained U-Net weights from: {pretrained_unet_path}")
            sd = torch.load(pretrained_unet_path, map_location="cpu", weights_only=True)
            if "model_state_dict" in sd:
                sd = sd["model_state_dict"]
            self.unet.load_state_dict(sd)
        self.classifier = nn.Sequential(
            nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Dropout(0.5), nn.Linear(FEATURE_DIM, 512),
            nn.ReLU(), nn.Dropout(0.3), nn.Linear(512, 256), nn.ReLU(), nn.Dropout(0.2),
            nn.Linear(256, num_classes))
        if pretrained_unet_path:
            self._freeze_encoder()
        self._enc = None

    def _freeze_encoder(self):
        for p in self.unet.parameters():
            p.requires_grad = False

    def unfreeze_encoder(self):
        for p in self.unet.parameters():
            p.requires_grad = True

    def _encoder(self):
        if self._enc is None:
            n_down = len(_LAYOUT[self.stage][1]) - 1
            g = self.unet.encoder_graph(n_down)
            params = [p for blk in g.blocks for p in blk.mod.parameters()]
            self._enc = (g, params)
        return self._enc

    def _extract_features(self, x):
        """Encoder feature map (B, 512, h, w), as the reference helper returns it."""
        g, params = self._encoder()
        return Fn.run_act(g, x, params)

    def forward(self, x):
        ensure_flat(self)
        g, params = self._encoder()
        h = Fn.run_pooled(g, x, params)  # (B, 512): AdaptiveAvgPool2d(1) + Flatten fused
        c = self.classifier
        for drop, lin, relu in ((c[2], c[3], True), (c[5], c[6], True), (c[8], c[9], False)):
            h = _dropout(h, drop.p, self.training)
            h = _LinearFn.apply(h, lin.weight, lin.bias, relu)
        return h


class HerlevTrainer:
    """The uncertainty-guided step of HerlevTrainer (train_herlev.py:124-357):
    stage configs, models, class-weighted criterion, Adam + ReduceLROnPlateau,
    classifier weight transfer, forward pass, train/validate epochs."""

    def __init__(self, config):
        self.config = config
        self.device = config["device"]
        e = config["epochs_per_stage"]
        res4 = config.get("stage4_resolution", 224)
        self.stage_configs = {1: {"resolution": 32, "epochs": e, "lr": 3e-4},
                              2: {"resolution": 64, "epochs": e, "lr": 1e-4},
                              3: {"resolution": 128, "epochs": e, "lr": 1e-4},
                              4: {"resolution": res4, "epochs": e, "lr": 1e-4}}
        self.current_stage = 1
        self.models, self.optimizers, self.schedulers = {}, {}, {}
        for stage in range(1, 5):
            self.models[stage] = HerlevClassificationModel(
                stage, config["num_classes"],
                config.get("pretrained_unet_paths", {}).get(stage)).to(self.device)
        self.setup_loss_function()
        self.uncertainty_loss = UncertaintyGuidedLoss(self.device)
        self.uncertainty_alpha = config.get("uncertainty_alpha", 1.0)
        self.history = {k: [] for k in ("train_loss", "val_loss", "train_acc", "val_acc",
                                        "uncertainty_weights_mean", "uncertainty_weights_std",
                                        "base_loss", "stage_transitions")}

    def setup_loss_function(self):
        cw = self.config.get("class_weights")
        self.class_weights = (torch.tensor(cw, dtype=torch.float32).to(self.device)
                              if cw is not None else None)
        self.criterion = nn.CrossEntropyLoss(weight=self.class_weights)

    def setup_optimizer_scheduler(self, stage):
        model = self.models[stage]
        self.optimizers[stage] = Adam(model.parameters(), lr=self.stage_configs[stage]["lr"],
                                      weight_decay=self.config.get("weight_decay", 1e-4))
        self.schedulers[stage] = torch.optim.lr_scheduler.ReduceLROnPlateau(
            self.optimizers[stage], mode="min", factor=0.5, patience=5)

    def transfer_weights(self, prev_stage, current_stage):
        print(f"Transferring weights from stage {prev_stage} to {current_stage}")
        src, dst = self.models[prev_stage].classifier, self.models[current_stage].classifier
        with torch.no_grad():
            for (_, ps), (name, cs) in zip(src.named_parameters(), dst.named_parameters()):
                if ps.shape == cs.shape:
                    cs.copy_(ps)
                    print(f"  Transferred {name}")

    def _forward_device(self, data, target, stage):
        output = self.models[stage](data)
        prev = None
        if stage > 1:
            pm = self.models[stage - 1]
            pm.eval()
            r = self.stage_configs[stage - 1]["resolution"]
            with torch.no_grad():
                prev = pm(ops.resize_nchw(data.float().contiguous(), r, r, ops.RESIZE_BILINEAR))
        if self.config["num_classes"] <= 2:
            raise NotImplementedError("binary Herlev heads are not supported (the reference's "
                                      "binary branch mis-broadcasts the sample weights)")
        out = torch.empty(5, dtype=torch.float32, device=output.device)
        final = _CEUGFn.apply(output, target.contiguous(), prev, self.class_weights,
                              float(self.uncertainty_alpha), out)
        return output, final, out

    def uncertainty_guided_forward_pass(self, data, target, stage):
        output, final, out = self._forward_device(data, target, stage)
        v = out.tolist()
        return final, {"final_loss": v[0], "base_loss": v[1], "output": output,
                       "uncertainty_weight_mean": v[2] if stage > 1 else 0.0,
                       "uncertainty_weight_std": v[3] if stage > 1 else 0.0}

    def train_step(self, data, target, stage):
        """One step on device tensors; returns the 5-float device metrics buffer."""
        opt = self.optimizers[stage]
        opt.zero_grad()
        _, final, out = self._forward_device(data, target, stage)
        final.backward()
        from .dist import allreduce_gradients
        opt.grad_scale = allreduce_gradients([p for g in opt.param_groups for p in g["params"]])
        opt.step()
        return out

    def _epoch(self, dataloader, stage, train):
        model = self.models[stage]
        model.train(train)
        if stage > 1:
            self.models[stage - 1].eval()
        tot, correct, total = [0.0] * 4, 0, 0
        for data, target in dataloader:
            data = data.to(self.device, non_blocking=True).float()
            target = target.to(self.device, non_blocking=True)
            if train:
                out = self.train_step(data, target, stage)
            else:
                with torch.no_grad():
                    _, _, out = self._forward_device(data, target, stage)
            v = out.tolist()
            tot = [a + b for a, b in zip(tot, (v[0], v[1], v[2] if stage > 1 else 0.0,
                                               v[3] if stage > 1 else 0.0))]
            correct += int(v[4])
            total += target.shape[0]
        n = len(dataloader)
        return tot[0] / n, tot[1] / n, 100.0 * correct / total, tot[2] / n, tot[3] / n

    def train_epoch(self, dataloader, stage):
        return self._epoch(dataloader, stage, True)

    def validate_epoch(self, dataloader, stage):
        return self._epoch(dataloader, stage, False)

