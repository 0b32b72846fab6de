"""Herlev cervical-cell classifier on libugpg (BASELINE config 4; drop-in for
HerlevClassificationModel and the uncertainty-guided step of HerlevTrainer,
reference Herlev/train_herlev.py:29-121, 124-296).

Model: the PGUNet{stage} encoder (InConv + every Down except down4) runs as one
UNetGraph whose output is global-average-pooled inside the same autograd node;
the head (Dropout -> Linear 512 -> ReLU -> Dropout -> Linear 256 -> ReLU ->
Dropout -> Linear K) runs on ugpg linear/dropout kernels.  state_dict keys are the
reference's (`unet.*`, `classifier.{3,6,9}.*`).

Constructor side effect: the reference runs a probe forward of the encoder on
``torch.randn(1, 3, res, res)`` to read the feature width (train_herlev.py:59-63).
That draws from the global RNG and, the module being in train mode, moves every
encoder BatchNorm's running statistics once (num_batches_tracked = 1).  ugpg draws
the same probe image at the same point of construction (so the RNG stream and the
classifier's initial weights equal the reference's) and runs the probe on the GPU
encoder the first time the model is moved to a ROCm device -- the state_dict of a
constructed-and-moved model therefore matches the reference's.
"""
from __future__ import annotations

import json
import math
import os
from datetime import datetime

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import functional as Fn
from . import ops
from .flat import ensure_flat
from .loss import UncertaintyGuidedLoss
from .dist import (allreduce_gradients, allreduce_metrics, broadcast_buffers,
                   broadcast_parameters, overlapped_allreduce, shard_batch,
                   sync_batchnorm_from_env, world)
from .optim import Adam
from .unet import STAGE_CLASSES, STAGE_RESOLUTIONS, _LAYOUT

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
        # the reference's feature-width probe: same RNG draw, same point (train_herlev.py:59-63)
        res = STAGE_RESOLUTIONS[stage]
        self._probe = torch.randn(1, 3, res, res)
        self.classifier = nn.Sequential(
            nn.AdaptiveAvgPool2d(1), nn.Flatten(), nn.Dropout(0.5), nn.Linear(FEATURE_DIM, 512),
            nn.ReLU(), nn.Dropout(0.3), nn.Linear(512, 256), nn.ReLU(), nn.Dropout(0.2),
            nn.Linear(256, num_classes))
        if pretrained_unet_path:
            self._freeze_encoder()
        self._enc = None

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        probe = self.__dict__.get("_probe")
        if probe is not None and next(self.unet.parameters()).is_cuda:
            self._probe = None
            self._run_probe(probe)
        return out

    def load_state_dict(self, state_dict, strict=True, assign=False):
        # the reference probes before any load, so a load that sets every encoder
        # buffer supersedes the probe's BatchNorm update
        if all(f"unet.{k}" in state_dict for k, _ in self.unet.named_buffers()):
            self._probe = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def _run_probe(self, probe):
        """Encoder forward in train mode (a freshly built module's mode) on the probe
        image, no grad: BatchNorm statistics move as in the reference's constructor."""
        was = self.unet.training
        self.unet.train(True)
        with torch.no_grad():
            dev = next(self.unet.parameters()).device
            self._extract_features(probe.to(dev))
        self.unet.train(was)

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
    """HerlevTrainer (train_herlev.py:124-489): stage configs, models,
    class-weighted criterion, Adam + ReduceLROnPlateau, classifier weight transfer,
    forward pass, train/validate epochs, progressive driver with early stop."""

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
        sync_batchnorm_from_env()
        if world()[1] > 1:  # data parallel: every replica starts from rank 0's weights
            for m in self.models.values():
                broadcast_parameters(m)

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
            return self._forward_binary(output, target, prev)
        out = torch.empty(5, dtype=torch.float32, device=output.device)
        final = _CEUGFn.apply(output, target.contiguous(), prev, self.class_weights,
                              float(self.uncertainty_alpha), out)
        return output, final, out

    def _forward_binary(self, output, target, prev):
        """The reference's num_classes <= 2 branch (train_herlev.py:258-261, 266-285):
        U = 1 - 2|sigmoid(prev) - 0.5| per logit, weights 1 + alpha*U.squeeze(), per-sample
        CE times the weights under torch broadcasting, mean.  The logits are (B, <=2), so
        this tail runs as torch device ops with the reference's exact expression --
        including its broadcast (an error for 2 logits unless B <= 2, as in the
        reference).  Same 5-float metrics buffer as the fused multi-class kernel."""
        base = self.criterion(output, target)
        if prev is None:
            final, w = base, None
        else:
            u = 1.0 - 2.0 * torch.abs(torch.sigmoid(prev) - 0.5)
            w = 1.0 + self.uncertainty_alpha * u.squeeze()
            if w.dim() == 0:
                w = w.unsqueeze(0)
            final = torch.mean(F.cross_entropy(output, target, reduction="none") * w.detach())
        zero = torch.zeros((), device=output.device)
        correct = output.argmax(dim=1).eq(target.view(-1)).sum().float()
        out = torch.stack([final.detach(), base.detach(),
                           w.mean() if w is not None else zero,
                           w.std() if w is not None else zero, correct]).float()
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
        with overlapped_allreduce():  # encoder gradient buckets go out during the backward
            final.backward()
        opt.grad_scale = allreduce_gradients([p for g in opt.param_groups for p in g["params"]])
        opt.step()
        self._reduce_metrics(out, data.shape[0], stage)
        return out

    @staticmethod
    def _reduce_metrics(out, batch, stage):
        """Data parallel: [final, base] averaged over ranks, the weight mean/std pooled
        over the global batch, the correct count summed (one all-reduce)."""
        allreduce_metrics(out, 2, batch if stage > 1 else 0, 0b11)

    def _epoch(self, dataloader, stage, train):
        model = self.models[stage]
        model.train(train)
        if stage > 1:
            self.models[stage - 1].eval()
        rank, ws = world()
        if not train and ws > 1:
            broadcast_buffers(model)  # every rank validates rank 0's BatchNorm state
        tot, correct, total, skipped = [0.0] * 4, 0, 0, 0
        for batch_idx, (data, target) in enumerate(dataloader):
            part = shard_batch(dataloader, data, target, check=batch_idx == 0)
            if part is None:
                skipped += 1
                continue
            data = part[0].to(self.device, non_blocking=True).float()
            target = part[1].to(self.device, non_blocking=True)
            if train:
                out = self.train_step(data, target, stage)
            else:
                with torch.no_grad():
                    _, _, out = self._forward_device(data, target, stage)
                    self._reduce_metrics(out, data.shape[0], stage)
            v = out.tolist()
            tot = [a + b for a, b in zip(tot, (v[0], v[1], v[2] if stage > 1 else 0.0,
                                               v[3] if stage > 1 else 0.0))]
            correct += int(round(v[4]))
            total += target.shape[0] * ws
        n = max(len(dataloader) - skipped, 1)
        return tot[0] / n, tot[1] / n, 100.0 * correct / max(total, 1), tot[2] / n, tot[3] / n

    def train_epoch(self, dataloader, stage):
        return self._epoch(dataloader, stage, True)

    def validate_epoch(self, dataloader, stage):
        return self._epoch(dataloader, stage, False)


    def train_progressive(self, train_loaders, val_loaders, save_dir):
        """Stage loop of train_herlev.py:404-489: per stage a fresh Adam +
        ReduceLROnPlateau(min, 0.5, 5) stepped on the validation loss, classifier
        transfer from the previous stage, a checkpoint whenever validation accuracy
        improves, early stop after `early_stopping_patience` (15) epochs without one,
        and the history JSON at the end.  Checkpoints carry the reference's keys."""
        os.makedirs(save_dir, exist_ok=True)
        rank, _ = world()
        for stage in self.config["stages"]:
            print(f"\n{'=' * 60}")
            print(f"Training Stage {stage} - Resolution: {self.stage_configs[stage]['resolution']}")
            print(f"{'=' * 60}")
            self.current_stage = stage
            self.setup_optimizer_scheduler(stage)
            if stage > 1 and (stage - 1) in self.models:
                self.transfer_weights(stage - 1, stage)
            train_loader, val_loader = train_loaders[stage], val_loaders[stage]
            best_val_loss, best_val_acc, stale = float("inf"), 0, 0
            for epoch in range(self.stage_configs[stage]["epochs"]):
                print(f"\nStage {stage}, Epoch {epoch + 1}/{self.stage_configs[stage]['epochs']}")
                tr_loss, tr_base, tr_acc, tr_um, tr_us = self.train_epoch(train_loader, stage)
                va_loss, va_base, va_acc, va_um, va_us = self.validate_epoch(val_loader, stage)
                self.schedulers[stage].step(va_loss)
                h = self.history
                h["train_loss"].append(tr_loss)
                h["val_loss"].append(va_loss)
                h["train_acc"].append(tr_acc)
                h["val_acc"].append(va_acc)
                h["uncertainty_weights_mean"].append(va_um)
                h["uncertainty_weights_std"].append(va_us)
                h["base_loss"].append(va_base)
                print(f"Train Loss: {tr_loss:.4f}, Base Loss: {tr_base:.4f}, Train Acc: {tr_acc:.2f}%")
                print(f"Val Loss: {va_loss:.4f}, Base Loss: {va_base:.4f}, Val Acc: {va_acc:.2f}%")
                if stage > 1:
                    print(f"Train Uncertainty - Mean: {tr_um:.4f}, Std: {tr_us:.4f}")
                    print(f"Val Uncertainty - Mean: {va_um:.4f}, Std: {va_us:.4f}")
                if va_acc > best_val_acc:
                    best_val_loss, best_val_acc, stale = va_loss, va_acc, 0
                    if rank == 0:
                        torch.save({"model_state_dict": self.models[stage].state_dict(),
                                    "optimizer_state_dict": self.optimizers[stage].state_dict(),
                                    "stage": stage, "epoch": epoch + 1,
                                    "train_loss": tr_loss, "val_loss": va_loss,
                                    "train_acc": tr_acc, "val_acc": va_acc,
                                    "config": self.config},
                                   os.path.join(save_dir, f"herlev_stage{stage}_best.pth"))
                    print(f"New best model saved! Val Acc: {va_acc:.2f}%")
                else:
                    stale += 1
                if stale >= self.config.get("early_stopping_patience", 15):
                    print(f"Early stopping after {stale} epochs without improvement")
                    break
            broadcast_buffers(self.models[stage])  # the next stage's U producer: one BN state
            self.history["stage_transitions"].append(
                {"stage": stage, "completed_at": datetime.now().isoformat(),
                 "best_val_acc": best_val_acc, "best_val_loss": best_val_loss})
            print(f"Stage {stage} completed. Best Val Acc: {best_val_acc:.2f}%")
        if rank == 0:
            path = os.path.join(save_dir, "training_history.json")
            with open(path, "w") as f:
                json.dump(self.history, f, indent=2)
            print(f"Training history saved to: {path}")
