"""UncertaintyGuidedProgressiveTrainer on libugpg (drop-in for
uncertainty_guided_trainer.py:25-525).

Public attributes and methods are the reference's, because subclasses such as
AugMoNuSegTrainer (MoNuSegImprove/train_aug_monuseg.py:36-121) override
``__init__`` and replace ``base_criterion``.  The per-batch hot path
(``train_epoch``: resize, forward, uncertainty map, weighted loss, backward,
RMSprop, Dice/accuracy) runs entirely in ugpg kernels and synchronises with the
host once per batch instead of the reference's six ``.item()``/``.cpu()`` calls.
"""
from __future__ import annotations

import json
import os
import time
from collections import OrderedDict
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .dist import (allreduce_gradients, allreduce_metrics, broadcast_buffers,
                   broadcast_parameters, overlapped_allreduce, shard_batch,
                   sync_batchnorm_enabled, sync_batchnorm_from_env, world)
from .graphs import StepGraph
from .loss import UncertaintyGuidedLoss, weighted_loss_tensors
from .optim import RMSprop
from .unet import PGUNet1, PGUNet2, PGUNet3, PGUNet4, ProgressiveUNet

try:  # plotting is optional, as in the reference
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    MATPLOTLIB_AVAILABLE = True
except Exception:  # pragma: no cover
    MATPLOTLIB_AVAILABLE = False


class MetricsReadback:
    """The 8-float device metrics buffer of one batch, copied to pinned host memory
    behind an event.  Reading batch k after batch k+1 has been enqueued keeps the GPU
    busy while Python prepares the next step (the host gap between a blocking
    ``.tolist()`` and the next batch's first kernel was ~0.45 ms of a 20 ms step)."""

    def __init__(self, mbuf):
        if mbuf.is_cuda:
            self.host = torch.empty(mbuf.shape, dtype=mbuf.dtype, pin_memory=True)
            self.host.copy_(mbuf, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record()
        else:
            self.host, self.event = mbuf, None

    def values(self):
        if self.event is not None:
            self.event.synchronize()
        return self.host.tolist()


class UncertaintyGuidedProgressiveTrainer:
    def __init__(self, in_channels=3, num_classes=1, device="cuda", uncertainty_alpha=1.0):
        self.device = device
        self.in_channels = in_channels
        self.num_classes = num_classes
        self.uncertainty_alpha = uncertainty_alpha
        self.stage_configs = {
            1: {"resolution": 32, "epochs_per_stage": 40, "lr": 3e-4},
            2: {"resolution": 64, "epochs_per_stage": 40, "lr": 1e-4},
            3: {"resolution": 128, "epochs_per_stage": 40, "lr": 1e-4},
            4: {"resolution": 256, "epochs_per_stage": 40, "lr": 1e-4},
        }
        self.models = {s: cls(in_channels, num_classes).to(device)
                       for s, cls in ((1, PGUNet1), (2, PGUNet2), (3, PGUNet3), (4, PGUNet4))}
        self.current_stage = 1
        self.current_model = self.models[1]
        self.uncertainty_loss = UncertaintyGuidedLoss(device)
        self.base_criterion = nn.BCEWithLogitsLoss(
            pos_weight=torch.tensor([5.0]).to(device), reduction="none")
        self.optimizer = None
        self.setup_optimizer(1)
        self.history = {k: [] for k in ("train_loss", "val_loss", "train_dice", "val_dice",
                                        "uncertainty_weights_mean", "uncertainty_weights_std",
                                        "base_loss", "stage_transitions")}
        sync_batchnorm_from_env()
        self.use_graphs = os.environ.get("UGPG_GRAPHS", "0") == "1"
        self._graphs, self._graph_warm, self.last_step_graph = OrderedDict(), [], None
        self.sync_replicas()

    def enable_graphs(self, on=True):
        """Opt-in (or UGPG_GRAPHS=1): run ``train_step`` as a replay of a captured hipGraph of
        the whole step (ugpg.graphs; bit-identical to the eager step; 1.5x the eager rate at
        bs2 x 64^2 and bs4 x 128^2, where the host's launch issue bounds the step, and equal at
        bs16 x 256^2: profiles/r6l_graph_probe.txt).  Single process only.  The first
        step of a key (shapes, stage, optimizer and its hyperparameters, the modules, the
        frozen previous stage's weights) runs eagerly, the second captures and replays,
        the rest replay; steps with the live kernel timer (bench.py's sampled roofline
        steps) run eagerly."""
        self.use_graphs = bool(on)
        self._graphs, self._graph_warm, self.last_step_graph = OrderedDict(), [], None

    # ------------------------------------------------------------ data parallel
    def sync_replicas(self, stages=None, buffers_only=False):
        """Under torch.distributed (one process per GPU) make every rank's stage models
        equal to rank 0's: parameters and buffers at construction / after loading
        weights, BatchNorm buffers before validation and at stage end.
        A no-op in a single process.  COLLECTIVE: under data parallelism every rank must
        call it (as it must call the constructor, load_stage_weights, train_epoch,
        validate_epoch and train_progressive); an ``if rank == 0:`` around any of them
        hangs the job."""
        if world()[1] <= 1:
            return
        for s in (stages or sorted(self.models)):
            (broadcast_buffers if buffers_only else broadcast_parameters)(self.models[s])

    # ------------------------------------------------------------ components
    def setup_optimizer(self, stage):
        self.optimizer = RMSprop(self.current_model.parameters(),
                                 lr=self.stage_configs[stage]["lr"], weight_decay=1e-4)
        # captured steps wrote through the old optimizer's state: never replay them
        self._drop_graphs()

    def _drop_graphs(self):
        if hasattr(self, "_graphs"):
            self._graphs.clear()
            self._graph_warm = []
            self.last_step_graph = None

    def dice_coefficient(self, pred, target, smooth=1):
        """Mean per-sample Dice (uncertainty_guided_trainer.py:90-107).  Host-side helper
        kept for API parity; the training loop uses the fused seg_metrics kernel."""
        p = pred.to(target.device).contiguous().float().view(pred.size(0), -1)
        t = target.to(p.device).contiguous().float().view(target.size(0), -1)
        inter = (p * t).sum(dim=1)
        return ((2.0 * inter + smooth) / (p.sum(dim=1) + t.sum(dim=1) + smooth)).mean()

    def get_predictions(self, output_batch):
        return (torch.sigmoid(output_batch) > 0.5).float().squeeze(1)

    def calculate_accuracy(self, pred, target):
        pred = pred.to(target.device)
        assert pred.size() == target.size()
        bs, h, w = pred.size()
        incorrect = pred.ne(target).cpu().sum().numpy()
        return 1 - incorrect / (bs * h * w)

    def transfer_weights(self, prev_stage, new_stage):
        print(f"Transferring weights from stage {prev_stage} to stage {new_stage}")
        prev_dict = self.models[prev_stage].state_dict()
        new_dict = self.models[new_stage].state_dict()
        # the reference builds a throwaway ProgressiveUNet here (uncertainty_guided_trainer.py:
        # 136); building ours on the host draws the same default-init random numbers, so the
        # global RNG -- DataLoader shuffles, augmentation seeds -- stays in step with it
        progressive_unet = ProgressiveUNet(self.in_channels, self.num_classes)
        new_state = progressive_unet.transfer_weights(prev_dict, new_dict, new_stage)
        del progressive_unet
        self.models[new_stage].load_state_dict(new_state)
        print(f"Weight transfer completed for stage {new_stage}")

    # ------------------------------------------------------------ hot path
    def _forward_device(self, data, target, stage, mbuf):
        """Forward + uncertainty map + weighted loss; results stay on the device.
        mbuf: 8-float device buffer [final, base, dice, acc, wrong, u_mean, u_std, 0]."""
        umap = None
        output = self.current_model(data)
        if stage > 1:
            umap = self.uncertainty_loss.generate_uncertainty_map(
                data, self.models[stage - 1], self.stage_configs[stage - 1]["resolution"],
                self.stage_configs[stage]["resolution"])
        final, base = weighted_loss_tensors(self.base_criterion, output, target, umap,
                                            self.uncertainty_alpha,
                                            out=mbuf[0:2] if mbuf is not None else None)
        return output, umap, final, base

    def _resize_batch(self, data, target, res):
        data = data.to(self.device, non_blocking=True).float()
        target = target.to(self.device, non_blocking=True).float()
        if data.shape[-2:] != (res, res):
            data = ops.resize_nchw(data, res, res, ops.RESIZE_BILINEAR)
        if target.shape[-2:] != (res, res):
            target = ops.resize_nchw(target, res, res, ops.RESIZE_NEAREST)
        return data.contiguous(), target.contiguous()

    def _metrics_device(self, output, target, umap, mbuf):
        if output.shape[1] != 1:
            # the reference's calculate_accuracy unpacks a 3-D prediction
            raise ValueError("too many values to unpack (expected 3)")
        ops.seg_metrics(output, target, out=mbuf[2:5])
        if umap is not None:
            ops.mean_std(umap, out=mbuf[5:7])

    def train_step(self, data, target, stage):
        """One uncertainty-guided training step on device tensors already at the
        stage resolution.  Returns the 8-float device metrics buffer (unsynced)."""
        if (self.use_graphs and data.is_cuda and world()[1] == 1 and not sync_batchnorm_enabled()
                and ops.TIMER is None):
            return self._train_step_graphed(data, target, stage)
        self.last_step_graph = None
        return self._train_step_eager(data, target, stage)

    def _graph_key(self, data, target, stage):
        """Everything a captured step bakes in besides the buffers it rewrites.  Objects
        (optimizer, modules, criterion) are held by the key itself and compare by identity,
        so a freed object's id can never match a new one; the optimizer state the
        replay writes through raw pointers (each square_avg) is keyed by storage, so
        ``optimizer.load_state_dict`` -- new state tensors -- captures again."""
        prev = self.models[stage - 1] if stage > 1 else None
        frozen = () if prev is None else tuple(
            (t.data_ptr(), t._version) for t in (*prev.parameters(), *prev.buffers()))
        groups = tuple((g["lr"], g["alpha"], g["eps"], g["weight_decay"])
                       for g in self.optimizer.param_groups)
        opt_state = tuple(
            (p.data_ptr(), st["square_avg"].data_ptr() if "square_avg" in st else None)
            for grp in self.optimizer.param_groups for p in grp["params"]
            for st in (self.optimizer.state.get(p, {}),))
        pw = getattr(self.base_criterion, "pos_weight", None)
        res = tuple(self.stage_configs[s]["resolution"] for s in (stage - 1, stage) if s >= 1)
        return (stage, tuple(data.shape), tuple(target.shape), data.dtype, target.dtype,
                str(data.device), ops.conv_math(), self.optimizer, groups, opt_state,
                self.current_model, self.current_model.training,
                tuple(p.data_ptr() for p in self.current_model.parameters()),
                None if prev is None else (prev, prev.training), frozen,
                self.uncertainty_alpha, self.base_criterion,
                None if pw is None else (pw.data_ptr(), pw._version), res)

    GRAPH_SLOTS = 2  # captured steps kept (an epoch's full batches and its last, shorter one)

    def _train_step_graphed(self, data, target, stage):
        key = self._graph_key(data, target, stage)
        g = self._graphs.get(key)
        if g is None:
            if key not in self._graph_warm:
                # the first step of a key runs eagerly: lazily built state (the frozen
                # stage's cached weight packs, the optimizer's buffers, the parameters'
                # flat layout) is then outside the capture instead of re-run by every
                # replay; the key is taken again after it
                out = self._train_step_eager(data, target, stage)
                self._graph_warm = (self._graph_warm + [self._graph_key(data, target, stage)])[-4:]
                self.last_step_graph = None
                return out
            while len(self._graphs) >= self.GRAPH_SLOTS:  # (releases a capture's pool first)
                self._graphs.pop(next(iter(self._graphs)))
            g = StepGraph(key, lambda x, t: self._train_step_eager(x, t, stage), (data, target))
            # capturing ran the step's Python side once (RMSprop's step counts, the
            # weights' version counters, the .grad tensors): the first replay is that step
            g.grads = [(p, p.grad) for grp in self.optimizer.param_groups for p in grp["params"]]
            self._graphs[key] = g
            fresh = True
        else:
            self._graphs.move_to_end(key)
            fresh = False
        out = g.replay((data, target))
        if not fresh:
            for p, gr in g.grads:  # the replay wrote these; an eager step may have swapped .grad
                p.grad = gr
            self.optimizer.replayed_step()
            # the replayed BatchNorm finalizes updated the running statistics in place (the
            # eager bn_finalize bumps their versions: eval-mode parameter caches key on them)
            ops.weights_written([b for b in self.current_model.buffers() if b.is_floating_point()])
        self.last_step_graph = g
        return out.clone()

    def _train_step_eager(self, data, target, stage):
        mbuf = torch.zeros(8, dtype=torch.float32, device=data.device)
        self.optimizer.zero_grad()
        output, umap, final, _ = self._forward_device(data, target, stage, mbuf)
        with overlapped_allreduce():  # data-parallel: buckets go to RCCL during the backward
            final.backward()
        self.optimizer.grad_scale = allreduce_gradients(
            [p for g in self.optimizer.param_groups for p in g["params"]])
        self.optimizer.step()
        self._metrics_device(output, target, umap, mbuf)
        self._reduce_metrics(mbuf, umap)
        return mbuf

    @staticmethod
    def _reduce_metrics(mbuf, umap):
        """Data parallel: [final, base, dice, acc] averaged over ranks (equal shards),
        the wrong-pixel count summed, the U mean/std pooled over the global batch."""
        allreduce_metrics(mbuf, 5, umap.numel() if umap is not None else 0, 0b1111)

    def uncertainty_guided_forward_pass(self, data, target, stage):
        mbuf = torch.zeros(8, dtype=torch.float32, device=data.device)
        output, umap, final, _ = self._forward_device(data, target, stage, mbuf)
        if umap is not None:
            ops.mean_std(umap, out=mbuf[5:7])
        v = mbuf.tolist()
        metrics = {"final_loss": v[0], "base_loss": v[1], "output": output,
                   "uncertainty_weight_mean": v[5] if umap is not None else 0.0,
                   "uncertainty_weight_std": v[6] if umap is not None else 0.0}
        return final, metrics

    def _epoch(self, dataloader, stage, train):
        model = self.current_model
        model.train(train)
        if stage > 1:
            self.models[stage - 1].eval()
        tot = np.zeros(6)
        res = self.stage_configs[stage]["resolution"]

        def consume(batch_idx, npx, rb):
            nonlocal tot
            v = rb.values()  # the one host synchronisation of the batch
            acc = 1 - v[4] / npx
            um, us = (v[5], v[6]) if stage > 1 else (0.0, 0.0)
            tot += (v[0], v[1], v[2], acc, um, us)
            if train and batch_idx % 10 == 0:
                extra = f", Unc_mean: {um:.4f}" if stage > 1 else ""
                print(f"Stage {stage}, Batch {batch_idx}, Loss: {v[0]:.4f}, Base_Loss: {v[1]:.4f}, "
                      f"Dice: {v[2]:.4f}, Acc: {acc:.4f}{extra}")

        _, ws = world()
        if not train:
            self.sync_replicas([stage], buffers_only=True)
        pending = None  # batch k is read back after batch k+1 is enqueued
        skipped = 0
        for batch_idx, (data, target) in enumerate(dataloader):
            part = shard_batch(dataloader, data, target, check=batch_idx == 0)  # this rank's rows
            if part is None:
                skipped += 1
                continue
            data, target = self._resize_batch(*part, res)
            if train:
                mbuf = self.train_step(data, target, stage)
            else:
                mbuf = torch.zeros(8, dtype=torch.float32, device=data.device)
                with torch.no_grad():
                    output, umap, _, _ = self._forward_device(data, target, stage, mbuf)
                    self._metrics_device(output, target, umap, mbuf)
                    self._reduce_metrics(mbuf, umap)
            cur = (batch_idx, data.shape[0] * ws * res * res, MetricsReadback(mbuf))
            if pending is not None:
                consume(*pending)
            pending = cur
        if pending is not None:
            consume(*pending)
        num = len(dataloader) - skipped
        avg = tot / max(num, 1)
        kind = "training" if train else "validation"
        print(f"Stage {stage} {kind} epoch completed. Batches processed: {num}")
        return tuple(float(a) for a in avg)

    def train_epoch(self, dataloader, stage):
        return self._epoch(dataloader, stage, True)

    def validate_epoch(self, dataloader, stage):
        return self._epoch(dataloader, stage, False)

    # ------------------------------------------------------------ driver
    def train_progressive(self, train_loader, val_loader, max_stages=4,
                          save_dir="./uncertainty_guided_weights"):
        save_path = Path(save_dir)
        save_path.mkdir(exist_ok=True)
        rank, _ = world()
        print("Starting Uncertainty-Guided Progressive Growing U-Net Training")
        print("=" * 60)
        for stage in range(1, max_stages + 1):
            res = self.stage_configs[stage]["resolution"]
            print(f"\nStarting Stage {stage}")
            print(f"Resolution: {res}x{res}")
            if stage > 1:
                print(f"Using uncertainty-guided loss weighting (alpha={self.uncertainty_alpha})")
            print("-" * 40)
            if stage > 1:
                self.transfer_weights(stage - 1, stage)
            self.current_stage = stage
            self.current_model = self.models[stage]
            self.setup_optimizer(stage)
            self.history["stage_transitions"].append(len(self.history["train_loss"]))
            best = 0
            epochs = self.stage_configs[stage]["epochs_per_stage"]
            for epoch in range(epochs):
                t0 = time.time()
                tr = self.train_epoch(train_loader, stage)
                va = self.validate_epoch(val_loader, stage)
                self.history["train_loss"].append(tr[0])
                self.history["val_loss"].append(va[0])
                self.history["train_dice"].append(tr[2])
                self.history["val_dice"].append(va[2])
                self.history["uncertainty_weights_mean"].append(va[4])
                self.history["uncertainty_weights_std"].append(va[5])
                self.history["base_loss"].append(va[1])
                print(f"Stage {stage}, Epoch {epoch + 1}/{epochs} ({time.time() - t0:.2f}s)")
                print(f"Train - Loss: {tr[0]:.4f}, Base: {tr[1]:.4f}, Dice: {tr[2]:.4f}, Acc: {tr[3]:.4f}")
                print(f"Val   - Loss: {va[0]:.4f}, Base: {va[1]:.4f}, Dice: {va[2]:.4f}, Acc: {va[3]:.4f}")
                if stage > 1:
                    print(f"Uncertainty - Mean: {va[4]:.4f}, Std: {va[5]:.4f}")
                # validation used rank 0's BatchNorm buffers on every rank, so the
                # checkpoint decision below is the same everywhere
                if va[2] > best:
                    best = va[2]
                    if rank == 0:
                        torch.save({"stage": stage, "epoch": epoch,
                                    "model_state_dict": self.current_model.state_dict(),
                                    "optimizer_state_dict": self.optimizer.state_dict(),
                                    "val_dice": va[2], "train_dice": tr[2],
                                    "uncertainty_alpha": self.uncertainty_alpha,
                                    "history": self.history},
                                   save_path / f"ug_pgunet_stage{stage}_best.pth")
                print("-" * 60)
            # the finished stage becomes the next stage's U-map producer: one BN state
            self.sync_replicas([stage], buffers_only=True)
        print("Uncertainty-guided progressive training completed!")
        if rank == 0:
            self.save_training_plots(save_path)

    def save_training_plots(self, save_path):
        if not MATPLOTLIB_AVAILABLE:
            print("Warning: matplotlib not available. Skipping plot generation.")
            return
        h = self.history
        ep = range(len(h["train_loss"]))
        fig, axs = plt.subplots(2, 2, figsize=(16, 12))
        axs[0, 0].plot(ep, h["train_loss"], label="Train Loss (Weighted)")
        axs[0, 0].plot(ep, h["val_loss"], label="Val Loss (Weighted)")
        axs[0, 0].plot(ep, h["base_loss"], "--", label="Base Loss (Unweighted)")
        axs[0, 1].plot(ep, h["train_dice"], label="Train Dice")
        axs[0, 1].plot(ep, h["val_dice"], label="Val Dice")
        m, s = np.array(h["uncertainty_weights_mean"]), np.array(h["uncertainty_weights_std"])
        axs[1, 0].plot(ep, m, label="Mean Uncertainty Weight")
        axs[1, 0].fill_between(ep, m - s, m + s, alpha=0.3, label="±1 Std")
        axs[1, 1].plot(ep, np.array(h["val_loss"]) - np.array(h["base_loss"]),
                       label="Loss Difference (Weighted - Base)")
        for ax in axs.flat:
            for t in h["stage_transitions"]:
                ax.axvline(x=t, color="red", linestyle="--", alpha=0.5)
            ax.legend()
        plt.tight_layout()
        plt.savefig(Path(save_path) / "uncertainty_guided_training_plots.png", dpi=100)
        plt.close(fig)

    def load_stage_weights(self, stage, checkpoint_path):
        """Load a checkpoint (dict with model_state_dict, or a raw state_dict) into
        models[stage] (uncertainty_guided_trainer.py:469-473).  COLLECTIVE under data
        parallelism: every rank calls it, then rank 0's weights are broadcast."""
        ck = torch.load(checkpoint_path, map_location=self.device, weights_only=True)
        self.models[stage].load_state_dict(ck["model_state_dict"] if "model_state_dict" in ck else ck)
        self.sync_replicas([stage])
        print(f"Loaded weights for stage {stage} from {checkpoint_path}")

    def save_uncertainty_analysis(self, data_loader, stage, save_path):
        if stage == 1:
            print("No uncertainty analysis for stage 1 (base stage)")
            return
        self.current_model.eval()
        self.models[stage - 1].eval()
        res = self.stage_configs[stage]["resolution"]
        prev_res = self.stage_configs[stage - 1]["resolution"]
        stats = []
        with torch.no_grad():
            for batch_idx, (data, target) in enumerate(data_loader):
                if batch_idx >= 10:
                    break
                data, _ = self._resize_batch(data, target, res)
                u = self.uncertainty_loss.generate_uncertainty_map(
                    data, self.models[stage - 1], prev_res, res)
                ms = ops.mean_std(u).tolist()
                stats.append({"batch_idx": batch_idx, "uncertainty_mean": ms[0],
                              "uncertainty_std": ms[1], "uncertainty_min": float(u.min()),
                              "uncertainty_max": float(u.max())})
        with open(Path(save_path) / f"uncertainty_stats_stage{stage}.json", "w") as f:
            json.dump(stats, f, indent=2)
        print(f"Uncertainty analysis saved for stage {stage}")
