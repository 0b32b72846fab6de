"""RMSprop on libugpg (drop-in for the ``optim.RMSprop(params, lr, weight_decay)``
the trainer builds at uncertainty_guided_trainer.py:81-88).

Same update rule and state layout as torch.optim.RMSprop (alpha .99, eps 1e-8,
no momentum, not centred): ``state[p] = {'step', 'square_avg'}``, so
``optimizer.state_dict()`` round-trips with reference checkpoints.  When the
parameters, their gradients and the square averages are each one contiguous
buffer (the normal case: flat.py + functional.py), a step is a single kernel
launch over all 13.4M Stage-4 parameters.
"""
from __future__ import annotations

import torch
from torch.optim import Optimizer

from . import ops
from .flat import contiguous_run


class RMSprop(Optimizer):
    def __init__(self, params, lr=1e-2, alpha=0.99, eps=1e-8, weight_decay=0, momentum=0,
                 centered=False, foreach=None, maximize=False, differentiable=False,
                 capturable=False):
        if momentum != 0 or centered or maximize or differentiable:
            raise NotImplementedError("ugpg RMSprop implements the reference configuration "
                                      "(momentum=0, centered=False)")
        defaults = dict(lr=lr, alpha=alpha, eps=eps, weight_decay=weight_decay, momentum=0,
                        centered=False, foreach=None, maximize=False, differentiable=False,
                        capturable=False)
        super().__init__(params, defaults)
        self.grad_scale = 1.0  # set by the data-parallel wrapper (1/world_size)

    def _flat_square_avg(self, params):
        """Allocate square_avg for all fresh params as one contiguous buffer."""
        fresh = [p for p in params if len(self.state[p]) == 0]
        if not fresh:
            return
        total = sum(p.numel() for p in fresh)
        buf = torch.zeros(total, dtype=torch.float32, device=fresh[0].device)
        off = 0
        for p in fresh:
            n = p.numel()
            self.state[p]["step"] = torch.tensor(0.0)
            self.state[p]["square_avg"] = buf[off:off + n].view_as(p)
            off += n

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            for p in params:
                if not p.is_cuda:
                    raise RuntimeError("ugpg RMSprop: parameters must be on the GPU")
            self._flat_square_avg(params)
            for p in params:
                self.state[p]["step"] += 1
            lr, a, eps, wd = group["lr"], group["alpha"], group["eps"], group["weight_decay"]
            runs = [contiguous_run([p for p in params]),
                    contiguous_run([p.grad for p in params]),
                    contiguous_run([self.state[p]["square_avg"] for p in params])]
            if all(r is not None for r in runs):
                (pf, _, _), (gf, _, _), (vf, _, _) = runs
                ops.rmsprop_step(pf, gf, vf, lr, a, eps, wd, self.grad_scale)
            else:
                for p in params:
                    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    ops.rmsprop_step(p.data, g, self.state[p]["square_avg"], lr, a, eps, wd,
                                     self.grad_scale)
            ops.weights_written(params)  # the kernels wrote through raw pointers
        return loss

    def replayed_step(self):
        """The host-side part of a step whose kernels ran as a graph replay
        (ugpg.graphs): step counts and the parameters' version counters."""
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            for p in params:
                self.state[p]["step"] += 1
            ops.weights_written(params)


class Adam(Optimizer):
    """torch.optim.Adam rule on libugpg (Herlev trainer, train_herlev.py:178-194);
    state layout {'step', 'exp_avg', 'exp_avg_sq'} as in torch; flat single launch
    when parameters, grads and moments are contiguous runs."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0,
                 amsgrad=False, foreach=None, maximize=False, capturable=False,
                 differentiable=False, fused=None):
        if amsgrad or maximize or differentiable:
            raise NotImplementedError("ugpg Adam implements amsgrad=False, maximize=False")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                        foreach=None, maximize=False, capturable=False, differentiable=False,
                        fused=None)
        super().__init__(params, defaults)
        self.grad_scale = 1.0

    def _init_state(self, params):
        fresh = [p for p in params if len(self.state[p]) == 0]
        if not fresh:
            return
        total = sum(p.numel() for p in fresh)
        m = torch.zeros(total, dtype=torch.float32, device=fresh[0].device)
        v = torch.zeros(total, dtype=torch.float32, device=fresh[0].device)
        off = 0
        for p in fresh:
            n = p.numel()
            self.state[p]["step"] = torch.tensor(0.0)
            self.state[p]["exp_avg"] = m[off:off + n].view_as(p)
            self.state[p]["exp_avg_sq"] = v[off:off + n].view_as(p)
            off += n

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            self._init_state(params)
            for p in params:
                self.state[p]["step"] += 1
            b1, b2 = group["betas"]
            lr, eps, wd = group["lr"], group["eps"], group["weight_decay"]
            steps = {int(self.state[p]["step"]) for p in params}
            runs = [contiguous_run(params), contiguous_run([p.grad for p in params]),
                    contiguous_run([self.state[p]["exp_avg"] for p in params]),
                    contiguous_run([self.state[p]["exp_avg_sq"] for p in params])]
            if len(steps) == 1 and all(r is not None for r in runs):
                (pf, _, _), (gf, _, _), (mf, _, _), (vf, _, _) = runs
                ops.adam_step(pf, gf, mf, vf, lr, b1, b2, eps, wd, steps.pop(), self.grad_scale)
            else:
                for p in params:
                    st = self.state[p]
                    g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
                    ops.adam_step(p.data, g, st["exp_avg"], st["exp_avg_sq"], lr, b1, b2, eps, wd,
                                  int(st["step"]), self.grad_scale)
            ops.weights_written(params)  # the kernels wrote through raw pointers
        return loss
