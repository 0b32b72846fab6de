"""autograd.Function bridge between nn.Module parameters and the UNetGraph executor.

One Function call covers a whole network (or a single block): forward runs the
graph on libugpg kernels and keeps the lazily-activated NHWC tensors; backward
allocates ONE flat fp32 gradient buffer laid out like the module's flat
parameter buffer (see ``flat.py``) and returns per-parameter views of it, which
autograd installs as ``p.grad`` without a copy.  The optimizer and the DP
all-reduce then work on that single buffer.
"""
from __future__ import annotations

import torch
from torch.autograd.function import once_differentiable

from . import ops
from .dist import overlap_reducer


def _check_device(x, params):
    if not x.is_cuda:
        raise RuntimeError("ugpg models run on ROCm/HIP devices only (move the model and the "
                           "input to 'cuda'); there is no CPU fallback")
    for p in params:
        if not p.is_cuda:
            raise RuntimeError("ugpg: model parameters are not on the GPU")


def _grad_views(params, needs):
    sizes = [p.numel() if n else 0 for p, n in zip(params, needs)]
    total = sum(sizes)
    flat = torch.empty(max(total, 1), dtype=torch.float32, device=params[0].device)
    views, off = [], 0
    for p, n, s in zip(params, needs, sizes):
        if n:
            views.append(flat[off:off + s].view_as(p))
            off += s
        else:
            views.append(None)
    return views


def _flat_of(views):
    """The 1-D flat buffer behind the gradient views of _grad_views."""
    v = next(t for t in views if t is not None)
    st = v.untyped_storage()
    return torch.empty(0, dtype=torch.float32, device=v.device).set_(
        st, 0, (st.nbytes() // 4,), (1,))


class _LogitsFn(torch.autograd.Function):
    """x (NCHW) -> combined deep-supervision logits (NCHW)."""

    @staticmethod
    def forward(ctx, graph, x, *params):
        logits, state = graph.forward(x, save=True)
        ctx.graph, ctx.state, ctx.params = graph, state, params
        return logits

    @staticmethod
    @once_differentiable
    def backward(ctx, dlogits):
        need = ctx.needs_input_grad
        views = _grad_views(ctx.params, need[2:])
        grads = {p: v for p, v in zip(ctx.params, views) if v is not None}
        red = overlap_reducer()
        if red is not None and grads:
            red.begin(_flat_of(views), list(grads.values()))
        dx = ctx.graph.backward(ctx.state, grads, dlogits=dlogits.contiguous(), need_dx=need[1],
                                on_done=red.done if red is not None and grads else None)
        if red is not None and grads:
            red.flush()
        ctx.state = None
        return (None, dx, *views)


class _PooledFeaturesFn(torch.autograd.Function):
    """x (NCHW) -> global-average-pooled last-block features (B, C) (Herlev encoder)."""

    @staticmethod
    def forward(ctx, graph, x, *params):
        act, state = graph.forward(x, save=True)
        feats = ops.avgpool_fwd(act)
        ctx.graph, ctx.state, ctx.params = graph, state, params
        ctx.act_shape = act.shape
        return feats

    @staticmethod
    @once_differentiable
    def backward(ctx, dfeat):
        need = ctx.needs_input_grad
        views = _grad_views(ctx.params, need[2:])
        grads = {p: v for p, v in zip(ctx.params, views) if v is not None}
        B, H, W, C = ctx.act_shape
        da = torch.empty(B, H, W, C, dtype=torch.float32, device=dfeat.device)
        ops.avgpool_bwd(dfeat.contiguous(), H, W, da)
        red = overlap_reducer()
        if red is not None and grads:
            red.begin(_flat_of(views), list(grads.values()))
        dx = ctx.graph.backward(ctx.state, grads, dout_act=da, need_dx=need[1],
                                on_done=red.done if red is not None and grads else None)
        if red is not None and grads:
            red.flush()
        ctx.state = None
        return (None, dx, *views)


class _ActOutFn(torch.autograd.Function):
    """x (NCHW) -> last block activation materialised as NCHW (standalone blocks)."""

    @staticmethod
    def forward(ctx, graph, x, *params):
        act, state = graph.forward(x, save=True)
        y = act.materialize()
        out = ops.nhwc_to_nchw(y, y.shape[-1])
        ctx.graph, ctx.state, ctx.params = graph, state, params
        return out

    @staticmethod
    @once_differentiable
    def backward(ctx, dout):
        need = ctx.needs_input_grad
        views = _grad_views(ctx.params, need[2:])
        grads = {p: v for p, v in zip(ctx.params, views) if v is not None}
        da = ops.nchw_to_nhwc(dout.contiguous(), dout.shape[1])
        dx = ctx.graph.backward(ctx.state, grads, dout_act=da, need_dx=need[1])
        ctx.state = None
        return (None, dx, *views)


def _run(fn, graph, x, params, no_grad_out):
    _check_device(x, params)
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        return fn.apply(graph, x, *params)
    out, _ = graph.forward(x, save=False)
    return no_grad_out(out)


def run_logits(graph, x, params):
    return _run(_LogitsFn, graph, x, params, lambda o: o)


def run_pooled(graph, x, params):
    return _run(_PooledFeaturesFn, graph, x, params, ops.avgpool_fwd)


def run_act(graph, x, params):
    def mat(act):
        y = act.materialize()
        return ops.nhwc_to_nchw(y, y.shape[-1])
    return _run(_ActOutFn, graph, x, params, mat)
