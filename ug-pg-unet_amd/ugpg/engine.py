"""Forward/backward executor for the Progressive U-Net graph on libugpg kernels.

A network is a list of DoubleConv *blocks* (InConv / Down / Up, reference
UG_unet_parts.py:5-81) plus optional 1x1 deep-supervision *heads*
(UG_unet_parts.py:84-91, UG_unet.py:294-303).  Every block output is kept as a
lazily-activated NHWC tensor ``Act(y, scale, shift)``: the second conv's raw
output plus its folded BatchNorm affine; consumers (max-pool, bilinear x2, the
next conv, the heads) apply ``relu(scale*y+shift)`` while loading.  The
backward pass is an explicit schedule (heads -> decoder -> encoder -> inc) that
writes parameter gradients straight into caller-provided tensors (views of one
flat gradient buffer) and accumulates activation gradients in place, so no
PyTorch arithmetic runs anywhere on the path.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from . import ops
from .ops import Act


def _store16(W: int) -> bool:
    """bf16 storage of activations of an image this wide: under the bf16 arithmetic
    (config 3) every conv output, and the upsampled input of an Up conv, of an image
    >= 32 wide is kept in bf16 only (torch.autocast keeps bf16 conv outputs): its readers
    -- the next conv, max-pool, bilinear x2, the heads, BatchNorm backward, the weight
    gradient -- read half the bytes.  BatchNorm's statistics describe the stored (rounded)
    values; the oracle models it as oracle.ref_cpu.BF16_STORE."""
    return ops.conv_math() == "bf16" and W >= 32


def ceil_to(v: int, m: int) -> int:
    return (v + m - 1) // m * m


@dataclass
class Block:
    """One DoubleConv application.  kind: 'inc' (image input), 'down' (maxpool of
    inputs[0]) or 'up' (cat([inputs[0] (skip), up2x(inputs[1])]))."""
    mod: torch.nn.Module
    kind: str
    inputs: tuple = ()


@dataclass
class Head:
    mod: torch.nn.Module  # OutConv (holds .conv 1x1)
    block: int


@dataclass
class BlockCtx:
    srcs: list
    y1: torch.Tensor = None
    st1: tuple = None
    y2: torch.Tensor = None
    st2: tuple = None
    extra: dict = field(default_factory=dict)
    part2: torch.Tensor = None  # BN2-backward partials written by the last producer of da2
    route2: tuple = None  # (route, has_base): the deferred last producer of da2 (bn_relu_bwd)


def _grad_like(y):
    """An fp32 gradient buffer shaped like activation y (whatever y's storage)."""
    return torch.empty(y.shape, dtype=torch.float32, device=y.device)


def _conv_bn(seq):
    return (seq[0], seq[1]), (seq[3], seq[4])


def _bn_mode(bn):
    return bn.training or not bn.track_running_stats


def double_conv_forward(mod, srcs, ctx: BlockCtx, save: bool):
    """conv3x3 -> BN -> ReLU, twice (UG_unet_parts.py:9-16) on Act inputs."""
    B, H, W, _ = srcs[0].shape
    cin = sum(s.C for s in srcs)
    cur = srcs
    for i, (conv, bn) in enumerate(_conv_bn(mod.conv_op)):
        w = conv.weight
        cout = w.shape[0]
        if w.shape[1] > cin:
            raise ValueError(f"conv expects {w.shape[1]} input channels, got {cin}")
        wpk = ops.pack_conv3x3(w.detach(), ops.conv_pack_k(cin), 0)
        # bf16 storage: the single-piece form writes it, and the image layer's fp32 kernel
        store16 = _store16(W) and (wpk.ugpg_fmt == ops.WFMT_BF16 or (cin == 8 and cout in (64, 128)))
        y = ops.empty(B, H, W, cout, like=srcs[0].y,
                      dtype=torch.bfloat16 if store16 else torch.float32)
        train = _bn_mode(bn)
        stats = None
        ntiles = 0
        if train:
            ntiles = ops.conv_ntiles(B, H, W, cin, cout, wpk)
            stats = ops.empty(3 * cout * ntiles, like=y)
        bias = conv.bias.detach() if conv.bias is not None else None
        ops.conv3x3_fwd(cur, wpk, bias, cout, [y], stats=stats,
                        flops=2.0 * B * H * W * cout * 9 * w.shape[1])
        if train:
            if bn.momentum is None:
                raise NotImplementedError("BatchNorm2d(momentum=None) is not supported")
            track = bn.track_running_stats and bn.running_mean is not None
            mean, invstd, scale, shift = ops.bn_finalize(
                stats, ntiles, bn.weight.detach(), bn.bias.detach(),
                bn.running_mean if track else None, bn.running_var if track else None,
                bn.num_batches_tracked if track else None, float(bn.momentum), float(bn.eps))
            st = (mean, invstd, scale, shift)
        else:
            scale, shift = ops.bn_eval_params(bn.weight.detach(), bn.bias.detach(),
                                              bn.running_mean, bn.running_var, float(bn.eps),
                                              owner=bn)
            st = (None, None, scale, shift)
        if save:
            if i == 0:
                ctx.y1, ctx.st1 = y, st
            else:
                ctx.y2, ctx.st2 = y, st
        cur = [Act(y, scale, shift)]
        cin = cout
    return cur[0]


def _bn_relu_wgrad(conv, bn, y, st, in_srcs, da, grads, part=None, route=None, need_dy=True):
    """dy = dL/d(conv output) from da = dL/d(relu(bn(y))) -- in place, or, where the bf16
    arithmetic stores the activations in bf16 (y is bf16), into a bf16 tensor: exactly the
    operand its weight and data gradients read -- then dW, db.  Returns dy.
    part: BatchNorm-backward partials written by the data gradient that produced da.
    route: the deferred last producer of da (BlockCtx.route2): da holds only the base
    gradient (nothing when route[1] is false) and the apply adds the producer's gradient.
    need_dy: the caller reads the returned dy (the data gradient); else None may return."""
    mean, invstd, scale, shift = st
    if mean is None:
        raise RuntimeError("backward through an eval-mode BatchNorm is not supported")
    # the conv bias gradient (sum of dy) comes out of the BN-backward reduction
    db = grads.get(conv.bias) if conv.bias is not None else None
    dw = grads.get(conv.weight)
    co = conv.weight.shape[0]
    # the apply pass folded into the weight gradient (the plain apply, from the partials of
    # da's producer; the split-bf16 arithmetic): the finalize here, then x6w forms dy while
    # loading (da, y) and writes it once for the data gradient, bit-identical to the apply
    # (in-process A/B: fp32 step -1.0 %, profiles/r5j_ab_step_folded_bn_apply.txt; the
    # single-piece form, whose loaders already wait on loads, was 1.6 % slower with it)
    # (a deferred max-pool backward is routed into da by the x6w loader too, -0.3 %,
    # profiles/r5o_ab_step_folded_apply_pool_route.txt; the head route keeps the apply pass)
    pool = route is not None and route[0][0] == "pool"
    plain = part is not None and dw is not None and co % 64 == 0 and da.dtype == torch.float32
    fold = (route is None or pool) and plain and ops.conv_math() == "x6" and y.dtype == torch.float32
    x6w = fold and all(s.C % 64 == 0 and s.y.dtype == torch.float32 for s in in_srcs)
    # the image layer's weight gradient (conv3x3_wgrad_img_kernel) forms it as well, under
    # either arithmetic (y fp32, or bf16 under the bf16 arithmetic); its dy has no other
    # reader (in-process A/B -0.2 %, profiles/r5m_ab_step_folded_apply_img.txt)
    # (only up to 3 real input channels: conv.hip's image-layer form, WGI_NCI; a 4-8 channel
    # image padded to 8 takes the apply pass and the narrow-input weight gradient)
    img = route is None and plain and not need_dy and co == 64 and len(in_srcs) == 1 and \
        in_srcs[0].C == 8 and conv.weight.shape[1] <= 3 and in_srcs[0].scale is None and \
        in_srcs[0].y.dtype == torch.float32
    if x6w or img:
        base = da if not pool or route[1] else None
        coef = ops.bn_relu_bwd(base, y, mean, invstd, scale, shift, None, grads.get(bn.weight),
                               grads.get(bn.bias), db, part=part)
        # dy_out only when the data gradient reads it (no dead full-size write)
        dy = ops.empty(*y.shape, like=y) if x6w and need_dy else None
        ci = conv.weight.shape[1]
        ops.conv3x3_wgrad(in_srcs, ops.BnLazyDy(base, y, mean, invstd, scale, shift, coef, dy,
                                                pool=route[0][1:3] if pool else None),
                          dw, None, ci, flops=2.0 * y.numel() / co * co * 9 * ci)
        return dy
    dy = da
    if y.dtype == torch.bfloat16 and all(s.C % 64 == 0 for s in in_srcs) and \
            da.dtype != torch.bfloat16:
        dy = ops.empty(*da.shape, like=da, dtype=torch.bfloat16)
    base = da if route is None or route[1] else None
    ops.bn_relu_bwd(base, y, mean, invstd, scale, shift, dy, grads.get(bn.weight),
                    grads.get(bn.bias), db, part=part, route=None if route is None else route[0])
    if dw is not None:
        ci = conv.weight.shape[1]
        ops.conv3x3_wgrad(in_srcs, dy, dw, None, ci, flops=2.0 * dy.numel() / co * co * 9 * ci)
    return dy


def double_conv_backward(mod, ctx: BlockCtx, da2, targets, acc_flags, grads, pad_out=None):
    """Backward of one DoubleConv given dL/d(block output) `da2` (overwritten).

    targets: per input source, a tensor to receive dL/d(source activation) (or
    None); acc_flags: accumulate into it.  grads: {param: destination or None}.
    pad_out: padded channel count of a single dgrad target (the image input)."""
    (c1, b1), (c2, b2) = _conv_bn(mod.conv_op)
    B, H, W, cout = ctx.y2.shape
    a1 = Act(ctx.y1, ctx.st1[2], ctx.st1[3])
    # stage 2: BN2/ReLU backward, wgrad(conv2), dgrad(conv2) -> dL/d(a1)
    dy2 = _bn_relu_wgrad(c2, b2, ctx.y2, ctx.st2, [a1], da2, grads, part=ctx.part2,
                         route=ctx.route2)
    cmid = c2.weight.shape[1]
    npix = B * H * W
    wpk2 = ops.pack_conv3x3(c2.weight.detach(), cmid, 1)
    # the data gradient also reduces BN1's backward sums over da1 while each tile is in
    # registers (ugpg_conv_t.bnb_*), so BN1's backward is finalize + apply only
    part = bnb = None
    # (in-process A/B: -0.9 % of the step fusing every layer, -0.2 % with K >= 128 only)
    if ctx.st1[0] is not None:
        part = ops.empty(3 * cmid * ops.conv_ntiles(B, H, W, cout, cmid, wpk2), like=da2)
        bnb = (ctx.y1, *ctx.st1, part)
    # the bf16 arithmetic stores da1 in bf16 (autocast's conv backward returns a bf16
    # grad_input; oracle.ref_cpu.BF16_DGRAD_STORE), with partials of the rounded values,
    # where y1 is bf16 and BN1's apply writes a bf16 dy (sources of 64-channel multiples)
    da16 = (bnb is not None and ctx.y1.dtype == torch.bfloat16 and _store16(W)
            and wpk2.ugpg_fmt == ops.WFMT_BF16 and all(s.C % 64 == 0 for s in ctx.srcs))
    da1 = ops.empty(B, H, W, cmid, like=da2, dtype=torch.bfloat16 if da16 else torch.float32)
    ops.conv3x3_fwd([Act(dy2)], wpk2, None, cmid, [da1], flops=2.0 * npix * cmid * 9 * cout,
                    bnb=bnb)
    # stage 1: BN1/ReLU backward, wgrad(conv1), dgrad(conv1) -> source targets
    dy1 = _bn_relu_wgrad(c1, b1, ctx.y1, ctx.st1, ctx.srcs, da1, grads, part=part,
                         need_dy=any(t is not None for t in targets))
    if not any(t is not None for t in targets):
        return
    cin = c1.weight.shape[1]
    fl = 2.0 * npix * cin * 9 * cmid
    if pad_out is not None:
        wpk = ops.pack_conv3x3(c1.weight.detach(), pad_out, 1)
        ops.conv3x3_fwd([Act(dy1)], wpk, None, pad_out, [targets[0]], accumulate=(acc_flags[0], 0),
                        flops=fl)
        return
    wpk = ops.pack_conv3x3(c1.weight.detach(), cin, 1)
    if len(targets) == 1:
        ops.conv3x3_fwd([Act(dy1)], wpk, None, cin, [targets[0]], accumulate=(acc_flags[0], 0),
                        flops=fl)
    else:
        ops.conv3x3_fwd([Act(dy1)], wpk, None, cin, [targets[0], targets[1]],
                        split=ctx.srcs[0].C, accumulate=(acc_flags[0], acc_flags[1]), flops=fl)


class UNetGraph:
    """Executes blocks + heads.  `heads` empty -> the output is the last block's
    activation (encoder-only graphs, e.g. the Herlev classifier)."""

    def __init__(self, blocks, heads=()):
        self.blocks = list(blocks)
        self.heads = list(heads)

    # -------------------------------------------------------------- weight packs
    def _pack_specs(self, cpad, save):
        """(weight, K, mode) of every 3x3 pack this forward (and, when saving for the
        backward, its data gradients) will request -- the arguments double_conv_forward
        and double_conv_backward pass to ops.pack_conv3x3."""
        specs = []
        for blk in self.blocks:
            (c1, _), (c2, _) = _conv_bn(blk.mod.conv_op)
            w1, w2 = c1.weight, c2.weight  # parameters: packs are cached on them
            cin = cpad if blk.kind == "inc" else w1.shape[1]
            specs += [(w1, ops.conv_pack_k(cin), 0), (w2, ops.conv_pack_k(w2.shape[1]), 0)]
            if save:
                specs.append((w2, w2.shape[1], 1))
                if blk.kind != "inc":  # the image input gets no data gradient by default
                    specs.append((w1, w1.shape[1], 1))
        return specs

    def prepare_eval_bn(self):
        """Eval-mode BatchNorm coefficients of every block, cached on the modules (the same
        call double_conv_forward makes), computed on the current stream."""
        for blk in self.blocks:
            for _, bn in _conv_bn(blk.mod.conv_op):
                if not _bn_mode(bn):
                    ops.bn_eval_params(bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                       bn.running_var, float(bn.eps), owner=bn)

    # -------------------------------------------------------------- forward
    def forward(self, x, save: bool):
        if x.dim() != 4:
            raise ValueError(f"expected NCHW input, got shape {tuple(x.shape)}")
        packs = ops.prepack(self._pack_specs(ceil_to(x.shape[1], 8), save))
        with ops.prepacked(packs):
            logits, state = self._forward(x, save)
        if save:  # the backward needs only the data-gradient (mode 1) packs
            state["packs"] = {k: v for k, v in packs.items() if k[4] == 1}
        return logits, state

    def _forward(self, x, save: bool):
        B, cx, H, W = x.shape
        cpad = ceil_to(cx, 8)
        x0 = ops.nchw_to_nhwc(x.detach().to(torch.float32), cpad)
        outs, ctxs = [], []
        for blk in self.blocks:
            ctx = BlockCtx(srcs=[])
            if blk.kind == "inc":
                srcs = [Act(x0)]
            elif blk.kind == "down":
                a = outs[blk.inputs[0]]
                p, am = ops.maxpool2_fwd(a, bf16=_store16(a.shape[2] // 2))
                ctx.extra["argmax"] = am
                ctx.extra["in_hw"] = a.shape[1:3]
                srcs = [Act(p)]
            elif blk.kind == "up":
                skip, low = outs[blk.inputs[0]], outs[blk.inputs[1]]
                _, h, w, _ = low.shape
                u = ops.bilinear_nhwc_fwd(low, 2 * h, 2 * w, bf16=_store16(2 * w))
                if u.shape[1:3] != skip.shape[1:3]:
                    raise ValueError("Up: upsampled size does not match the skip connection")
                ctx.extra["low_hw"] = (h, w)
                srcs = [skip, Act(u)]
            else:
                raise ValueError(blk.kind)
            ctx.srcs = srcs
            outs.append(double_conv_forward(blk.mod, srcs, ctx, save))
            ctxs.append(ctx if save else None)
        state = dict(outs=outs, ctxs=ctxs, x_shape=(B, cx, H, W), cpad=cpad)
        if not self.heads:
            return outs[-1], state
        hs = []
        for hd in self.heads:
            conv = hd.mod.conv
            w = conv.weight.detach().reshape(conv.weight.shape[0], -1)
            hs.append(ops.head_fwd(outs[hd.block], w.contiguous(), conv.bias.detach()))
        fin = hs[-1]
        nc = fin.shape[-1]
        logits = ops.heads_combine(hs, B, fin.shape[1], fin.shape[2], nc)
        state["hres"] = [h.shape[1] for h in hs]
        return logits, state

    # -------------------------------------------------------------- backward
    def backward(self, state, grads, dlogits=None, dout_act=None, need_dx=False, on_done=None):
        with ops.prepacked(state.get("packs")):
            return self._backward(state, grads, dlogits, dout_act, need_dx, on_done)

    def _backward(self, state, grads, dlogits=None, dout_act=None, need_dx=False, on_done=None):
        """dlogits: NCHW gradient of the combined head output, or dout_act: NHWC
        gradient w.r.t. the last block's activation (encoder-only graphs).
        grads: {param: destination tensor or None}.  on_done(views) is called with the
        gradient views of each block (and of the heads) once they are final (the
        data-parallel reducer overlaps its all-reduce with the rest of the backward).
        Returns dx (NCHW) or None."""
        outs, ctxs = state["outs"], state["ctxs"]
        nb = len(self.blocks)
        da = [None] * nb
        # the backward walks heads, then blocks in reverse: a block's output gradient is
        # final after its lowest-indexed block consumer (or, with none, its last head),
        # which may then also reduce the block's BN2 backward sums
        first_use = {}
        for bi, blk in enumerate(self.blocks):
            for src in blk.inputs:
                first_use.setdefault(src, bi)
        last_head = {hd.block: i for i, hd in enumerate(self.heads)}

        def bn2_state(src, bi):
            c = ctxs[src]
            if first_use.get(src) != bi or c.st2 is None or c.st2[0] is None:
                return None
            return (c.y2, *c.st2)
        if self.heads:
            dhs = ops.heads_split_bwd(dlogits.contiguous(), state["hres"])
            for hi, (hd, dh) in enumerate(zip(self.heads, dhs)):
                conv = hd.mod.conv
                w = conv.weight.detach().reshape(conv.weight.shape[0], -1).contiguous()
                a = outs[hd.block]
                acc = da[hd.block] is not None
                if not acc:
                    da[hd.block] = _grad_like(a.y)
                dw = grads.get(conv.weight)
                dw_flat = dw.view(w.shape) if dw is not None else torch.empty_like(w)
                db = grads.get(conv.bias)
                c = ctxs[hd.block]
                # the last head of a block no block consumes (the top decoder block): it
                # writes only the BN2-backward partials, and the block's BN2-backward apply
                # recomputes dh @ w per pixel instead of reading a full-resolution da
                defer = (hd.block not in first_use and last_head[hd.block] == hi
                         and c.st2 is not None and c.st2[0] is not None and a.y is c.y2)
                dh = dh.contiguous()
                part = ops.head_bwd(a, w, dh, dw_flat, db, da[hd.block], acc,
                                    bnb=c.st2[:2] if defer else None, defer=defer)
                if part is not None:
                    c.part2 = part
                if defer:
                    c.route2 = (("head", dh, w), acc)
            if on_done is not None:
                on_done([grads.get(p) for hd in self.heads for p in hd.mod.parameters()])
        else:
            da[nb - 1] = dout_act
        dx0 = None
        for bi in range(nb - 1, -1, -1):
            blk, ctx, g = self.blocks[bi], ctxs[bi], da[bi]
            if g is None:
                raise RuntimeError(f"block {bi} output received no gradient")
            if blk.kind == "inc":
                if need_dx:
                    B, cx, H, W = state["x_shape"]
                    padc = ceil_to(state["cpad"], 64)
                    dx0 = ops.empty(B, H, W, padc, like=g)
                    double_conv_backward(blk.mod, ctx, g, [dx0], [0], grads, pad_out=padc)
                else:
                    double_conv_backward(blk.mod, ctx, g, [None], [0], grads)
            elif blk.kind == "down":
                src = blk.inputs[0]
                dp = _grad_like(ctx.srcs[0].y)
                double_conv_backward(blk.mod, ctx, g, [dp], [0], grads)
                H, W = ctx.extra["in_hw"]
                acc = da[src] is not None
                if not acc:
                    da[src] = _grad_like(outs[src].y)
                st = bn2_state(src, bi)
                am = ctx.extra["argmax"]
                if st is not None:
                    # the last contribution to da[src]: only its partials here; the apply of
                    # src's BN2 backward recomputes the routing (no full-resolution write:
                    # DESIGN §3, maxpool2 row)
                    ctxs[src].part2 = ops.maxpool2_bwd(dp, am, H, W, da[src], acc, bnb=st,
                                                       defer=True)
                    ctxs[src].route2 = (("pool", dp, am, H, W), acc)
                else:
                    part = ops.maxpool2_bwd(dp, am, H, W, da[src], acc, bnb=st)
                    if part is not None:
                        ctxs[src].part2 = part
            else:
                skip, low = blk.inputs
                acc_s = da[skip] is not None
                if not acc_s:
                    da[skip] = _grad_like(outs[skip].y)
                du = _grad_like(ctx.srcs[1].y)
                double_conv_backward(blk.mod, ctx, g, [da[skip], du], [acc_s, 0], grads)
                h, w = ctx.extra["low_hw"]
                acc_l = da[low] is not None
                if not acc_l:
                    da[low] = _grad_like(outs[low].y)
                part = ops.bilinear_nhwc_bwd(du, h, w, da[low], acc_l, bnb=bn2_state(low, bi))
                if part is not None:
                    ctxs[low].part2 = part
            if on_done is not None:
                on_done([grads.get(p) for p in blk.mod.parameters()])
            da[bi] = None
            ctxs[bi] = None
        if dx0 is not None:
            return ops.nhwc_to_nchw(dx0, state["x_shape"][1])
        return None
