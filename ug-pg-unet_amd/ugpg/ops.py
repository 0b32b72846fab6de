"""Tensor-level wrappers over the libugpg C-ABI (one function per entry point).

PyTorch is used only for device memory (the caching allocator) and the current
HIP stream; every arithmetic op below runs in a hand-written gfx950 kernel.
Activations are NHWC fp32 ``(B, H, W, C)`` tensors.
"""
from __future__ import annotations

import ctypes as C
import os

import torch

from ._C import Bnb, BnLazy, BwdRoute, ConvDesc, PackItem, Src, WgradDesc, check, lib

F32 = torch.float32


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("ugpg: tensor is not on a ROCm/HIP device (no CPU fallback)")
    if not t.is_contiguous():
        raise RuntimeError("ugpg: tensor must be contiguous")
    return t.data_ptr()


def _f32(t):
    if t.dtype != F32:
        raise TypeError(f"ugpg: expected float32, got {t.dtype}")
    return ptr(t)


def empty(*shape, like=None, device=None, dtype=F32):
    dev = device if device is not None else like.device
    return torch.empty(*shape, dtype=dtype, device=dev)


def _yargs(y):
    """(fp32 pointer, bf16 pointer) of a BatchNorm input stored in either precision."""
    return (None, ptr(y)) if y.dtype == torch.bfloat16 else (ptr(y), None)


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


class Act:
    """A lazily-activated NHWC tensor: value = relu(scale*y + shift) when scale is set.

    BatchNorm + ReLU of a DoubleConv (UG_unet_parts.py:11-12) is folded into the
    consumer's load, so the normalised activation is never written to HBM.  y is fp32,
    or bf16 under the bf16 arithmetic (the storage of conv outputs of images >= 32 wide:
    ugpg_src_t.data_bf16)."""
    __slots__ = ("y", "scale", "shift")

    def __init__(self, y, scale=None, shift=None):
        self.y, self.scale, self.shift = y, scale, shift

    @property
    def shape(self):
        return tuple(self.y.shape)

    @property
    def C(self):
        return self.y.shape[-1]

    def src(self) -> Src:
        y, y16 = _yargs(self.y)
        return Src(y, ptr(self.scale), ptr(self.shift), self.C, y16)

    def materialize(self) -> torch.Tensor:
        if self.scale is None and self.y.dtype == F32:
            return self.y
        out = torch.empty(self.y.shape, dtype=F32, device=self.y.device)
        check(lib.ugpg_bn_relu_apply(self.src(), self.y.numel() // self.C, ptr(out), stream()),
              "bn_relu_apply")
        return out


NULL_SRC = Src(None, None, None, 0, None)


# ------------------------------------------------------------------ conv
WFMT_F32, WFMT_X6, WFMT_BF16 = 0, 1, 2
_MATHS = ("x6", "f32", "bf16")
_MATH_FMT = {"x6": WFMT_X6, "bf16": WFMT_BF16, "f32": WFMT_F32}
_conv_math = os.environ.get("UGPG_CONV_MATH", "x6")
if _conv_math not in _MATHS:
    raise ValueError(f"UGPG_CONV_MATH must be one of {_MATHS}, got {_conv_math!r}")


def set_conv_math(math: str) -> None:
    """'x6': split-bf16 MFMA (fp32-accurate, 2.67x the fp32 MFMA rate) wherever the
    shape allows; 'f32': v_mfma_f32_32x32x2_f32 everywhere; 'bf16': bf16 arithmetic
    (operands rounded to bf16, fp32 accumulation and storage -- BASELINE config 3)
    wherever the shape allows, fp32 MFMA elsewhere (the 3-channel image layer)."""
    global _conv_math
    if math not in _MATHS:
        raise ValueError(f"conv math must be one of {_MATHS}")
    _conv_math = math


def conv_math() -> str:
    return _conv_math


def conv_weight_format(n: int, k: int) -> int:
    """Pack format for a conv GEMM with N output columns and K input channels."""
    fmt = _MATH_FMT[_conv_math]
    return fmt if n % 64 == 0 and k % 16 == 0 else WFMT_F32


def conv_pack_k(cin: int) -> int:
    """K the forward weights are packed with for `cin` source channels: an 8-channel
    source (the padded image) is zero-extended by the split-bf16 kernels to one
    16-channel chunk, so under math x6 its weights are packed with K = 16 (fp32-class
    like every x6 conv).  Math bf16 keeps the image layer in fp32 (its weight gradient
    is the fp32 narrow-input kernel; §3b)."""
    return 16 if cin == 8 and _conv_math == "x6" else cin


# packs made ahead for the running forward/backward (see prepack / UNetGraph); a miss
# (or None) packs on the spot, so the table only saves launches, never changes results
_PREPACK = None


def _pack_key(w, cin_pad, mode):
    return (w.data_ptr(), w._version, tuple(w.shape), int(cin_pad), int(mode), _conv_math)


def _cache_key(cin_pad, mode):
    return (int(cin_pad), int(mode), _conv_math)


def prepack(specs):
    """Pack many (parameter, cin_pad, mode) in one launch (split-bf16 formats only);
    returns {key: packed} for pack_conv3x3 to consult while the table is active.

    Packs persist on the parameter (``_ugpg_packs``), keyed by its storage address and
    version counter: a weight that has not changed since its last pack -- the frozen
    previous stage that produces the uncertainty map -- is not repacked every step.
    Every writer of parameters bumps the version (ugpg's optimizers, broadcasts,
    load_state_dict), so a stale pack is never used."""
    table = {}
    if _conv_math not in ("x6", "bf16") or not specs:
        return table
    items, outs = [], []
    for p, cin_pad, mode in specs:
        w = p.detach()
        cout, cin = w.shape[0], w.shape[1]
        fmt = conv_weight_format(cout, cin_pad) if mode == 0 else conv_weight_format(cin_pad, cout)
        if fmt != _MATH_FMT[_conv_math] or not w.is_contiguous() or w.dtype != F32:
            continue
        key = _pack_key(w, cin_pad, mode)
        if key in table:
            continue
        cache = p.__dict__.setdefault("_ugpg_packs", {}) if isinstance(p, torch.nn.Parameter) else {}
        hit = cache.get(_cache_key(cin_pad, mode))
        if hit is not None and hit[0] == key:
            table[key] = hit[1]
            continue
        out = torch.empty(lib.ugpg_pack_conv3x3_bytes(cout, cin_pad, fmt), dtype=torch.uint8,
                          device=w.device)
        out.ugpg_fmt = fmt
        table[key] = out
        cache[_cache_key(cin_pad, mode)] = (key, out)
        items.append(PackItem(ptr(w), ptr(out), cout, cin, int(cin_pad), int(mode)))
        outs.append(out)
    if items:
        arr = (PackItem * len(items))(*items)
        check(lib.ugpg_pack_conv3x3_batch(arr, len(items), _MATH_FMT[_conv_math], stream()),
              "pack_conv3x3_batch")
    return table


def weights_written(params):
    """Record an in-place write to `params` that bypassed autograd (raw-pointer kernels,
    collectives): bump their version counters so cached packs are not reused."""
    from torch.autograd.graph import increment_version
    increment_version([p for p in params])


class prepacked:
    """Context manager: make `table` visible to pack_conv3x3 (restores the previous)."""

    def __init__(self, table):
        self.table = table

    def __enter__(self):
        global _PREPACK
        self.prev, _PREPACK = _PREPACK, self.table
        return self.table

    def __exit__(self, *exc):
        global _PREPACK
        _PREPACK = self.prev
        return False


def pack_conv3x3(w, cin_pad: int, mode: int) -> torch.Tensor:
    """Repack OIHW weights for conv3x3_fwd (mode 0) or its data gradient (mode 1).
    The result carries its pack format in ``.ugpg_fmt``."""
    if _PREPACK:
        hit = _PREPACK.get(_pack_key(w, cin_pad, mode))
        if hit is not None:
            return hit
    cout, cin = w.shape[0], w.shape[1]
    fmt = conv_weight_format(cout, cin_pad) if mode == 0 else conv_weight_format(cin_pad, cout)
    out = torch.empty(lib.ugpg_pack_conv3x3_bytes(cout, cin_pad, fmt), dtype=torch.uint8,
                      device=w.device)
    check(lib.ugpg_pack_conv3x3(_f32(w.contiguous()), ptr(out), cout, cin, cin_pad, mode, fmt,
                                stream()), "pack_conv3x3")
    out.ugpg_fmt = fmt
    return out


def conv_ntiles(B, H, W, cin, cout, wpk) -> int:
    """BatchNorm partial-tile count of conv3x3_fwd with these packed weights."""
    return lib.ugpg_conv3x3_fwd_ntiles(B, H, W, cin, cout, wpk.ugpg_fmt)


class KernelTimer:
    """Brackets selected launches with HIP events on the launching stream (used by
    bench.py for the live per-kernel roofline).  Records (name, flops, ev0, ev1)."""

    def __init__(self):
        self.records = []

    def wrap(self, name, flops, fn):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        self.records.append((name, flops, e0, e1))

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for name, flops, e0, e1 in self.records:
            d = out.setdefault(name, {"launches": 0, "flops": 0.0, "ms": 0.0})
            d["launches"] += 1
            d["flops"] += flops
            d["ms"] += e0.elapsed_time(e1)
        return out


TIMER = None  # set to a KernelTimer to time conv launches


def _timed(name, flops, fn):
    if TIMER is None or flops is None:
        fn()
    else:
        TIMER.wrap(name, flops, fn)


def conv3x3_fwd(srcs, wpk, bias, cout, outs, split=None, accumulate=(0, 0), stats=None,
                flops=None, bnb=None):
    """srcs: 1-2 Act; outs: 1-2 NHWC tensors (channel split at `split`); a bf16 outs[0]
    (one output) stores the result in bf16 only (the bf16 arithmetic's storage).
    flops: algorithmic FLOPs of this call (for the optional KernelTimer).
    bnb: (y, mean, invstd, scale, shift, part) -- also write the BatchNorm-backward
    partials of outs[0] = dL/d(relu(bn(y))) into `part` (3*cout*conv_ntiles floats) for
    bn_relu_bwd(..., part=part)."""
    B, H, W, _ = srcs[0].shape
    d = ConvDesc()
    d.B, d.H, d.W = B, H, W
    d.src[0] = srcs[0].src()
    d.src[1] = srcs[1].src() if len(srcs) > 1 else NULL_SRC
    d.wpk, d.bias, d.Cout = ptr(wpk), ptr(bias), cout
    if outs[0].dtype == torch.bfloat16:
        d.out[0], d.out_bf16 = None, ptr(outs[0])
    else:
        d.out[0] = ptr(outs[0])
    d.out[1] = ptr(outs[1]) if len(outs) > 1 else None
    d.out_split = cout if split is None else split
    d.accumulate[0], d.accumulate[1] = int(accumulate[0]), int(accumulate[1])
    d.stats = ptr(stats)
    if stats is not None:  # capacity in slots: the library refuses a call that would overflow
        d.stats_slots = stats.numel() // (3 * cout)
    d.wfmt = wpk.ugpg_fmt
    if bnb is not None:
        d.bnb_y, d.bnb_y_bf16 = _yargs(bnb[0])
        d.bnb_mean, d.bnb_invstd, d.bnb_scale, d.bnb_shift, d.bnb_part = (ptr(t) for t in bnb[1:])
        d.bnb_slots = bnb[5].numel() // (3 * cout)
    _timed("conv3x3_fwd", flops,
           lambda: check(lib.ugpg_conv3x3_fwd(C.byref(d), stream()), "conv3x3_fwd"))


class BnLazyDy:
    """dy of a weight gradient formed while loading from the following BatchNorm(+ReLU)
    backward (ugpg_wgrad_t.dy_bn): da, the BN input y and its statistics, `coef` the
    workspace bn_relu_bwd(..., dy=None, part=...) returned (its finalize only), and dy_out
    receiving dy for the data gradient (bit-identical to the apply pass).  pool: (dout,
    argmax) of a deferred MaxPool2d backward routed into da (bn_relu_bwd's "pool" route;
    da then holds only the base gradient, or None)."""
    __slots__ = ("da", "y", "mean", "invstd", "scale", "shift", "coef", "dy_out", "pool")

    def __init__(self, da, y, mean, invstd, scale, shift, coef, dy_out, pool=None):
        self.da, self.y, self.mean, self.invstd = da, y, mean, invstd
        self.scale, self.shift, self.coef, self.dy_out = scale, shift, coef, dy_out
        self.pool = pool

    @property
    def shape(self):
        return tuple(self.y.shape)



def conv3x3_wgrad(srcs, dy, dw, db, cin_real, accumulate=0, flops=None):
    """dy: fp32, bf16 (the bf16 arithmetic's storage) or a BnLazyDy."""
    B, H, W, _ = srcs[0].shape
    d = WgradDesc()
    d.B, d.H, d.W = B, H, W
    d.src[0] = srcs[0].src()
    d.src[1] = srcs[1].src() if len(srcs) > 1 else NULL_SRC
    lazy = None
    if isinstance(dy, BnLazyDy):
        pool = dy.pool or (None, None)
        y32, y16 = _yargs(dy.y)  # (a bf16 y: the image layer's kernel only)
        lazy = BnLazy(ptr(dy.da), y32, ptr(dy.mean), ptr(dy.invstd), ptr(dy.scale),
                      ptr(dy.shift), ptr(dy.coef), ptr(dy.dy_out), ptr(pool[0]), ptr(pool[1]), y16)
        d.dy_bn = C.pointer(lazy)
        dy = dy.y
    else:
        d.dy, d.dy_bf16 = _yargs(dy)  # dy fp32, or bf16 (the bf16 arithmetic's storage)
    d.Cout = dy.shape[-1]
    d.dw, d.Cin_real, d.db, d.accumulate = ptr(dw), cin_real, ptr(db), int(accumulate)
    d.math = _MATH_FMT[_conv_math]
    nbytes = lib.ugpg_conv3x3_wgrad_workspace(C.byref(d))
    if nbytes == 0:
        check(-1, "conv3x3_wgrad_workspace")
    ws = workspace(nbytes, dy.device)
    _timed("conv3x3_wgrad", flops,
           lambda: check(lib.ugpg_conv3x3_wgrad(C.byref(d), ptr(ws), ws.numel(), stream()),
                         "conv3x3_wgrad"))


# ------------------------------------------------------------------ BN
# Synchronised BatchNorm across data-parallel ranks (ugpg.dist.enable_sync_batchnorm): None
# (local BatchNorm, the default), or an object with `rank`, `nranks` and `all_reduce(t)`
# (SUM, in place, ordered on the current stream).  Every train-mode BatchNorm then
# normalises over the global batch: its forward statistics are gathered before the
# finalize, its backward sums all-reduced before the backward finalize.
_BN_SYNC = None


def bn_finalize(stats, ntiles, gamma, beta, rm, rv, nbt, momentum, eps):
    c = gamma.numel()
    mean, invstd, scale, shift = (empty(c, like=gamma) for _ in range(4))
    sync = _BN_SYNC
    if sync is not None:
        # this rank's (N, mean, M2) per channel in its row of a zeroed [nranks][3][C] fp64
        # buffer; the SUM all-reduce is an exact gather; every rank merges the rows in order
        g = torch.zeros(sync.nranks, 3, c, dtype=torch.float64, device=stats.device)
        check(lib.ugpg_bn_stats_pack(ptr(stats), ntiles, c, ptr(g[sync.rank]), stream()),
              "bn_stats_pack")
        sync.all_reduce(g)
        check(lib.ugpg_bn_finalize_merged(ptr(g), sync.nranks, c, _f32(gamma), _f32(beta), ptr(rm),
                                          ptr(rv), ptr(nbt), momentum, eps, ptr(mean), ptr(invstd),
                                          ptr(scale), ptr(shift), stream()), "bn_finalize_merged")
    else:
        check(lib.ugpg_bn_finalize(ptr(stats), ntiles, c, _f32(gamma), _f32(beta), ptr(rm), ptr(rv),
                                   ptr(nbt), momentum, eps, ptr(mean), ptr(invstd), ptr(scale),
                                   ptr(shift), stream()), "bn_finalize")
    if rm is not None:
        weights_written([rm, rv])  # running stats updated in place (eval-param cache keys)
    return mean, invstd, scale, shift


def bn_eval_params(gamma, beta, rm, rv, eps, owner=None):
    """(scale, shift) of an eval-mode BatchNorm.  With `owner` (the module) the result is
    cached on it, keyed on the storage and version counter of gamma, beta and the running
    stats -- every writer of those bumps the version (optimizers, bn_finalize, the DP
    broadcasts, load_state_dict's copy_) -- so a frozen previous stage (the U-map
    producer) costs no launch per step."""
    key = None
    if owner is not None:
        key = tuple((t.data_ptr(), t._version) for t in (gamma, beta, rm, rv)) + (float(eps),)
        hit = getattr(owner, "_ugpg_eval_params", None)
        if hit is not None and hit[0] == key:
            return hit[1]
    c = gamma.numel()
    scale, shift = empty(c, like=gamma), empty(c, like=gamma)
    check(lib.ugpg_bn_eval_params(_f32(gamma), _f32(beta), _f32(rm), _f32(rv), eps, c,
                                  ptr(scale), ptr(shift), stream()), "bn_eval_params")
    if key is not None:
        owner._ugpg_eval_params = (key, (scale, shift))
    return scale, shift


def bn_relu_bwd(da, y, mean, invstd, scale, shift, dy, dgamma, dbeta, dconv_bias=None,
                accumulate=0, part=None, route=None):
    """part: partials the data gradient producing `da` wrote (conv3x3_fwd(bnb=...)):
    only the finalize and apply passes run.  dy: fp32, or a bf16 tensor receiving dy
    rounded to bf16 (what the bf16 arithmetic's data and weight gradients read).
    route: the deferred last producer of da, which returned `part` and wrote no da:
    ("pool", dout, argmax, H, W) from maxpool2_bwd(defer=True) or ("head", dh, w) from
    head_bwd(defer=True); the apply adds its gradient to da (da None: nothing to add)."""
    c = y.shape[-1]
    npix = y.numel() // c
    sync = _BN_SYNC
    if sync is not None:
        if part is None:  # no producer wrote the partials: the reduction as a pass
            part = empty(3 * c * lib.ugpg_bnb_slots(npix, c), like=y, dtype=F32)
            check(lib.ugpg_bn_relu_bwd_reduce(ptr(da), *_yargs(y), npix, c, ptr(mean), ptr(invstd),
                                              ptr(scale), ptr(shift), ptr(part),
                                              part.numel() // (3 * c), stream()), "bn_relu_bwd_reduce")
        # (sum g, sum g*xhat, sum xhat) and the pixel count summed over ranks, written back
        # as one slot scaled by npix / N_global (any shard sizes: ADVICE r5)
        sums = empty(3 * c + 1, like=y, dtype=torch.float64)
        nslots = part.numel() // (3 * c)
        check(lib.ugpg_bn_bwd_partials_pack(ptr(part), nslots, c, npix, ptr(sums), stream()),
              "bn_bwd_partials_pack")
        sync.all_reduce(sums)
        check(lib.ugpg_bn_bwd_partials_unpack(ptr(sums), npix, ptr(part), nslots, c, stream()),
              "bn_bwd_partials_unpack")
    if route is not None:
        if route[0] == "pool":
            _, dout, am, H, W = route
            r = BwdRoute(1, ptr(dout), ptr(am), None, 0, npix // (H * W), H, W)
        elif route[0] == "head":
            _, dh, w = route
            r = BwdRoute(2, ptr(dh), None, _f32(w), w.shape[0], 0, 0, 0)
        else:
            raise ValueError(f"unknown backward route {route[0]!r}")
        ws = workspace(lib.ugpg_bn_relu_bwd_partials_workspace(c), y.device)
        check(lib.ugpg_bn_relu_bwd_partials_routed(
            C.byref(r), ptr(part), part.numel() // (3 * c), ptr(da), *_yargs(y), npix, c, ptr(mean),
            ptr(invstd), ptr(scale), ptr(shift), *_yargs(dy), ptr(dgamma), ptr(dbeta),
            ptr(dconv_bias), int(accumulate), ptr(ws), ws.numel(), stream()),
            "bn_relu_bwd_partials_routed")
        return
    if part is not None:
        # dy None: the finalize only; the returned workspace holds the apply's coefficients
        # (its first 2*C floats) for conv3x3_wgrad(dy=BnLazyDy(..., coef=ws, ...))
        ws = workspace(lib.ugpg_bn_relu_bwd_partials_workspace(c), y.device)
        check(lib.ugpg_bn_relu_bwd_partials(
            ptr(part), part.numel() // (3 * c), *(_yargs(da) if da is not None else (None, None)),
            *_yargs(y), npix, c, ptr(mean), ptr(invstd),
            ptr(scale), ptr(shift), *(_yargs(dy) if dy is not None else (None, None)), ptr(dgamma),
            ptr(dbeta), ptr(dconv_bias), int(accumulate), ptr(ws), ws.numel(), stream()),
            "bn_relu_bwd_partials")
        return ws
    ws = workspace(lib.ugpg_bn_relu_bwd_workspace(npix, c), y.device)
    check(lib.ugpg_bn_relu_bwd(ptr(da), *_yargs(y), npix, c, ptr(mean), ptr(invstd), ptr(scale),
                               ptr(shift), *_yargs(dy), ptr(dgamma), ptr(dbeta), ptr(dconv_bias),
                               int(accumulate), ptr(ws), ws.numel(), stream()), "bn_relu_bwd")


# ------------------------------------------------------------------ pool / resize
def maxpool2_fwd(a: Act, bf16=False):
    """bf16: the output stored in bf16 (RNE) only -- the next conv's operand under the bf16
    arithmetic, exactly."""
    B, H, W, c = a.shape
    out = empty(B, H // 2, W // 2, c, like=a.y, dtype=torch.bfloat16 if bf16 else F32)
    am = empty(B, H // 2, W // 2, c, like=a.y, dtype=torch.uint8)
    check(lib.ugpg_maxpool2_fwd(a.src(), B, H, W, *_yargs(out), ptr(am), stream()), "maxpool2_fwd")
    return out, am


def bnb_desc(bn_state, npix, c, like, nslots=None):
    """(ugpg_bnb_t, partials tensor) for a kernel that last writes da of relu(bn(y)):
    bn_state = (y, mean, invstd, scale, shift); nslots: the kernel's own slot count
    (default ugpg_bnb_slots)."""
    n = lib.ugpg_bnb_slots(npix, c) if nslots is None else nslots
    if n <= 0:
        raise ValueError(f"no BatchNorm-backward partials for C={c}")
    part = empty(3 * c * n, like=like)
    d = Bnb()
    d.y, d.y_bf16 = _yargs(bn_state[0])
    d.mean, d.invstd, d.scale, d.shift = (ptr(t) for t in bn_state[1:])
    d.part, d.nslots = ptr(part), n
    return d, part


def maxpool2_bwd(dout, am, H, W, din, accumulate, bnb=None, defer=False):
    """bnb: (y, mean, invstd, scale, shift) of the BatchNorm whose output was pooled ->
    also returns its backward partials (for bn_relu_bwd(part=...)).  defer (with bnb): din
    is not written (read as the base gradient when accumulate); the partials are those of
    din + the routed gradient, which bn_relu_bwd(part=..., route=(dout, am, H, W))
    recomputes."""
    B, _, _, c = dout.shape
    if bnb is not None and defer:
        d, part = bnb_desc(bnb, B * H * W, c, dout)
        check(lib.ugpg_maxpool2_bwd_partials(ptr(dout), ptr(am), B, H, W, c,
                                             ptr(din) if accumulate else None, C.byref(d), stream()),
              "maxpool2_bwd_partials")
        return part
    if bnb is not None:
        d, part = bnb_desc(bnb, B * H * W, c, din)
        check(lib.ugpg_maxpool2_bwd_bnb(ptr(dout), ptr(am), B, H, W, c, ptr(din), int(accumulate),
                                        C.byref(d), stream()), "maxpool2_bwd_bnb")
        return part
    check(lib.ugpg_maxpool2_bwd(ptr(dout), ptr(am), B, H, W, c, ptr(din), int(accumulate),
                                stream()), "maxpool2_bwd")
    return None


def bilinear_nhwc_fwd(a: Act, Ho, Wo, bf16=False):
    """bf16: store the result in bf16 (an Up conv's input under the bf16 arithmetic, which
    that conv and its weight gradient round to bf16 anyway)."""
    B, Hi, Wi, c = a.shape
    out = empty(B, Ho, Wo, c, like=a.y, dtype=torch.bfloat16 if bf16 else F32)
    o32, o16 = _yargs(out)
    check(lib.ugpg_bilinear_nhwc_fwd(a.src(), B, Hi, Wi, o32, Ho, Wo, o16, stream()),
          "bilinear_nhwc_fwd")
    return out


def bilinear_nhwc_bwd(dout, Hi, Wi, din, accumulate, bnb=None):
    """bnb: (y, mean, invstd, scale, shift) of the BatchNorm whose output was upsampled
    -> also returns its backward partials (for bn_relu_bwd(part=...))."""
    B, Ho, Wo, c = dout.shape
    if bnb is not None:
        d, part = bnb_desc(bnb, B * Hi * Wi, c, din, nslots=B * Hi)
        check(lib.ugpg_bilinear_nhwc_bwd_bnb(ptr(dout), B, Ho, Wo, c, ptr(din), Hi, Wi,
                                             int(accumulate), C.byref(d), stream()),
              "bilinear_nhwc_bwd_bnb")
        return part
    check(lib.ugpg_bilinear_nhwc_bwd(ptr(dout), B, Ho, Wo, c, ptr(din), Hi, Wi, int(accumulate),
                                     stream()), "bilinear_nhwc_bwd")
    return None


def cast_f32_bf16(src, dst):
    check(lib.ugpg_cast_f32_bf16(ptr(src), ptr(dst), src.numel(), stream()), "cast_f32_bf16")


def cast_bf16_f32(src, dst):
    check(lib.ugpg_cast_bf16_f32(ptr(src), ptr(dst), src.numel(), stream()), "cast_bf16_f32")


RESIZE_BILINEAR, RESIZE_NEAREST, RESIZE_UNCERTAINTY = 0, 1, 2


def resize_nchw(x, Ho, Wo, mode):
    x = x.contiguous()
    B, c, Hi, Wi = x.shape
    out = empty(B, c, Ho, Wo, like=x)
    check(lib.ugpg_resize_nchw(_f32(x), B, c, Hi, Wi, ptr(out), Ho, Wo, mode, stream()),
          "resize_nchw")
    return out


def resize_nchw_bwd(dout, Hi, Wi):
    """Input gradient of resize_nchw(..., RESIZE_BILINEAR)."""
    B, C, Ho, Wo = dout.shape
    din = empty(B, C, Hi, Wi, like=dout)
    check(lib.ugpg_resize_nchw_bwd(_f32(dout.contiguous()), B, C, Ho, Wo, ptr(din), Hi, Wi,
                                   stream()), "resize_nchw_bwd")
    return din


def nchw_to_nhwc(x, cpad):
    x = x.contiguous()
    B, c, H, W = x.shape
    out = empty(B, H, W, cpad, like=x)
    check(lib.ugpg_nchw_to_nhwc(_f32(x), B, c, H, W, ptr(out), cpad, stream()), "nchw_to_nhwc")
    return out


def nhwc_to_nchw(y, c, out=None, accumulate=0):
    B, H, W, cs = y.shape
    if out is None:
        out = empty(B, c, H, W, like=y)
    check(lib.ugpg_nhwc_to_nchw(ptr(y), B, c, H, W, cs, ptr(out), int(accumulate), stream()),
          "nhwc_to_nchw")
    return out


# ------------------------------------------------------------------ heads
def head_fwd(a: Act, w, b):
    B, H, W, c = a.shape
    nc = w.shape[0]
    h = empty(B, H, W, nc, like=a.y)
    check(lib.ugpg_head_fwd(a.src(), B * H * W, _f32(w), _f32(b), nc, ptr(h), stream()),
          "head_fwd")
    return h


def heads_combine(hs, B, H, W, nc):
    n = len(hs)
    arr = (C.c_void_p * n)(*[ptr(h) for h in hs])
    res = (C.c_int * n)(*[h.shape[1] for h in hs])
    out = empty(B, nc, H, W, like=hs[0])
    check(lib.ugpg_heads_combine(arr, res, n, B, H, W, nc, ptr(out), stream()), "heads_combine")
    return out


def heads_split_bwd(dlogits, hres):
    B, nc, H, W = dlogits.shape
    dhs = [empty(B, r, r, nc, like=dlogits) for r in hres]
    n = len(hres)
    arr = (C.c_void_p * n)(*[ptr(d) for d in dhs])
    res = (C.c_int * n)(*hres)
    check(lib.ugpg_heads_split_bwd(ptr(dlogits), B, H, W, nc, arr, res, n, stream()),
          "heads_split_bwd")
    return dhs


def head_bwd(a: Act, w, dh, dw, db, da, accumulate, bnb=None, defer=False):
    """bnb: (mean, invstd) of the BatchNorm behind `a` (its scale/shift are a's) -> also
    returns the BatchNorm-backward partials of da (for bn_relu_bwd(part=...)).  defer (with
    bnb): da is not written (read as the base gradient when accumulate); the partials are
    those of da + dh @ w, which bn_relu_bwd(part=..., route=("head", dh, w)) recomputes."""
    B, H, W, c = a.shape
    nc = w.shape[0]
    npix = B * H * W
    ws = workspace(lib.ugpg_head_bwd_workspace(npix, c, nc), dh.device)
    if bnb is not None:
        n = lib.ugpg_head_bwd_bnb_slots(npix)
        part = empty(3 * c * n, like=da)
        d = Bnb()
        d.y, d.y_bf16 = _yargs(a.y)
        d.mean, d.invstd, d.scale, d.shift = (ptr(t) for t in (*bnb, a.scale, a.shift))
        d.part, d.nslots = ptr(part), n
        check(lib.ugpg_head_bwd_bnb(a.src(), npix, _f32(w), nc, ptr(dh), ptr(dw), ptr(db),
                                    ptr(da) if accumulate or not defer else None,
                                    int(accumulate) | (2 if defer else 0), ptr(ws), ws.numel(),
                                    C.byref(d), stream()), "head_bwd_bnb")
        return part
    check(lib.ugpg_head_bwd(a.src(), npix, _f32(w), nc, ptr(dh), ptr(dw), ptr(db), ptr(da),
                            int(accumulate), ptr(ws), ws.numel(), stream()), "head_bwd")
    return None


# ------------------------------------------------------------------ loss / metrics
def _umap_args(umap, logits):
    if umap is None:
        return None, 1
    if umap.shape[0] != logits.shape[0] or umap.shape[2:] != logits.shape[2:]:
        raise ValueError(f"uncertainty map shape {tuple(umap.shape)} vs output {tuple(logits.shape)}")
    return umap.contiguous(), umap.shape[1]


def ug_loss_fwd(logits, target, umap, pos_weight, alpha, out=None):
    B, c = logits.shape[:2]
    hw = logits.numel() // (B * c)
    u, cu = _umap_args(umap, logits)
    out = empty(2, like=logits) if out is None else out
    ws = workspace(lib.ugpg_ug_loss_workspace(logits.numel()), logits.device)
    check(lib.ugpg_ug_loss_fwd(_f32(logits), _f32(target), ptr(u), B, c, hw, cu, ptr(pos_weight),
                               float(alpha), ptr(out), ptr(ws), ws.numel(), stream()), "ug_loss_fwd")
    return out


def ug_loss_bwd(logits, target, umap, pos_weight, alpha, gout):
    B, c = logits.shape[:2]
    hw = logits.numel() // (B * c)
    u, cu = _umap_args(umap, logits)
    dx = torch.empty_like(logits)
    check(lib.ugpg_ug_loss_bwd(ptr(logits), ptr(target), ptr(u), B, c, hw, cu, ptr(pos_weight),
                               float(alpha), ptr(gout), ptr(dx), stream()), "ug_loss_bwd")
    return dx


def weighted_mean_fwd(pixel_loss, umap, alpha):
    B, c = pixel_loss.shape[:2]
    hw = pixel_loss.numel() // (B * c)
    u, cu = _umap_args(umap, pixel_loss)
    out = empty(2, like=pixel_loss)
    ws = workspace(lib.ugpg_ug_loss_workspace(pixel_loss.numel()), pixel_loss.device)
    check(lib.ugpg_weighted_mean_fwd(_f32(pixel_loss), ptr(u), B, c, hw, cu, float(alpha), ptr(out),
                                     ptr(ws), ws.numel(), stream()), "weighted_mean_fwd")
    return out


def weighted_mean_bwd(pixel_loss, umap, alpha, gout):
    B, c = pixel_loss.shape[:2]
    hw = pixel_loss.numel() // (B * c)
    u, cu = _umap_args(umap, pixel_loss)
    d = torch.empty_like(pixel_loss)
    check(lib.ugpg_weighted_mean_bwd(ptr(u), B, c, hw, cu, float(alpha), ptr(gout), ptr(d),
                                     stream()), "weighted_mean_bwd")
    return d


def seg_metrics(logits, target, out=None):
    """-> device tensor [dice, acc, wrong_count] (single-channel segmentation)."""
    B = logits.shape[0]
    hw = logits.numel() // B
    out = empty(3, like=logits) if out is None else out
    ws = workspace(lib.ugpg_seg_metrics_workspace(B), logits.device)
    check(lib.ugpg_seg_metrics(_f32(logits.contiguous()), _f32(target.contiguous()), B, hw,
                               ptr(out), ptr(ws), ws.numel(), stream()), "seg_metrics")
    return out


EVAL_KEYS = ("iou", "dice", "accuracy", "precision", "recall", "specificity", "confidence", "tp")


def seg_eval(logits, gt):
    """Per-sample evaluation metrics of single-channel logits (B,1,H,W) against masks
    (B,1,H,W) -> device tensor (B, 8) with columns EVAL_KEYS (test_monuseg.py:264-297)."""
    B = logits.shape[0]
    hw = logits.numel() // B
    if gt.numel() != logits.numel():
        raise ValueError(f"seg_eval: mask {tuple(gt.shape)} does not match logits {tuple(logits.shape)}")
    out = empty((B, 8), like=logits)
    ws = workspace(lib.ugpg_seg_eval_workspace(B, hw), logits.device)
    check(lib.ugpg_seg_eval(_f32(logits.contiguous()), _f32(gt.contiguous()), B, hw, ptr(out),
                            ptr(ws), ws.numel(), stream()), "seg_eval")
    return out


def predict_mask(logits, size):
    """(sigmoid(x) > 0.5) nearest-resized to `size` = (Ho, Wo) -> (B,1,Ho,Wo) float."""
    B, C, H, W = logits.shape
    if C != 1:
        raise ValueError("predict_mask: single-channel logits expected")
    Ho, Wo = size
    out = empty((B, 1, Ho, Wo), like=logits)
    check(lib.ugpg_predict_mask(_f32(logits.contiguous()), B, H, W, ptr(out), Ho, Wo, stream()),
          "predict_mask")
    return out


def metrics_pack(m, ip, n_stat):
    """-> float64 device tensor of n+2 sums for a SUM all-reduce (see include/ugpg.h)."""
    sums = torch.empty(m.numel() + 2, dtype=torch.float64, device=m.device)
    check(lib.ugpg_metrics_pack(_f32(m), m.numel(), int(ip), float(n_stat), ptr(sums), stream()),
          "metrics_pack")
    return sums


def metrics_unpack(sums, m, ip, avg_mask):
    check(lib.ugpg_metrics_unpack(ptr(sums), m.numel(), int(ip), int(avg_mask), _f32(m), stream()),
          "metrics_unpack")
    return m


def mean_std(x, out=None):
    x = x.contiguous()
    out = empty(2, like=x) if out is None else out
    ws = workspace(lib.ugpg_mean_std_workspace(x.numel()), x.device)
    check(lib.ugpg_mean_std(_f32(x), x.numel(), ptr(out), ptr(ws), ws.numel(), stream()),
          "mean_std")
    return out


def rmsprop_step(p, g, v, lr, alpha, eps, weight_decay, grad_scale=1.0):
    check(lib.ugpg_rmsprop_step(_f32(p), _f32(g), _f32(v), p.numel(), float(lr), float(alpha),
                                float(eps), float(weight_decay), float(grad_scale), stream()),
          "rmsprop_step")


# ------------------------------------------------------------------ Herlev head
def avgpool_fwd(a: Act):
    B, H, W, c = a.shape
    out = empty(B, c, like=a.y)
    check(lib.ugpg_avgpool_fwd(a.src(), B, H * W, ptr(out), stream()), "avgpool_fwd")
    return out


def avgpool_bwd(dout, H, W, da, accumulate=0):
    B, c = dout.shape
    check(lib.ugpg_avgpool_bwd(ptr(dout), B, H * W, c, ptr(da), int(accumulate), stream()),
          "avgpool_bwd")


def linear_fwd(x, w, b, relu):
    M, K = x.shape
    N = w.shape[0]
    y = empty(M, N, like=x)
    check(lib.ugpg_linear_fwd(_f32(x.contiguous()), _f32(w), ptr(b), M, N, K, int(relu), ptr(y),
                              stream()), "linear_fwd")
    return y


def linear_bwd(x, w, dy, dx, dw, db):
    M, K = x.shape
    N = w.shape[0]
    check(lib.ugpg_linear_bwd(ptr(x), ptr(w), ptr(dy), M, N, K, ptr(dx), ptr(dw), ptr(db),
                              stream()), "linear_bwd")


def dropout_mask(n, p, seed, device):
    m = torch.empty(n, dtype=F32, device=device)
    check(lib.ugpg_dropout_mask(ptr(m), n, float(p), int(seed) & ((1 << 64) - 1), stream()),
          "dropout_mask")
    return m


def ce_ug_fwd(x, y, prev, class_weights, alpha, out=None):
    B, K = x.shape
    out = empty(5, like=x) if out is None else out
    wts = empty(B, like=x) if prev is not None else None
    check(lib.ugpg_ce_ug_fwd(_f32(x.contiguous()), ptr(y.contiguous()), ptr(prev), ptr(class_weights),
                             B, K, float(alpha), ptr(out), ptr(wts), stream()), "ce_ug_fwd")
    return out, wts


def ce_ug_bwd(x, y, wts, class_weights, gout):
    B, K = x.shape
    dx = torch.empty_like(x)
    check(lib.ugpg_ce_ug_bwd(ptr(x), ptr(y), ptr(wts), ptr(class_weights), B, K, ptr(gout),
                             ptr(dx), stream()), "ce_ug_bwd")
    return dx


def adam_step(p, g, m, v, lr, beta1, beta2, eps, weight_decay, step, grad_scale=1.0):
    check(lib.ugpg_adam_step(_f32(p), _f32(g), _f32(m), _f32(v), p.numel(), float(lr),
                             float(beta1), float(beta2), float(eps), float(weight_decay), int(step),
                             float(grad_scale), stream()), "adam_step")


def relu_bwd(y, dy, out=None):
    dx = torch.empty_like(dy) if out is None else out
    check(lib.ugpg_relu_bwd(ptr(y), ptr(dy), ptr(dx), y.numel(), stream()), "relu_bwd")
    return dx


def mul(x, m):
    y = torch.empty_like(x)
    check(lib.ugpg_mul(ptr(x), ptr(m), ptr(y), x.numel(), stream()), "mul")
    return y
