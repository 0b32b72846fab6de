"""Kernel-level parity: every libugpg entry point vs the same op in PyTorch on the
CPU (fp64 where it sharpens the reference).  Sizes cover every conv tile
configuration, ragged (non tile-multiple) images, concat inputs and the
fused BatchNorm-apply prologue."""
import pytest
import torch
import torch.nn.functional as F

from oracle import detgen as G

pytestmark = pytest.mark.gpu


def rnd(shape, seed, name="t", scale=1.0):
    return G.randn(seed, shape, name) * scale


def nhwc(t):  # NCHW cpu -> NHWC contiguous
    return t.permute(0, 2, 3, 1).contiguous()


def rnd_nhwc(shape, seed, name, dev):
    """NHWC normal tensor on dev: detgen's for small shapes, a seeded device generator for
    the large ones (bit-identity tests only need fixed inputs)."""
    B, C, H, W = shape
    if B * C * H * W > (1 << 22):
        g = torch.Generator(device=dev).manual_seed(seed)
        return torch.randn((B, H, W, C), generator=g, device=dev)
    return nhwc(rnd(shape, seed, name)).to(dev)


def nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def close(a, b, tol, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    err = (a - b).abs().max().item()
    scale = max(b.abs().max().item(), 1e-30)
    assert err <= tol * scale, f"{what}: max|diff| {err:.3e} > {tol:.1e} * {scale:.3e}"


def bq(t, on=True):
    """The operand as the bf16 arithmetic sees it: rounded to bf16 (nearest even)."""
    return t.to(torch.bfloat16).to(t.dtype) if on else t


def act_ref(y, scale, shift):
    """relu(scale*y + shift) rounded once to fp32, as the kernels' fmaf computes it
    (a twice-rounded reference can sit one fp32 ulp off, which the bf16 arithmetic
    turns into a whole bf16 rounding step)."""
    if scale is None:
        return y
    a = y.double() * scale.double().view(1, -1, 1, 1) + shift.double().view(1, -1, 1, 1)
    return torch.relu(a.float())


CONV_CASES = [
    # B, H, W, C0, C1, Cout, affine
    (2, 16, 16, 64, 0, 64, False),
    (2, 32, 32, 64, 0, 128, True),     # CFG_W candidate / CFG_S
    (1, 24, 20, 8, 0, 64, False),      # ragged tiles, BKC 8
    (2, 16, 16, 128, 128, 256, True),  # concat, CFG_S
    (4, 64, 64, 64, 64, 64, True),     # concat, CFG_L
    (16, 32, 32, 256, 0, 128, False),  # CFG_W
    (1, 8, 8, 512, 512, 256, True),    # deep K, tiny image
    (2, 256, 256, 64, 0, 64, True),    # CFG_L (16x16 tile), multi-tile wgrad splits
    (4, 128, 128, 64, 0, 128, False),  # CFG_W (8x16 x 128)
    (2, 256, 256, 64, 64, 64, True),   # Up4-shaped: concat dgrad must not straddle the split
    (4, 256, 256, 8, 0, 64, False),    # Inc-shaped image layer: narrow-input wgrad, many splits
    (3, 40, 24, 8, 0, 128, True),      # ragged 8x16 wgrad tiles, 2 co blocks, lazy affine
    (2, 4, 4, 512, 0, 512, True),      # Down4 of a 64^2 stage: 4x4 image in a 8x16 tile
    (2, 8, 8, 256, 256, 256, True),    # Up1 of a 64^2 stage
    (2, 20, 24, 64, 0, 64, True),      # 16x16-item persistent form: ragged rows and columns
    (1, 18, 17, 128, 64, 128, True),   # same, concat input, 2 partial tiles per side
    (1, 16, 16, 512, 512, 512, True),  # Up-shaped 16-wide concat: 4-way split-K forward/dgrad
    (2, 45, 70, 8, 0, 64, False),      # image layer, ragged 8 x 32 tiles (direct fp32 kernel)
    (3, 16, 40, 512, 0, 64, True),     # 16-high, 40-wide: 8 x 32 items, ragged columns
    (2, 250, 254, 64, 0, 64, True),    # bf16: 16 x 32-pixel items, ragged rows and columns
]
BIG = {5, 6, 7}


@pytest.fixture(params=["x6", "f32", "bf16"])
def math(request):
    """Every conv arithmetic form: split-bf16 (default), fp32 MFMA, and bf16 (BASELINE
    config 3: operands rounded to bf16, fp32 accumulation).  The kernel form within an
    arithmetic is chosen by shape alone; CONV_CASES covers every form (persistent 8 x 32
    and 8 x 16 items, the single-stage kernel, the direct image-layer kernel)."""
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math(request.param)
    yield request.param
    ops.set_conv_math(old)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv3x3_fwd_stats(dev, case, math):
    from ugpg import ops
    B, H, W, C0, C1, Cout, affine = case
    cin = C0 + C1
    x0 = rnd((B, C0, H, W), 1, "x0")
    x1 = rnd((B, C1, H, W), 2, "x1") if C1 else None
    w = rnd((Cout, cin, 3, 3), 3, "w", 1.0 / (3 * cin ** 0.5))
    b = rnd((Cout,), 4, "b", 0.1)
    sc0 = sh0 = sc1 = sh1 = None
    if affine:
        sc0, sh0 = rnd((C0,), 5, "s0", 0.5) + 1, rnd((C0,), 6, "h0", 0.2)
        if C1:
            sc1, sh1 = rnd((C1,), 7, "s1", 0.5) + 1, rnd((C1,), 8, "h1", 0.2)
    inp = act_ref(x0, sc0, sh0)
    if C1:
        inp = torch.cat([inp, act_ref(x1, sc1, sh1) if affine else x1], 1)
    kp = ops.conv_pack_k(cin)  # 8-channel sources: zero-extended to K = 16 (x6 / bf16)
    half = math == "bf16" and kp % 16 == 0  # runs in bf16 arithmetic
    ref = F.conv2d(bq(inp, half).double(), bq(w, half).double(), b.double(), padding=1)

    g = lambda t: None if t is None else t.to(dev)
    srcs = [ops.Act(nhwc(x0).to(dev), g(sc0), g(sh0))]
    if C1:
        srcs.append(ops.Act(nhwc(x1).to(dev), g(sc1), g(sh1)))
    wpk = ops.pack_conv3x3(w.to(dev), kp, 0)
    out = torch.empty(B, H, W, Cout, device=dev)
    fmt = {"f32": ops.WFMT_F32, "bf16": ops.WFMT_BF16}.get(math, ops.WFMT_X6)
    assert wpk.ugpg_fmt == (fmt if kp % 16 == 0 else ops.WFMT_F32)
    nt = ops.conv_ntiles(B, H, W, cin, Cout, wpk)
    stats = torch.empty(3 * Cout * nt, device=dev)
    ops.conv3x3_fwd(srcs, wpk, b.to(dev), Cout, [out], stats=stats)
    close(nchw(out.cpu()), ref, 2e-5, "conv fwd")
    # BatchNorm finalize from the fused partials
    gam, bet = rnd((Cout,), 9, "g", 0.3) + 1, rnd((Cout,), 10, "be", 0.1)
    rm, rv = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    mean, invstd, scale, shift = ops.bn_finalize(stats, nt, gam.to(dev), bet.to(dev), rm, rv, nbt,
                                                 0.1, 1e-5)
    rmean = ref.mean(dim=(0, 2, 3))
    rvar = ref.var(dim=(0, 2, 3), unbiased=False)
    close(mean.cpu(), rmean, 1e-5, "bn mean")
    close(invstd.cpu(), 1 / torch.sqrt(rvar + 1e-5), 1e-5, "bn invstd")
    n = B * H * W
    close(rv.cpu(), 0.9 + 0.1 * rvar * n / (n - 1), 1e-5, "running_var")
    close(rm.cpu(), 0.1 * rmean, 1e-5, "running_mean")
    assert int(nbt.item()) == 1


@pytest.mark.parametrize("case", CONV_CASES[:5] + CONV_CASES[7:])
def test_conv3x3_dgrad_wgrad(dev, case, math):
    from ugpg import ops
    B, H, W, C0, C1, Cout, affine = case
    cin = C0 + C1
    cin_real = 3 if cin == 8 else cin
    x = rnd((B, cin, H, W), 11, "x")
    if cin_real < cin:
        x[:, cin_real:] = 0
    sc = rnd((cin,), 12, "s", 0.5) + 1 if affine else None
    sh = rnd((cin,), 13, "h", 0.2) if affine else None
    w = rnd((Cout, cin_real, 3, 3), 14, "w", 0.05)
    dy = rnd((B, Cout, H, W), 15, "dy")
    xin = act_ref(x, sc, sh).double()[:, :cin_real].clone().requires_grad_(True)
    wd = w.double().requires_grad_(True)
    bd = torch.zeros(Cout, dtype=torch.float64, requires_grad=True)
    y = F.conv2d(xin, wd, bd, padding=1)
    y.backward(dy.double())
    # bf16 arithmetic: the same gradients of bf16-rounded operands (dgrad: dy, W;
    # wgrad: dy, act(x)), accumulated exactly
    half = math == "bf16"
    xq = bq(xin.detach(), half).clone().requires_grad_(True)
    wq = bq(wd.detach(), half).clone().requires_grad_(True)
    F.conv2d(xq, wq, None, padding=1).backward(bq(dy.double(), half))
    # dgrad (only for real input channels that are multiples of 64)
    if cin_real % 64 == 0:
        wpk = ops.pack_conv3x3(w.to(dev), cin_real, 1)
        if C1:
            d0 = torch.empty(B, H, W, C0, device=dev)
            d1 = torch.full((B, H, W, C1), 0.5, device=dev)
            ops.conv3x3_fwd([ops.Act(nhwc(dy).to(dev))], wpk, None, cin_real, [d0, d1], split=C0,
                            accumulate=(0, 1))
            close(nchw(d0.cpu()), xq.grad[:, :C0], 2e-5, "dgrad src0")
            close(nchw(d1.cpu()) - 0.5, xq.grad[:, C0:], 2e-5, "dgrad src1 (accumulate)")
        else:
            dx = torch.empty(B, H, W, cin_real, device=dev)
            ops.conv3x3_fwd([ops.Act(nhwc(dy).to(dev))], wpk, None, cin_real, [dx])
            close(nchw(dx.cpu()), xq.grad, 2e-5, "dgrad")
    # wgrad on the activated (lazy) source
    g = lambda t: None if t is None else t.to(dev)
    xs = nhwc(x).to(dev)
    if C1:
        srcs = [ops.Act(xs[..., :C0].contiguous(), g(sc[:C0] if affine else None), g(sh[:C0] if affine else None)),
                ops.Act(xs[..., C0:].contiguous(), g(sc[C0:] if affine else None), g(sh[C0:] if affine else None))]
    else:
        srcs = [ops.Act(xs, g(sc), g(sh))]
    dw = torch.empty(Cout, cin_real, 3, 3, device=dev)
    db = torch.empty(Cout, device=dev)
    ops.conv3x3_wgrad(srcs, nhwc(dy).to(dev), dw, db, cin_real)
    close(dw.cpu(), wd.grad, 2e-5, "wgrad")
    close(db.cpu(), bd.grad, 2e-5, "bias grad")
    # without a bias grad (the model's call): the narrow-input kernel for the image
    # layer, the split-bf16 kernel for 64-channel sources under math "x6"
    dw2 = torch.empty(Cout, cin_real, 3, 3, device=dev)
    ops.conv3x3_wgrad(srcs, nhwc(dy).to(dev), dw2, None, cin_real)
    split = cin_real % 64 == 0 and C0 % 64 == 0  # the split-bf16 / bf16 wgrad kernel
    close(dw2.cpu(), wq.grad if split else wd.grad, 2e-5, f"wgrad without db ({math})")


@pytest.mark.parametrize("shape", [(4, 64, 64, 64, 64), (2, 32, 32, 512, 512), (2, 16, 16, 256, 128)])
def test_conv_x6_is_fp32_class(dev, shape):
    """The split-bf16 form must be as accurate as fp32 MFMA: error vs an fp64
    reference (max and RMS over the output) within 1.5x of the fp32 path's."""
    from ugpg import ops
    B, H, W, cin, cout = shape
    x = rnd((B, cin, H, W), 31, "x")
    w = rnd((cout, cin, 3, 3), 32, "w", 1.0 / (3 * cin ** 0.5))
    ref = F.conv2d(x.double(), w.double(), None, padding=1)
    errs = {}
    old = ops.conv_math()
    try:
        for m in ("x6", "f32"):
            ops.set_conv_math(m)
            wpk = ops.pack_conv3x3(w.to(dev), cin, 0)
            out = torch.empty(B, H, W, cout, device=dev)
            ops.conv3x3_fwd([ops.Act(nhwc(x).to(dev))], wpk, None, cout, [out])
            d = nchw(out.cpu()).double() - ref
            errs[m] = (d.abs().max().item(), d.pow(2).mean().sqrt().item())
    finally:
        ops.set_conv_math(old)
    print("conv error vs fp64 (max, rms):", errs)
    assert errs["x6"][0] <= 1.5 * errs["f32"][0] and errs["x6"][1] <= 1.5 * errs["f32"][1], errs


@pytest.mark.parametrize("C,npix", [(64, 5000), (512, 300), (128, 70000)])
def test_bn_relu_bwd(dev, C, npix):
    from ugpg import ops
    y = rnd((npix, C), 20, "y") * 2 + 0.3
    gam = rnd((C,), 21, "g", 0.3) + 1
    bet = rnd((C,), 22, "b", 0.3)
    da = rnd((npix, C), 23, "da")
    yd = y.double().requires_grad_(True)
    gd = gam.double().requires_grad_(True)
    bd = bet.double().requires_grad_(True)
    a = torch.relu(F.batch_norm(yd.t().unsqueeze(0), None, None, gd, bd, True, 0.1, 1e-5))
    a.backward(da.double().t().unsqueeze(0))
    mean = y.double().mean(0)
    var = y.double().var(0, unbiased=False)
    invstd = 1 / torch.sqrt(var + 1e-5)
    scale = (gam.double() * invstd)
    shift = bet.double() - mean * scale
    f = lambda t: t.float().to(dev)
    dy = torch.empty(npix, C, device=dev)
    dg, dbt = torch.empty(C, device=dev), torch.empty(C, device=dev)
    dcb = torch.empty(C, device=dev)
    ops.bn_relu_bwd(f(da), f(y), f(mean), f(invstd), f(scale), f(shift), dy, dg, dbt, dcb)
    close(dy.cpu(), yd.grad, 1e-4, "bn bwd dx")
    # bias grad of the producing conv = sum_p dy (true value ~0)
    assert (dcb.cpu().double() - yd.grad.sum(0)).abs().max() <= 1e-6 * yd.grad.abs().sum(0).max()
    close(dg.cpu(), gd.grad, 1e-4, "dgamma")
    close(dbt.cpu(), bd.grad, 1e-4, "dbeta")


# (B, H, W, K = channels of dy, C = channels of da): the fused epilogue on the 8 x 32
# and 8 x 16 persistent forms (ragged tiles included), the separate pass elsewhere
BNB_CASES = [(2, 32, 32, 64, 64), (1, 20, 37, 64, 64), (2, 16, 16, 128, 128),
             (1, 24, 18, 128, 64), (2, 8, 8, 128, 64),
             # the bf16 arithmetic's wide single-piece forms (512 x 64 and 256 x 128 items),
             # with y stored in bf16 (fused) and in fp32 (their partials come from the pass)
             (2, 256, 256, 64, 64, True), (2, 256, 256, 64, 64), (4, 128, 128, 128, 128, True),
             (4, 128, 128, 128, 128), (2, 250, 254, 64, 64, True)]


@pytest.mark.parametrize("case", BNB_CASES)
def test_dgrad_fused_bn_bwd_partials(dev, case, math):
    """conv3x3_fwd(bnb=...) + bn_relu_bwd(part=...) == conv3x3_fwd + bn_relu_bwd: the
    data gradient is unchanged and the BatchNorm backward (dy, dgamma, dbeta, the conv
    bias grad) equals the standalone reduction's up to summation order."""
    from ugpg import ops
    B, H, W, K, Cc = case[:5]
    y16 = len(case) > 5 and case[5]
    dy2 = rnd((B, K, H, W), 30, "dy2")
    w = rnd((K, Cc, 3, 3), 31, "w", 0.05)
    y = rnd((B, Cc, H, W), 32, "y") * 2 + 0.3
    if y16:
        y = y.to(torch.bfloat16).float()
    gam, bet = rnd((Cc,), 33, "g", 0.3) + 1, rnd((Cc,), 34, "b", 0.3)
    yd = y.double()
    mean = yd.mean((0, 2, 3))
    invstd = 1 / torch.sqrt(yd.var((0, 2, 3), unbiased=False) + 1e-5)
    scale = gam.double() * invstd
    shift = bet.double() - mean * scale
    f = lambda t: t.float().to(dev)
    st = [f(mean), f(invstd), f(scale), f(shift)]
    ys, d2 = nhwc(y).to(dev), nhwc(dy2).to(dev)
    if y16:
        ys = ys.to(torch.bfloat16)
    wpk = ops.pack_conv3x3(w.to(dev), Cc, 1)
    nt = ops.conv_ntiles(B, H, W, K, Cc, wpk)
    part = torch.full((3 * Cc * nt,), float("nan"), device=dev)  # every slot must be written
    da_f = torch.empty(B, H, W, Cc, device=dev)
    ops.conv3x3_fwd([ops.Act(d2)], wpk, None, Cc, [da_f], bnb=(ys, *st, part))
    da_r = torch.empty_like(da_f)
    ops.conv3x3_fwd([ops.Act(d2)], wpk, None, Cc, [da_r])
    assert torch.equal(da_f, da_r), "the partials must not change the data gradient"
    assert torch.isfinite(part).all()
    outs = []
    for p in (part, None):
        dy = torch.empty_like(da_f)
        dg, dbt, dcb = (torch.empty(Cc, device=dev) for _ in range(3))
        ops.bn_relu_bwd(da_f, ys, *st, dy, dg, dbt, dcb, part=p)
        outs.append((dy.cpu(), dg.cpu(), dbt.cpu(), dcb.cpu()))
    for name, a_, b_ in zip(("dy", "dgamma", "dbeta"), outs[0], outs[1]):
        close(a_.double(), b_.double(), 1e-5, f"fused partials: {name}")
    # the conv-bias gradient is a cancellation (~0): compare on the scale of |dy| sums
    tol = 1e-6 * outs[1][0].abs().sum((0, 1, 2)).max().item()
    assert (outs[0][3] - outs[1][3]).abs().max().item() <= tol


@pytest.mark.parametrize("C,acc", [(64, 0), (64, 1), (128, 1), (512, 0)])
def test_maxpool2_bwd_fused_bn_partials(dev, C, acc):
    """maxpool2_bwd(bnb=...) writes the same din and the BatchNorm-backward partials that
    make bn_relu_bwd(part=...) equal the standalone reduction."""
    from ugpg import ops
    B, H, W = 2, 18, 22
    x = nhwc(rnd((B, C, H, W), 50, "x")).to(dev)
    out, am = ops.maxpool2_fwd(ops.Act(x))
    dout = nhwc(rnd((B, C, H // 2, W // 2), 51, "dp")).to(dev)
    base = nhwc(rnd((B, C, H, W), 52, "base")).to(dev)
    y = nhwc(rnd((B, C, H, W), 53, "y") * 2 + 0.3).to(dev)
    st = [rnd((C,), 54 + i, f"s{i}").abs().to(dev) + 0.1 for i in range(4)]
    st[3] = st[3] - 0.5
    d1, d2 = base.clone(), base.clone()
    part = ops.maxpool2_bwd(dout, am, H, W, d1, acc, bnb=(y, *st))
    ops.maxpool2_bwd(dout, am, H, W, d2, acc)
    assert torch.equal(d1, d2)
    outs = []
    for p in (part, None):
        dy = torch.empty_like(d1)
        dg, dbt, dcb = (torch.empty(C, device=dev) for _ in range(3))
        ops.bn_relu_bwd(d1, y, *st, dy, dg, dbt, dcb, part=p)
        outs.append((dy.cpu(), dg.cpu(), dbt.cpu()))
    for name, a_, b_ in zip(("dy", "dgamma", "dbeta"), outs[0], outs[1]):
        close(a_, b_, 1e-5, f"maxpool-fused partials: {name}")


# large shapes: n4 = B*H*W*C/4 above 4x the apply's 524,288-thread grid, so
# every thread runs the 4-way unrolled loop and steps its (x, row, image) position across
# row and image boundaries; odd sizes whose pixel count is not a multiple of the grid's
# pixel stride; the real step's shape (bs16 x 256^2 x 64)
ROUTE_BIG = [(4, 64, 1, 250, 254, True), (4, 64, 0, 250, 254, False), (3, 64, 1, 255, 253, False),
             (16, 64, 1, 256, 256, True), (5, 128, 1, 129, 127, True)]


@pytest.mark.parametrize("B,C,acc,H,W,y16", [(2, 64, 0, 18, 22, False), (2, 64, 1, 19, 22, False),
                                             (2, 128, 1, 18, 21, True), (2, 512, 0, 8, 8, True),
                                             (2, 64, 1, 32, 32, True)] + ROUTE_BIG)
def test_maxpool2_bwd_deferred_route_bit_identical(dev, B, C, acc, H, W, y16):
    """maxpool2_bwd(defer=True) + bn_relu_bwd(route=...) -- the routed gradient recomputed by
    the apply, never stored -- equals maxpool2_bwd(bnb=...) writing din followed by
    bn_relu_bwd(part=...) bit for bit (fp32 and bf16 storage of y, odd sizes, with and
    without a base gradient, grid-stride loops over many rows and images)."""
    from ugpg import ops
    x = rnd_nhwc((B, C, H, W), 60, "x", dev)
    _, am = ops.maxpool2_fwd(ops.Act(x))
    dout = rnd_nhwc((B, C, H // 2, W // 2), 61, "dp", dev)
    base = rnd_nhwc((B, C, H, W), 62, "base", dev)
    y = rnd_nhwc((B, C, H, W), 63, "y", dev) * 2 + 0.3
    if y16:
        y = y.to(torch.bfloat16)
    st = [rnd((C,), 64 + i, f"s{i}").abs().to(dev) + 0.1 for i in range(4)]
    st[3] = st[3] - 0.5
    outs = []
    for defer in (False, True):
        d = base.clone()
        part = ops.maxpool2_bwd(dout, am, H, W, d, acc, bnb=(y, *st), defer=defer)
        if defer:
            assert torch.equal(d, base)  # nothing written
        dy = torch.empty(d.shape, device=dev, dtype=torch.bfloat16 if y16 else torch.float32)
        dg, dbt, dcb = (torch.empty(C, device=dev) for _ in range(3))
        ops.bn_relu_bwd(d if (acc or not defer) else None, y, *st, dy, dg, dbt, dcb, part=part,
                        route=("pool", dout, am, H, W) if defer else None)
        outs.append((part.cpu(), dy.cpu(), dg.cpu(), dbt.cpu(), dcb.cpu()))
    for name, a_, b_ in zip(("partials", "dy", "dgamma", "dbeta", "dconv_bias"), *outs):
        assert torch.equal(a_, b_), f"deferred pool backward differs: {name}"


@pytest.mark.parametrize("C,nc,acc", [(64, 1, 0), (64, 2, 1), (128, 1, 1)])
def test_head_bwd_fused_bn_partials(dev, C, nc, acc):
    """head_bwd(bnb=...) = head_bwd + the standalone BatchNorm-backward reduction."""
    from ugpg import ops
    B, H, W = 2, 20, 24
    y = nhwc(rnd((B, C, H, W), 60, "y") * 2 + 0.3).to(dev)
    mean, invstd = rnd((C,), 61, "m").to(dev), rnd((C,), 62, "i").abs().to(dev) + 0.2
    sc, sh = rnd((C,), 63, "s").abs().to(dev) + 0.1, rnd((C,), 64, "h").to(dev)
    a = ops.Act(y, sc, sh)
    w = rnd((nc, C), 65, "w", 0.1).to(dev)
    dh = rnd((B * H * W, nc), 66, "dh").to(dev)
    base = nhwc(rnd((B, C, H, W), 67, "base")).to(dev)
    res = []
    for fused in (True, False):
        da = base.clone()
        dw, db = torch.empty(nc, C, device=dev), torch.empty(nc, device=dev)
        part = ops.head_bwd(a, w, dh, dw, db, da, acc, bnb=(mean, invstd) if fused else None)
        dy = torch.empty_like(da)
        dg, dbt, dcb = (torch.empty(C, device=dev) for _ in range(3))
        ops.bn_relu_bwd(da, y, mean, invstd, sc, sh, dy, dg, dbt, dcb, part=part)
        res.append((da.cpu(), dw.cpu(), db.cpu(), dy.cpu(), dg.cpu(), dbt.cpu()))
    assert all(torch.equal(x_, y_) for x_, y_ in zip(res[0][:3], res[1][:3]))
    for name, a_, b_ in zip(("dy", "dgamma", "dbeta"), res[0][3:], res[1][3:]):
        close(a_, b_, 1e-5, f"head-fused partials: {name}")


@pytest.mark.parametrize("B,H,W,C,nc,acc,y16", [(2, 20, 24, 64, 1, 0, False), (2, 20, 24, 64, 2, 1, False),
                                                (2, 20, 24, 128, 1, 1, True), (2, 20, 24, 64, 4, 0, True),
                                                (2, 20, 24, 256, 3, 1, False),
                                                (4, 250, 254, 64, 1, 1, True), (3, 255, 253, 64, 2, 0, False),
                                                (16, 256, 256, 64, 1, 0, True)])
def test_head_bwd_deferred_route_bit_identical(dev, B, H, W, C, nc, acc, y16):
    """head_bwd(bnb=..., defer=True) + bn_relu_bwd(route=("head", dh, w)) -- the head's input
    gradient recomputed by the apply, never stored -- equals head_bwd(bnb=...) writing da
    followed by bn_relu_bwd(part=...) bit for bit, dW and db included (large shapes: the
    apply's grid-stride loop)."""
    from ugpg import ops
    y = rnd_nhwc((B, C, H, W), 80, "y", dev) * 2 + 0.3
    if y16:
        y = y.to(torch.bfloat16)
    mean, invstd = rnd((C,), 81, "m").to(dev), rnd((C,), 82, "i").abs().to(dev) + 0.2
    sc, sh = rnd((C,), 83, "s").abs().to(dev) + 0.1, rnd((C,), 84, "h").to(dev)
    a = ops.Act(y, sc, sh)
    w = rnd((nc, C), 85, "w", 0.1).to(dev)
    dh = rnd_nhwc((B, nc, H, W), 86, "dh", dev).reshape(B * H * W, nc)
    base = rnd_nhwc((B, C, H, W), 87, "base", dev)
    res = []
    for defer in (False, True):
        da = base.clone()
        dw, db = torch.empty(nc, C, device=dev), torch.empty(nc, device=dev)
        part = ops.head_bwd(a, w, dh, dw, db, da, acc, bnb=(mean, invstd), defer=defer)
        if defer:
            assert torch.equal(da, base)  # nothing written
        dy = torch.empty(da.shape, device=dev, dtype=torch.bfloat16 if y16 else torch.float32)
        dg, dbt, dcb = (torch.empty(C, device=dev) for _ in range(3))
        ops.bn_relu_bwd(da if (acc or not defer) else None, y, mean, invstd, sc, sh, dy, dg, dbt,
                        dcb, part=part, route=("head", dh, w) if defer else None)
        res.append((part.cpu(), dw.cpu(), db.cpu(), dy.cpu(), dg.cpu(), dbt.cpu(), dcb.cpu()))
    for name, a_, b_ in zip(("partials", "dw", "db", "dy", "dgamma", "dbeta", "dconv_bias"), *res):
        assert torch.equal(a_, b_), f"deferred head backward differs: {name}"


@pytest.mark.parametrize("h,C,acc", [(16, 512, 0), (32, 256, 1), (13, 64, 1)])
def test_bilinear_bwd_fused_bn_partials(dev, h, C, acc):
    """bilinear_nhwc_bwd(bnb=...) writes a bit-identical din plus the BatchNorm-backward
    partials that make bn_relu_bwd(part=...) equal the standalone reduction."""
    from ugpg import ops
    B, H = 2, 2 * h
    dout = nhwc(rnd((B, C, H, H), 70, "du")).to(dev)
    base = nhwc(rnd((B, C, h, h), 71, "base")).to(dev)
    y = nhwc(rnd((B, C, h, h), 72, "y") * 2 + 0.3).to(dev)
    st = [rnd((C,), 73 + i, f"s{i}").abs().to(dev) + 0.1 for i in range(4)]
    st[3] = st[3] - 0.5
    d1, d2 = base.clone(), base.clone()
    part = ops.bilinear_nhwc_bwd(dout, h, h, d1, acc, bnb=(y, *st))
    ops.bilinear_nhwc_bwd(dout, h, h, d2, acc)
    assert torch.equal(d1, d2)
    outs = []
    for p in (part, None):
        dy = torch.empty_like(d1)
        dg, dbt, dcb = (torch.empty(C, device=dev) for _ in range(3))
        ops.bn_relu_bwd(d1, y, *st, dy, dg, dbt, dcb, part=p)
        outs.append((dy.cpu(), dg.cpu(), dbt.cpu()))
    for name, a_, b_ in zip(("dy", "dgamma", "dbeta"), outs[0], outs[1]):
        close(a_, b_, 1e-5, f"bilinear-fused partials: {name}")


def test_bf16_casts(dev):
    """The bf16 gradient exchange's casts: round to nearest even exactly as torch's
    .to(bfloat16) (ties, subnormals, inf, NaN), and back exactly."""
    from ugpg import ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(100003, generator=g) * torch.exp(torch.randn(100003, generator=g) * 20)
    ties = torch.tensor([1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, -1.0 - 2 ** -8, 2 ** -130, -2 ** -133,
                         float("inf"), -float("inf"), 3.0e38, -3.4e38], dtype=torch.float32)
    x = torch.cat([x, ties]).to(dev)
    h = torch.empty(x.numel(), dtype=torch.bfloat16, device=dev)
    ops.cast_f32_bf16(x, h)
    assert torch.equal(h.view(torch.int16).cpu(), x.cpu().to(torch.bfloat16).view(torch.int16))
    y = torch.empty_like(x)
    ops.cast_bf16_f32(h, y)
    assert torch.equal(y.cpu(), h.cpu().float())
    n = torch.tensor([float("nan")], device=dev)
    hn = torch.empty(1, dtype=torch.bfloat16, device=dev)
    ops.cast_f32_bf16(n, hn)
    assert torch.isnan(hn.float()).all()


@pytest.mark.parametrize("case", [(2, 32, 40, 64, 0, 128), (1, 36, 64, 64, 64, 64),
                                  (2, 40, 48, 8, 0, 64),
                                  # the wide single-piece forms: 512 x 64 items (ragged
                                  # rows too) and 256 x 128 items with a concat input
                                  (2, 256, 256, 64, 0, 64), (2, 250, 254, 64, 0, 64),
                                  (4, 128, 128, 64, 64, 128)])
def test_conv_bf16_storage(dev, case):
    """bf16 activation storage (the bf16 arithmetic's, config 3): a conv whose output is
    stored in bf16 only writes exactly bf16(the fp32 output) -- persistent single-piece
    epilogue and the image-layer kernel -- with BatchNorm statistics of the rounded values;
    a source stored in bf16 gives the same output as its fp32 form (bf16-exact values)."""
    from ugpg import ops
    B, H, W, C0, C1, Cout = case
    old = ops.conv_math()
    ops.set_conv_math("bf16")
    try:
        cin = C0 + C1
        q = lambda t: t.to(torch.bfloat16).float()
        y0 = q(nhwc(rnd((B, C0, H, W), 80, "y0"))).to(dev)
        y1 = q(nhwc(rnd((B, C1, H, W), 81, "y1"))).to(dev) if C1 else None
        sc = (rnd((C0,), 82, "s", 0.5) + 1).to(dev) if C0 % 16 == 0 else None
        sh = rnd((C0,), 83, "h", 0.2).to(dev) if sc is not None else None
        w = rnd((Cout, cin, 3, 3), 84, "w", 0.05).to(dev)
        b = rnd((Cout,), 85, "b", 0.1).to(dev)
        wpk = ops.pack_conv3x3(w, ops.conv_pack_k(cin), 0)
        nt = ops.conv_ntiles(B, H, W, cin, Cout, wpk)
        res = {}
        for src16 in (False, True):
            if src16 and C0 == 8:
                continue  # the image is an fp32 input
            s0 = ops.Act(y0.to(torch.bfloat16) if src16 else y0, sc, sh)
            srcs = [s0] + ([ops.Act(y1.to(torch.bfloat16) if src16 else y1)] if C1 else [])
            for out16 in (False, True):
                out = torch.empty(B, H, W, Cout, device=dev,
                                  dtype=torch.bfloat16 if out16 else torch.float32)
                st = torch.empty(3 * Cout * nt, device=dev)
                ops.conv3x3_fwd(srcs, wpk, b, Cout, [out], stats=st)
                res[src16, out16] = (out, st)
        ref, st_ref = res[False, False]
        for (src16, out16), (out, st) in res.items():
            want = ref.to(torch.bfloat16) if out16 else ref
            assert torch.equal(out, want), (src16, out16)
            # statistics of the stored values
            gam, bet = torch.ones(Cout, device=dev), torch.zeros(Cout, device=dev)
            mean, invstd, _, _ = ops.bn_finalize(st, nt, gam, bet, None, None, None, 0.1, 1e-5)
            v = out.float().reshape(-1, Cout).double()
            close(mean.cpu(), v.mean(0).cpu(), 1e-5, "bn mean of the stored values")
            close(invstd.cpu(), (1 / torch.sqrt(v.var(0, unbiased=False) + 1e-5)).cpu(), 1e-5,
                  "bn invstd of the stored values")
    finally:
        ops.set_conv_math(old)


@pytest.mark.parametrize("math", ["bf16", "x6"])
def test_bf16_stored_bn_input(dev, math):
    """Every reader of a BatchNorm input y (a conv output) accepts its bf16 storage and
    gives exactly the result of the fp32 form of the same (bf16-exact) values: max-pool,
    bilinear x2 (also storing its result in bf16), the heads forward/backward, BatchNorm
    backward (reduce, apply, and the partials fused into max-pool / bilinear / head
    backward and the data gradient's epilogue) and the bf16 weight gradient."""
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math(math)
    try:
        B, H, W, C = 2, 32, 40, 64
        q = lambda t: t.to(torch.bfloat16).float()
        y = q(nhwc(rnd((B, C, H, W), 90, "y") * 2 + 0.3)).to(dev)
        y16 = y.to(torch.bfloat16)
        sc, sh = (rnd((C,), 91, "s", 0.5) + 1).to(dev), rnd((C,), 92, "h", 0.3).to(dev)
        mean, invstd = rnd((C,), 93, "m", 0.1).to(dev), (rnd((C,), 94, "i").abs() + 0.5).to(dev)
        st = (mean, invstd, sc, sh)
        eq = lambda a_, b_, what: (torch.equal(a_, b_) or pytest.fail(what))
        # max-pool forward / backward with fused partials
        (p32, am32), (p16, am16) = (ops.maxpool2_fwd(ops.Act(t, sc, sh)) for t in (y, y16))
        eq(p32, p16, "maxpool fwd")
        eq(am32, am16, "maxpool argmax")
        dout = nhwc(rnd((B, C, H // 2, W // 2), 95, "dp")).to(dev)
        parts = []
        for t in (y, y16):
            din = torch.empty(B, H, W, C, device=dev)
            parts.append((din, ops.maxpool2_bwd(dout, am32, H, W, din, 0, bnb=(t, *st))))
        eq(parts[0][0], parts[1][0], "maxpool bwd")
        eq(parts[0][1], parts[1][1], "maxpool bwd partials")
        # BatchNorm backward, standalone and from partials
        outs = []
        for t in (y, y16):
            dy = torch.empty(B, H, W, C, device=dev)
            dg, dbt, dcb = (torch.empty(C, device=dev) for _ in range(3))
            ops.bn_relu_bwd(parts[0][0], t, *st, dy, dg, dbt, dcb)
            dy2 = torch.empty_like(dy)
            ops.bn_relu_bwd(parts[0][0], t, *st, dy2, dg, dbt, dcb, part=parts[0][1])
            outs.append((dy, dy2, dg, dbt))
        for a_, b_ in zip(*outs):
            eq(a_, b_, "bn_relu_bwd")
        # bilinear x2: fp32 and bf16 results; backward partials
        u32 = ops.bilinear_nhwc_fwd(ops.Act(y, sc, sh), 2 * H, 2 * W)
        u16 = ops.bilinear_nhwc_fwd(ops.Act(y16, sc, sh), 2 * H, 2 * W, bf16=True)
        eq(u16, u32.to(torch.bfloat16), "bilinear fwd bf16 output")
        eq(ops.bilinear_nhwc_fwd(ops.Act(y16, sc, sh), 2 * H, 2 * W), u32, "bilinear fwd")
        du = nhwc(rnd((B, C, 2 * H, 2 * W), 96, "du")).to(dev)
        bp = []
        for t in (y, y16):
            din = torch.empty(B, H, W, C, device=dev)
            bp.append((din, ops.bilinear_nhwc_bwd(du, H, W, din, 0, bnb=(t, *st))))
        eq(bp[0][0], bp[1][0], "bilinear bwd")
        eq(bp[0][1], bp[1][1], "bilinear bwd partials")
        # heads
        wh, bh = rnd((1, C), 97, "wh").to(dev), rnd((1,), 98, "bh").to(dev)
        eq(ops.head_fwd(ops.Act(y, sc, sh), wh, bh), ops.head_fwd(ops.Act(y16, sc, sh), wh, bh),
           "head fwd")
        dh = nhwc(rnd((B, 1, H, W), 99, "dh")).to(dev)
        hb = []
        for t in (y, y16):
            dw, db = torch.empty(1, C, device=dev), torch.empty(1, device=dev)
            da = torch.empty(B, H, W, C, device=dev)
            part = ops.head_bwd(ops.Act(t, sc, sh), wh, dh, dw, db, da, 0, bnb=(mean, invstd))
            hb.append((dw, db, da, part))
        for a_, b_ in zip(*hb):
            eq(a_, b_, "head bwd")
        # data gradient with the BN1 partials fused in its epilogue, y1 stored in bf16
        wd = rnd((C, C, 3, 3), 100, "wd", 0.05).to(dev)
        wpk = ops.pack_conv3x3(wd, C, 1)
        nt = ops.conv_ntiles(B, H, W, C, C, wpk)
        dg_ = []
        for t in (y, y16):
            part = torch.empty(3 * C * nt, device=dev)
            da = torch.empty(B, H, W, C, device=dev)
            ops.conv3x3_fwd([ops.Act(du[:, :H, :W].contiguous())], wpk, None, C, [da],
                            bnb=(t, *st, part))
            dg_.append((da, part))
        eq(dg_[0][0], dg_[1][0], "dgrad")
        eq(dg_[0][1], dg_[1][1], "dgrad fused partials")
        if math == "bf16":  # the weight gradient of bf16-stored sources (one and two)
            dyw = nhwc(rnd((B, 128, H, W), 101, "dyw")).to(dev)
            for two in (False, True):
                ws_ = []
                for t in (y, y16):
                    srcs = [ops.Act(t, sc, sh)] + ([ops.Act(t)] if two else [])
                    dw = torch.empty(128, C * (2 if two else 1), 3, 3, device=dev)
                    ops.conv3x3_wgrad(srcs, dyw, dw, None, C * (2 if two else 1))
                    ws_.append(dw)
                eq(ws_[0], ws_[1], f"bf16 wgrad of bf16-stored sources (two={two})")
            # dy stored in bf16 by the BatchNorm backward (standalone and from partials):
            # the round-to-nearest-even of the fp32 dy; the weight gradient (fp32 or bf16
            # sources) and the data gradient reading it give exactly the fp32-dy results
            dy32 = torch.empty(B, H, W, C, device=dev)
            ops.bn_relu_bwd(parts[0][0], y16, *st, dy32, *(torch.empty(C, device=dev)
                                                           for _ in range(3)))
            for use_part in (False, True):
                dy16 = torch.empty(B, H, W, C, device=dev, dtype=torch.bfloat16)
                ops.bn_relu_bwd(parts[0][0], y16, *st, dy16,
                                *(torch.empty(C, device=dev) for _ in range(3)),
                                part=parts[0][1] if use_part else None)
                eq(dy16, dy32.to(torch.bfloat16), f"bf16 dy (partials={use_part})")
            for t in (y, y16):
                w2 = []
                for d in (dy32, dy16):
                    dw = torch.empty(C, C, 3, 3, device=dev)
                    ops.conv3x3_wgrad([ops.Act(t, sc, sh)], d, dw, None, C)
                    w2.append(dw)
                eq(w2[0], w2[1], f"bf16 wgrad of a bf16-stored dy (x {t.dtype})")
            d2 = []
            for d in (dy32, dy16):
                da = torch.empty(B, H, W, C, device=dev)
                ops.conv3x3_fwd([ops.Act(d)], wpk, None, C, [da])
                d2.append(da)
            eq(d2[0], d2[1], "bf16 dgrad of a bf16-stored dy")
            # max-pool output stored in bf16: the rounded fp32 output, same argmax
            p16b, am16b = ops.maxpool2_fwd(ops.Act(y16, sc, sh), bf16=True)
            eq(p16b, p32.to(torch.bfloat16), "maxpool fwd bf16 output")
            eq(am16b, am32, "maxpool argmax (bf16 output)")
        # avgpool (Herlev)
        eq(ops.avgpool_fwd(ops.Act(y, sc, sh)), ops.avgpool_fwd(ops.Act(y16, sc, sh)), "avgpool")
    finally:
        ops.set_conv_math(old)


def test_bn_eval_params_cache(dev):
    """Eval-mode BN (scale, shift) cached on the module: reused while gamma, beta and the
    running stats are unchanged, recomputed after any in-place write (torch ops, the
    optimizers' and bn_finalize's raw-pointer writes bump the version counter)."""
    from ugpg import ops
    bn = torch.nn.BatchNorm2d(64).to(dev)
    with torch.no_grad():
        bn.running_mean.copy_(rnd((64,), 40, "rm").to(dev))
        bn.running_var.copy_(rnd((64,), 41, "rv").abs().to(dev) + 0.5)
        bn.weight.copy_(rnd((64,), 42, "g").to(dev))

    def ref():
        sc = bn.weight.double() / torch.sqrt(bn.running_var.double() + bn.eps)
        return sc, bn.bias.double() - bn.running_mean.double() * sc

    def get():
        return ops.bn_eval_params(bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                                  bn.running_var, bn.eps, owner=bn)
    s1, h1 = get()
    s2, h2 = get()
    assert s2 is s1 and h2 is h1, "unchanged parameters: cached"
    close(s1, ref()[0], 1e-6, "scale")
    with torch.no_grad():
        bn.running_var.mul_(2.0)
    s3, h3 = get()
    assert s3 is not s1
    close(s3, ref()[0], 1e-6, "scale after running_var write")
    # bn_finalize updates the running stats through a raw pointer: must invalidate too
    stats = torch.zeros(3 * 64 * 4, device=dev)
    stats[:64 * 4] = 10.0
    stats[64 * 4:2 * 64 * 4] = 5.0
    stats[2 * 64 * 4:] = 7.0
    nbt = torch.zeros((), dtype=torch.int64, device=dev)
    ops.bn_finalize(stats, 4, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                    bn.running_var, nbt, 0.1, bn.eps)
    s4, h4 = get()
    assert s4 is not s3
    close(s4, ref()[0], 1e-6, "scale after bn_finalize")
    close(h4, ref()[1], 1e-6, "shift after bn_finalize")


def test_maxpool(dev):
    from ugpg import ops
    B, H, W, C = 2, 18, 22, 64
    y = rnd((B, C, H, W), 30, "y")
    sc, sh = rnd((C,), 31, "s", 0.5) + 1, rnd((C,), 32, "h", 0.3)
    a = act_ref(y, sc, sh).double().requires_grad_(True)
    ref = F.max_pool2d(a, 2)
    d = rnd(tuple(ref.shape), 33, "d")
    ref.backward(d.double())
    out, am = ops.maxpool2_fwd(ops.Act(nhwc(y).to(dev), sc.to(dev), sh.to(dev)))
    close(nchw(out.cpu()), ref, 1e-6, "maxpool fwd")
    din = torch.full((B, H, W, C), 1.0, device=dev)
    ops.maxpool2_bwd(nhwc(d).to(dev), am, H, W, din, 1)
    close(nchw(din.cpu()) - 1.0, a.grad, 1e-6, "maxpool bwd")


@pytest.mark.parametrize("hi,wi,ho,wo,C", [(16, 16, 32, 32, 64), (8, 8, 16, 16, 64), (7, 5, 13, 11, 64),
                                            (32, 32, 16, 16, 64), (64, 64, 128, 128, 128),
                                            (9, 11, 18, 22, 96), (16, 16, 32, 32, 1024)])
def test_bilinear_nhwc(dev, hi, wi, ho, wo, C):
    from ugpg import ops
    B = 2
    y = rnd((B, C, hi, wi), 40, "y")
    sc, sh = rnd((C,), 41, "s", 0.5) + 1, rnd((C,), 42, "h", 0.3)
    # fp32 reference: ATen derives the align_corners weights in fp32 (fp64 rounds differently)
    a = act_ref(y, sc, sh).requires_grad_(True)
    ref = F.interpolate(a, size=(ho, wo), mode="bilinear", align_corners=True)
    d = rnd(tuple(ref.shape), 43, "d")
    ref.backward(d)
    out = ops.bilinear_nhwc_fwd(ops.Act(nhwc(y).to(dev), sc.to(dev), sh.to(dev)), ho, wo)
    close(nchw(out.cpu()), ref, 2e-6, "bilinear fwd")
    din = torch.empty(B, hi, wi, C, device=dev)
    ops.bilinear_nhwc_bwd(nhwc(d).to(dev), hi, wi, din, 0)
    close(nchw(din.cpu()), a.grad, 1e-5, "bilinear bwd")


@pytest.mark.parametrize("mode", [0, 1, 2])
@pytest.mark.parametrize("hi,ho", [(256, 128), (128, 256), (64, 64), (30, 47)])
def test_resize_nchw(dev, mode, hi, ho):
    from ugpg import ops
    x = rnd((2, 3, hi, hi), 50, "x")
    if mode == 0:
        ref = F.interpolate(x, size=(ho, ho), mode="bilinear", align_corners=True)
    elif mode == 1:
        ref = F.interpolate(x, size=(ho, ho), mode="nearest")
    else:
        p = F.interpolate(torch.sigmoid(x), size=(ho, ho), mode="bilinear", align_corners=True)
        ref = 1.0 - 2.0 * torch.abs(p - 0.5)
    out = ops.resize_nchw(x.to(dev), ho, ho, mode)
    close(out.cpu(), ref, 2e-6, f"resize mode {mode}")
    if mode == 1:
        assert torch.equal(out.cpu(), ref)


@pytest.mark.parametrize("nc", [1, 2])
def test_heads(dev, nc):
    from ugpg import ops
    B = 2
    specs = [(256, 8), (128, 16), (64, 32), (64, 64)]
    ys, acts, ws, bs, refs, leaf = [], [], [], [], [], []
    for i, (C, R) in enumerate(specs):
        y = rnd((B, C, R, R), 60 + i, "y")
        sc, sh = rnd((C,), 70 + i, "s", 0.5) + 1, rnd((C,), 80 + i, "h", 0.3)
        a = act_ref(y, sc, sh).double().requires_grad_(True)
        w = rnd((nc, C, 1, 1), 90 + i, "w", 0.1).double().requires_grad_(True)
        b = rnd((nc,), 95 + i, "b", 0.1).double().requires_grad_(True)
        h = F.conv2d(a, w, b)
        if R != 64:
            h = F.interpolate(h, scale_factor=64 // R, mode="bilinear", align_corners=True)
        refs.append(h)
        leaf.append((a, w, b))
        acts.append(ops.Act(nhwc(y).to(dev), sc.to(dev), sh.to(dev)))
        ws.append(w.detach().float().reshape(nc, C).contiguous().to(dev))
        bs.append(b.detach().float().to(dev))
    ref = refs[0] + refs[1] + refs[2] + refs[3]
    dl = rnd(tuple(ref.shape), 99, "dl")
    ref.backward(dl.double())
    hs = [ops.head_fwd(a, w, b) for a, w, b in zip(acts, ws, bs)]
    logits = ops.heads_combine(hs, B, 64, 64, nc)
    close(logits.cpu(), ref, 1e-5, "heads fwd")
    dhs = ops.heads_split_bwd(dl.to(dev), [R for _, R in specs])
    for i, (a, w, b) in enumerate(leaf):
        dw = torch.empty_like(ws[i])
        db = torch.empty(nc, device=dev)
        da = torch.empty_like(acts[i].y)
        ops.head_bwd(acts[i], ws[i], dhs[i].contiguous(), dw, db, da, 0)
        close(dw.cpu(), w.grad.reshape(nc, -1), 1e-5, f"head{i} dw")
        # db is a heavily cancelling sum: bound it relative to sum|terms|
        dh64 = dhs[i].double().cpu()
        assert (db.cpu().double() - b.grad).abs().max() <= 1e-6 * dh64.abs().sum(), f"head{i} db"
        close(nchw(da.cpu()), a.grad, 1e-5, f"head{i} da")


@pytest.mark.parametrize("nc", [1, 3])
def test_heads_split_bwd_full(dev, nc):
    """dh of each deep-supervision head at the Stage-4 shapes (x8/x4/x2/x1 to 256^2,
    PGUNet4.forward, UG_unet.py:294-303) against fp64 autograd of F.interpolate."""
    from ugpg import ops
    B, H = 2, 256
    dl = rnd((B, nc, H, H), 97, "dl")
    hres = [32, 64, 128, 256]
    dhs = ops.heads_split_bwd(dl.to(dev), hres)
    for R, dh in zip(hres, dhs):
        h = torch.zeros(B, nc, R, R, dtype=torch.float64, requires_grad=True)
        up = h if R == H else F.interpolate(h, size=(H, H), mode="bilinear", align_corners=True)
        up.backward(dl.double())
        close(nchw(dh.reshape(B, R, R, nc).cpu()), h.grad, 1e-5, f"split bwd R={R}")


@pytest.mark.parametrize("pw,with_u,cu", [(5.0, True, 1), (None, True, 1), (5.0, False, 1), (2.0, True, 2)])
def test_ug_loss(dev, pw, with_u, cu):
    from ugpg import ops
    B, C, H = 3, 2 if cu == 2 else 1, 40
    x = rnd((B, C, H, H), 100, "x", 3.0)
    t = G.bernoulli(101, (B, C, H, H), 0.4, "t")
    u = torch.from_numpy(G.uniform(102, B * cu * H * H, "u").reshape(B, cu, H, H)).float() if with_u else None
    alpha = 1.5
    xd = x.double().requires_grad_(True)
    pwt = None if pw is None else torch.tensor([pw], dtype=torch.float64)
    pl = F.binary_cross_entropy_with_logits(xd, t.double(), pos_weight=pwt, reduction="none")
    final = (pl * (1 + alpha * u.double())).mean() if with_u else pl.mean()
    final.backward()
    g = lambda v: None if v is None else v.to(dev)
    pw_dev = None if pw is None else torch.tensor([pw], device=dev)
    out = ops.ug_loss_fwd(x.to(dev), t.to(dev), g(u), pw_dev, alpha if with_u else 0.0)
    close(out[0:1].cpu(), final.reshape(1), 1e-6, "final")
    close(out[1:2].cpu(), pl.mean().reshape(1), 1e-6, "base")
    gout = torch.tensor([1.0], device=dev)
    dx = ops.ug_loss_bwd(x.to(dev), t.to(dev), g(u), pw_dev, alpha if with_u else 0.0, gout)
    close(dx.cpu(), xd.grad, 1e-5, "dlogits")


def test_seg_metrics_and_mean_std(dev):
    from ugpg import ops
    B, H = 4, 64
    x = rnd((B, 1, H, H), 110, "x", 2.0)
    x[0, 0, 0, :4] = torch.tensor([1e-9, -1e-9, 0.0, 1e-3])  # around the 0.5 threshold
    t = G.bernoulli(111, (B, 1, H, H), 0.3, "t")
    pred = (torch.sigmoid(x) > 0.5).float().squeeze(1)
    ts = t.squeeze(1)
    inter = (pred * ts).view(B, -1).sum(1)
    dice = ((2 * inter + 1) / (pred.view(B, -1).sum(1) + ts.view(B, -1).sum(1) + 1)).mean()
    wrong = pred.ne(ts.long()).sum().item()
    out = ops.seg_metrics(x.to(dev), t.to(dev)).cpu()
    assert abs(out[0].item() - dice.item()) < 1e-6
    assert int(out[2].item()) == wrong
    u = torch.from_numpy(G.uniform(112, 3 * 100003, "u")).float()
    ms = ops.mean_std(u.to(dev)).cpu()
    close(ms[0:1], u.double().mean().reshape(1), 1e-6, "mean")
    close(ms[1:2], u.double().std().reshape(1), 1e-6, "std")


@pytest.mark.parametrize("n,off", [(4096, 0), (1001, 3)])
def test_rmsprop(dev, n, off):
    from ugpg import ops
    p = rnd((n + off,), 120, "p")
    g = rnd((n + off,), 121, "g", 0.1)
    ref_p = p[off:].clone().requires_grad_(True)
    ref_p.grad = g[off:].clone()
    opt = torch.optim.RMSprop([ref_p], lr=1e-3, weight_decay=1e-4)
    pd, gd = p.to(dev), g.to(dev)
    v = torch.zeros(n + off, device=dev)
    for _ in range(3):
        opt.step()
        ops.rmsprop_step(pd[off:], gd[off:], v[off:], 1e-3, 0.99, 1e-8, 1e-4)
    close(pd[off:].cpu(), ref_p.detach(), 1e-6, "rmsprop params")


def test_avgpool_linear(dev):
    from ugpg import ops
    B, C, H = 4, 512, 8
    y = rnd((B, C, H, H), 130, "y")
    sc, sh = rnd((C,), 131, "s", 0.5) + 1, rnd((C,), 132, "h", 0.3)
    a = act_ref(y, sc, sh)
    ref = F.adaptive_avg_pool2d(a, 1).flatten(1)
    out = ops.avgpool_fwd(ops.Act(nhwc(y).to(dev), sc.to(dev), sh.to(dev)))
    close(out.cpu(), ref, 1e-6, "avgpool")
    w = rnd((256, C), 133, "w", 0.05).double().requires_grad_(True)
    b = rnd((256,), 134, "b", 0.05).double().requires_grad_(True)
    xin = ref.double().requires_grad_(True)
    yr = torch.relu(F.linear(xin, w, b))
    dy = rnd(tuple(yr.shape), 135, "dy")
    yr.backward(dy.double())
    yo = ops.linear_fwd(out, w.detach().float().to(dev), b.detach().float().to(dev), True)
    close(yo.cpu(), yr, 1e-5, "linear fwd")
    dyd = dy.to(dev).contiguous()
    dyd = ops.relu_bwd(yo, dyd)
    dx = torch.empty(B, C, device=dev)
    dw = torch.empty(256, C, device=dev)
    db = torch.empty(256, device=dev)
    ops.linear_bwd(out, w.detach().float().to(dev), dyd, dx, dw, db)
    close(dx.cpu(), xin.grad, 1e-5, "linear dx")
    close(dw.cpu(), w.grad, 1e-5, "linear dw")
    close(db.cpu(), b.grad, 1e-5, "linear db")


@pytest.mark.parametrize("conv_math", ["x6", "bf16"])
def test_pack_batch_matches_single_packs(dev, conv_math):
    """ugpg_pack_conv3x3_batch writes the same bytes as one ugpg_pack_conv3x3 per item
    (forward and data-gradient layouts, the 16-channel image layer, > 48 items)."""
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math(conv_math)
    try:
        shapes = [(64, 3, 16, 0), (64, 64, 64, 0), (128, 64, 64, 1), (64, 128, 128, 1),
                  (512, 1024, 1024, 0), (256, 512, 512, 1)] * 9
        ws = [rnd((co, ci, 3, 3), 200 + i, "pw").to(dev) for i, (co, ci, _, _) in enumerate(shapes)]
        specs = [(w, k, m) for w, (_, _, k, m) in zip(ws, shapes)]
        table = ops.prepack(specs)
        assert len(table) == len(specs)
        for w, k, m in specs:
            got = table[ops._pack_key(w, k, m)]
            want = ops.pack_conv3x3(w, k, m)
            assert got.ugpg_fmt == want.ugpg_fmt
            assert torch.equal(got.cpu(), want.cpu())
        with ops.prepacked(table):
            w, k, m = specs[1]
            assert ops.pack_conv3x3(w, k, m) is table[ops._pack_key(w, k, m)]
            w.add_(0.5)  # an in-place change retires the entry (version counter)
            assert ops.pack_conv3x3(w, k, m) is not table.get(ops._pack_key(w, k, m), None)
    finally:
        ops.set_conv_math(old)


@pytest.mark.parametrize("hi,wi,ho,wo", [(96, 80, 64, 64), (32, 32, 256, 256), (256, 256, 128, 128),
                                         (17, 29, 40, 33), (64, 64, 64, 64)])
def test_resize_bilinear_backward(dev, hi, wi, ho, wo):
    """Input gradient of the align-corners resize (ProgressiveUNet.forward's F.interpolate)
    vs torch autograd of F.interpolate in fp32 on the CPU: the same fp32 source-index and
    weight arithmetic (an fp64 reference computes different weights: src = o*(in-1)/(out-1)
    carries ~1e-5 of fp32 rounding at o ~ 127), summed in a different order."""
    from ugpg import ops
    x = torch.randn(2, 3, hi, wi, requires_grad=True)
    g = torch.randn(2, 3, ho, wo)
    torch.nn.functional.interpolate(x, size=(ho, wo), mode="bilinear", align_corners=True).backward(g)
    got = ops.resize_nchw_bwd(g.to(dev), hi, wi).cpu().double()
    ref = x.grad.double()
    assert (got - ref).abs().max().item() <= 1e-5 * max(1.0, ref.abs().max().item())


class _Guards:
    """Device tensors placed inside NaN-canary guard bands (tests/_guard.py); check() asserts
    that no kernel of the test wrote past either end of any of them."""

    def __init__(self, dev):
        self.dev, self.all = dev, []

    def __call__(self, host, name):
        from tests._guard import guarded
        g = guarded(tuple(host.shape), self.dev, host.dtype, fill=host.to(self.dev))
        self.all.append((g, name))
        return g.t

    def empty(self, shape, name, dtype=torch.float32):
        from tests._guard import guarded
        g = guarded(shape, self.dev, dtype)
        self.all.append((g, name))
        return g.t

    def check(self):
        torch.cuda.synchronize()
        for g, name in self.all:
            g.check(name)


LAZY_CASES = [  # B, H, W, C0, C1, Cout: one / two sources, partial tiles, 2 ci and 2 co blocks
    (2, 20, 36, 64, 0, 64),
    (2, 33, 40, 64, 64, 128),
    (1, 64, 64, 128, 0, 64),
    (3, 16, 16, 64, 0, 192),
]


@pytest.mark.parametrize("case", LAZY_CASES)
def test_wgrad_lazy_bn_dy_is_the_apply(dev, case):
    """The BatchNorm-backward apply folded into the split-bf16 weight gradient
    (ugpg_wgrad_t.dy_bn, ops.BnLazyDy): dy formed while loading (da, y) and written once per
    pixel equals the apply pass's dy bit for bit, and so do dW and the finalize's dgamma,
    dbeta and conv bias gradient."""
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math("x6")
    try:
        B, H, W, C0, C1, Cout = case
        cin = C0 + C1
        x0 = nhwc(rnd((B, C0, H, W), 201, "x0")).to(dev)
        x1 = nhwc(rnd((B, C1, H, W), 202, "x1")).to(dev) if C1 else None
        sc0, sh0 = (rnd((C0,), 203, "s", 0.5) + 1).to(dev), rnd((C0,), 204, "h", 0.2).to(dev)
        srcs = [ops.Act(x0, sc0, sh0)] + ([ops.Act(x1)] if C1 else [])
        gd = _Guards(dev)
        y = gd(nhwc(rnd((B, Cout, H, W), 205, "y") + 0.2), "y")
        da = gd(nhwc(rnd((B, Cout, H, W), 206, "da")), "da")
        mean, invstd = rnd((Cout,), 207, "m", 0.1).to(dev), (rnd((Cout,), 208, "i").abs() + 0.5).to(dev)
        scale, shift = (rnd((Cout,), 209, "s", 0.5) + 1).to(dev), rnd((Cout,), 210, "h", 0.3).to(dev)
        # one partial slot: (sum g, sum g*xhat, sum xhat) per channel
        yd, dd = y.double(), da.double()
        g = torch.where(yd * scale.double() + shift.double() > 0, dd, torch.zeros_like(dd))
        xh = (yd - mean.double()) * invstd.double()
        part = torch.stack([g.sum((0, 1, 2)), (g * xh).sum((0, 1, 2)), xh.sum((0, 1, 2))]).float()
        part = gd(part.reshape(3 * Cout, 1).cpu(), "part")
        outs = []
        for lazy in (False, True):
            dg, dbt, dcb = (gd(torch.zeros(Cout), n) for n in ("dgamma", "dbeta", "dbias"))
            dw = gd.empty((Cout, cin, 3, 3), "dW")
            dy = gd.empty(tuple(da.shape), "dy")
            if lazy:
                coef = ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, None, dg, dbt, dcb,
                                       part=part)
                ops.conv3x3_wgrad(srcs, ops.BnLazyDy(da, y, mean, invstd, scale, shift, coef, dy),
                                  dw, None, cin)
            else:
                ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, dy, dg, dbt, dcb, part=part)
                ops.conv3x3_wgrad(srcs, dy, dw, None, cin)
            outs.append((dy, dw, dg, dbt, dcb))
        gd.check()
        for name, a_, b_ in zip(("dy", "dW", "dgamma", "dbeta", "dbias"), *outs):
            assert torch.equal(a_, b_), name
    finally:
        ops.set_conv_math(old)


@pytest.mark.parametrize("math", ["x6", "bf16"])
@pytest.mark.parametrize("shape", [(2, 36, 70), (1, 256, 256)])
def test_wgrad_img_lazy_bn_dy_is_the_apply(dev, shape, math):
    """The image layer's weight gradient (3 real channels of an 8-channel image, 64 outputs)
    forming dy from the following BatchNorm backward (dy_out NULL: no other reader): dW and
    the finalize's outputs bit-identical to the apply pass + the same kernel.  Under the
    bf16 arithmetic y is stored in bf16 (the image layer's output) and the apply writes an
    fp32 dy (the image layer's weight gradient is fp32)."""
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math(math)
    try:
        B, H, W = shape
        C = 64
        img = torch.zeros(B, H, W, 8)
        img[..., :3] = nhwc(rnd((B, 3, H, W), 301, "img"))
        srcs = [ops.Act(img.to(dev))]
        gd = _Guards(dev)
        yh = nhwc(rnd((B, C, H, W), 302, "y") + 0.2)
        y = gd(yh.to(torch.bfloat16) if math == "bf16" else yh, "y")
        da = gd(nhwc(rnd((B, C, H, W), 303, "da")), "da")
        mean, invstd = rnd((C,), 304, "m", 0.1).to(dev), (rnd((C,), 305, "i").abs() + 0.5).to(dev)
        scale, shift = (rnd((C,), 306, "s", 0.5) + 1).to(dev), rnd((C,), 307, "h", 0.3).to(dev)
        part = gd(torch.randn(3 * C, 1, generator=torch.Generator().manual_seed(308)), "part")
        outs = []
        for lazy in (False, True):
            dg, dbt, dcb = (gd(torch.zeros(C), n) for n in ("dgamma", "dbeta", "dbias"))
            dw = gd.empty((C, 3, 3, 3), "dW")
            if lazy:
                coef = ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, None, dg, dbt, dcb,
                                       part=part)
                ops.conv3x3_wgrad(srcs, ops.BnLazyDy(da, y, mean, invstd, scale, shift, coef, None),
                                  dw, None, 3)
            else:
                dy = gd.empty(tuple(da.shape), "dy")
                ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, dy, dg, dbt, dcb, part=part)
                ops.conv3x3_wgrad(srcs, dy, dw, None, 3)
            outs.append((dw, dg, dbt, dcb))
        gd.check()
        for name, a_, b_ in zip(("dW", "dgamma", "dbeta", "dbias"), *outs):
            assert torch.equal(a_, b_), name
    finally:
        ops.set_conv_math(old)


@pytest.mark.parametrize("case", [(2, 20, 36, 64, 0, 64), (2, 33, 41, 64, 64, 128), (1, 64, 64, 128, 0, 64)])
@pytest.mark.parametrize("base", [True, False])
def test_wgrad_lazy_bn_dy_pool_route_is_the_apply(dev, case, base):
    """The folded apply with a deferred MaxPool2d backward routed into da (BlockCtx.route2
    "pool"): the x6w loader adds the routed pooled gradient (argmax window match) to the
    base gradient, as the routed apply does -- dy, dW and the finalize's outputs bit-identical
    to bn_relu_bwd(route=("pool", ...)) + the weight gradient; odd sizes leave the last
    row / column outside the pooled area."""
    from ugpg import ops
    old = ops.conv_math()
    ops.set_conv_math("x6")
    try:
        B, H, W, C0, C1, Cout = case
        cin = C0 + C1
        x0 = nhwc(rnd((B, C0, H, W), 401, "x0")).to(dev)
        x1 = nhwc(rnd((B, C1, H, W), 402, "x1")).to(dev) if C1 else None
        sc0, sh0 = (rnd((C0,), 403, "s", 0.5) + 1).to(dev), rnd((C0,), 404, "h", 0.2).to(dev)
        srcs = [ops.Act(x0, sc0, sh0)] + ([ops.Act(x1)] if C1 else [])
        gd = _Guards(dev)
        y = gd(nhwc(rnd((B, Cout, H, W), 405, "y") + 0.2), "y")
        mean, invstd = rnd((Cout,), 407, "m", 0.1).to(dev), (rnd((Cout,), 408, "i").abs() + 0.5).to(dev)
        scale, shift = (rnd((Cout,), 409, "s", 0.5) + 1).to(dev), rnd((Cout,), 410, "h", 0.3).to(dev)
        _, am = ops.maxpool2_fwd(ops.Act(y, scale, shift))
        am = gd(am.cpu(), "argmax")
        dout = gd(nhwc(rnd((B, Cout, H // 2, W // 2), 411, "dp")), "dout")
        da = gd(nhwc(rnd((B, Cout, H, W), 406, "da")), "da") if base else None
        part = gd(torch.randn(3 * Cout, 1, generator=torch.Generator().manual_seed(412)), "part")
        outs = []
        for lazy in (False, True):
            dg, dbt, dcb = (gd(torch.zeros(Cout), n) for n in ("dgamma", "dbeta", "dbias"))
            dw = gd.empty((Cout, cin, 3, 3), "dW")
            dy = gd.empty(tuple(y.shape), "dy")
            if lazy:
                coef = ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, None, dg, dbt, dcb,
                                       part=part)
                ops.conv3x3_wgrad(srcs, ops.BnLazyDy(da, y, mean, invstd, scale, shift, coef, dy,
                                                     pool=(dout, am)), dw, None, cin)
            else:
                ops.bn_relu_bwd(da, y, mean, invstd, scale, shift, dy, dg, dbt, dcb, part=part,
                                route=("pool", dout, am, H, W))
                ops.conv3x3_wgrad(srcs, dy, dw, None, cin)
            outs.append((dy, dw, dg, dbt, dcb))
        gd.check()
        for name, a_, b_ in zip(("dy", "dW", "dgamma", "dbeta", "dbias"), *outs):
            assert torch.equal(a_, b_), name
    finally:
        ops.set_conv_math(old)


@pytest.mark.parametrize("B,C,H,W,cp", [(2, 3, 17, 19, 8), (16, 3, 64, 64, 8), (2, 1, 9, 7, 1),
                                        (3, 5, 8, 8, 6), (2, 8, 16, 16, 8)])
def test_nchw_to_nhwc_pads_and_copies(dev, B, C, H, W, cp):
    """The image / gradient layout conversion: a pure copy with zero channel padding."""
    from ugpg import ops
    x = rnd((B, C, H, W), 310, "x").to(dev)
    out = ops.nchw_to_nhwc(x, cp)
    ref = torch.zeros(B, H, W, cp, device=dev)
    ref[..., :C] = x.permute(0, 2, 3, 1)
    assert torch.equal(out, ref)
