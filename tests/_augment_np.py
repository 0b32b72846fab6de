"""numpy restatement of csrc/augment.hip (test infrastructure): the same per-pixel
formulas as the kernels, driven by the product's host tables and parameter packing,
so the CPU suite checks the algorithm against PIL without a GPU."""
import numpy as np

from ugpg import augment as A


def resample_pass(img, axis, n_out):
    n_in = img.shape[axis]
    b, k = A.resample_coeffs(n_in, n_out)
    x = np.moveaxis(img, axis, 0).astype(np.int64)
    out = np.zeros((n_out,) + x.shape[1:], np.uint8)
    for o in range(n_out):
        lo, n = b[o]
        acc = np.full(x.shape[1:], 1 << (A.PRECISION_BITS - 1), np.int64)
        for t in range(n):
            acc += x[lo + t] * int(k[o, t])
        out[o] = np.clip(acc >> A.PRECISION_BITS, 0, 255)
    return np.moveaxis(out, 0, axis)


def resize(img, mask, S):
    H, W, _ = img.shape
    if W != S:
        img = resample_pass(img, 1, S)
    if H != S:
        img = resample_pass(img, 0, S)
    if (H, W) != (S, S):
        mask = mask[A.nearest_table(H, S)][:, A.nearest_table(W, S)]
    return img, mask


def blend(in1, in2, alpha):
    a = np.float32(alpha)
    t = np.float32(in1) + a * (np.float32(in2) - np.float32(in1))
    t = t.astype(np.float32)
    return np.where(t <= 0, 0, np.where(t >= 255, 255, np.trunc(t))).astype(np.int64)


def lum(r, g, b):
    return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16


def geom(img, mask, g):
    S = img.shape[0]
    y, x = np.mgrid[0:S, 0:S]
    fx = (lambda v: S - 1 - v) if g["hflip"] else (lambda v: v)
    fy = (lambda v: S - 1 - v) if g["vflip"] else (lambda v: v)
    src = img.astype(np.float64)
    if not g["rotate"]:
        rgb = img[fy(y), fx(x)].astype(np.int64)
        mv = mask[fy(y), fx(x)]
    else:
        a = g["a"]
        xi, yi = x + 0.5, y + 0.5
        xin = (a[0] * xi + a[1] * yi) + a[2]
        yin = (a[3] * xi + a[4] * yi) + a[5]
        ok = (xin >= 0) & (xin < S) & (yin >= 0) & (yin < S)
        xin, yin = xin - 0.5, yin - 0.5
        xf, yf = np.floor(xin).astype(np.int64), np.floor(yin).astype(np.int64)
        dx, dy = xin - xf, yin - yf
        x0, x1 = np.clip(xf, 0, S - 1), np.clip(xf + 1, 0, S - 1)
        y0 = np.clip(yf, 0, S - 1)
        has1 = (yf + 1 >= 0) & (yf + 1 < S)
        y1 = np.where(has1, yf + 1, y0)
        rgb = np.zeros((S, S, 3), np.int64)
        for c in range(3):
            a0, b0 = src[fy(y0), fx(x0), c], src[fy(y0), fx(x1), c]
            v1 = a0 + (b0 - a0) * dx
            a1, b1 = src[fy(y1), fx(x0), c], src[fy(y1), fx(x1), c]
            v2 = np.where(has1, a1 + (b1 - a1) * dx, v1)
            v = v1 + (v2 - v1) * dy
            rgb[..., c] = np.where(ok, np.clip(np.trunc(v), 0, 255), 0)
        fa = [int(v) for v in g["fa"]]
        xx = fa[2] + y * fa[1] + x * fa[0]
        yy = fa[5] + y * fa[4] + x * fa[3]
        sx, sy = xx >> 16, yy >> 16
        okm = (sx >= 0) & (sx < S) & (sy >= 0) & (sy < S)
        mv = np.where(okm, mask[fy(np.clip(sy, 0, S - 1)), fx(np.clip(sx, 0, S - 1))], 0)
    if g["brightness"] != np.float32(1.0):
        rgb = blend(0, rgb, g["brightness"])
    return rgb, mv.astype(np.uint8)


def rgb2hsv(r, g, b):
    rgb = np.stack([r, g, b], -1)
    maxc = rgb.max(-1); minc = rgb.min(-1)
    with np.errstate(divide="ignore", invalid="ignore"):
        cr = (maxc - minc).astype(np.float32)
        s = cr / maxc.astype(np.float32)
        rc = (maxc - r).astype(np.float32) / cr
        gc = (maxc - g).astype(np.float32) / cr
        bc = (maxc - b).astype(np.float32) / cr
        rc64, gc64, bc64 = (v.astype(np.float64) for v in (rc, gc, bc))
        h = np.where(r == maxc, (bc - gc).astype(np.float64),
                     np.where(g == maxc, (2.0 + rc64 - bc64).astype(np.float32).astype(np.float64),
                              (4.0 + gc64 - rc64).astype(np.float32).astype(np.float64)))
        h = np.fmod(h / 6.0 + 1.0, 1.0).astype(np.float32)
        uh = np.clip(np.nan_to_num(h.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
        us = np.clip(np.nan_to_num(s.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    eq = maxc == minc
    return np.where(eq, 0, uh), np.where(eq, 0, us), maxc


def hsv2rgb(h, s, v):
    h6 = h.astype(np.float32).astype(np.float64) * 6.0 / 255.0
    i = np.floor(h6).astype(np.int64)
    f = (h6 - i.astype(np.float64)).astype(np.float32)
    fs = (s.astype(np.float32).astype(np.float64) / 255.0).astype(np.float32)
    vf = v.astype(np.float64)

    def rnd(z):
        return np.clip(np.floor(z + 0.5).astype(np.int64), 0, 255)
    p = rnd(vf * (1.0 - fs.astype(np.float64)))
    q = rnd(vf * (1.0 - (fs * f).astype(np.float64)))
    t = rnd(vf * (1.0 - fs.astype(np.float64) * (1.0 - f.astype(np.float64))))
    i6 = i % 6
    r = np.choose(i6, [v, q, p, p, t, v]); g = np.choose(i6, [t, v, v, q, p, p])
    b = np.choose(i6, [p, p, t, v, v, q])
    sz = s == 0
    return np.where(sz, v, r), np.where(sz, v, g), np.where(sz, v, b)


def color(rgb, mask, c):
    r, g, b = (rgb[..., i].astype(np.int64) for i in range(3))
    if c["jitter"]:
        mean = int(float(lum(r, g, b).sum()) / r.size + 0.5)
        if c["contrast"] != np.float32(1.0):
            r, g, b = (blend(mean, v, c["contrast"]) for v in (r, g, b))
        if c["saturation"] != np.float32(1.0):
            l = lum(r, g, b)
            r, g, b = (blend(l, v, c["saturation"]) for v in (r, g, b))
        h, s, v = rgb2hsv(r, g, b)
        h = (h + int(c["hue_shift"])) & 255
        r, g, b = hsv2rgb(h, s, v)
    x = np.stack([r, g, b]).astype(np.float32) / np.float32(255)
    return x, mask.astype(np.float32)[None]


def pipeline(img, mask, S, params):
    img, mask = resize(img, mask, S)
    if params is None:
        params = {"hflip": False, "vflip": False, "angle": 0.0, "jitter": False,
                  "b": 1.0, "c": 1.0, "s": 1.0, "h": 0.0}
    g, c = A.pack_params([params], S)
    rgb, mv = geom(img, mask, g[0])
    return color(rgb, mv, c[0])
