"""Polygon test cases for the MoNuSeg mask rasteriser (TEST INFRASTRUCTURE).

Deterministic canvases of polygons in the shapes the reference's XML annotations
produce (MoNuSegImprove/monuseg_dataset.py:97-135: float vertex coordinates, one filled
polygon per nucleus, all regions of an image drawn into one uint8 mask) plus the cases a
scan converter gets wrong: concave, self-intersecting, integer and half-integer vertices,
axis-aligned runs (Pillow merges consecutive horizontal edges), repeated vertices,
collinear and sub-pixel polygons, polygons partly or wholly off the canvas, negative
coordinates.  ``render_pil`` is the reference's own call (PIL ImageDraw.polygon,
fill=1), used only to make fixtures and as the checker in tests.
"""
from __future__ import annotations

import math
import random
from typing import List, Sequence, Tuple

import numpy as np

Poly = List[Tuple[float, float]]


def nucleus(rng: random.Random, cx: float, cy: float, r: float, n: int, ndp: int = 4) -> Poly:
    """A star-shaped nucleus outline, vertices rounded to `ndp` decimals (the XML's)."""
    angs = sorted(rng.uniform(0, 2 * math.pi) for _ in range(n))
    pts = []
    for a in angs:
        rr = r * rng.uniform(0.6, 1.0)
        pts.append((round(cx + rr * math.cos(a), ndp), round(cy + rr * math.sin(a), ndp)))
    return pts


def odd_polygon(rng: random.Random, H: int, W: int, kind: int) -> Poly:
    n = rng.randint(3, 40)
    cx, cy = rng.uniform(-10, W + 10), rng.uniform(-10, H + 10)
    r = rng.uniform(0.3, 25)
    pts: Poly = []
    if kind == 0:      # star-shaped, full precision
        pts = nucleus(rng, cx, cy, r, n, ndp=12)
    elif kind == 1:    # random vertices: self-intersecting
        pts = [(cx + rng.uniform(-r, r), cy + rng.uniform(-r, r)) for _ in range(n)]
    elif kind == 2:    # integer / half-integer / near-half vertices
        for _ in range(n):
            pts.append((round(cx + rng.uniform(-r, r)) + rng.choice([0, 0.5, -0.5, 0.49, 0.51]),
                        round(cy + rng.uniform(-r, r)) + rng.choice([0, 0.5, -0.5, 0.999])))
    elif kind == 3:    # axis-aligned walks: horizontal runs, repeats, collinear
        x, y = cx, cy
        for _ in range(n):
            if rng.random() < 0.5:
                x += rng.choice([-1, 1]) * rng.randint(0, 6)
            else:
                y += rng.choice([-1, 1]) * rng.randint(0, 6)
            pts.append((x, y))
    elif kind == 4:    # sub-pixel and thin slivers
        pts = [(cx + rng.uniform(-0.9, 0.9), cy + rng.uniform(-0.9, 0.9)) for _ in range(n % 6 + 3)]
        if rng.random() < 0.5:  # a long thin sliver
            pts = [(cx, cy), (cx + rng.uniform(-30, 30), cy + rng.uniform(-30, 30)),
                   (cx + rng.uniform(-1, 1), cy + rng.uniform(-1, 1))]
    else:              # repeated vertices and a closing vertex equal to the first
        base = nucleus(rng, cx, cy, r, max(3, n // 2), ndp=2)
        pts = []
        for p in base:
            pts += [p] * rng.randint(1, 3)
        if rng.random() < 0.5:
            pts.append(pts[0])
    return pts


def canvases(seed: int = 13, n_small: int = 360) -> List[Tuple[int, int, List[Poly]]]:
    """(H, W, polygons) cases: one MoNuSeg-sized 1000 x 1000 canvas of 600 nuclei (radius
    3-14 px, 8-36 vertices, 4 decimals, some touching the border or overlapping), and
    n_small small canvases of 1-3 odd polygons each."""
    rng = random.Random(seed)
    out = []
    big = []
    for _ in range(600):
        big.append(nucleus(rng, rng.uniform(-5, 1005), rng.uniform(-5, 1005),
                           rng.uniform(3, 14), rng.randint(8, 36)))
    out.append((1000, 1000, big))
    for t in range(n_small):
        H, W = rng.randint(5, 64), rng.randint(5, 64)
        polys = [odd_polygon(rng, H, W, (t + j) % 6) for j in range(1 + t % 3)]
        out.append((H, W, polys))
    return out


def render_pil(H: int, W: int, polys: Sequence[Poly]) -> np.ndarray:
    """The reference's rasterisation: each polygon filled with 1 into one "L" mask."""
    from PIL import Image, ImageDraw
    m = Image.fromarray(np.zeros((H, W), np.uint8))
    d = ImageDraw.Draw(m)
    for p in polys:
        d.polygon(p, fill=1)
    return np.array(m)


def pack(cases) -> dict:
    """Flat arrays: verts (N, 2) float64, poly_off (P+1), case_poly (C+1), hw (C, 2)."""
    verts, poly_off, case_poly, hw = [], [0], [0], []
    for H, W, polys in cases:
        for p in polys:
            verts.extend(p)
            poly_off.append(len(verts))
        case_poly.append(len(poly_off) - 1)
        hw.append((H, W))
    return {"verts": np.asarray(verts, np.float64).reshape(-1, 2),
            "poly_off": np.asarray(poly_off, np.int64),
            "case_poly": np.asarray(case_poly, np.int64), "hw": np.asarray(hw, np.int64)}


def unpack(fx) -> List[Tuple[int, int, List[Poly]]]:
    verts, po, cp, hw = fx["verts"], fx["poly_off"], fx["case_poly"], fx["hw"]
    out = []
    for c in range(len(hw)):
        polys = [[(float(x), float(y)) for x, y in verts[po[p]:po[p + 1]]]
                 for p in range(cp[c], cp[c + 1])]
        out.append((int(hw[c][0]), int(hw[c][1]), polys))
    return out
