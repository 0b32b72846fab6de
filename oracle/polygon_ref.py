"""CPU restatement of Pillow's filled-polygon scan converter (TEST INFRASTRUCTURE -- only
tests/ and oracle/make_goldens.py use it; the product path is the HIP kernel
ugpg_rasterize_polygons in csrc/augment.hip).

The reference rasterises every MoNuSeg nucleus with ``ImageDraw.Draw(mask).polygon(pts,
fill=1)`` on a uint8 "L" image (MoNuSegImprove/monuseg_dataset.py:126-132,
aug_monuseg_dataset.py:89-111).  Pillow is a third-party dependency, not vendored in the
reference; the version here is Pillow 12.2.0 (PIL.__version__).  Its C source is not in
this container, so the algorithm below was restated from the behaviour and the machine
code of the installed ``PIL/_imaging`` module (``_draw_polygon``, ``ImagingDrawPolygon``,
``polygon_generic``, ``hline8`` of libImaging/Draw.c, read with objdump), then pinned
against Pillow itself on random, concave, self-intersecting, degenerate, sub-pixel and
off-canvas polygons (tests/golden/g13_polygons.npz, tests/test_polygon_oracle.py):

1. vertices: Python floats -> C int by truncation toward zero (``cvttpd2dq``);
2. edges, in vertex order, closing edge last unless the last vertex equals the first;
   a horizontal edge that continues a horizontal edge in the same x direction extends
   the previous edge instead (xmax / xmin); dx = float(x1-x0) / float(y1-y0) in float;
3. horizontal edges are drawn as spans [xmin, xmax] on their row; the polygon's row
   range is [max(ymin, 0), min(ymax, H)] over ALL edges;
4. per row y, per non-horizontal edge i with ymin <= y <= ymax, in edge order:
   x = float(y - y0) * dx + float(x0) (float, no fused multiply-add);
   if y == ymax_edge and y < ymax_poly: x is entered twice; otherwise, if y is the
   edge's ymin or ymax and dx != 0, the first earlier edge k < i that also ends or
   starts on row y, has dx != 0, roundf-matches x on row y and spans the adjacent row
   (y - 1 when y is edge i's ymax, else y + 1) decides a corner: with a_i, a_k the two
   edges' x on the adjacent row, x > a_i + 1 and x > a_k + 1 -> x = roundf(max) + 1;
   x < a_i - 1 and x < a_k - 1 -> x = roundf(min) - 1 (float);
5. the row's x values sorted ascending; pairs (x[2m], x[2m+1]) filled from
   ROUND_UP(x[2m]) to ROUND_DOWN(x[2m+1]) inclusive, where for f >= 0
   ROUND_UP = floor(f + 0.5f), ROUND_DOWN = ceil(f - 0.5f) in float, and for f < 0
   ROUND_UP = -floor(|f| + 0.5), ROUND_DOWN = -ceil(|f| - 0.5) in double;
6. a span is clipped to [0, W-1]; nothing is drawn when it is empty after clipping or
   its row is outside [0, H).
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np

f32 = np.float32
INT_MIN = -(1 << 31)


def _trunc_int(v: float) -> int:
    """C (int) of a double: toward zero; out of range -> INT_MIN (x86 cvttpd2dq)."""
    if not math.isfinite(v) or v >= 2 ** 31 or v <= -(2 ** 31) - 1:
        return INT_MIN
    return int(v)


def _roundf(v) -> float:
    """C roundf: half away from zero."""
    v = float(v)
    return float(math.floor(v + 0.5)) if v >= 0 else -float(math.floor(-v + 0.5))


def _round_up(f) -> int:
    f = f32(f)
    if f >= 0:
        return int(math.floor(f32(f + f32(0.5))))
    return -int(math.floor(abs(float(f)) + 0.5))


def _round_down(f) -> int:
    f = f32(f)
    if f >= 0:
        return int(math.ceil(f32(f - f32(0.5))))
    return -int(math.ceil(abs(float(f)) - 0.5))


class _Edge:
    __slots__ = ("x0", "y0", "xmin", "xmax", "ymin", "ymax", "dx")

    def __init__(self, x0, y0, x1, y1):
        self.xmin, self.xmax = (x0, x1) if x0 <= x1 else (x1, x0)
        self.ymin, self.ymax = (y0, y1) if y0 <= y1 else (y1, y0)
        self.dx = f32(0) if y0 == y1 else f32(f32(x1 - x0) / f32(y1 - y0))
        self.x0, self.y0 = x0, y0

    def x_at(self, y):
        return f32(f32(f32(y - self.y0) * self.dx) + f32(self.x0))


def _edges(xy: List[int]) -> List[_Edge]:
    count = len(xy) // 2
    e: List[_Edge] = []
    i = 0
    for i in range(count - 1):
        x0, y0, x1, y1 = xy[2 * i], xy[2 * i + 1], xy[2 * i + 2], xy[2 * i + 3]
        if y0 == y1 and i != 0 and y0 == xy[2 * i - 1]:
            # a horizontal edge continuing a horizontal edge in the same direction
            if x1 > x0 and x0 > xy[2 * i - 2]:
                e[-1].xmax = x1
                continue
            if x1 < x0 and x0 < xy[2 * i - 2]:
                e[-1].xmin = x1
                continue
        e.append(_Edge(x0, y0, x1, y1))
    i = count - 1
    if xy[2 * i] != xy[0] or xy[2 * i + 1] != xy[1]:
        e.append(_Edge(xy[2 * i], xy[2 * i + 1], xy[0], xy[1]))
    return e


def fill_polygon(mask: np.ndarray, points: Sequence[Tuple[float, float]], ink: int = 1) -> None:
    """ImageDraw.Draw(Image.fromarray(mask)).polygon(points, fill=ink), in place, on a
    uint8 (H, W) array."""
    H, W = mask.shape
    if len(points) < 2:
        raise TypeError("coordinate list must contain at least 2 coordinates")
    xy: List[int] = []
    for x, y in points:
        xy += [_trunc_int(float(x)), _trunc_int(float(y))]

    def hline(x0, y, x1):
        if y < 0 or y >= H:
            return
        if x0 < 0:
            if x1 < 0:
                return
            x0 = 0
        elif x0 >= W or x1 < 0:
            return
        if x1 >= W:
            x1 = W - 1
        if x1 >= x0:
            mask[y, x0:x1 + 1] = ink

    ymin, ymax = H - 1, 0
    table: List[_Edge] = []
    for ed in _edges(xy):
        ymin = min(ymin, ed.ymin)
        ymax = max(ymax, ed.ymax)
        if ed.ymin == ed.ymax:
            hline(ed.xmin, ed.ymin, ed.xmax)
            continue
        table.append(ed)
    ymin = max(ymin, 0)
    ymax = min(ymax, H)
    for y in range(ymin, ymax + 1):
        xx = []
        for i, cur in enumerate(table):
            if not (cur.ymin <= y <= cur.ymax):
                continue
            x = cur.x_at(y)
            if y == cur.ymax and y < ymax:
                xx += [x, x]
                continue
            if (y == cur.ymin or y == cur.ymax) and cur.dx != 0:
                adj = y - 1 if y == cur.ymax else y + 1
                for k in range(i):
                    oth = table[k]
                    if not ((y == oth.ymin or y == oth.ymax) and oth.dx != 0):
                        continue
                    if _roundf(x) != _roundf(oth.x_at(y)):
                        continue
                    if not (oth.ymin <= adj <= oth.ymax):
                        continue
                    ac, ao = cur.x_at(adj), oth.x_at(adj)
                    if x > f32(ac + f32(1)) and x > f32(ao + f32(1)):
                        x = f32(f32(_roundf(max(float(ac), float(ao)))) + f32(1))
                    elif x < f32(ac - f32(1)) and x < f32(ao - f32(1)):
                        x = f32(f32(_roundf(min(float(ac), float(ao)))) - f32(1))
                    break
            xx.append(x)
        xx.sort()
        for m in range(1, len(xx), 2):
            hline(_round_up(xx[m - 1]), y, _round_down(xx[m]))


def rasterize(H: int, W: int, polygons: Sequence[Sequence[Tuple[float, float]]],
              ink: int = 1) -> np.ndarray:
    """A fresh (H, W) uint8 mask with every polygon filled in order (the reference's
    region loop, monuseg_dataset.py:117-132, without its < 3 vertex filter)."""
    m = np.zeros((H, W), np.uint8)
    for p in polygons:
        fill_polygon(m, p, ink)
    return m
