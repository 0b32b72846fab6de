"""The polygon-fill oracle (oracle/polygon_ref.py) pinned by the reference's own
rasteriser: the masks PIL ImageDraw.polygon(fill=1) drew for tests/golden/g13 (SURVEY
§8f row 3, monuseg_dataset.py:126-132), and live Pillow on further random cases."""
import random

import numpy as np
import pytest

from oracle import polygon_cases as PC
from oracle import polygon_ref as PR


def _golden():
    fx = np.load("tests/golden/g13_polygons.npz")
    cases = PC.unpack(fx)
    masks = []
    for c, (H, W, _) in enumerate(cases):
        b = fx["mask_bits"][fx["mask_off"][c]:fx["mask_off"][c + 1]]
        masks.append(np.unpackbits(b)[:H * W].reshape(H, W))
    return cases, masks


def test_oracle_reproduces_pillow_golden_masks():
    cases, masks = _golden()
    assert len(cases) == 361 and cases[0][:2] == (1000, 1000)
    for (H, W, polys), want in zip(cases, masks):
        assert np.array_equal(PR.rasterize(H, W, polys), want)


def test_golden_covers_the_hard_cases():
    """The fixture exercises what a scan converter gets wrong: the corner rule fires,
    horizontal runs merge, spans clip at both borders, polygons lie wholly outside."""
    cases, masks = _golden()
    big = masks[0]
    assert 0.02 < big.mean() < 0.5                       # MoNuSeg-like coverage
    assert big[0].any() and big[-1].any() and big[:, 0].any() and big[:, -1].any()
    assert any(not m.any() for m in masks[1:])           # wholly off-canvas
    verts = np.load("tests/golden/g13_polygons.npz")["verts"]
    assert (verts < 0).any() and (verts == np.round(verts)).any()


@pytest.mark.parametrize("seed", [101, 202])
def test_oracle_matches_live_pillow(seed):
    pytest.importorskip("PIL")
    rng = random.Random(seed)
    for t in range(400):
        H, W = rng.randint(4, 48), rng.randint(4, 48)
        polys = [PC.odd_polygon(rng, H, W, (t + j) % 6) for j in range(1 + t % 2)]
        assert np.array_equal(PR.rasterize(H, W, polys), PC.render_pil(H, W, polys)), polys
