"""GPU polygon rasterisation (the reference's XML -> mask step,
MoNuSegImprove/monuseg_dataset.py:117-132, PIL ImageDraw.polygon(fill=1)) against the
masks Pillow drew (tests/golden/g13) and live Pillow: bit-exact, torch.equal."""
import random

import numpy as np
import pytest
import torch

from oracle import polygon_cases as PC

pytestmark = pytest.mark.gpu


def _golden():
    fx = np.load("tests/golden/g13_polygons.npz")
    cases = PC.unpack(fx)
    masks = []
    for c, (H, W, _) in enumerate(cases):
        b = fx["mask_bits"][fx["mask_off"][c]:fx["mask_off"][c + 1]]
        masks.append(np.unpackbits(b)[:H * W].reshape(H, W))
    return cases, masks


def test_rasterize_matches_pillow_golden_masks(dev):
    from ugpg.augment import rasterize_polygons
    cases, masks = _golden()
    bad = []
    for c, ((H, W, polys), want) in enumerate(zip(cases, masks)):
        got = rasterize_polygons(polys, H, W, dev).cpu().numpy()
        if not np.array_equal(got, want):
            bad.append((c, int((got != want).sum())))
    assert not bad, f"{len(bad)} of {len(cases)} canvases differ (case, pixels): {bad[:10]}"


@pytest.mark.parametrize("seed", [7, 8, 9])
def test_rasterize_matches_live_pillow(dev, seed):
    from ugpg.augment import rasterize_polygons
    rng = random.Random(seed)
    for t in range(150):
        H, W = rng.randint(4, 80), rng.randint(4, 80)
        polys = [PC.odd_polygon(rng, H, W, (t + j) % 6) for j in range(1 + t % 4)]
        got = rasterize_polygons(polys, H, W, dev).cpu().numpy()
        assert np.array_equal(got, PC.render_pil(H, W, polys)), (H, W, polys)


def test_rasterize_draws_into_an_existing_mask_with_ink(dev):
    """`out` is drawn into, not cleared, and `ink` is the fill value (PIL's fill=ink)."""
    from ugpg.augment import rasterize_polygons
    rng = random.Random(3)
    a = [PC.nucleus(rng, 20, 20, 9, 16)]
    b = [PC.nucleus(rng, 30, 26, 7, 12)]
    m = rasterize_polygons(a, 48, 50, dev, ink=7)
    rasterize_polygons(b, 48, 50, dev, ink=200, out=m)
    from PIL import Image, ImageDraw
    ref = Image.fromarray(np.zeros((48, 50), np.uint8))
    d = ImageDraw.Draw(ref)
    d.polygon(a[0], fill=7)
    d.polygon(b[0], fill=200)
    assert np.array_equal(m.cpu().numpy(), np.asarray(ref))
    with pytest.raises(TypeError):
        rasterize_polygons([[(1.0, 2.0)]], 8, 8, dev)


def test_monuseg_sized_mask_throughput(dev):
    """One MoNuSeg image's annotation (1000 x 1000, ~600 nuclei) in one launch pair;
    reported, and checked against Pillow."""
    import time
    from ugpg.augment import rasterize_polygons
    cases, masks = _golden()
    H, W, polys = cases[0]
    rasterize_polygons(polys, H, W, dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        m = rasterize_polygons(polys, H, W, dev)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    t1 = time.perf_counter()
    ref = PC.render_pil(H, W, polys)
    dp = time.perf_counter() - t1
    assert np.array_equal(m.cpu().numpy(), ref)
    print(f"1000x1000 mask, {len(polys)} polygons: GPU {dt * 1e3:.2f} ms per mask "
          f"(incl. host packing and upload), PIL {dp * 1e3:.2f} ms")
