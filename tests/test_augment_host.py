"""MoNuSeg augmentation, CPU side: the product's host tables / parameter packing, run
through a numpy restatement of csrc/augment.hip, against PIL (oracle/augment_ref.py).
The GPU kernels themselves are checked against PIL in tests/test_gpu_augment.py."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import augment_ref as R
from ugpg import augment as A

import _augment_np as N


def _img(rng, h, w):
    return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("w,h,s", [(1000, 1000, 256), (200, 150, 64), (57, 61, 64), (96, 96, 32)])
def test_resample_tables_match_pil(w, h, s):
    rng = np.random.default_rng(w * 7 + s)
    a = _img(rng, h, w)
    m = rng.integers(0, 2, (h, w), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(a).resize((s, s), Image.BILINEAR))
    refm = np.asarray(Image.fromarray(m).resize((s, s), Image.NEAREST))
    img, msk = N.resize(a, m, s)
    assert np.array_equal(img, ref) and np.array_equal(msk, refm)


def test_nearest_table_matches_pil_over_many_sizes():
    rng = np.random.default_rng(1)
    for _ in range(200):
        w, o = int(rng.integers(20, 1300)), int(rng.integers(8, 300))
        row = np.arange(w, dtype=np.int32)[None, :]
        ref = np.asarray(Image.fromarray(row, mode="I").resize((o, 1), Image.NEAREST))[0]
        assert np.array_equal(A.nearest_table(w, o), ref), (w, o)


def test_draw_params_follow_the_reference_rng():
    for seed in (0, 1, 12345, 2 ** 32 - 1):
        assert A.draw_params(seed) == R.draw_params(seed)
    assert A.hue_shift_u8(-0.05) == 244 and A.hue_shift_u8(0.05) == 12 and A.hue_shift_u8(0.001) == 0


@pytest.mark.parametrize("seed", range(12))
def test_pipeline_restatement_matches_pil(seed):
    rng = np.random.default_rng(seed)
    a = _img(rng, 53, 47)
    m = (rng.random((53, 47)) < 0.3).astype(np.uint8)
    p = R.draw_params(seed * 7919)
    if seed % 4 == 0:
        p["angle"] = 0.0  # no-rotation branch
    x, mm = N.pipeline(a, m, 40, p)
    rx, rm = R.joint_transform(Image.fromarray(a), Image.fromarray(m), 40, p)
    assert torch.equal(torch.from_numpy(x), rx)
    assert torch.equal(torch.from_numpy(mm), rm)


def test_hsv_round_trip_matches_pil_on_a_colour_sample():
    rng = np.random.default_rng(3)
    a = rng.integers(0, 256, (256, 256, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(a).convert("HSV"))
    h, s, v = N.rgb2hsv(*(a[..., i].astype(np.int64) for i in range(3)))
    assert np.array_equal(np.stack([h, s, v], -1), ref)
    hsv = rng.integers(0, 256, (256, 256, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(hsv, "HSV").convert("RGB"))
    r, g, b = N.hsv2rgb(*(hsv[..., i].astype(np.int64) for i in range(3)))
    assert np.array_equal(np.stack([r, g, b], -1), ref)


def test_xml_annotations_rasterise_like_the_reference(tmp_path):
    xml = tmp_path / "a.xml"
    xml.write_text('<Annotations MicronsPerPixel="0.252"><Annotation><Regions>'
                   '<Region><Vertices><Vertex X="3.2" Y="4.9"/><Vertex X="20.7" Y="6.1"/>'
                   '<Vertex X="11.5" Y="18.4"/></Vertices></Region>'
                   '<Region><Vertices><Vertex X="1" Y="1"/><Vertex X="2" Y="2"/></Vertices></Region>'
                   '</Regions></Annotation></Annotations>')
    polys = A.xml_polygons(str(xml))  # regions with < 3 vertices skipped, as the reference
    assert polys == [[(3.2, 4.9), (20.7, 6.1), (11.5, 18.4)]]
    from PIL import ImageDraw
    from oracle import polygon_ref as PR
    ref = Image.fromarray(np.zeros((24, 32), np.uint8))
    ImageDraw.Draw(ref).polygon([(3.2, 4.9), (20.7, 6.1), (11.5, 18.4)], fill=1)
    m = PR.rasterize(24, 32, polys)   # the restatement the GPU kernel is held to
    assert np.array_equal(m, np.asarray(ref)) and m.sum() > 0
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        A.rasterize_polygons(polys, 24, 32, "cpu")


def test_parameter_records_match_the_library_layout():
    A._check_layout()  # struct sizes from the C-ABI (no GPU needed)
    assert A.GEOM_DTYPE.fields["fa"][1] == 48 and A.GEOM_DTYPE.fields["brightness"][1] == 84


def test_create_train_val_split_follows_the_reference_sampling(tmp_path):
    import os
    import random
    for d in ("images", "annots"):
        os.makedirs(tmp_path / "train" / d)
    names = [f"t{k:02d}.tif" for k in range(10)]
    for n in names:
        (tmp_path / "train" / "images" / n).write_bytes(b"x")
        (tmp_path / "train" / "annots" / n.replace(".tif", ".xml")).write_text("<a/>")
    got = A.create_train_val_split(str(tmp_path), val_ratio=0.3, seed=7)
    random.seed(7)
    assert got == random.sample(sorted(names), 3)
    assert sorted(os.listdir(tmp_path / "val" / "images")) == sorted(got)
    assert len(os.listdir(tmp_path / "train" / "images")) == 10  # copy, not move
