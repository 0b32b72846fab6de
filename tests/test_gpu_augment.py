"""MoNuSeg augmentation on the GPU vs PIL (oracle/augment_ref.py, the reference's
_apply_joint_transforms on PIL images): every output tensor must be identical."""
import numpy as np
import pytest
import torch
from PIL import Image

from oracle import augment_ref as R

pytestmark = pytest.mark.gpu


def _batch(rng, B, h, w):
    imgs = rng.integers(0, 256, (B, h, w, 3), dtype=np.uint8)
    masks = (rng.random((B, h, w)) < 0.35).astype(np.uint8)
    return imgs, masks


def _check(aug, imgs, masks, params, S):
    dev = torch.device("cuda")
    x, m = aug(torch.from_numpy(imgs).to(dev), torch.from_numpy(masks).to(dev), params)
    x, m = x.cpu(), m.cpu()
    for i in range(len(imgs)):
        rx, rm = R.joint_transform(Image.fromarray(imgs[i]), Image.fromarray(masks[i]), S,
                                   None if params is None else params[i])
        assert torch.equal(x[i], rx), (i, (x[i] != rx).sum().item())
        assert torch.equal(m[i], rm), (i, (m[i] != rm).sum().item())


@pytest.mark.parametrize("h,w,S,B", [(1000, 1000, 256, 4), (150, 200, 64, 3), (64, 64, 64, 2)])
def test_augment_matches_pil(dev, h, w, S, B):
    from ugpg.augment import MoNuSegAugmenter
    rng = np.random.default_rng(h + S)
    imgs, masks = _batch(rng, B, h, w)
    params = [R.draw_params(int(s)) for s in rng.integers(0, 2 ** 32, B)]
    params[0] = dict(params[0], angle=0.0)          # no-rotation branch
    if B > 2:
        params[2] = dict(params[2], jitter=False)    # no colour jitter
    _check(MoNuSegAugmenter(S, dev), imgs, masks, params, S)


def test_resize_only_matches_pil(dev):
    from ugpg.augment import MoNuSegAugmenter
    rng = np.random.default_rng(5)
    imgs, masks = _batch(rng, 3, 333, 257)
    _check(MoNuSegAugmenter(128, dev), imgs, masks, None, 128)


def test_many_seeds_small(dev):
    from ugpg.augment import MoNuSegAugmenter
    rng = np.random.default_rng(9)
    imgs, masks = _batch(rng, 32, 90, 110)
    params = [R.draw_params(int(s)) for s in rng.integers(0, 2 ** 32, 32)]
    _check(MoNuSegAugmenter(48, dev), imgs, masks, params, 48)


def _write_dataset(root, split_dir, n, size, rng):
    import os
    idir, adir = os.path.join(root, *split_dir, "images"), os.path.join(root, *split_dir, "annots")
    os.makedirs(idir)
    os.makedirs(adir)
    for k in range(n):
        Image.fromarray(rng.integers(0, 256, (size, size, 3), dtype=np.uint8)).save(
            os.path.join(idir, f"s{k}.tif"))
        regs = []
        for _ in range(6):
            cx, cy = rng.uniform(10, size - 10, 2)
            ang = np.sort(rng.uniform(0, 2 * np.pi, 8))
            pts = "".join(f'<Vertex X="{cx + 8 * np.cos(a):.3f}" Y="{cy + 6 * np.sin(a):.3f}"/>'
                          for a in ang)
            regs.append(f"<Region><Vertices>{pts}</Vertices></Region>")
        with open(os.path.join(adir, f"s{k}.xml"), "w") as f:
            f.write('<Annotations><Annotation><Regions>' + "".join(regs) +
                    "</Regions></Annotation></Annotations>")


def test_datasets_match_reference_behaviour(dev, tmp_path):
    from ugpg.augment import AugMoNuSegDataset, MoNuSegDataset, xml_polygons
    from oracle.polygon_cases import render_pil

    def parse_xml_annotations(path, size):  # the reference's PIL rasterisation
        return render_pil(size[1], size[0], xml_polygons(path))
    rng = np.random.default_rng(11)
    _write_dataset(str(tmp_path), ("train", "aug"), 3, 120, rng)
    _write_dataset(str(tmp_path), ("test",), 2, 120, rng)
    ds = AugMoNuSegDataset(str(tmp_path), image_size=64, device=dev)
    assert len(ds) == 3 and ds.get_sample_info(0)["num_nuclei"] == 6
    torch.manual_seed(123)
    got = [ds[i] for i in range(3)]
    torch.manual_seed(123)
    for i in range(3):
        img_path, ann_path = ds.samples[i]
        image = Image.open(img_path).convert("RGB")
        mask = Image.fromarray(parse_xml_annotations(ann_path, image.size))
        p = R.draw_params(torch.randint(0, 2 ** 32, (1,)).item())
        rx, rm = R.joint_transform(image, mask, 64, p)
        assert torch.equal(got[i][0].cpu(), rx) and torch.equal(got[i][1].cpu(), rm)
    # test split: no augmentation, resize only; batch form = per-item form
    ts = MoNuSegDataset(str(tmp_path), image_size=32, split="test", device=dev)
    xb, mb = ts.get_batch([0, 1])
    for i in range(2):
        img_path, ann_path = ts.samples[i]
        image = Image.open(img_path).convert("RGB")
        mask = Image.fromarray(parse_xml_annotations(ann_path, image.size))
        rx, rm = R.joint_transform(image, mask, 32, None)
        assert torch.equal(xb[i].cpu(), rx) and torch.equal(mb[i].cpu(), rm)
