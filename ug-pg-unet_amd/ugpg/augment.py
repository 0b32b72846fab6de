"""MoNuSeg data pipeline with the per-sample augmentation on the GPU.

Reference behaviour: ``aug_monuseg_dataset.py:22-188``
(``AugMoNuSegDataset``) and ``monuseg_dataset.py:21-242`` (``MoNuSegDataset``):
XML polygons rasterised with ``ImageDraw.polygon(fill=1)`` (:89-111), then per sample
``Image.resize`` BILINEAR / NEAREST, hflip, vflip, ``rotate(angle)`` BILINEAR /
NEAREST, ``TF.adjust_brightness/contrast/saturation/hue`` and ``ToTensor`` (:113-148),
the random parameters drawn from ``random.Random(torch.randint(0, 2**32))``.

Here the decode (PIL ``Image.open``) runs once per image on the host; the XML polygons
are rasterised on the GPU by Pillow's own scan converter reproduced bit for bit
(``rasterize_polygons``, ``ugpg_rasterize_polygons``); image and mask are cached in HBM,
and every random transform runs on the GPU (``csrc/augment.hip``) with PIL's own 8-bit
arithmetic, so the tensors equal the reference's bit for bit for the same torch RNG
state (``tests/test_gpu_augment.py`` and ``tests/test_gpu_polygons.py`` check against
PIL).  The product path needs the HIP library: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import random
import xml.etree.ElementTree as ET
from typing import Any, Dict, List, Tuple

import numpy as np
import torch

from ._C import check, lib

PRECISION_BITS = 22  # PIL Resample.c, 8-bit images

GEOM_DTYPE = np.dtype([("a", "<f8", (6,)), ("fa", "<i4", (6,)), ("rotate", "<i4"),
                       ("hflip", "<i4"), ("vflip", "<i4"), ("brightness", "<f4"),
                       ("pad", "<i4")], align=True)   # C struct AugGeom (augment.hip)
COLOR_DTYPE = np.dtype([("jitter", "<i4"), ("contrast", "<f4"), ("saturation", "<f4"),
                        ("hue_shift", "<i4")], align=True)


def _check_layout():
    g, c = C.c_int(0), C.c_int(0)
    check(lib.ugpg_augment_param_sizes(C.byref(g), C.byref(c)), "augment_param_sizes")
    if g.value != GEOM_DTYPE.itemsize or c.value != COLOR_DTYPE.itemsize:
        raise RuntimeError(f"augment parameter layout mismatch: library {g.value}/{c.value} B, "
                           f"host {GEOM_DTYPE.itemsize}/{COLOR_DTYPE.itemsize} B")


# ----------------------------------------------------------------- PIL geometry tables
def resample_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray]:
    """PIL's bilinear antialiasing coefficients (Resample.c precompute_coeffs +
    normalize_coeffs_8bpc): bounds (out, 2) = (first tap, tap count) and the 22-bit
    fixed-point taps (out, ksize)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.float64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = np.zeros(xmax)
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            w[x] = 1.0 - t if t < 1.0 else 0.0
        ww = float(np.sum(w)) if xmax else 0.0
        # sequential sum as in C
        ww = 0.0
        for x in range(xmax):
            ww += w[x]
        for x in range(xmax):
            kk[xx, x] = w[x] / ww if ww != 0.0 else w[x]
        bounds[xx] = (xmin, xmax)
    scaled = kk * (1 << PRECISION_BITS)
    ik = np.where(kk < 0, np.trunc(-0.5 + scaled), np.trunc(0.5 + scaled)).astype(np.int32)
    return bounds, ik


def nearest_table(in_size: int, out_size: int) -> np.ndarray:
    """Source index per output position of Image.resize NEAREST (accumulated double
    coordinate, as ImagingScaleAffine)."""
    a = in_size / out_size
    out = np.zeros(out_size, np.int32)
    xo = a * 0.5
    for x in range(out_size):
        out[x] = -1 if xo < 0.0 else int(xo)
        xo += a
    return out


def rotation_params(angle: float, w: int, h: int):
    """Image.rotate(angle) (expand=0, centre, no translate): the affine map PIL builds
    (cos/sin rounded to 15 digits) and its 16.16 fixed-point form.  None when PIL
    returns a copy (angle % 360 == 0)."""
    angle = angle % 360.0
    if angle == 0:
        return None
    ang = -math.radians(angle)
    m = [round(math.cos(ang), 15), round(math.sin(ang), 15), 0.0,
         round(-math.sin(ang), 15), round(math.cos(ang), 15), 0.0]
    cx, cy = w / 2.0, h / 2.0
    m[2] = m[0] * -cx + m[1] * -cy + m[2]
    m[5] = m[3] * -cx + m[4] * -cy + m[5]
    m[2] += cx
    m[5] += cy

    def fix(v):
        return int(math.floor(v * 65536.0 + 0.5))

    fa = [fix(m[0]), fix(m[1]), fix(m[2] + m[1] * 0.5 + m[0] * 0.5),
          fix(m[3]), fix(m[4]), fix(m[5] + m[4] * 0.5 + m[3] * 0.5)]
    return m, fa


def hue_shift_u8(h: float) -> int:
    """np.array(h * 255).astype(np.uint8) as torchvision's adjust_hue adds it
    (truncation toward zero, wrapped mod 256)."""
    return int(math.trunc(h * 255.0)) % 256


def draw_params(seed: int) -> Dict[str, Any]:
    """The reference's per-sample draws from random.Random(seed), in its order
    (aug_monuseg_dataset.py:117-142)."""
    rng = random.Random(seed)
    p = {"hflip": rng.random() < 0.5, "vflip": rng.random() < 0.5,
         "angle": rng.uniform(-90, 90), "jitter": False,
         "b": 1.0, "c": 1.0, "s": 1.0, "h": 0.0}
    if rng.random() < 0.8:
        p["jitter"] = True
        p["b"] = 1.0 + rng.uniform(-0.2, 0.2)
        p["c"] = 1.0 + rng.uniform(-0.2, 0.2)
        p["s"] = 1.0 + rng.uniform(-0.2, 0.2)
        p["h"] = rng.uniform(-0.05, 0.05)
    return p


def pack_params(params: List[Dict[str, Any]], size: int):
    g = np.zeros(len(params), GEOM_DTYPE)
    c = np.zeros(len(params), COLOR_DTYPE)
    for i, p in enumerate(params):
        g[i]["hflip"], g[i]["vflip"] = int(p["hflip"]), int(p["vflip"])
        g[i]["brightness"] = np.float32(p["b"]) if p["jitter"] else np.float32(1.0)
        rot = rotation_params(p["angle"], size, size) if abs(p["angle"]) > 1e-3 else None
        if rot is not None:
            g[i]["a"], g[i]["fa"] = rot[0], rot[1]
            g[i]["rotate"] = 1
        c[i]["jitter"] = int(p["jitter"])
        c[i]["contrast"] = np.float32(p["c"])
        c[i]["saturation"] = np.float32(p["s"])
        c[i]["hue_shift"] = hue_shift_u8(p["h"])
    return g, c


# the exact float32 values torch's ToTensor produces (v.float().div(255))
_U8_TO_F32 = (torch.arange(256, dtype=torch.uint8).float().div(255)).numpy()


class MoNuSegAugmenter:
    """Batched GPU form of ``_apply_joint_transforms``: uint8 images (B,H,W,3) and masks
    (B,H,W) on the device -> image (B,3,S,S) float32, mask (B,1,S,S) float32."""

    def __init__(self, image_size: int, device=None):
        _check_layout()
        self.image_size = image_size
        self.device = torch.device(device or "cuda")
        self._tables: Dict[Tuple[str, int, int], Any] = {}
        self._u8f = torch.from_numpy(_U8_TO_F32).to(self.device)

    def _dev(self, a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(self.device)

    def _coeffs(self, n_in, n_out):
        key = ("aa", n_in, n_out)
        if key not in self._tables:
            b, k = resample_coeffs(n_in, n_out)
            self._tables[key] = (self._dev(b), self._dev(k), k.shape[1])
        return self._tables[key]

    def _nearest(self, n_in, n_out):
        key = ("nn", n_in, n_out)
        if key not in self._tables:
            self._tables[key] = self._dev(nearest_table(n_in, n_out))
        return self._tables[key]

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def resize(self, images: torch.Tensor, masks: torch.Tensor):
        """Image.resize((S, S), BILINEAR) of the images, NEAREST of the masks."""
        B, H, W, _ = images.shape
        S = self.image_size
        st = self._stream()
        img = images.contiguous()
        if W != S:  # horizontal pass over B*H rows of W*3 bytes
            b, k, ks = self._coeffs(W, S)
            out = torch.empty(B, H, S, 3, dtype=torch.uint8, device=self.device)
            check(lib.ugpg_resample_aa_u8(img.data_ptr(), B * H, W, S, 3, b.data_ptr(),
                                          k.data_ptr(), ks, out.data_ptr(), st), "resample_aa")
            img = out
        if H != S:  # vertical pass over B images of H rows of S*3 bytes
            b, k, ks = self._coeffs(H, S)
            out = torch.empty(B, S, S, 3, dtype=torch.uint8, device=self.device)
            check(lib.ugpg_resample_aa_u8(img.data_ptr(), B, H, S, S * 3, b.data_ptr(),
                                          k.data_ptr(), ks, out.data_ptr(), st), "resample_aa")
            img = out
        msk = masks.contiguous()
        if (H, W) != (S, S):
            out = torch.empty(B, S, S, dtype=torch.uint8, device=self.device)
            check(lib.ugpg_resize_nearest_u8(msk.data_ptr(), B, H, W, 1,
                                             self._nearest(H, S).data_ptr(),
                                             self._nearest(W, S).data_ptr(), out.data_ptr(), S,
                                             S, st), "resize_nearest")
            msk = out
        return img, msk

    def __call__(self, images: torch.Tensor, masks: torch.Tensor,
                 params: List[Dict[str, Any]] | None):
        """params: one ``draw_params`` dict per sample, or None for no augmentation."""
        if images.dtype != torch.uint8 or masks.dtype != torch.uint8 or images.dim() != 4 \
                or images.shape[-1] != 3 or masks.shape != images.shape[:3]:
            raise ValueError("expected uint8 images (B,H,W,3) and masks (B,H,W)")
        B = images.shape[0]
        S = self.image_size
        img, msk = self.resize(images, masks)
        if params is None:
            params = [{"hflip": False, "vflip": False, "angle": 0.0, "jitter": False,
                       "b": 1.0, "c": 1.0, "s": 1.0, "h": 0.0}] * B
        if len(params) != B:
            raise ValueError(f"{len(params)} parameter sets for {B} samples")
        g, c = pack_params(params, S)
        gd = self._dev(g.view(np.uint8))
        cd = self._dev(c.view(np.uint8))
        st = self._stream()
        gimg = torch.empty_like(img)
        gmsk = torch.empty_like(msk)
        lsum = torch.empty(B, dtype=torch.int32, device=self.device)
        check(lib.ugpg_augment_geom(img.data_ptr(), msk.data_ptr(), S, B, gd.data_ptr(),
                                    gimg.data_ptr(), gmsk.data_ptr(), lsum.data_ptr(), st),
              "augment_geom")
        out = torch.empty(B, 3, S, S, dtype=torch.float32, device=self.device)
        omask = torch.empty(B, 1, S, S, dtype=torch.float32, device=self.device)
        check(lib.ugpg_augment_color(gimg.data_ptr(), gmsk.data_ptr(), S, B, cd.data_ptr(),
                                     lsum.data_ptr(), self._u8f.data_ptr(), out.data_ptr(),
                                     omask.data_ptr(), st), "augment_color")
        return out, omask


# ----------------------------------------------------------------- masks
def rasterize_polygons(polygons, H: int, W: int, device, ink: int = 1,
                       out: torch.Tensor = None) -> torch.Tensor:
    """Fill every polygon (a sequence of (x, y) floats) with `ink` into an (H, W) uint8
    device mask, exactly as ``ImageDraw.Draw(mask).polygon(points, fill=ink)`` called
    per polygon in order does (monuseg_dataset.py:126-132): one launch pair for all of
    them.  `out` (default: a new zero mask) is drawn into, not cleared."""
    dev = torch.device(device)
    if dev.type != "cuda":
        raise RuntimeError("rasterize_polygons: the HIP kernel needs a GPU tensor device "
                           "(no CPU fallback)")
    mask = torch.zeros(H, W, dtype=torch.uint8, device=dev) if out is None else out
    if mask.shape != (H, W) or mask.dtype != torch.uint8 or not mask.is_contiguous():
        raise ValueError("rasterize_polygons: out must be a contiguous (H, W) uint8 tensor")
    polys = [p for p in polygons]
    if not polys:
        return mask
    counts = [len(p) for p in polys]
    if min(counts) < 2:
        # PIL: "coordinate list must contain at least 2 coordinates"
        raise TypeError("coordinate list must contain at least 2 coordinates")
    off = np.zeros(len(polys) + 1, np.int64)
    np.cumsum(counts, out=off[1:])
    xy = np.asarray([c for p in polys for pt in p for c in pt], np.float64)
    xy_d = torch.from_numpy(xy).to(dev)
    off_d = torch.from_numpy(off).to(dev)
    nv, npoly = int(off[-1]), len(polys)
    wsb = int(lib.ugpg_rasterize_polygons_ws_size(nv, npoly))
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    check(lib.ugpg_rasterize_polygons(xy_d.data_ptr(), off_d.data_ptr(), npoly, nv,
                                      mask.data_ptr(), H, W, int(ink), ws.data_ptr(), wsb, st),
          "rasterize_polygons")
    return mask


def xml_polygons(xml_path: str):
    """The reference's region list (aug_monuseg_dataset.py:89-111 / monuseg_dataset.py:
    114-126): the float vertices of every Region with >= 3 vertices, in file order."""
    root = ET.parse(xml_path).getroot()
    polys = []
    for region in root.findall(".//Region"):
        vertices = region.findall(".//Vertex")
        if len(vertices) < 3:
            continue
        polys.append([(float(v.attrib["X"]), float(v.attrib["Y"])) for v in vertices])
    return polys


# ----------------------------------------------------------------- datasets
def parse_xml_annotations(xml_path: str, image_size: Tuple[int, int], device="cuda") -> torch.Tensor:
    """aug_monuseg_dataset.py:89-111 / monuseg_dataset.py:97-135: the binary mask
    (H, W) uint8 of every Region with >= 3 vertices filled with 1, rasterised on the GPU
    (``rasterize_polygons``: PIL ImageDraw's result bit for bit).  image_size = (W, H)."""
    W, H = image_size
    return rasterize_polygons(xml_polygons(xml_path), H, W, device)


class _MoNuSegBase:
    """Shared sample list, host cache (decoded RGB + rasterised mask) and GPU transforms."""

    def _scan(self, images_dir, annotations_dir):
        files = sorted(f for f in os.listdir(images_dir) if f.lower().endswith(".tif"))
        samples, missing = [], []
        for name in files:
            ann = os.path.join(annotations_dir, name.rsplit(".", 1)[0] + ".xml")
            if os.path.exists(ann):
                samples.append((os.path.join(images_dir, name), ann))
            else:
                missing.append(name)
        if missing:
            print(f"Warning: {len(missing)} images have no matching annotation and will be "
                  f"skipped\nExamples: {missing[:5]}")
        if not samples:
            raise RuntimeError(f"No image-annotation pairs found in {images_dir} / "
                               f"{annotations_dir}")
        self.samples = samples
        self.image_files = [os.path.basename(s[0]) for s in samples]
        self.annotation_files = [os.path.basename(s[1]) for s in samples]
        self._cache: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        self._aug = None

    def _load(self, idx):
        if idx not in self._cache:
            from PIL import Image
            image_path, annotation_path = self.samples[idx]
            image = Image.open(image_path).convert("RGB")
            dev = self.device
            mask = parse_xml_annotations(annotation_path, image.size, dev)
            self._cache[idx] = (torch.from_numpy(np.array(image)).to(dev), mask)
        return self._cache[idx]

    def _augmenter(self):
        if self._aug is None or self._aug.image_size != self.image_size:
            self._aug = MoNuSegAugmenter(self.image_size, self.device)
        return self._aug

    def _augmenting(self):
        return self.augment

    def __len__(self):
        return len(self.samples)

    def get_batch(self, indices):
        """Batched form of __getitem__ (same RNG draws, in index order): images of one
        original size are transformed in one launch sequence."""
        imgs, masks = zip(*(self._load(i) for i in indices))
        if not self.transform:
            return (torch.stack([m.permute(2, 0, 1).float().div(255) for m in imgs]),
                    torch.stack([m.float().unsqueeze(0) for m in masks]))
        params = None
        if self._augmenting():
            params = [draw_params(torch.randint(0, 2 ** 32, (1,)).item()) for _ in indices]
        return self._augmenter()(torch.stack(imgs), torch.stack(masks), params)

    def __getitem__(self, idx):
        x, m = self.get_batch([idx])
        return x[0], m[0]

    def update_image_size(self, new_size: int):
        self.image_size = new_size
        print(f"Updated dataset image size to {new_size}x{new_size}")

    def get_sample_info(self, idx: int) -> Dict[str, Any]:
        from PIL import Image
        image_path, annotation_path = self.samples[idx]
        root = ET.parse(annotation_path).getroot()
        return {"image_file": self.image_files[idx],
                "annotation_file": self.annotation_files[idx],
                "original_size": Image.open(image_path).size,
                "num_nuclei": len(root.findall(".//Region")),
                "microns_per_pixel": float(root.attrib.get("MicronsPerPixel", 0.252))}


class AugMoNuSegDataset(_MoNuSegBase):
    """aug_monuseg_dataset.py:22-188 (<data_dir>/train/aug/{images,annots}); items are
    device tensors (image (3,S,S), mask (1,S,S))."""

    def __init__(self, data_dir: str, image_size: int = 256, transform: bool = True,
                 augment: bool = True, device=None):
        self.data_dir, self.image_size = data_dir, image_size
        self.transform, self.augment = transform, augment
        self.device = torch.device(device or "cuda")
        self.images_dir = os.path.join(data_dir, "train", "aug", "images")
        self.annotations_dir = os.path.join(data_dir, "train", "aug", "annots")
        self._scan(self.images_dir, self.annotations_dir)
        print(f"Augmented MoNuSeg (train/aug) dataset: {len(self.image_files)} samples")


class MoNuSegDataset(_MoNuSegBase):
    """monuseg_dataset.py:21-242 (<data_dir>/<split>/{images,annots}); augmentation only
    for split 'train' (:146)."""

    def __init__(self, data_dir: str, image_size: int = 256, split: str = "train",
                 transform: bool = True, augment: bool = True, device=None):
        self.data_dir, self.image_size, self.split = data_dir, image_size, split
        self.transform, self.augment = transform, augment
        self.device = torch.device(device or "cuda")
        self.images_dir = os.path.join(data_dir, split, "images")
        self.annotations_dir = os.path.join(data_dir, split, "annots")
        self._scan(self.images_dir, self.annotations_dir)
        print(f"MoNuSeg {split} dataset: {len(self.image_files)} samples")

    def _augmenting(self):
        return self.augment and self.split == "train"


def create_train_val_split(data_dir: str, val_ratio: float = 0.2, seed: int = 42,
                           move: bool = False):
    """monuseg_dataset.py:245-299: copy (or move) a seeded random sample of
    train/images/*.tif and their annots/*.xml into val/ (random.seed(seed);
    random.sample over the sorted file list, as the reference)."""
    import shutil
    train_dir, val_dir = os.path.join(data_dir, "train"), os.path.join(data_dir, "val")
    os.makedirs(os.path.join(val_dir, "images"), exist_ok=True)
    os.makedirs(os.path.join(val_dir, "annots"), exist_ok=True)
    image_files = sorted(f for f in os.listdir(os.path.join(train_dir, "images"))
                         if f.endswith(".tif"))
    random.seed(seed)
    n_val = int(len(image_files) * val_ratio)
    val_files = random.sample(image_files, n_val)
    action = "move" if move else "copy"
    print(f"{action.title()}ing {n_val} files to validation set (move={move})...")
    op = shutil.move if move else shutil.copy2
    for img_file in val_files:
        annot_file = img_file.replace(".tif", ".xml")
        op(os.path.join(train_dir, "images", img_file), os.path.join(val_dir, "images", img_file))
        src_annot = os.path.join(train_dir, "annots", annot_file)
        if os.path.exists(src_annot):
            op(src_annot, os.path.join(val_dir, "annots", annot_file))
    print("Train/Val split complete:")
    print(f"  Training: {len(os.listdir(os.path.join(train_dir, 'images')))} samples")
    print(f"  Validation: {len(os.listdir(os.path.join(val_dir, 'images')))} samples")
    return val_files
