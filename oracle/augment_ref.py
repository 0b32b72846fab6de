"""CPU oracle for the MoNuSeg augmentation (TEST INFRASTRUCTURE -- never shipped).

The reference's per-sample transform, aug_monuseg_dataset.py:113-148 (identical in
monuseg_dataset.py:137-190), restated on PIL images with PIL itself -- the library the
reference calls -- so the GPU kernels are checked against PIL's own 8-bit arithmetic:

  Image.resize((S, S), BILINEAR) / resize NEAREST (mask)          :114-115
  TF.hflip / TF.vflip  = Image.transpose(FLIP_LEFT_RIGHT / TOP_BOTTOM)   :121-127
  Image.rotate(angle, BILINEAR) / rotate(angle, NEAREST)          :129-132
  TF.adjust_brightness / contrast / saturation = ImageEnhance.Brightness / Contrast /
      Color(...).enhance(factor)                                  :139-141
  TF.adjust_hue: H channel of img.convert("HSV") += uint8(h * 255), merge, convert
      back to RGB                                                  :142
  ToTensor: uint8 -> float32 / 255, CHW; mask -> float (1, S, S)  :144-147

torchvision is not installed here: its PIL-backend functions above are restated from
its published source (torchvision/transforms/_functional_pil.py), which calls exactly
these PIL operations.  The parameter draws are the reference's (random.Random(seed)).
"""
from __future__ import annotations

import math
import random

import numpy as np
import torch
from PIL import Image, ImageEnhance


def draw_params(seed: int) -> dict:
    """aug_monuseg_dataset.py:117-142, same call order."""
    rng = random.Random(seed)
    p = {"hflip": rng.random() < 0.5, "vflip": rng.random() < 0.5,
         "angle": rng.uniform(-90, 90), "jitter": False, "b": 1.0, "c": 1.0, "s": 1.0, "h": 0.0}
    if rng.random() < 0.8:
        p["jitter"] = True
        p["b"] = 1.0 + rng.uniform(-0.2, 0.2)
        p["c"] = 1.0 + rng.uniform(-0.2, 0.2)
        p["s"] = 1.0 + rng.uniform(-0.2, 0.2)
        p["h"] = rng.uniform(-0.05, 0.05)
    return p


def adjust_hue(img: Image.Image, hue_factor: float) -> Image.Image:
    """torchvision _functional_pil.adjust_hue for an RGB image."""
    h, s, v = img.convert("HSV").split()
    np_h = np.array(h, dtype=np.uint8)
    # np.array(hue_factor * 255).astype(np.uint8): truncation, wrapped mod 256
    np_h = (np_h.astype(np.int64) + (int(math.trunc(hue_factor * 255.0)) % 256)) % 256
    h = Image.fromarray(np_h.astype(np.uint8), "L")
    return Image.merge("HSV", (h, s, v)).convert("RGB")


def joint_transform(image: Image.Image, mask: Image.Image, size: int, params: dict | None):
    """One sample; params None = resize + ToTensor only (augment off)."""
    image = image.resize((size, size), Image.BILINEAR)
    mask = mask.resize((size, size), Image.NEAREST)
    if params is not None:
        if params["hflip"]:
            image = image.transpose(Image.FLIP_LEFT_RIGHT)
            mask = mask.transpose(Image.FLIP_LEFT_RIGHT)
        if params["vflip"]:
            image = image.transpose(Image.FLIP_TOP_BOTTOM)
            mask = mask.transpose(Image.FLIP_TOP_BOTTOM)
        angle = params["angle"]
        if abs(angle) > 1e-3:
            image = image.rotate(angle, resample=Image.BILINEAR)
            mask = mask.rotate(angle, resample=Image.NEAREST)
        if params["jitter"]:
            image = ImageEnhance.Brightness(image).enhance(params["b"])
            image = ImageEnhance.Contrast(image).enhance(params["c"])
            image = ImageEnhance.Color(image).enhance(params["s"])
            image = adjust_hue(image, params["h"])
    x = torch.from_numpy(np.array(image, dtype=np.uint8)).permute(2, 0, 1).contiguous()
    x = x.float().div(255)
    m = torch.from_numpy(np.array(mask)).float().unsqueeze(0)
    return x, m
