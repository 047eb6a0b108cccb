"""CPU restatement of the reference's image preprocessing - TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module; the
product path (image_caption_amd.preprocess -> libicap icap_preprocess) never does.

What it restates: the eval transforms of the reference scripts on a
decoded RGB uint8 image -
  * ViT:  Resize(256) + CenterCrop(224) + ToTensor + Normalize   (scripts/inference_vit_transformer.py:75-80,
          utils/deepfashion_dataset.py:223-228)
  * Grid: Resize((224, 224)) + ToTensor + Normalize              (scripts/inference_grid_transformer.py:43-47,
          scripts/inference.py:47-53)
torchvision (absent here) hands PIL images to Pillow's Image.resize(BILINEAR), so the algorithm
is Pillow's 8-bit resampler (third-party dependency; Pillow 12.2.0 is importable here and on the
GPU box, so this restatement is PINNED against Pillow itself in tests/test_preprocess.py):
  precompute_coeffs  - per output coordinate xx: center = (xx + 0.5) * scale, support =
                       max(scale, 1), taps x in [int(center - support + 0.5), int(center + support + 0.5))
                       clipped to the image, triangle weights w = 1 - |(x - center + 0.5) / max(scale, 1)|,
                       normalised by their (sequential, double) sum;
  normalize_coeffs_8bpc - weights to Q22 fixed point: int(w * 2^22 + 0.5) (w >= 0);
  ResampleHorizontal/Vertical_8bpc - acc = 2^21 + sum(pixel * k), out = clamp(acc >> 22, 0, 255);
  ImagingResampleInner - horizontal pass first (uint8 intermediate), then vertical; a pass whose
                       size does not change is skipped.
torchvision's size rules: Resize(int) keeps the aspect (short side -> 256, long side ->
int(256 * long / short)); CenterCrop offsets int(round((size_in - size_out) / 2.0)) (banker's
rounding); ToTensor = float32 / 255; Normalize = (x - mean) / std in float32.
"""
from __future__ import annotations

import math
from typing import List, Tuple

import numpy as np

PRECISION_BITS = 22
MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def resample_coeffs(in_size: int, out_size: int) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Pillow precompute_coeffs + normalize_coeffs_8bpc (bilinear): (xmin (out,), n (out,), k (out, ksize) int64)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 1.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    xmin_a = np.zeros(out_size, np.int64)
    n_a = np.zeros(out_size, np.int64)
    k_a = np.zeros((out_size, ksize), np.int64)
    ss = 1.0 / filterscale
    for xx in range(out_size):
        center = (xx + 0.5) * scale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        w = []
        ww = 0.0
        for x in range(xmax):
            t = abs((x + xmin - center + 0.5) * ss)
            wx = 1.0 - t if t < 1.0 else 0.0
            w.append(wx)
            ww += wx
        for x in range(xmax):
            v = w[x] / ww if ww != 0.0 else w[x]
            k_a[xx, x] = int(v * (1 << PRECISION_BITS) + 0.5) if v >= 0 else int(-0.5 + v * (1 << PRECISION_BITS))
        xmin_a[xx], n_a[xx] = xmin, xmax
    return xmin_a, n_a, k_a


def _pass(img: np.ndarray, axis: int, out_size: int) -> np.ndarray:
    """One 8-bpc resampling pass along axis 0 (rows) or 1 (columns) of an (H, W, 3) uint8 image."""
    in_size = img.shape[axis]
    xmin, n, k = resample_coeffs(in_size, out_size)
    src = np.moveaxis(img.astype(np.int64), axis, 0)  # (in, other, 3)
    out = np.empty((out_size,) + src.shape[1:], np.int64)
    for xx in range(out_size):
        taps = src[xmin[xx]: xmin[xx] + n[xx]]
        out[xx] = (1 << (PRECISION_BITS - 1)) + np.tensordot(k[xx, : n[xx]], taps, axes=(0, 0))
    out = np.clip(out >> PRECISION_BITS, 0, 255).astype(np.uint8)
    return np.moveaxis(out, 0, axis)


def pil_bilinear_resize(img: np.ndarray, out_h: int, out_w: int) -> np.ndarray:
    """Image.resize((out_w, out_h), BILINEAR) of an (H, W, 3) uint8 RGB image."""
    h, w = img.shape[:2]
    if out_w != w:
        img = _pass(img, 1, out_w)
    if out_h != h:
        img = _pass(img, 0, out_h)
    return img


def resized_size(h: int, w: int, size: int) -> Tuple[int, int]:
    """torchvision Resize(size) output (h, w) for an int size: short side -> size."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def crop_offsets(h: int, w: int, size: int) -> Tuple[int, int]:
    """torchvision CenterCrop(size) (top, left) for an image at least `size` on both sides."""
    return int(round((h - size) / 2.0)), int(round((w - size) / 2.0))


def preprocess(img: np.ndarray, mode: str = "crop", size: int = 224, resize_to: int = 256) -> np.ndarray:
    """(H, W, 3) uint8 -> (3, size, size) float32; mode "crop" (ViT) or "square" (Grid)."""
    h, w = img.shape[:2]
    if mode == "crop":
        rh, rw = resized_size(h, w, resize_to)
        r = pil_bilinear_resize(img, rh, rw)
        top, left = crop_offsets(rh, rw, size)
        r = r[top: top + size, left: left + size]
    elif mode == "square":
        r = pil_bilinear_resize(img, size, size)
    else:
        raise ValueError(mode)
    a = r.astype(np.float32) / np.float32(255.0)
    a = (a - MEAN) / STD
    return np.ascontiguousarray(a.transpose(2, 0, 1))


def preprocess_batch(imgs: List[np.ndarray], mode: str = "crop", size: int = 224) -> np.ndarray:
    return np.stack([preprocess(i, mode, size) for i in imgs])
