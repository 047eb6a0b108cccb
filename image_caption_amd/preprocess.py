"""Batched eval preprocessing on the GPU through libicap icap_preprocess.

Decoded RGB uint8 images of any size -> the normalised (B, 3, 224, 224) fp32 batch, bit-identical
to the reference scripts' torchvision transforms on PIL images:
  mode "crop"   : Resize(256) + CenterCrop(224)  (scripts/inference_vit_transformer.py:75-80,
                  utils/deepfashion_dataset.py:223-228)
  mode "square" : Resize((224, 224))            (scripts/inference_grid_transformer.py:43-47,
                  scripts/inference.py:47-53)
followed by ToTensor + Normalize(ImageNet mean/std).  The host side here only computes the per-image
geometry with torchvision's size rules; the resampling itself (Pillow's 8-bit bilinear) runs in
preprocess.hip.  There is no CPU fallback: the HIP library must be loaded.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch

from . import _lib

MODES = ("crop", "square")


def resized_size(h: int, w: int, size: int) -> Tuple[int, int]:
    """torchvision Resize(int) on a PIL image: short side -> size, long side -> int(size * long / short)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = size, int(size * long / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def _tap_range(in_size: int, out_size: int, xx: int) -> Tuple[int, int]:
    """[first, end) source index Pillow's bilinear resampler reads for output coordinate xx."""
    scale = in_size / out_size
    support = max(scale, 1.0)
    center = (xx + 0.5) * scale
    return max(int(center - support + 0.5), 0), min(int(center + support + 0.5), in_size)


def geometry(h: int, w: int, mode: str, size: int = 224, resize_to: int = 256) -> List[int]:
    """icap_preprocess geometry row: in_h, in_w, rs_h, rs_w, top, left, y0, nrows."""
    if mode == "crop":
        rs_h, rs_w = resized_size(h, w, resize_to)
        if rs_h < size or rs_w < size:
            raise ValueError(f"Resize({resize_to}) of a {h}x{w} image is smaller than the {size} crop")
        top, left = int(round((rs_h - size) / 2.0)), int(round((rs_w - size) / 2.0))
    elif mode == "square":
        rs_h, rs_w, top, left = size, size, 0, 0
    else:
        raise ValueError(f"mode must be one of {MODES}")
    if rs_h == h:  # no vertical pass: the kept rows themselves
        y0, y1 = top, top + size
    else:
        y0 = _tap_range(h, rs_h, top)[0]
        y1 = _tap_range(h, rs_h, top + size - 1)[1]
    return [h, w, rs_h, rs_w, top, left, y0, y1 - y0]


def preprocess_batch(images: Sequence, mode: str = "crop", size: int = 224,
                     device: torch.device | str | None = None) -> torch.Tensor:
    """images: (H, W, 3) uint8 arrays / tensors (RGB, any sizes) -> (B, 3, size, size) fp32 on `device`."""
    lib = _lib.load()
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if device.type != "cuda":
        raise _lib.IcapError("icap_preprocess needs a GPU device")
    arrs = [np.ascontiguousarray(np.asarray(im.cpu() if isinstance(im, torch.Tensor) else im)) for im in images]
    for a in arrs:
        if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
            raise ValueError(f"expected (H, W, 3) uint8 RGB images, got {a.dtype} {a.shape}")
    B = len(arrs)
    if B == 0:
        return torch.empty(0, 3, size, size, device=device)
    geom = np.array([geometry(a.shape[0], a.shape[1], mode, size) for a in arrs], dtype=np.int32)
    sizes = np.array([a.size for a in arrs], dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    flat = torch.from_numpy(np.concatenate([a.reshape(-1) for a in arrs])).pin_memory()
    px = flat.to(device, non_blocking=True)
    offs_d = torch.from_numpy(offs).to(device)
    geom_d = torch.from_numpy(geom).to(device)
    max_rows = int(geom[:, 7].max())
    tmp = torch.empty(B * max_rows * size * 4, dtype=torch.uint8, device=device)
    out = torch.empty(B, 3, size, size, dtype=torch.float32, device=device)
    with torch.cuda.device(device):
        _lib.check(lib.icap_preprocess(px.data_ptr(), offs_d.data_ptr(), geom_d.data_ptr(), B, size, max_rows,
                                       tmp.data_ptr(), out.data_ptr(), _lib.stream_ptr(device)), "icap_preprocess")
    return out

