"""Image preprocessing and checkpoint loading shared by the drop-in inference scripts.

torchvision is absent here, so the transforms of the reference scripts are restated on PIL +
numpy with torchvision's semantics for PIL inputs:
  * Resize(256) + CenterCrop(224)  (scripts/inference_vit_transformer.py:75-80)
  * Resize((224, 224))            (scripts/inference_grid_transformer.py:43-47, scripts/inference.py:47-53)
  * ToTensor + Normalize(ImageNet mean/std)
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def _pil():
    from PIL import Image

    return Image


def resize_shorter(img, size: int):
    w, h = img.size
    if w <= h:
        nw, nh = size, int(size * h / w)
    else:
        nw, nh = int(size * w / h), size
    return img.resize((nw, nh), _pil().BILINEAR)


def center_crop(img, size: int):
    w, h = img.size
    top = int(round((h - size) / 2.0))
    left = int(round((w - size) / 2.0))
    return img.crop((left, top, left + size, top + size))


def to_normalized_tensor(img) -> torch.Tensor:
    a = np.asarray(img.convert("RGB"), dtype=np.float32) / 255.0
    a = (a - MEAN) / STD
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))


def preprocess(image_path: str, mode: str = "crop", image_size: int = 224) -> torch.Tensor:
    """(3,H,W) normalised tensor; mode "crop" = Resize(256)+CenterCrop, "square" = Resize((s,s))."""
    img = _pil().open(image_path).convert("RGB")
    if mode == "crop":
        img = center_crop(resize_shorter(img, 256), image_size)
    else:
        img = img.resize((image_size, image_size), _pil().BILINEAR)
    return to_normalized_tensor(img)


def decode_rgb(image_path: str) -> np.ndarray:
    """Image.open(path).convert('RGB') as an (H, W, 3) uint8 array."""
    return np.asarray(_pil().open(image_path).convert("RGB"))


def preprocess_to_device(image_paths, mode: str, device, image_size: int = 224) -> torch.Tensor:
    """(B,3,S,S) batch on `device`: decode on the host, then on a GPU the whole batch is resized,
    cropped and normalised by the HIP kernels (image_caption_amd.preprocess, bit-identical to the
    PIL path of preprocess() above); on the CPU that PIL path itself."""
    if torch.device(device).type == "cuda":
        from image_caption_amd.preprocess import preprocess_batch

        return preprocess_batch([decode_rgb(p) for p in image_paths], mode, image_size, device)
    return torch.stack([preprocess(p, mode, image_size) for p in image_paths])


def _numpy_safe_globals() -> list:
    """The numpy names a reference checkpoint pickles besides tensors: its `scores` / `loss` / `cider` values and the
    LR scheduler's `best` are numpy scalars (pycocoevalcap returns numpy floats; train_vit_transformer.py:413-423,
    train_*_scst_optimized.py:509-520).  Scalars reduce to multiarray.scalar(dtype, bytes) and dtypes to
    numpy.dtype(str, ...): plain data constructors, nothing that runs code from the file.  Checkpoints written under
    numpy 1.x name the module numpy.core (the reference's own loader shims numpy._core for the other direction,
    scripts/inference_vit_transformer.py:37-42), so both spellings are allowlisted."""
    import numpy as np

    core = np._core if hasattr(np, "_core") else np.core
    objs = [core.multiarray.scalar, np.dtype, np.ndarray, core.multiarray._reconstruct]
    out = list(objs)
    for mod in ("numpy.core.multiarray", "numpy._core.multiarray"):
        out += [(core.multiarray.scalar, f"{mod}.scalar"), (core.multiarray._reconstruct, f"{mod}._reconstruct")]
    out += [type(np.dtype(t)) for t in ("f2", "f4", "f8", "i1", "i2", "i4", "i8", "u1", "b1")]
    return out


def load_checkpoint(path: str, device):
    """torch.load with weights_only=True (no unpickling of arbitrary objects), with numpy scalars / dtypes / arrays
    allowlisted so the reference's training checkpoints (numpy-float scores and losses) load as they are."""
    try:
        with torch.serialization.safe_globals(_numpy_safe_globals()):
            return torch.load(path, map_location=device, weights_only=True)
    except Exception as e:
        raise RuntimeError(f"{path}: cannot be loaded with weights_only=True ({e}); re-save it as a plain "
                           "{'model_state_dict': ..., 'config': {...}} dict of tensors and primitives") from e


def load_vocab(path: str) -> dict:
    with open(path, "r", encoding="utf-8") as f:
        return json.load(f)


def default_vocab_path() -> str:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(here, "data", "vocab.json")
