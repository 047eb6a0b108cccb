"""Data-only helpers for the golden fixtures: inputs that are regenerated from a seed instead of stored.

Nothing here imports the reference or the fixture generator (tests/golden/make_golden.py), so GPU tests
may import it on the GPU box, where /root/reference does not exist."""
from __future__ import annotations

import numpy as np


SCRIPT_IMAGE_SHAPES = ((240, 320), (300, 256), (375, 500), (224, 224))  # (H, W): landscape, portrait, large, exact


def script_images() -> list:
    """The RGB uint8 images of scripts.json (seeded; smooth gradients plus noise, so the resampler's taps differ)."""
    rng = np.random.Generator(np.random.PCG64(12))
    out = []
    for h, w in SCRIPT_IMAGE_SHAPES:
        yy, xx = np.meshgrid(np.linspace(0, 1, h), np.linspace(0, 1, w), indexing="ij")
        base = np.stack([yy * 200, xx * 180, (1 - yy) * 150], -1) + rng.integers(0, 56, size=(h, w, 3))
        out.append(np.clip(base, 0, 255).astype(np.uint8))
    return out


def write_pngs(arrays, directory) -> list:
    """Write each array as <directory>/img<i>.png (lossless: decoding gives the array back); returns the paths."""
    import os

    from PIL import Image

    paths = []
    for i, a in enumerate(arrays):
        p = os.path.join(str(directory), f"img{i}.png")
        Image.fromarray(a, "RGB").save(p)
        paths.append(p)
    return paths


def decoder_ops_memory() -> np.ndarray:
    """The (3,196,512) memory of decoder_ops.npz, regenerated from its seed (not stored)."""
    return np.random.Generator(np.random.PCG64(8)).standard_normal((3, 196, 512)).astype(np.float32)
