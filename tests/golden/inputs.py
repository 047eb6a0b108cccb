"""Data-only helpers for the golden fixtures: inputs that are regenerated from a seed instead of stored.

Nothing here imports the reference or the fixture generator (tests/golden/make_golden.py), so GPU tests
may import it on the GPU box, where /root/reference does not exist."""
from __future__ import annotations

import numpy as np


def decoder_ops_memory() -> np.ndarray:
    """The (3,196,512) memory of decoder_ops.npz, regenerated from its seed (not stored)."""
    return np.random.Generator(np.random.PCG64(8)).standard_normal((3, 196, 512)).astype(np.float32)
