"""ORACLE — test infrastructure only (imported by tests/ and nothing in the product path).

numpy restatement of the decoder's counter-based dropout masks (image_caption_amd/csrc/common.h
icap_drop_hash, DropCfg): keep(seed, site, layer, row, pos, idx) = hash >= round(p 2^32), kept elements
scaled by 1 / (1 - p) in fp32 (torch.nn.Dropout's scale).  A mask element depends only on its image row,
query position and index, so a full-prefix recompute (the reference loop, this oracle) and the KV-cached
HIP sampler / teacher-forced HIP training pass draw the same masks.

Sites: 0 positional-encoding output (idx = column), 1 self-attention probabilities (idx = head * 128 +
key), 2 self-attention output, 3 cross-attention probabilities (idx = head * 256 + memory token), 4
cross-attention output, 5 feed-forward hidden, 6 feed-forward output.

Reference: nn.Dropout inside PositionalEncoding (models/vit_transformer_model.py:14-33) and
nn.TransformerDecoderLayer (dropout on both attention maps, dropout1/2/3, and the FFN hidden dropout,
torch/nn/modules/transformer.py), active while the reference samples in train mode
(utils/scst_loss.py:161, 222-223).  The reference draws its masks from torch's RNG, freshly for every
full-prefix recompute; these are a deterministic stand-in with the same keep probability - parity with
the reference's masks is not defined (documented deviation)."""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch

_U = np.uint32


def mix32(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint32, copy=True)
    x ^= x >> _U(16)
    x *= _U(0x7FEB352D)
    x ^= x >> _U(15)
    x *= _U(0x846CA68B)
    x ^= x >> _U(16)
    return x


def drop_hash(seed: int, site: int, layer: int, row, pos, idx) -> np.ndarray:
    """icap_drop_hash over broadcast integer arrays (uint32 arithmetic, wrapping)."""
    with np.errstate(over="ignore"):
        idx, pos, row = (np.asarray(a, dtype=np.uint32) for a in (idx, pos, row))
        h = mix32(idx * _U(0x9E3779B1) + _U(0x7F4A7C15))
        h = mix32(h ^ (pos * _U(0x85EBCA77) + _U(0xC2B2AE3D)))
        h = mix32(h ^ (row * _U(0x27D4EB2F) + _U(0x165667B1)))
        h = mix32(h ^ (_U((site * 16 + layer) & 0xFFFFFFFF) * _U(0x94D049BB) + _U(0x2545F491)))
        return mix32(h ^ _U(seed & 0xFFFFFFFF))


def threshold(p: float) -> int:
    return int(min(4294967295, np.floor(p * 4294967296.0 + 0.5)))


def _mask(p, seed, site, layer, row, pos, idx) -> torch.Tensor:
    keep = drop_hash(seed, site, layer, row, pos, idx) >= _U(threshold(p))
    scale = np.float32(1.0) / (np.float32(1.0) - np.float32(p))
    return torch.from_numpy(np.where(keep, scale, np.float32(0.0)).astype(np.float32))


def decoder_masks(p: float, seed: int, B: int, T: int, S: int, n_layers: int = 6, nhead: int = 8, d: int = 512,
                  dim_ff: int = 2048) -> Dict[str, torch.Tensor]:
    """Every mask of a (B images) x (T positions) teacher-forced decoder pass over S memory tokens:
    'pe' (B,T,d); per layer l: 'sa_p.l' (B,H,T,T), 'sa_o.l' (B,T,d), 'ca_p.l' (B,H,T,S), 'ca_o.l' (B,T,d),
    'ff_h.l' (B,T,dim_ff), 'ff_o.l' (B,T,d) - fp32 tensors of 0 or 1/(1-p)."""
    b = np.arange(B)[:, None, None]
    t = np.arange(T)[None, :, None]
    bh = np.arange(B)[:, None, None, None]
    hh = np.arange(nhead)[None, :, None, None]
    th = np.arange(T)[None, None, :, None]
    m = {"pe": _mask(p, seed, 0, 0, b, t, np.arange(d)[None, None, :])}
    for l in range(n_layers):
        m[f"sa_p.{l}"] = _mask(p, seed, 1, l, bh, th, hh * 128 + np.arange(T)[None, None, None, :])
        m[f"sa_o.{l}"] = _mask(p, seed, 2, l, b, t, np.arange(d)[None, None, :])
        m[f"ca_p.{l}"] = _mask(p, seed, 3, l, bh, th, hh * 256 + np.arange(S)[None, None, None, :])
        m[f"ca_o.{l}"] = _mask(p, seed, 4, l, b, t, np.arange(d)[None, None, :])
        m[f"ff_h.{l}"] = _mask(p, seed, 5, l, b, t, np.arange(dim_ff)[None, None, :])
        m[f"ff_o.{l}"] = _mask(p, seed, 6, l, b, t, np.arange(d)[None, None, :])
    return m
