"""Seeded synthetic weights for the captioning models (no checkpoints exist offline).

The reference's trained checkpoints are Git-LFS stubs
(`checkpoints/vit_transformer/best_model.pth`), and the pretrained
torchvision ViT/ResNet weights need the network.  Every run here therefore uses
random-init weights from this generator.  It is deterministic across machines
(numpy PCG64), so the GPU box regenerates exactly the weights the golden
fixtures in `tests/golden/` were made with.

Key names follow the reference's `state_dict` exactly:
  * ViT model  — `models/vit_transformer_model.py:185-214` (encoder.vit.* are
    torchvision `VisionTransformer` names, encoder.projection vit:61, decoder.*
    vit:103-137).
  * Grid model — `models/grid_transformer_model.py:161-183` (encoder.cnn.{0,1,4..7}
    are torchvision `resnet101` children[:-2] names, grid:51).

Init scales mimic the reference (decoder embedding / fc_out U(-0.1,0.1), vit:142-147;
MHA xavier-uniform in_proj with zero biases; nn.Linear kaiming-uniform bounds;
ViT pos-embedding N(0,0.02)).  LayerNorm affines are perturbed around (1, 0) so that a
kernel that drops gamma/beta fails parity.  With `bf16_exact=True` every floating
weight is rounded once to a bf16-representable fp32 value, so the fp32 CPU oracle and
the bf16-weight GPU path see identical parameters.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

VOCAB_SIZE = 109
START_TOKEN = 107
END_TOKEN = 108
PAD_TOKEN = 0

DEFAULT_CONFIG = {
    "d_model": 512,
    "nhead": 8,
    "num_encoder_layers": 6,
    "num_decoder_layers": 6,
    "dim_feedforward": 2048,
    "dropout": 0.1,
    "max_len": 100,
}

VIT_DIM = 768
VIT_LAYERS = 12
VIT_HEADS = 12
VIT_MLP = 3072
VIT_PATCH = 16
VIT_IMAGE = 224
RESNET101_BLOCKS = (3, 4, 23, 3)


def round_to_bf16(a: np.ndarray) -> np.ndarray:
    """Round fp32 -> nearest-even bf16, returned as fp32 (exactly representable)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    u = a.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32)
    # keep NaN/inf untouched (none are generated, but be exact about it)
    bad = ~np.isfinite(a)
    if bad.any():
        out = out.copy()
        out[bad] = a[bad]
    return out


def positional_encoding(max_len: int, d_model: int) -> np.ndarray:
    """The sinusoidal table of `PositionalEncoding.__init__` (vit:19-24), computed with
    the same torch CPU ops so the buffer is bit-identical to the reference's."""
    import torch

    pe = torch.zeros(max_len, d_model)
    position = torch.arange(0, max_len, dtype=torch.float).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, d_model, 2).float() * (-math.log(10000.0) / d_model))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe.unsqueeze(0).numpy()


class _Gen:
    def __init__(self, seed: int):
        self.rng = np.random.Generator(np.random.PCG64(seed))

    def uniform(self, shape, bound):
        return self.rng.uniform(-bound, bound, size=shape).astype(np.float32)

    def normal(self, shape, std, mean=0.0):
        return (mean + std * self.rng.standard_normal(size=shape)).astype(np.float32)

    def xavier(self, shape):
        fan_out, fan_in = shape[0], int(np.prod(shape[1:]))
        return self.uniform(shape, math.sqrt(6.0 / (fan_in + fan_out)))

    def kaiming_linear(self, shape):
        fan_in = int(np.prod(shape[1:]))
        return self.uniform(shape, 1.0 / math.sqrt(fan_in))

    def ln(self, sd, prefix, dim):
        sd[prefix + ".weight"] = self.normal((dim,), 0.1, 1.0)
        sd[prefix + ".bias"] = self.normal((dim,), 0.05)

    def mha(self, sd, prefix, dim):
        sd[prefix + ".in_proj_weight"] = self.xavier((3 * dim, dim))
        sd[prefix + ".in_proj_bias"] = self.normal((3 * dim,), 0.02)
        sd[prefix + ".out_proj.weight"] = self.kaiming_linear((dim, dim))
        sd[prefix + ".out_proj.bias"] = self.normal((dim,), 0.02)

    def linear(self, sd, prefix, out_f, in_f):
        sd[prefix + ".weight"] = self.kaiming_linear((out_f, in_f))
        sd[prefix + ".bias"] = self.uniform((out_f,), 1.0 / math.sqrt(in_f))


def _decoder_weights(g: _Gen, sd: Dict[str, np.ndarray], cfg: dict, vocab_size: int):
    d, ff = cfg["d_model"], cfg["dim_feedforward"]
    sd["decoder.embedding.weight"] = g.uniform((vocab_size, d), 0.1)
    sd["decoder.pos_encoder.pe"] = positional_encoding(cfg["max_len"], d)
    for i in range(cfg["num_decoder_layers"]):
        p = f"decoder.transformer_decoder.layers.{i}"
        g.mha(sd, p + ".self_attn", d)
        g.mha(sd, p + ".multihead_attn", d)
        g.linear(sd, p + ".linear1", ff, d)
        g.linear(sd, p + ".linear2", d, ff)
        g.ln(sd, p + ".norm1", d)
        g.ln(sd, p + ".norm2", d)
        g.ln(sd, p + ".norm3", d)
    sd["decoder.fc_out.weight"] = g.uniform((vocab_size, d), 0.1)
    sd["decoder.fc_out.bias"] = g.normal((vocab_size,), 0.01)


def _finish(sd: Dict[str, np.ndarray], bf16_exact: bool) -> Dict[str, np.ndarray]:
    out = {}
    for k, v in sd.items():
        if v.dtype == np.float32 and bf16_exact and not k.endswith(".pe"):
            v = round_to_bf16(v)
        out[k] = np.ascontiguousarray(v)
    return out


def vit_state_dict(seed: int = 0, config: dict | None = None, vocab_size: int = VOCAB_SIZE,
                   bf16_exact: bool = True) -> Dict[str, np.ndarray]:
    """state_dict of `ViTTransformerCaptioning` (vit:185) with synthetic weights."""
    cfg = dict(DEFAULT_CONFIG, **(config or {}))
    g = _Gen(seed)
    sd: Dict[str, np.ndarray] = {}
    D = VIT_DIM
    n_patch = (VIT_IMAGE // VIT_PATCH) ** 2
    sd["encoder.vit.class_token"] = g.normal((1, 1, D), 0.02)
    # torchvision: trunc_normal(std=sqrt(1/fan_in)) for conv_proj, zero bias
    sd["encoder.vit.conv_proj.weight"] = np.clip(
        g.normal((D, 3, VIT_PATCH, VIT_PATCH), math.sqrt(1.0 / (3 * VIT_PATCH * VIT_PATCH))),
        -2 * math.sqrt(1.0 / 768), 2 * math.sqrt(1.0 / 768)).astype(np.float32)
    sd["encoder.vit.conv_proj.bias"] = g.normal((D,), 0.02)
    sd["encoder.vit.encoder.pos_embedding"] = g.normal((1, n_patch + 1, D), 0.02)
    for i in range(VIT_LAYERS):
        p = f"encoder.vit.encoder.layers.encoder_layer_{i}"
        g.ln(sd, p + ".ln_1", D)
        g.mha(sd, p + ".self_attention", D)
        g.ln(sd, p + ".ln_2", D)
        sd[p + ".mlp.0.weight"] = g.xavier((VIT_MLP, D))
        sd[p + ".mlp.0.bias"] = g.normal((VIT_MLP,), 0.02)
        sd[p + ".mlp.3.weight"] = g.xavier((D, VIT_MLP))
        sd[p + ".mlp.3.bias"] = g.normal((D,), 0.02)
    g.ln(sd, "encoder.vit.encoder.ln", D)
    g.linear(sd, "encoder.projection", cfg["d_model"], D)
    _decoder_weights(g, sd, cfg, vocab_size)
    return _finish(sd, bf16_exact)


def _bn(g: _Gen, sd, prefix, ch, gamma_scale=1.0):
    sd[prefix + ".weight"] = g.normal((ch,), 0.1 * gamma_scale, gamma_scale)
    sd[prefix + ".bias"] = g.normal((ch,), 0.05)
    sd[prefix + ".running_mean"] = g.normal((ch,), 0.05)
    sd[prefix + ".running_var"] = (1.0 + 0.2 * np.abs(g.normal((ch,), 1.0))).astype(np.float32)
    sd[prefix + ".num_batches_tracked"] = np.array(0, dtype=np.int64)


def _conv(g: _Gen, shape):
    # kaiming_normal_(mode="fan_out", nonlinearity="relu") as torchvision's ResNet init
    fan_out = shape[0] * int(np.prod(shape[2:]))
    return g.normal(shape, math.sqrt(2.0 / fan_out))


def grid_state_dict(seed: int = 0, config: dict | None = None, vocab_size: int = VOCAB_SIZE,
                    bf16_exact: bool = True) -> Dict[str, np.ndarray]:
    """state_dict of `GridTransformerCaptioning` (grid:161) with synthetic weights.

    The residual branch's last BN gamma is scaled by 0.2 so 33 stacked bottlenecks stay
    in a sane fp32 range with random weights (torchvision's `zero_init_residual` idea).  The 1x1
    projection is initialised at 10x torch's kaiming-uniform bound: the random trunk's features are
    small (mean |f| 0.16) and at torch's scale the projected features drown under the positional
    encoding, so the memory of different images differed by ~0.3% and every golden row decoded the
    same ids; at 10x the memory differs by ~3% between images and the rows do not."""
    cfg = dict(DEFAULT_CONFIG, **(config or {}))
    g = _Gen(seed + 1000003)
    sd: Dict[str, np.ndarray] = {}
    sd["encoder.cnn.0.weight"] = _conv(g, (64, 3, 7, 7))
    _bn(g, sd, "encoder.cnn.1", 64)
    inplanes = 64
    for li, (planes, blocks) in enumerate(zip((64, 128, 256, 512), RESNET101_BLOCKS)):
        for b in range(blocks):
            p = f"encoder.cnn.{4 + li}.{b}"
            sd[p + ".conv1.weight"] = _conv(g, (planes, inplanes, 1, 1))
            _bn(g, sd, p + ".bn1", planes)
            sd[p + ".conv2.weight"] = _conv(g, (planes, planes, 3, 3))
            _bn(g, sd, p + ".bn2", planes)
            sd[p + ".conv3.weight"] = _conv(g, (planes * 4, planes, 1, 1))
            _bn(g, sd, p + ".bn3", planes * 4, gamma_scale=0.2)
            if b == 0:
                sd[p + ".downsample.0.weight"] = _conv(g, (planes * 4, inplanes, 1, 1))
                _bn(g, sd, p + ".downsample.1", planes * 4)
            inplanes = planes * 4
    d = cfg["d_model"]
    sd["encoder.projection.weight"] = 10.0 * g.kaiming_linear((d, 2048, 1, 1))
    sd["encoder.projection.bias"] = g.uniform((d,), 1.0 / math.sqrt(2048))
    for i in range(cfg["num_encoder_layers"]):
        p = f"encoder.transformer_encoder.layers.{i}"
        g.mha(sd, p + ".self_attn", d)
        g.linear(sd, p + ".linear1", cfg["dim_feedforward"], d)
        g.linear(sd, p + ".linear2", d, cfg["dim_feedforward"])
        g.ln(sd, p + ".norm1", d)
        g.ln(sd, p + ".norm2", d)
    sd["encoder.pos_encoder.pe"] = positional_encoding(100, d)
    _decoder_weights(g, sd, cfg, vocab_size)
    return _finish(sd, bf16_exact)


def synthetic_images(batch: int, seed: int = 0, size: int = VIT_IMAGE) -> np.ndarray:
    """ImageNet-normalised-space synthetic images, N(0,1), NCHW fp32."""
    rng = np.random.Generator(np.random.PCG64(seed + 77))
    return rng.standard_normal(size=(batch, 3, size, size)).astype(np.float32)


def to_torch(sd: Dict[str, np.ndarray]):
    import torch

    return {k: torch.from_numpy(np.array(v)) for k, v in sd.items()}
