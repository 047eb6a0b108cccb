"""Drop-in `models.vit_transformer_model` (reference: models/vit_transformer_model.py).

Same classes, constructor arguments, config keys, attribute names and state_dict keys as the
reference; `generate` / `encoder(...)` / `decoder(...)` on GPU tensors in eval/no-grad run the
MI355X HIP engine (libicap.so) instead of torch modules.  Extra, build-owned config keys:
`backend` ("auto" | "hip" | "torch") and `hip_precision` ("f16" default: fp16 encoder operands, bf16x2 decoder; "i8x2", "bf16x2" or "bf16").
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn

from ._common import PositionalEncoding, TransformerDecoder, beam_search, greedy_torch, padding_mask
from ._hip import HipRouted, attach_owner, owner_of
from ._vision import load_trunks

__all__ = ["PositionalEncoding", "VisionTransformerEncoder", "TransformerDecoder", "ViTTransformerCaptioning",
           "build_model"]


class VisionTransformerEncoder(nn.Module):
    """ViT-B/16 trunk (classification head removed) + Linear(768 -> d_model) (vit:36-100).
    Output: patch features (B, 196, d_model); the CLS token is dropped."""

    def __init__(self, model_name="vit_b_16", pretrained=True, d_model=512):
        super().__init__()
        vit_b_16, weights_enum, _, _ = load_trunks()
        try:
            self.vit = vit_b_16(weights=weights_enum.DEFAULT) if pretrained else vit_b_16()
        except Exception as e:  # no network / no torchvision: random init, a checkpoint overwrites it
            warnings.warn(f"pretrained ViT weights unavailable ({e}); using random init")
            self.vit = vit_b_16()
        self.vit.heads = nn.Identity()
        self.projection = nn.Linear(768, d_model)
        self.set_trainable(False)

    def set_trainable(self, trainable=True):
        for p in self.vit.parameters():
            p.requires_grad = trainable

    def forward(self, images):
        owner = owner_of(self)
        if owner is not None and not self.training and owner.use_hip(images):
            return owner.checked_encode(images)[1]  # f16 range guard: bf16x2 re-encode on overflow
        x = self.vit._process_input(images)
        x = torch.cat([self.vit.class_token.expand(x.shape[0], -1, -1), x], dim=1)
        x = self.vit.encoder(x)
        return self.projection(x[:, 1:, :])


class ViTTransformerCaptioning(HipRouted, nn.Module):
    """ViT encoder + Transformer decoder captioner (vit:185-420)."""

    _hip_kind = "vit"

    def __init__(self, vocab_size, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, max_len=100, pretrained_vit=True, backend="auto",
                 hip_precision="f16"):
        super().__init__()
        self._hip_setup(backend, hip_precision)
        self.vocab_size = vocab_size
        self.d_model = d_model
        self.encoder = VisionTransformerEncoder(model_name="vit_b_16", pretrained=pretrained_vit, d_model=d_model)
        self.decoder = TransformerDecoder(vocab_size=vocab_size, d_model=d_model, nhead=nhead,
                                          num_layers=num_decoder_layers, dim_feedforward=dim_feedforward,
                                          dropout=dropout, max_len=max_len)
        attach_owner(self.encoder, self)
        attach_owner(self.decoder, self)

    def forward(self, images, captions, caption_lengths=None):
        """Teacher-forced training forward (vit:216-255): logits for captions[:, :-1]."""
        memory = self.encoder(images)
        tgt = captions[:, :-1]
        mask = self.decoder.generate_square_subsequent_mask(tgt.size(1), images.device)
        pad = self._generate_padding_mask(tgt, caption_lengths) if caption_lengths is not None else None
        return self.decoder(tgt, memory, tgt_mask=mask, tgt_key_padding_mask=pad)

    def _generate_padding_mask(self, tgt, lengths):
        return padding_mask(tgt, lengths)

    def generate(self, images, start_token, end_token, max_len=50, method="greedy"):
        if method == "greedy":
            return self._greedy_search(images, start_token, end_token, max_len)
        if method == "beam_search":
            return self._beam_search(images, start_token, end_token, max_len, beam_size=5)
        raise ValueError(f"Unknown generation method: {method}")

    def _greedy_search(self, images, start_token, end_token, max_len):
        self.eval()
        with torch.no_grad():
            if self.use_hip(images):
                eng = self.hip_engine(images.device)
                ids = eng.greedy(eng.encode(images), start_token, end_token, max_len)
                if eng.range_overflowed():  # an fp16 encoder activation overflowed: bf16x2 again
                    eng = self.hip_engine(images.device, precision="bf16x2")
                    ids = eng.greedy(eng.encode(images), start_token, end_token, max_len)
                return ids
            return greedy_torch(self, images, start_token, end_token, max_len)

    def _beam_search(self, images, start_token, end_token, max_len, beam_size=5):
        self.eval()
        return beam_search(self, images, start_token, end_token, max_len, beam_size, grid_variant=False)


def build_model(vocab_size, config):
    """Config dict -> model, same keys and defaults as the reference (vit:423-444)."""
    return ViTTransformerCaptioning(
        vocab_size=vocab_size,
        d_model=config.get("d_model", 512),
        nhead=config.get("nhead", 8),
        num_decoder_layers=config.get("num_decoder_layers", 6),
        dim_feedforward=config.get("dim_feedforward", 2048),
        dropout=config.get("dropout", 0.1),
        max_len=config.get("max_len", 100),
        pretrained_vit=config.get("pretrained_vit", True),
        backend=config.get("backend", "auto"),
        hip_precision=config.get("hip_precision", "f16"),
    )
