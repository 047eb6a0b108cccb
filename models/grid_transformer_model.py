"""Drop-in `models.grid_transformer_model` (reference: models/grid_transformer_model.py).

ResNet-101 grid features -> 1x1 conv -> sinusoidal PE -> 6 post-LN Transformer encoder layers ->
the shared Transformer decoder.  On the HIP path everything runs in libicap.so: the ResNet-101
trunk as MFMA GEMMs over NHWC activation planes (BatchNorm folded into the GEMM epilogue,
SURVEY.md §8(f)3), then projection, PE, encoder layers, decoder and the decode loops.
"""
from __future__ import annotations

import warnings

import torch
import torch.nn as nn

from ._common import PositionalEncoding, TransformerDecoder, beam_search, greedy_torch, padding_mask
from ._hip import HipRouted, attach_owner, owner_of
from ._vision import load_trunks

__all__ = ["PositionalEncoding", "GridFeatureEncoder", "TransformerDecoder", "GridTransformerCaptioning",
           "build_model"]


class GridFeatureEncoder(nn.Module):
    """(B,3,H,W) -> (B, 49, d_model) grid features (grid:34-110)."""

    def __init__(self, d_model=512, nhead=8, num_encoder_layers=6, dim_feedforward=2048, dropout=0.1,
                 pretrained_cnn=True):
        super().__init__()
        _, _, resnet101, weights_enum = load_trunks()
        try:
            trunk = resnet101(weights=weights_enum.DEFAULT) if pretrained_cnn else resnet101()
        except Exception as e:
            warnings.warn(f"pretrained ResNet-101 weights unavailable ({e}); using random init")
            trunk = resnet101()
        self.cnn = nn.Sequential(*list(trunk.children())[:-2])
        self.projection = nn.Conv2d(2048, d_model, kernel_size=1)
        layer = nn.TransformerEncoderLayer(d_model=d_model, nhead=nhead, dim_feedforward=dim_feedforward,
                                           dropout=dropout, batch_first=True)
        self.transformer_encoder = nn.TransformerEncoder(layer, num_layers=num_encoder_layers,
                                                         enable_nested_tensor=False)
        self.pos_encoder = PositionalEncoding(d_model, dropout, max_len=100)
        self.d_model = d_model
        self.set_cnn_trainable(False)

    def set_cnn_trainable(self, trainable=True):
        for p in self.cnn.parameters():
            p.requires_grad = trainable

    def forward(self, images):
        owner = owner_of(self)
        if owner is not None and not self.training and owner.use_hip(images):
            eng = owner.hip_engine(images.device)
            if eng.has_trunk and images.dim() == 4 and images.shape[1] == 3:
                h, w = images.shape[2], images.shape[3]
                if eng.grid_tokens(h, w) <= eng.enc_pe_len:
                    # HIP trunk + tail, any image size; the f16 trunk's range guard re-encodes in bf16x2 on overflow
                    return owner.checked_encode(images)[1]
            # grids larger than the PE table: the reference's own modules (the PE add raises there as well)
        return self.tail(self.cnn(images))

    def tail(self, feats):
        """Everything after self.cnn (grid:97-108): 1x1 projection, flatten, PE, encoder layers."""
        x = self.projection(feats)
        x = x.flatten(2).permute(0, 2, 1)
        return self.transformer_encoder(self.pos_encoder(x))


class GridTransformerCaptioning(HipRouted, nn.Module):
    """CNN grid features + Transformer encoder + Transformer decoder (grid:161-322)."""

    _hip_kind = "grid"

    def __init__(self, vocab_size, d_model=512, nhead=8, num_encoder_layers=6, num_decoder_layers=6,
                 dim_feedforward=2048, dropout=0.1, max_len=100, pretrained_cnn=True, backend="auto",
                 hip_precision="f16"):
        super().__init__()
        self._hip_setup(backend, hip_precision)
        self.vocab_size = vocab_size
        self.d_model = d_model
        self.encoder = GridFeatureEncoder(d_model=d_model, nhead=nhead, num_encoder_layers=num_encoder_layers,
                                          dim_feedforward=dim_feedforward, dropout=dropout,
                                          pretrained_cnn=pretrained_cnn)
        self.decoder = TransformerDecoder(vocab_size=vocab_size, d_model=d_model, nhead=nhead,
                                          num_layers=num_decoder_layers, dim_feedforward=dim_feedforward,
                                          dropout=dropout, max_len=max_len)
        attach_owner(self.encoder, self)
        attach_owner(self.decoder, self)

    def forward(self, images, captions, caption_lengths=None):
        """Teacher-forced training forward (grid:185-210); note the reference pads from
        caption_lengths - 1 here (grid:200), unlike the ViT model."""
        memory = self.encoder(images)
        tgt = captions[:, :-1]
        mask = self.decoder.generate_square_subsequent_mask(tgt.size(1), images.device)
        pad = None
        if caption_lengths is not None:
            pad = self._generate_padding_mask(tgt, [int(l) - 1 for l in caption_lengths])
        return self.decoder(tgt, memory, tgt_mask=mask, tgt_key_padding_mask=pad)

    def _generate_padding_mask(self, tgt, lengths):
        return padding_mask(tgt, lengths)

    def generate(self, images, start_token, end_token, max_len=50, method="greedy", beam_size=5):
        if method == "greedy":
            return self._greedy_search(images, start_token, end_token, max_len)
        if method == "beam_search":
            return self._beam_search(images, start_token, end_token, max_len, beam_size)
        raise ValueError(f"Unknown generation method: {method}")

    def _greedy_search(self, images, start_token, end_token, max_len):
        self.eval()
        with torch.no_grad():
            if self.use_hip(images):
                eng = self.hip_engine(images.device)
                return eng.greedy(self.encoder(images), start_token, end_token, max_len)
            return greedy_torch(self, images, start_token, end_token, max_len)

    def _beam_search(self, images, start_token, end_token, max_len, beam_size=5):
        self.eval()
        return beam_search(self, images, start_token, end_token, max_len, beam_size, grid_variant=True)


def build_model(vocab_size, config):
    """Config dict -> model, same keys and defaults as the reference (grid:325-338)."""
    return GridTransformerCaptioning(
        vocab_size=vocab_size,
        d_model=config.get("d_model", 512),
        nhead=config.get("nhead", 8),
        num_encoder_layers=config.get("num_encoder_layers", 6),
        num_decoder_layers=config.get("num_decoder_layers", 6),
        dim_feedforward=config.get("dim_feedforward", 2048),
        dropout=config.get("dropout", 0.1),
        max_len=config.get("max_len", 100),
        pretrained_cnn=config.get("pretrained_cnn", True),
        backend=config.get("backend", "auto"),
        hip_precision=config.get("hip_precision", "f16"),
    )
