"""Pieces shared by the ViT and Grid captioning models: positional encoding, the Transformer
decoder, and the generation loops' PyTorch forms (used off the HIP path: CPU tensors, or
backend="torch").  Behaviour follows the reference file:line cited on each piece."""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn

from image_caption_amd.weights import positional_encoding
from ._hip import is_causal_mask, owner_of


class PositionalEncoding(nn.Module):
    """x + pe[:, :T] then dropout; sinusoidal table, base 10000 (vit:11-33, grid:11-31)."""

    def __init__(self, d_model, dropout=0.1, max_len=5000):
        super().__init__()
        self.dropout = nn.Dropout(p=dropout)
        self.register_buffer("pe", torch.from_numpy(positional_encoding(max_len, d_model)))

    def forward(self, x):
        return self.dropout(x + self.pe[:, : x.size(1), :])


class TransformerDecoder(nn.Module):
    """Token embedding * sqrt(d) + PE -> 6 post-LN nn.TransformerDecoderLayer -> fc_out
    (vit:103-182, grid:113-158).  In eval on a GPU the forward runs on the HIP engine
    (icap_decoder_forward): causal mask or no mask, with or without a tgt_key_padding_mask of the
    form the captioners build (True on a suffix of each row = key lengths)."""

    def __init__(self, vocab_size, d_model=512, nhead=8, num_layers=6, dim_feedforward=2048, dropout=0.1,
                 max_len=100):
        super().__init__()
        self.d_model = d_model
        self.vocab_size = vocab_size
        self.embedding = nn.Embedding(vocab_size, d_model)
        self.pos_encoder = PositionalEncoding(d_model, dropout, max_len)
        layer = nn.TransformerDecoderLayer(d_model=d_model, nhead=nhead, dim_feedforward=dim_feedforward,
                                           dropout=dropout, batch_first=True)
        self.transformer_decoder = nn.TransformerDecoder(layer, num_layers=num_layers)
        self.fc_out = nn.Linear(d_model, vocab_size)
        self.init_weights()

    def init_weights(self):
        r = 0.1
        self.embedding.weight.data.uniform_(-r, r)
        self.fc_out.weight.data.uniform_(-r, r)
        self.fc_out.bias.data.zero_()

    def generate_square_subsequent_mask(self, sz, device):
        upper = torch.triu(torch.ones(sz, sz, device=device), diagonal=1)
        return upper.masked_fill(upper == 1, float("-inf"))

    def forward(self, tgt, memory, tgt_mask=None, tgt_key_padding_mask=None, memory_key_padding_mask=None):
        owner = owner_of(self)
        T = tgt.shape[1]
        if (owner is not None and memory_key_padding_mask is None
                and (tgt_mask is None or is_causal_mask(tgt_mask, T)) and not self.training
                and owner.use_hip(memory)):
            klen = suffix_mask_lengths(tgt_key_padding_mask, T) if tgt_key_padding_mask is not None else None
            if tgt_key_padding_mask is None or klen is not None:
                return owner.hip_engine(memory.device).decoder_forward(tgt, memory, causal=tgt_mask is not None,
                                                                       key_lengths=klen)
        x = self.pos_encoder(self.embedding(tgt) * math.sqrt(self.d_model))
        x = self.transformer_decoder(x, memory, tgt_mask=tgt_mask, tgt_key_padding_mask=tgt_key_padding_mask,
                                     memory_key_padding_mask=memory_key_padding_mask)
        return self.fc_out(x)


def padding_mask(tgt: torch.Tensor, lengths) -> torch.Tensor:
    """vit:257-274 / grid:209-216: mask[i, length:] = True when length < seq_len - Python slicing,
    so a negative length (grid's lengths - 1 of an empty caption) masks only the last -length keys."""
    B, T = tgt.shape
    starts = []
    for l in lengths:
        l = int(l)
        starts.append(T if l >= T else (l if l >= 0 else max(T + l, 0)))
    lens = torch.as_tensor(starts, device=tgt.device)
    return torch.arange(T, device=tgt.device)[None, :] >= lens[:, None]


def suffix_mask_lengths(mask: torch.Tensor, T: int):
    """(B,) key lengths of a bool key-padding mask that is True exactly on a suffix of every row
    (what padding_mask builds), else None (the mask then stays on the PyTorch path)."""
    if mask.dtype != torch.bool or mask.dim() != 2 or mask.shape[1] != T:
        return None
    klen = (~mask).sum(1)
    if not torch.equal(mask, torch.arange(T, device=mask.device)[None, :] >= klen[:, None]):
        return None
    return klen


def greedy_torch(model, images, start_token, end_token, max_len):
    """PyTorch form of `_greedy_search` (vit:296-325): full-prefix recompute every step."""
    B = images.size(0)
    memory = model.encoder(images)
    generated = torch.full((B, 1), start_token, dtype=torch.long, device=images.device)
    for _ in range(max_len - 1):
        mask = model.decoder.generate_square_subsequent_mask(generated.size(1), images.device)
        nxt = model.decoder(generated, memory, tgt_mask=mask)[:, -1, :].argmax(dim=-1)
        generated = torch.cat([generated, nxt.unsqueeze(1)], dim=1)
        if bool((nxt == end_token).all()):
            break
    return generated


def beam_search(model, images, start_token, end_token, max_len, beam_size, grid_variant: bool):
    """`_beam_search` (vit:327-420 / grid:253-322): one image at a time, log-softmax scores,
    pruning of finished beams (the live beam count shrinks).  The two reference variants differ
    in their stop tests, selected by `grid_variant`."""
    if getattr(model, "use_hip", None) is not None and not model.training and model.use_hip(images):
        # every image at once on the GPU (icap_decode_beam: B*K rows of the KV-cached decoder), then
        # the reference's per-image results concatenated as it does (vit:335-341)
        with torch.no_grad():
            memory = model.encoder(images)
            ids, lens = model.hip_engine(images.device).beam(memory, start_token, end_token, max_len, beam_size,
                                                             grid_variant)
        ids, lens = ids.long(), lens.tolist()
        return torch.cat([ids[i:i + 1, :lens[i]] for i in range(ids.shape[0])], dim=0)
    if images.size(0) != 1:
        return torch.cat([beam_search(model, images[i:i + 1], start_token, end_token, max_len, beam_size,
                                      grid_variant) for i in range(images.size(0))], dim=0)
    dev = images.device
    V = model.vocab_size
    with torch.no_grad():
        memory = model.encoder(images).expand(beam_size, -1, -1)
        seqs = torch.full((beam_size, 1), start_token, dtype=torch.long, device=dev)
        scores = torch.zeros(beam_size, device=dev)
        done, done_scores = [], []
        for step in range(max_len - 1):
            if grid_variant and seqs.size(0) == 0:
                break
            mask = model.decoder.generate_square_subsequent_mask(seqs.size(1), dev)
            logp = torch.log_softmax(model.decoder(seqs, memory, tgt_mask=mask)[:, -1, :], dim=-1)
            if step == 0:
                top_s, top_w = logp[0].topk(beam_size)
                seqs = torch.cat([seqs[0:1].expand(beam_size, -1), top_w.unsqueeze(1)], dim=1)
            else:
                top_s, top_i = (scores.unsqueeze(1) + logp).view(-1).topk(beam_size)
                seqs = torch.cat([seqs[top_i // V], (top_i % V).unsqueeze(1)], dim=1)
            scores = top_s
            ended = seqs[:, -1] == end_token
            if bool(ended.any()):
                for i in ended.nonzero(as_tuple=True)[0]:
                    done.append(seqs[i])
                    done_scores.append(scores[i])
                if grid_variant:
                    if len(done) >= beam_size:
                        break
                elif bool(ended.all()):
                    break
                keep = ~ended
                seqs, scores, memory = seqs[keep], scores[keep], memory[keep]
                if grid_variant and seqs.size(0) == 0:
                    break
                beam_size = seqs.size(0)
        if done:
            return done[int(torch.tensor(done_scores).argmax())].unsqueeze(0)
        return seqs[scores.argmax()].unsqueeze(0)


def decode_ids(ids, idx2word, end_token, pad_token, start_token):
    """ids -> caption strings: stop at <end>, drop <start>/<pad> (scst_loss:256-269,
    scripts/inference_vit_transformer.py:117-127)."""
    out = []
    for row in ids.tolist() if torch.is_tensor(ids) else ids:
        words = []
        for t in row:
            if t == end_token:
                break
            if t not in (start_token, pad_token):
                words.append(idx2word.get(t, "<unk>"))
        out.append(" ".join(words))
    return out
