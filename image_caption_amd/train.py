"""HIP training pass of the TransformerDecoder: the teacher-forced log-prob recompute of
the SCST step and its backward as one torch.autograd.Function over libicap's icap_decoder_train_forward /
icap_decoder_train_backward (train.hip), so the optimizer, DDP's gradient all-reduce and the encoder's
autograd (projection / Grid tail) see ordinary parameter gradients.

Reference: the autograd graph SCSTLoss._sample_with_log_probs builds (utils/scst_loss.py:210-254 of the
reference: decoder forward, log_softmax, gather, masked_fill after <end>) and loss.backward()
(scripts/train_vit_transformer_scst_optimized.py:261).  Eval-mode forward: no dropout, the same as the HIP
sampler; or train mode with the sampler's counter-based dropout masks (p, seed): the same masks, so the
distribution sampled from is the one differentiated either way."""
from __future__ import annotations

import ctypes
from typing import List, Tuple

import torch
import torch.nn as nn

from . import _lib
from ._lib import DecLayerW, LnW, MhaW, ModelDesc, check, stream_ptr

_MHA = ("in_proj_weight", "in_proj_bias", "out_proj.weight", "out_proj.bias")


def decoder_param_names(n_layers: int) -> List[str]:
    """The TransformerDecoder parameters in the order of the autograd Function's inputs."""
    names = ["embedding.weight", "fc_out.weight", "fc_out.bias"]
    for i in range(n_layers):
        p = f"transformer_decoder.layers.{i}."
        names += [p + "self_attn." + k for k in _MHA] + [p + "multihead_attn." + k for k in _MHA]
        names += [p + k for k in ("linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias",
                                  "norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias",
                                  "norm3.weight", "norm3.bias")]
    return names


def _desc(t: dict, n_layers: int, d_model: int, nhead: int, pe: torch.Tensor):
    """icap_model_desc with the decoder fields over the tensors `t` (name -> fp32 contiguous device tensor)."""
    ptr = lambda k: t[k].data_ptr()
    dec = (DecLayerW * n_layers)()
    for i in range(n_layers):
        p = f"transformer_decoder.layers.{i}."
        mha = lambda q: MhaW(*(ptr(p + q + "." + k) for k in _MHA))
        ln = lambda q: LnW(ptr(p + q + ".weight"), ptr(p + q + ".bias"))
        dec[i] = DecLayerW(mha("self_attn"), mha("multihead_attn"), ptr(p + "linear1.weight"), ptr(p + "linear1.bias"),
                           ptr(p + "linear2.weight"), ptr(p + "linear2.bias"), ln("norm1"), ln("norm2"), ln("norm3"))
    d = ModelDesc()
    d.d_model, d.nhead = d_model, nhead
    d.dim_ff = t["transformer_decoder.layers.0.linear1.weight"].shape[0]
    d.n_dec_layers, d.vocab, d.pe_len = n_layers, t["embedding.weight"].shape[0], pe.shape[1]
    d.emb, d.pe = ptr("embedding.weight"), pe.data_ptr()
    d.fc_w, d.fc_b = ptr("fc_out.weight"), ptr("fc_out.bias")
    d.dec_layers = ctypes.cast(dec, ctypes.POINTER(DecLayerW))
    return d, dec


class _DecoderLogProbs(torch.autograd.Function):
    @staticmethod
    def forward(ctx, cfg, memory, ids, *params):
        lib, n_layers, d_model, nhead, pe, end, drop_p, seed = cfg
        names = decoder_param_names(n_layers)
        t = dict(zip(names, params))
        desc, keep = _desc(t, n_layers, d_model, nhead, pe)
        B, L = ids.shape
        T, S = L - 1, memory.shape[1]
        mem = memory.detach().float().contiguous()
        ids32 = ids.to(torch.int32).contiguous()
        nbytes = lib.icap_decoder_train_workspace(ctypes.byref(desc), B, T, S, drop_p)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=memory.device)
        logp = torch.empty(B, T, dtype=torch.float32, device=memory.device)
        check(lib.icap_decoder_train_forward(ctypes.byref(desc), ids32.data_ptr(), B, T, mem.data_ptr(), S, end,
                                             drop_p, seed, logp.data_ptr(), ws.data_ptr(), nbytes,
                                             stream_ptr(memory.device)),
              "icap_decoder_train_forward")
        ctx.cfg, ctx.ws, ctx.keep = cfg, ws, keep
        ctx.save_for_backward(mem, ids32, *params)
        ctx.mem_grad = memory.requires_grad
        return logp

    @staticmethod
    def backward(ctx, dlogp):
        lib, n_layers, d_model, nhead, pe, end, drop_p, _ = ctx.cfg
        mem, ids32, *params = ctx.saved_tensors
        names = decoder_param_names(n_layers)
        t = dict(zip(names, params))
        desc, keep = _desc(t, n_layers, d_model, nhead, pe)
        grads = {k: torch.empty_like(v) for k, v in t.items()}
        gdesc, gkeep = _desc(grads, n_layers, d_model, nhead, pe)
        B, L = ids32.shape
        dmem = torch.empty_like(mem) if ctx.mem_grad else None
        dl = dlogp.float().contiguous()
        check(lib.icap_decoder_train_backward(ctypes.byref(desc), ctypes.byref(gdesc), ids32.data_ptr(), B, L - 1,
                                              mem.data_ptr(), mem.shape[1], end, drop_p, dl.data_ptr(),
                                              None if dmem is None else dmem.data_ptr(), ctx.ws.data_ptr(),
                                              ctx.ws.numel(), stream_ptr(mem.device)),
              "icap_decoder_train_backward")
        ctx.ws = None
        return (None, dmem, None) + tuple(grads[k] for k in names)


def decoder_dropout(decoder: nn.Module) -> float:
    """The dropout p of a TransformerDecoder in train mode (PositionalEncoding and every decoder layer share
    the config's value, vit:103-147), 0 in eval mode."""
    if not decoder.training:
        return 0.0
    ps = {decoder.pos_encoder.dropout.p}
    for layer in decoder.transformer_decoder.layers:
        ps |= {layer.dropout.p, layer.dropout1.p, layer.dropout2.p, layer.dropout3.p, layer.self_attn.dropout,
               layer.multihead_attn.dropout}
    if len(ps) != 1:
        raise ValueError(f"the HIP decoder needs one dropout p for every site, got {sorted(ps)}")
    return float(ps.pop())


def decoder_token_logp(decoder: nn.Module, memory: torch.Tensor, ids: torch.Tensor, end_token: int,
                       dropout: Tuple[float, int] = (0.0, 0)) -> torch.Tensor:
    """(B, L-1) log p(ids[:, t+1] | ids[:, :t+1], memory), zeroed after a row's first <end>: the HIP forward
    and backward of `decoder` (a TransformerDecoder: vit:103-182 / grid's) - the same values as
    utils.scst_loss.masked_token_logp(decoder(ids[:, :-1], memory, causal mask), ids, end) in eval mode;
    dropout = (p, seed) > 0: train mode with the masks of Engine.sample(..., dropout=(p, seed))."""
    n_layers = len(decoder.transformer_decoder.layers)
    names = decoder_param_names(n_layers)
    named = dict(decoder.named_parameters())
    params = [named[k] for k in names]
    for p in params:
        if p.dtype != torch.float32 or not p.is_contiguous() or not p.is_cuda:
            raise ValueError("the HIP decoder training pass needs contiguous fp32 parameters on the GPU")
    pe = decoder.pos_encoder.pe.detach().float().contiguous()
    nhead = decoder.transformer_decoder.layers[0].self_attn.num_heads
    cfg = (_lib.load(), n_layers, decoder.d_model, nhead, pe, int(end_token), float(dropout[0]),
           int(dropout[1]) & 0xFFFFFFFF)
    return _DecoderLogProbs.apply(cfg, memory, ids, *params)


def vit_trunk_frozen(model: nn.Module) -> bool:
    """A ViT captioner whose vit_b_16 trunk takes no gradient (the reference default, vit:64): its output
    can come from the HIP encoder and only encoder.projection needs PyTorch autograd."""
    enc = getattr(model, "encoder", None)
    vit = getattr(enc, "vit", None)
    return vit is not None and getattr(model, "_hip_kind", "") == "vit" and not any(
        p.requires_grad for p in vit.parameters())


def hip_memory_with_grad(model: nn.Module, images: torch.Tensor) -> torch.Tensor:
    """encoder(images) with autograd through its trainable parameters: the HIP trunk's output through
    encoder.projection when the ViT is frozen, the PyTorch encoder otherwise."""
    if vit_trunk_frozen(model) and tuple(images.shape[1:]) == (3, 224, 224):
        with torch.no_grad():
            _, feats = model.hip_engine(images.device).encode_vit_features(images)
        return model.encoder.projection(feats)
    return model.encoder(images)
