"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import
this module, and only as the checker / CPU baseline.  The product path
(`image_caption_amd`, `models/`, `scripts/`, `utils/`) never calls it.

It restates, with explicit torch fp32 CPU tensor math (no nn.Transformer* modules, no
reference import), the algorithm of:

  * `PositionalEncoding.forward`            models/vit_transformer_model.py:27-33
  * `VisionTransformerEncoder.forward`      models/vit_transformer_model.py:71-100
      + torchvision 0.x `VisionTransformer._process_input / Encoder / EncoderBlock /
        MLPBlock` (third-party, absent here; published algorithm: pre-LN eps 1e-6,
        12 heads, exact-erf GELU MLP 3072, final LN) — pinned against HF
        `transformers.ViTModel` in tests/test_oracle.py.
  * `GridFeatureEncoder.forward`            models/grid_transformer_model.py:86-110
      + torchvision `resnet101` children[:-2] (Bottleneck v1.5, eval BN eps 1e-5) —
        pinned against HF `transformers.ResNetModel` in tests/test_oracle.py;
      + `nn.TransformerEncoderLayer` post-LN ReLU (torch/nn/modules/transformer.py).
  * `TransformerDecoder.forward`            models/vit_transformer_model.py:155-182
      + `nn.TransformerDecoderLayer.forward` post-LN (torch/nn/modules/transformer.py
        :1144-1153), ReLU FFN, eps 1e-5, causal self-attn, cross-attn over memory.
  * `ViTTransformerCaptioning._greedy_search` models/vit_transformer_model.py:296-325
      (full-prefix recompute every step, argmax first-index on ties, stop iff every
      latest token == end).
  * `scripts/inference.py:generate_caption` :60-101 (no causal mask, B=1, stops at end).
  * `SCSTLoss._sample_with_log_probs`       utils/scst_loss.py:202-254 with
      `torch.multinomial` replaced by inverse-CDF on injected uniforms (documented
      deviation).

The oracle is pinned by `tests/golden/*.npz`, produced by running the reference's own code from
/root/reference (tests/golden/make_golden.py): the ViT and Grid models' encoders, greedy and beam
loops and training forwards, SCSTLoss._sample_with_log_probs and scripts/inference.py's loop.
The functions are device-agnostic torch fp32 math: the B = 256 GPU parity tests run the same code on
the GPU in fp32 (gfx950 has no TF32 path) and tie it to the CPU run on a subset of rows.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch

Tensor = torch.Tensor


# --------------------------------------------------------------------------- primitives
def linear(x: Tensor, w: Tensor, b: Optional[Tensor]) -> Tensor:
    y = x @ w.t()
    return y + b if b is not None else y


def layer_norm(x: Tensor, w: Tensor, b: Tensor, eps: float) -> Tensor:
    """(x - mean) / sqrt(biased var + eps) * w + b over the last dim (torch's LayerNorm definition)."""
    return torch.nn.functional.layer_norm(x, (x.shape[-1],), w, b, eps)


def gelu_erf(x: Tensor) -> Tensor:
    """0.5 x (1 + erf(x / sqrt 2)) - the exact GELU of torchvision's MLPBlock."""
    return torch.nn.functional.gelu(x)


def mha(q_in: Tensor, kv_in: Tensor, in_w: Tensor, in_b: Tensor, out_w: Tensor,
        out_b: Tensor, nhead: int, causal: bool, key_pad: Optional[Tensor] = None,
        p_mask: Optional[Tensor] = None) -> Tensor:
    """torch `F.multi_head_attention_forward` semantics (batch_first).  key_pad (B,S)
    bool masks keys; a query left with no key gets a zero context, which is what the
    scaled_dot_product_attention path (need_weights=False, the TransformerDecoderLayer call) returns.
    p_mask (B,H,T,S): dropout on the attention probabilities (train mode, oracle/dropout.py)."""
    B, T, D = q_in.shape
    S = kv_in.shape[1]
    hd = D // nhead
    if q_in is kv_in:  # self-attention: one packed projection (the same products as three)
        q, k, v = linear(q_in, in_w, in_b).chunk(3, dim=-1)
    else:
        q = linear(q_in, in_w[:D], in_b[:D])
        k, v = linear(kv_in, in_w[D:], in_b[D:]).chunk(2, dim=-1)
    q = q.reshape(B, T, nhead, hd).transpose(1, 2)
    k = k.reshape(B, S, nhead, hd).transpose(1, 2)
    v = v.reshape(B, S, nhead, hd).transpose(1, 2)
    if key_pad is None and p_mask is None:  # softmax(q k^T / sqrt(hd) [+ causal -inf]) v as one fused CPU primitive
        causal_mask = None
        if causal:
            causal_mask = torch.ones(T, S, dtype=torch.bool, device=q.device).tril(S - T)
        o = torch.nn.functional.scaled_dot_product_attention(q, k, v, attn_mask=causal_mask)
        return linear(o.transpose(1, 2).reshape(B, T, D), out_w, out_b)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    if causal:
        m = torch.ones(T, S, dtype=torch.bool, device=s.device).triu(1 + S - T)
        s = s.masked_fill(m, float("-inf"))
    if key_pad is not None:
        s = s.masked_fill(key_pad[:, None, None, :], float("-inf"))
    p = torch.softmax(s, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)  # fully masked rows
    if p_mask is not None:
        p = p * p_mask
    o = (p @ v).transpose(1, 2).reshape(B, T, D)
    return linear(o, out_w, out_b)


# --------------------------------------------------------------------------- encoders
def vit_encode(sd: Dict[str, Tensor], images: Tensor) -> Tensor:
    """images (B,3,224,224) fp32 -> memory (B,196,512).  vit:71-100."""
    P = "encoder.vit."
    B = images.shape[0]
    w = sd[P + "conv_proj.weight"]                     # (768,3,16,16)
    D = w.shape[0]
    # _process_input: conv k16 s16 == GEMM over 16x16 patches, (c,kh,kw) order
    patches = images.reshape(B, 3, 14, 16, 14, 16).permute(0, 2, 4, 1, 3, 5).reshape(B, 196, 768)
    x = linear(patches, w.reshape(D, -1), sd[P + "conv_proj.bias"])
    x = torch.cat([sd[P + "class_token"].expand(B, -1, -1), x], dim=1)
    x = x + sd[P + "encoder.pos_embedding"]
    i = 0
    while (P + f"encoder.layers.encoder_layer_{i}.ln_1.weight") in sd:
        L = P + f"encoder.layers.encoder_layer_{i}."
        h = layer_norm(x, sd[L + "ln_1.weight"], sd[L + "ln_1.bias"], 1e-6)
        h = mha(h, h, sd[L + "self_attention.in_proj_weight"], sd[L + "self_attention.in_proj_bias"],
                sd[L + "self_attention.out_proj.weight"], sd[L + "self_attention.out_proj.bias"],
                nhead=12, causal=False)
        x = x + h
        y = layer_norm(x, sd[L + "ln_2.weight"], sd[L + "ln_2.bias"], 1e-6)
        y = gelu_erf(linear(y, sd[L + "mlp.0.weight"], sd[L + "mlp.0.bias"]))
        y = linear(y, sd[L + "mlp.3.weight"], sd[L + "mlp.3.bias"])
        x = x + y
        i += 1
    x = layer_norm(x, sd[P + "encoder.ln.weight"], sd[P + "encoder.ln.bias"], 1e-6)
    return linear(x[:, 1:], sd["encoder.projection.weight"], sd["encoder.projection.bias"])


def _bn_eval(x: Tensor, sd, p: str) -> Tensor:
    scale = sd[p + ".weight"] / torch.sqrt(sd[p + ".running_var"] + 1e-5)
    shift = sd[p + ".bias"] - sd[p + ".running_mean"] * scale
    return x * scale[None, :, None, None] + shift[None, :, None, None]


def resnet101_trunk(sd: Dict[str, Tensor], images: Tensor) -> Tensor:
    """torchvision resnet101 children[:-2] in eval mode -> (B,2048,7,7)."""
    F = torch.nn.functional
    P = "encoder.cnn."
    x = F.conv2d(images, sd[P + "0.weight"], stride=2, padding=3)
    x = torch.relu(_bn_eval(x, sd, P + "1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nblk in enumerate((3, 4, 23, 3)):
        for b in range(nblk):
            p = P + f"{4 + li}.{b}."
            stride = 2 if (b == 0 and li > 0) else 1
            y = torch.relu(_bn_eval(F.conv2d(x, sd[p + "conv1.weight"]), sd, p + "bn1"))
            y = torch.relu(_bn_eval(F.conv2d(y, sd[p + "conv2.weight"], stride=stride, padding=1), sd, p + "bn2"))
            y = _bn_eval(F.conv2d(y, sd[p + "conv3.weight"]), sd, p + "bn3")
            if b == 0:
                x = _bn_eval(F.conv2d(x, sd[p + "downsample.0.weight"], stride=stride), sd, p + "downsample.1")
            x = torch.relu(x + y)
    return x


def encoder_layer_postln(x: Tensor, sd, p: str, nhead: int) -> Tensor:
    """nn.TransformerEncoderLayer (post-LN, ReLU, eps 1e-5), eval."""
    h = mha(x, x, sd[p + "self_attn.in_proj_weight"], sd[p + "self_attn.in_proj_bias"],
            sd[p + "self_attn.out_proj.weight"], sd[p + "self_attn.out_proj.bias"], nhead, False)
    x = layer_norm(x + h, sd[p + "norm1.weight"], sd[p + "norm1.bias"], 1e-5)
    f = linear(torch.relu(linear(x, sd[p + "linear1.weight"], sd[p + "linear1.bias"])),
               sd[p + "linear2.weight"], sd[p + "linear2.bias"])
    return layer_norm(x + f, sd[p + "norm2.weight"], sd[p + "norm2.bias"], 1e-5)


def grid_encode_tail(sd: Dict[str, Tensor], feats: Tensor, nhead: int = 8) -> Tensor:
    """(B,2048,7,7) trunk features -> memory (B,49,512).  grid:97-108."""
    B = feats.shape[0]
    w = sd["encoder.projection.weight"]
    x = feats.flatten(2).transpose(1, 2)                       # (B,49,2048)
    x = linear(x, w.reshape(w.shape[0], -1), sd["encoder.projection.bias"])
    x = x + sd["encoder.pos_encoder.pe"][:, : x.shape[1]]
    i = 0
    while f"encoder.transformer_encoder.layers.{i}.norm1.weight" in sd:
        x = encoder_layer_postln(x, sd, f"encoder.transformer_encoder.layers.{i}.", nhead)
        i += 1
    return x


def grid_encode(sd: Dict[str, Tensor], images: Tensor) -> Tensor:
    return grid_encode_tail(sd, resnet101_trunk(sd, images))


# --------------------------------------------------------------------------- decoder
def padding_mask(tgt: Tensor, lengths) -> Tensor:
    """`_generate_padding_mask` (vit:257-274): mask[i, length:] = True when length < seq_len, with
    Python slicing (a negative length masks the last -length positions)."""
    B, T = tgt.shape
    mask = torch.zeros(B, T, dtype=torch.bool)
    for i, length in enumerate(lengths):
        if int(length) < T:
            mask[i, int(length):] = True
    return mask


def training_forward(sd: Dict[str, Tensor], memory: Tensor, captions: Tensor, lengths, grid: bool = False) -> Tensor:
    """Teacher-forced forward after the encoder: vit:216-255 (padding from lengths) or grid:185-207
    (padding from lengths - 1)."""
    tgt = captions[:, :-1]
    lens = [int(l) - 1 for l in lengths] if grid else lengths
    return decoder_forward(sd, tgt, memory, True, key_pad=padding_mask(tgt, lens))


def decoder_forward(sd: Dict[str, Tensor], tgt: Tensor, memory: Tensor, causal: bool = True,
                    nhead: int = 8, key_pad: Optional[Tensor] = None, masks: Optional[dict] = None) -> Tensor:
    """`TransformerDecoder.forward` (vit:155-182): tgt (B,T) int -> logits (B,T,V).  masks (train mode,
    oracle/dropout.py decoder_masks over at least T positions): the dropout of PositionalEncoding and of
    every TransformerDecoderLayer (attention maps, dropout1/2/3, FFN hidden)."""
    emb = sd["decoder.embedding.weight"]
    d = emb.shape[1]
    T = tgt.shape[1]
    m = (lambda k: masks[k][:, :T]) if masks is not None else (lambda k: None)
    ma = (lambda k, S: masks[k][:, :, :T, :S]) if masks is not None else (lambda k, S: None)
    drop = lambda x, k: x if masks is None else x * m(k)
    x = emb[tgt] * math.sqrt(d)
    x = drop(x + sd["decoder.pos_encoder.pe"][:, : tgt.shape[1]], "pe")
    i = 0
    while f"decoder.transformer_decoder.layers.{i}.norm1.weight" in sd:
        p = f"decoder.transformer_decoder.layers.{i}."
        h = mha(x, x, sd[p + "self_attn.in_proj_weight"], sd[p + "self_attn.in_proj_bias"],
                sd[p + "self_attn.out_proj.weight"], sd[p + "self_attn.out_proj.bias"], nhead, causal, key_pad,
                p_mask=ma(f"sa_p.{i}", T))
        x = layer_norm(x + drop(h, f"sa_o.{i}"), sd[p + "norm1.weight"], sd[p + "norm1.bias"], 1e-5)
        h = mha(x, memory, sd[p + "multihead_attn.in_proj_weight"], sd[p + "multihead_attn.in_proj_bias"],
                sd[p + "multihead_attn.out_proj.weight"], sd[p + "multihead_attn.out_proj.bias"], nhead, False,
                p_mask=ma(f"ca_p.{i}", memory.shape[1]))
        x = layer_norm(x + drop(h, f"ca_o.{i}"), sd[p + "norm2.weight"], sd[p + "norm2.bias"], 1e-5)
        hid = drop(torch.relu(linear(x, sd[p + "linear1.weight"], sd[p + "linear1.bias"])), f"ff_h.{i}")
        f = linear(hid, sd[p + "linear2.weight"], sd[p + "linear2.bias"])
        x = layer_norm(x + drop(f, f"ff_o.{i}"), sd[p + "norm3.weight"], sd[p + "norm3.bias"], 1e-5)
        i += 1
    return linear(x, sd["decoder.fc_out.weight"], sd["decoder.fc_out.bias"])


def greedy_from_memory(sd, memory: Tensor, start: int, end: int, max_len: int,
                       return_trace: bool = False):
    """`_greedy_search` loop (vit:306-325): returns generated (B,L) int64 and, if asked,
    the per-step last-position logits (steps,B,V)."""
    B = memory.shape[0]
    generated = torch.full((B, 1), start, dtype=torch.long, device=memory.device)
    trace = []
    for _ in range(max_len - 1):
        out = decoder_forward(sd, generated, memory, causal=True)
        logits = out[:, -1, :]
        trace.append(logits)
        nxt = logits.argmax(dim=-1)
        generated = torch.cat([generated, nxt.unsqueeze(1)], dim=1)
        if bool((nxt == end).all()):
            break
    if return_trace:
        return generated, torch.stack(trace, 0)
    return generated


def greedy_search(sd, images: Tensor, start: int, end: int, max_len: int, encoder: str = "vit",
                  return_trace: bool = False):
    with torch.no_grad():
        mem = vit_encode(sd, images) if encoder == "vit" else grid_encode(sd, images)
        return greedy_from_memory(sd, mem, start, end, max_len, return_trace)


def teacher_forced_logits(sd, memory: Tensor, ids: Tensor) -> Tensor:
    """Logits of every step given a fixed id prefix (B,L): row t = prediction after ids[:, :t+1]."""
    with torch.no_grad():
        return decoder_forward(sd, ids[:, :-1], memory, causal=True)


def inference_py_generate(sd, memory: Tensor, start: int, end: int, max_len: int = 50):
    """`scripts/inference.py:generate_caption` loop (:75-99): NO causal mask, batch 1,
    breaks at <end> without appending it.  Returns the list of predicted ids."""
    inputs = torch.tensor([[start]])
    out_ids = []
    for _ in range(max_len):
        logits = decoder_forward(sd, inputs, memory, causal=False)[:, -1, :]
        pid = int(logits.max(1)[1].item())
        if pid == end:
            break
        out_ids.append(pid)
        inputs = torch.cat([inputs, torch.tensor([[pid]])], dim=1)
    return out_ids


def beam_from_memory(sd, memory: Tensor, start: int, end: int, max_len: int, beam_size: int,
                     grid_variant: bool = False, return_margins: bool = False):
    """`_beam_search` for ONE image (memory (1,S,d)), full-prefix recompute each step:
    vit:327-420 (stop when every live beam ended) or grid:253-322 (stop when the completed count
    reaches the live beam count, or no live beam is left).  Returns the chosen sequence (1,L)
    int64; with return_margins also the smallest gap, over all steps, between the k-th selected
    candidate score and the best rejected one (how far the selection is from a tie)."""
    V = sd["decoder.fc_out.weight"].shape[0]
    with torch.no_grad():
        mem = memory.expand(beam_size, -1, -1)
        seqs = torch.full((beam_size, 1), start, dtype=torch.long)
        scores = torch.zeros(beam_size)
        done, done_scores = [], []
        margin = float("inf")
        for step in range(max_len - 1):
            if grid_variant and seqs.size(0) == 0:
                break
            logp = torch.log_softmax(decoder_forward(sd, seqs, mem, causal=True)[:, -1, :], dim=-1)
            cand = logp[0] if step == 0 else (scores.unsqueeze(1) + logp).view(-1)
            top = cand.topk(min(beam_size + 1, cand.numel()))
            if top.values.numel() > beam_size:
                margin = min(margin, float(top.values[beam_size - 1] - top.values[beam_size]))
            top_s, top_i = top.values[:beam_size], top.indices[:beam_size]
            if step == 0:
                seqs = torch.cat([seqs[0:1].expand(beam_size, -1), top_i.unsqueeze(1)], dim=1)
            else:
                seqs = torch.cat([seqs[top_i // V], (top_i % V).unsqueeze(1)], dim=1)
            scores = top_s
            ended = seqs[:, -1] == end
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
                seqs, scores, mem = seqs[keep], scores[keep], mem[keep]
                if grid_variant and seqs.size(0) == 0:
                    break
                beam_size = seqs.size(0)
        out = (done[int(torch.tensor(done_scores).argmax())] if done else seqs[scores.argmax()]).unsqueeze(0)
    return (out, margin) if return_margins else out


def inverse_cdf_sample(logits: Tensor, u: Tensor) -> Tuple[Tensor, Tensor]:
    """Categorical sample from softmax(logits) with injected uniforms u in [0,1):
    first index whose inclusive prefix sum of probabilities exceeds u * total."""
    probs = torch.softmax(logits, dim=-1)
    cdf = torch.cumsum(probs, dim=-1)
    thr = u.unsqueeze(-1) * cdf[:, -1:]
    idx = (cdf <= thr).sum(-1).clamp_max(logits.shape[-1] - 1)
    logp = torch.log_softmax(logits, dim=-1).gather(1, idx.unsqueeze(1)).squeeze(1)
    return idx, logp


def sample_with_log_probs(sd, memory: Tensor, uniforms: Tensor, start: int, end: int, max_len: int,
                          masks: Optional[dict] = None):
    """`_sample_with_log_probs` (scst_loss:202-254) with injected uniforms (max_len-1, B); masks: train-mode
    dropout (oracle/dropout.py decoder_masks over max_len - 1 positions), applied to every full-prefix
    recompute by position, as the KV-cached HIP sampler does."""
    B = memory.shape[0]
    generated = torch.full((B, 1), start, dtype=torch.long, device=memory.device)
    finished = torch.zeros(B, dtype=torch.bool, device=memory.device)
    lps = []
    with torch.no_grad():
        for step in range(max_len - 1):
            logits = decoder_forward(sd, generated, memory, causal=True, masks=masks)[:, -1, :]
            nxt, lp = inverse_cdf_sample(logits, uniforms[step])
            lps.append(lp.masked_fill(finished, 0.0))
            generated = torch.cat([generated, nxt.unsqueeze(1)], dim=1)
            finished = finished | (nxt == end)
            if bool(finished.all()):
                break
    return generated, torch.stack(lps, dim=1)


def top2_margin(logits: Tensor) -> Tensor:
    t = logits.topk(2, dim=-1).values
    return t[..., 0] - t[..., 1]
