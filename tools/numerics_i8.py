"""CPU emulation of an int8-sliced (Ozaki-style) encoder GEMM for the LayerNorm-fed GEMMs
(ViT QKV and MLP-1): activation rows and weight rows as two int8 slices under a per-row scale
(x = s_x (256 a1 + a2), w = s_w (256 b1 + b2), 16-bit fixed point relative to the row maximum),
product 65536 a1.b1 + 256 (a1.b2 + a2.b1) accumulated exactly in int32 (the a2.b2 term dropped).
The other GEMMs stay bf16x2 (hi/lo bf16 activation planes, bf16 weights), attention products the
3-term split, the decoder bf16x2.  Counts greedy-token divergences vs the fp32 oracle.
Measurement tool used to decide the encoder precision scheme; not part of the product.
usage: python tools/numerics_i8.py B [drop_a2b2=1]"""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import weights as W
from oracle import captioner as O

torch.set_num_threads(8)
bf = lambda x: x.to(torch.bfloat16).float()
DROP = True


def split2(a, b_t):  # bf16x2 activation x bf16 weight
    ah = bf(a)
    al = bf(a - ah)
    return ah @ bf(b_t) + al @ bf(b_t)


def split3(a, b):  # attention products: hi.hi + lo.hi + hi.lo
    ah, bh = bf(a), bf(b)
    al, bl = bf(a - ah), bf(b - bh)
    return ah @ bh + al @ bh + ah @ bl


def q2(x):
    s = x.abs().amax(-1, keepdim=True).clamp_min(1e-30) / 32639.0
    q = torch.round(x / s)
    a1 = torch.floor((q + 128) / 256)
    a2 = q - 256 * a1
    assert a1.abs().max() <= 127 and a2.min() >= -128 and a2.max() <= 127
    return a1.double(), a2.double(), s.double()


def i8_linear(x, w, b):
    a1, a2, sx = q2(x)
    b1, b2, sw = q2(w)
    acc = 65536 * (a1 @ b1.t()) + 256 * (a1 @ b2.t() + a2 @ b1.t())
    if not DROP:
        acc = acc + a2 @ b2.t()
    y = (acc * sx * sw.t()).float()
    return y + b


def lin2(x, w, b):
    return split2(x, w.t()) + b


def enc_mha(h, L, sd, qkv_lin):
    B, T, D = h.shape
    in_w, in_b = sd[L + "self_attention.in_proj_weight"], sd[L + "self_attention.in_proj_bias"]
    qkv = qkv_lin(h, in_w, in_b)
    q, k, v = qkv.split(D, -1)
    q = q.view(B, T, 12, 64).transpose(1, 2)
    k = k.view(B, T, 12, 64).transpose(1, 2)
    v = v.view(B, T, 12, 64).transpose(1, 2)
    s = split3(q, k.transpose(-1, -2)) / 8.0
    p = torch.softmax(s, -1)
    o = split3(p, v).transpose(1, 2).reshape(B, T, D)
    return lin2(o, sd[L + "self_attention.out_proj.weight"], sd[L + "self_attention.out_proj.bias"])


def vit_encode(sd, images, mode):
    P = "encoder.vit."
    B = images.shape[0]
    w = sd[P + "conv_proj.weight"]
    patches = images.reshape(B, 3, 14, 16, 14, 16).permute(0, 2, 4, 1, 3, 5).reshape(B, 196, 768)
    x = lin2(patches, w.reshape(768, -1), sd[P + "conv_proj.bias"])
    x = torch.cat([sd[P + "class_token"].expand(B, -1, -1), x], dim=1) + sd[P + "encoder.pos_embedding"]
    ln_lin = i8_linear if mode == "i8" else lin2
    for i in range(12):
        L = P + f"encoder.layers.encoder_layer_{i}."
        h = O.layer_norm(x, sd[L + "ln_1.weight"], sd[L + "ln_1.bias"], 1e-6)
        x = x + enc_mha(h, L, sd, ln_lin)
        y = O.layer_norm(x, sd[L + "ln_2.weight"], sd[L + "ln_2.bias"], 1e-6)
        y = O.gelu_erf(ln_lin(y, sd[L + "mlp.0.weight"], sd[L + "mlp.0.bias"]))
        x = x + lin2(y, sd[L + "mlp.3.weight"], sd[L + "mlp.3.bias"])
    x = O.layer_norm(x, sd[P + "encoder.ln.weight"], sd[P + "encoder.ln.bias"], 1e-6)
    return lin2(x[:, 1:], sd["encoder.projection.weight"], sd["encoder.projection.bias"])


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    DROP = (sys.argv[2] != "0") if len(sys.argv) > 2 else True
    sd = W.to_torch(W.vit_state_dict(0))
    img = torch.from_numpy(W.synthetic_images(B, seed=1))
    with torch.no_grad():
        t = time.time()
        mem0 = O.vit_encode(sd, img)
        ids0, tr0 = O.greedy_from_memory(sd, mem0, 107, 108, 30, return_trace=True)
        print("fp32", time.time() - t, flush=True)
        marg = O.top2_margin(tr0)
        print("min margin", marg.min().item(), "frac<1e-3", (marg < 1e-3).float().mean().item())
        for mode in ("i8", "bf16x2"):
            mem = vit_encode(sd, img, mode)
            # decoder in fp32 here: isolates the encoder scheme's effect on the logits
            ids, tr = O.greedy_from_memory(sd, mem, 107, 108, 30, return_trace=True)
            L = min(ids.shape[1], ids0.shape[1])
            diff = ids[:, :L] != ids0[:, :L]
            dl = max((a - b).abs().max().item() for a, b in zip(tr[:L - 1], tr0[:L - 1]))
            rel = ((mem - mem0).norm() / mem0.norm()).item()
            print(f"{mode:7s} mem max err {(mem - mem0).abs().max().item():.2e} rel {rel:.2e} "
                  f"logit err (all steps) {dl:.2e} tokens diff {int(diff.sum())}/{diff.numel()}", flush=True)
