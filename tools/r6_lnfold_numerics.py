"""Round 6: CPU emulation of folding the encoder's pre-LayerNorms (ln_1 -> QKV, ln_2 -> MLP-1) into the GEMMs they feed,
against the product's f16 encoder (tools/numerics_fp16.py mode f16a).  Product: a = fp16(LN(x)), y = a W^T + b.
Fold: y = rstd (fp16(x) fp16(W')^T) - rstd mu s + c with W' = W diag(gamma), s = row sums of fp16(W'),
c = W beta + b, mu / rstd of the fp32 row - the LN's normalisation applied after the product, so no LN pass runs
and the GEMM reads the residual stream's fp16 copy.  Prints memory and logit errors against the fp32 oracle.
usage: python tools/r6_lnfold_numerics.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import numerics_fp16 as F
from image_caption_amd import weights as W
from oracle import captioner as O

h16 = F.h16


def folded(x, gamma, beta, w, b, eps=1e-6):
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    rstd = torch.rsqrt(var + eps)
    wp = h16(w * gamma)
    s = wp.sum(-1)
    c = w @ beta + b
    return rstd * (h16(x) @ wp.t()) - rstd * mu * s + c


def vit_encode(sd, images, fold):
    P = "encoder.vit."
    B = images.shape[0]
    w = sd[P + "conv_proj.weight"]
    patches = images.reshape(B, 3, 14, 16, 14, 16).permute(0, 2, 4, 1, 3, 5).reshape(B, 196, 768)
    x = F.lin_h(patches, w.reshape(768, -1), sd[P + "conv_proj.bias"])
    x = torch.cat([sd[P + "class_token"].expand(B, -1, -1), x], dim=1) + sd[P + "encoder.pos_embedding"]
    for i in range(12):
        L = P + f"encoder.layers.encoder_layer_{i}."
        g1, b1 = sd[L + "ln_1.weight"], sd[L + "ln_1.bias"]
        wq, bq = sd[L + "self_attention.in_proj_weight"], sd[L + "self_attention.in_proj_bias"]
        if fold:
            qkv = folded(x, g1, b1, wq, bq)
        else:
            qkv = F.lin_h(O.layer_norm(x, g1, b1, 1e-6), wq, bq)
        B_, T, D = x.shape
        q, k, v = (t.view(B_, T, 12, 64).transpose(1, 2) for t in qkv.split(D, -1))
        s = (h16(q) @ h16(k).transpose(-1, -2)) / 8.0
        o = (h16(torch.softmax(s, -1)) @ h16(v)).transpose(1, 2).reshape(B_, T, D)
        x = x + F.lin_h(o, sd[L + "self_attention.out_proj.weight"], sd[L + "self_attention.out_proj.bias"])
        g2, b2 = sd[L + "ln_2.weight"], sd[L + "ln_2.bias"]
        w0, bb0 = sd[L + "mlp.0.weight"], sd[L + "mlp.0.bias"]
        y = folded(x, g2, b2, w0, bb0) if fold else F.lin_h(O.layer_norm(x, g2, b2, 1e-6), w0, bb0)
        x = x + F.lin_h(O.gelu_erf(y), sd[L + "mlp.3.weight"], sd[L + "mlp.3.bias"])
    x = O.layer_norm(x, sd[P + "encoder.ln.weight"], sd[P + "encoder.ln.bias"], 1e-6)
    return F.lin_h(x[:, 1:], sd["encoder.projection.weight"], sd["encoder.projection.bias"])


def outliers(sd):
    sd = {k: v.clone() for k, v in sd.items()}
    for i in range(2, 12):
        p = f"encoder.vit.encoder.layers.encoder_layer_{i}.mlp.3"
        sd[p + ".weight"][[7, 200, 411, 650]] *= 20.0
        sd[p + ".bias"][[7, 200, 411, 650]] *= 20.0
    return sd


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    torch.set_num_threads(8)
    img = torch.from_numpy(W.synthetic_images(B, seed=1))
    for name, sd in (("seed0 bf16-exact", W.to_torch(W.vit_state_dict(0))),
                     ("seed3 fp32", W.to_torch(W.vit_state_dict(3, bf16_exact=False))),
                     ("seed3 fp32 + outliers x20", outliers(W.to_torch(W.vit_state_dict(3, bf16_exact=False))))):
        with torch.no_grad():
            mem0 = O.vit_encode(sd, img)
            _, tr0 = O.greedy_from_memory(sd, mem0, 107, 108, 30, return_trace=True)
            ids0 = O.greedy_from_memory(sd, mem0, 107, 108, 30)
            for fold in (False, True):
                mem = vit_encode(sd, img, fold)
                tf = O.teacher_forced_logits(sd, mem, ids0)
                dl = (tf - tr0.permute(1, 0, 2)).abs().max().item()
                print(f"{name:28s} {'fold' if fold else 'f16a'}: memory err {(mem - mem0).abs().max().item():.2e} "
                      f"logit err {dl:.2e}", flush=True)
