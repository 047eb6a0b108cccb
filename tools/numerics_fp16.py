"""CPU emulation of fp16 single-plane operands for the encoder GEMMs fed by the attention output and the
GELU output (out-projection, MLP-2), against the current i8x2 + bf16x2 scheme and fp32.  Weights of those
GEMMs in fp16 too.  Decoder fp32 (isolates the encoder).  Measurement tool, not product.
usage: python tools/numerics_fp16.py B"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

import numerics_i8 as N
from image_caption_amd import weights as W
from oracle import captioner as O

h16 = lambda x: x.to(torch.float16).float()


def lin_h(x, w, b):
    return h16(x) @ h16(w).t() + b


def vit_encode(sd, images, mode):
    P = "encoder.vit."
    B = images.shape[0]
    w = sd[P + "conv_proj.weight"]
    patches = images.reshape(B, 3, 14, 16, 14, 16).permute(0, 2, 4, 1, 3, 5).reshape(B, 196, 768)
    x = N.lin2(patches, w.reshape(768, -1), sd[P + "conv_proj.bias"])
    x = torch.cat([sd[P + "class_token"].expand(B, -1, -1), x], dim=1) + sd[P + "encoder.pos_embedding"]
    ln_lin = N.i8_linear if mode in ("i8", "i8+f16") else lin_h
    res_lin = lin_h if mode in ("i8+f16", "f16", "f16a") else N.lin2
    for i in range(12):
        L = P + f"encoder.layers.encoder_layer_{i}."
        h = O.layer_norm(x, sd[L + "ln_1.weight"], sd[L + "ln_1.bias"], 1e-6)
        B_, T, D = h.shape
        qkv = ln_lin(h, sd[L + "self_attention.in_proj_weight"], sd[L + "self_attention.in_proj_bias"])
        q, k, v = qkv.split(D, -1)
        q = q.view(B_, T, 12, 64).transpose(1, 2)
        k = k.view(B_, T, 12, 64).transpose(1, 2)
        v = v.view(B_, T, 12, 64).transpose(1, 2)
        if mode == "f16a":  # fp16 attention operands too (q, k, v and the probabilities)
            s = (h16(q) @ h16(k).transpose(-1, -2)) / 8.0
            pm = torch.softmax(s, -1)
            o = (h16(pm) @ h16(v)).transpose(1, 2).reshape(B_, T, D)
        else:
            s = N.split3(q, k.transpose(-1, -2)) / 8.0
            pm = torch.softmax(s, -1)
            o = N.split3(pm, v).transpose(1, 2).reshape(B_, T, D)
        x = x + res_lin(o, sd[L + "self_attention.out_proj.weight"], sd[L + "self_attention.out_proj.bias"])
        y = O.layer_norm(x, sd[L + "ln_2.weight"], sd[L + "ln_2.bias"], 1e-6)
        y = O.gelu_erf(ln_lin(y, sd[L + "mlp.0.weight"], sd[L + "mlp.0.bias"]))
        x = x + res_lin(y, sd[L + "mlp.3.weight"], sd[L + "mlp.3.bias"])
    x = O.layer_norm(x, sd[P + "encoder.ln.weight"], sd[P + "encoder.ln.bias"], 1e-6)
    return ln_lin(x[:, 1:], sd["encoder.projection.weight"], sd["encoder.projection.bias"])


if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    torch.set_num_threads(8)
    sd = W.to_torch(W.vit_state_dict(0))
    img = torch.from_numpy(W.synthetic_images(B, seed=1))
    with torch.no_grad():
        mem0 = O.vit_encode(sd, img)
        ids0, tr0 = O.greedy_from_memory(sd, mem0, 107, 108, 30, return_trace=True)
        marg = O.top2_margin(tr0)
        print("min margin", marg.min().item(), flush=True)
        for mode in sys.argv[2].split(",") if len(sys.argv) > 2 else ("i8", "i8+f16", "f16", "f16a"):
            t = time.time()
            mem = vit_encode(sd, img, mode)
            ids, tr = O.greedy_from_memory(sd, mem, 107, 108, 30, return_trace=True)
            L = min(ids.shape[1], ids0.shape[1])
            diff = ids[:, :L] != ids0[:, :L]
            dl = max((a - b).abs().max().item() for a, b in zip(tr[:L - 1], tr0[:L - 1]))
            print(f"{mode:7s} mem max err {(mem - mem0).abs().max().item():.2e} (|mem| max {mem0.abs().max().item():.2f}) logit err {dl:.2e} "
                  f"tokens diff {int(diff.sum())}/{diff.numel()}  ({time.time() - t:.0f}s)", flush=True)
