"""CPU emulation (round 3): the Grid encoder tail (1x1 projection + 6 post-LN encoder layers) on fp16 planes - GEMM
inputs, weights, Q / K / V, attention probabilities and context, ReLU output rounded to fp16; fp32 accumulation, residual
stream and LayerNorm - on the built fp16 trunk (conv1 hi-plane form), against the fp32 oracle.  B = 4 synthetic images."""
import importlib.util
import sys

import torch

sys.path.insert(0, '/root/repo')
from image_caption_amd import weights as W
from oracle import captioner as O

spec = importlib.util.spec_from_file_location("t16", "/root/repo/tools/numerics_trunk16_c1.py")
torch.set_num_threads(8)
sd = W.to_torch(W.grid_state_dict(0))
imgs = torch.from_numpy(W.synthetic_images(4, seed=3))
F = torch.nn.functional


def q(x):
    return x.to(torch.float16).float()


def trunk_f16():
    t = importlib.util.module_from_spec(spec)
    old = sys.stdout
    sys.stdout = open('/dev/null', 'w')
    try:
        spec.loader.exec_module(t)  # (prints its own table)
    finally:
        sys.stdout = old
    return t.trunk(True)


def layer16(x, p, nhead=8):
    B, T, D = x.shape
    hd = D // nhead
    qkv = q(q(x) @ q(sd[p + "self_attn.in_proj_weight"]).t() + sd[p + "self_attn.in_proj_bias"])
    qq, k, v = qkv.chunk(3, dim=-1)
    sp = lambda t: t.reshape(B, T, nhead, hd).transpose(1, 2)
    s = sp(qq) @ sp(k).transpose(-1, -2) / hd ** 0.5
    pr = q(torch.softmax(s, -1))
    ctx = q((pr @ sp(v)).transpose(1, 2).reshape(B, T, D))
    h = ctx @ q(sd[p + "self_attn.out_proj.weight"]).t() + sd[p + "self_attn.out_proj.bias"]
    x = O.layer_norm(x + h, sd[p + "norm1.weight"], sd[p + "norm1.bias"], 1e-5)
    f = q(torch.relu(q(x) @ q(sd[p + "linear1.weight"]).t() + sd[p + "linear1.bias"]))
    f = f @ q(sd[p + "linear2.weight"]).t() + sd[p + "linear2.bias"]
    return O.layer_norm(x + f, sd[p + "norm2.weight"], sd[p + "norm2.bias"], 1e-5)


def tail(feats, half):
    if not half:
        return O.grid_encode_tail(sd, feats)
    w = sd["encoder.projection.weight"]
    x = feats.flatten(2).transpose(1, 2)
    x = O.linear(x, w.reshape(w.shape[0], -1), sd["encoder.projection.bias"])  # (bf16 hi/lo planes: ~fp32)
    x = x + sd["encoder.pos_encoder.pe"][:, : x.shape[1]]
    i = 0
    while f"encoder.transformer_encoder.layers.{i}.norm1.weight" in sd:
        x = layer16(x, f"encoder.transformer_encoder.layers.{i}.")
        i += 1
    return x


with torch.no_grad():
    ref = O.resnet101_trunk(sd, imgs)
    mem_o = O.grid_encode_tail(sd, ref)
    ids = O.greedy_from_memory(sd, mem_o, W.START_TOKEN, W.END_TOKEN, 30)
    a = O.teacher_forced_logits(sd, mem_o, ids.long())
    x = trunk_f16()
    for name, half in (("bf16x2 tail", False), ("fp16 tail", True)):
        mem = tail(x, half)
        b = O.teacher_forced_logits(sd, mem, ids.long())
        gid = O.greedy_from_memory(sd, mem, W.START_TOKEN, W.END_TOKEN, 30)
        print(f"fp16 trunk + {name}: memory {(mem - mem_o).abs().max().item():.3e}  logits {(a - b).abs().max().item():.3e}"
              f"  ids equal {bool((gid == ids).all())}")
