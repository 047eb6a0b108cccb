"""Round 6: where the fp32-checkpoint logit error of config 2 comes from, and how the f16 encoder
fares on a weight draw with ViT-style residual outliers.  At B = 256, max_len 30, for each weight set:
  memory error (HIP f16 encoder vs the fp32 oracle encoder);
  logits: teacher-forced on the HIP greedy ids, max |.| over every row and step, of
    full   HIP encoder -> HIP decoder           vs oracle encoder -> oracle decoder
    dec    oracle memory -> HIP decoder          vs oracle (the decoder's own share)
    enc    HIP memory -> oracle decoder          vs oracle (the encoder's share)
for precision f16 (the default) and bf16x2.  Weight sets: seed 3 fp32 (not bf16-exact, config 2's fp32-weights test),
and the same with outliers: in ViT layers 2-11 the MLP-2 rows (and biases) of 4 residual channels scaled by OUTLIER
(default 20; trained ViT-B/16 carries residual channels two orders above the rest).  Measurement tool.
usage: python tools/r6_precision.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import weights as W
from image_caption_amd.engine import Engine
from oracle import captioner as O

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
L = 30
OUT = float(os.environ.get("OUTLIER", 20))
CH = [7, 200, 411, 650]


def outliers(sd):
    sd = {k: v.clone() for k, v in sd.items()}
    for i in range(2, 12):
        p = f"encoder.vit.encoder.layers.encoder_layer_{i}.mlp.3"
        sd[p + ".weight"][CH] *= OUT
        sd[p + ".bias"][CH] *= OUT
    return sd


def oracle_mem(sdd, imgs):
    with torch.no_grad():
        return torch.cat([O.vit_encode(sdd, imgs[i:i + 64]) for i in range(0, imgs.shape[0], 64)])


def tf(sdd, mem, ids):
    with torch.no_grad():
        return torch.cat([O.teacher_forced_logits(sdd, mem[i:i + 64], ids[i:i + 64]) for i in range(0, ids.shape[0], 64)])


base = W.to_torch(W.vit_state_dict(3, bf16_exact=False))
imgs = torch.from_numpy(W.synthetic_images(B, seed=7)).to(dev)
for name, sd in (("seed3 fp32", base), (f"seed3 fp32 + outliers x{OUT:g}", outliers(base))):
    sdd = {k: v.to(dev) for k, v in sd.items()}
    mem_o = oracle_mem(sdd, imgs)
    print(f"== {name}: oracle memory max |m| {mem_o.abs().max().item():.2f}", flush=True)
    for prec in ("f16", "bf16x2"):
        eng = Engine(sd, "vit", {}, precision=prec, device=dev)
        mem = eng.encode(imgs)
        over = eng.range_overflowed() if prec == "f16" else False
        ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
        ids = ids.long()
        ref = tf(sdd, mem_o, ids)
        full = (lg.permute(1, 0, 2) - ref).abs().max().item()
        dec = (eng.decoder_forward(ids[:, :-1], mem_o, causal=True) - ref).abs().max().item()
        enc = (tf(sdd, mem, ids) - ref).abs().max().item()
        merr = (mem - mem_o).abs().max().item()
        print(f"  {prec:7s} memory err {merr:.2e}  logits: full {full:.2e}  decoder share {dec:.2e}  encoder share "
              f"{enc:.2e}  fp16 range flag {over}", flush=True)
        del eng
        torch.cuda.empty_cache()
