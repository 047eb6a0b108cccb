"""Round 6: the ViT encode's GPU time in three step contexts (events around engine.encode, mean of 10): L1 encode +
decode + host sync (the bench's step), L2 encode + decode without a host sync (the host runs ahead), L3 host sync +
encode alone.  Measurement tool.  usage: python tools/r6_enc_ctx2.py LIB.so"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib

_lib.load(sys.argv[1])
from image_caption_amd import weights as W
from image_caption_amd.engine import Engine

dev = torch.device("cuda", 0)
eng = Engine(W.to_torch(W.vit_state_dict(0)), "vit", {}, device=dev)
if os.environ.get("R6_EAGER"):  # eager decode launches (rocprofv3 --pmc crashed on the decode graph's replays)
    eng.set_graphs(False)
imgs = torch.from_numpy(W.synthetic_images(256, seed=1)).to(dev)
m = eng.encode(imgs)
eng.greedy_raw(m, W.START_TOKEN, W.END_TOKEN, 30)
eng.greedy_raw(m, W.START_TOKEN, W.END_TOKEN, 30)
torch.cuda.synchronize()
name = os.path.basename(sys.argv[1])
for ctx in ("L1", "L2", "L3", "L1", "L2", "L3"):
    ev = []
    for _ in range(10):
        if ctx != "L2":
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        mm = eng.encode(imgs)
        e1.record()
        if ctx != "L3":
            eng.greedy_raw(mm, W.START_TOKEN, W.END_TOKEN, 30)
        ev.append((e0, e1))
    torch.cuda.synchronize()
    print(f"{name:22s} {ctx}: encode {sum(a.elapsed_time(b) for a, b in ev) / 10:.3f} ms", flush=True)
