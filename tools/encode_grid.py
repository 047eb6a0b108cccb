"""Run an encoder ITERS times at batch B, for kernel profiles (default the Grid encoder: HIP ResNet
trunk + tail).  usage: python tools/encode_grid.py [ITERS] [B] [vit|grid]   (ICAP_LIB: a variant library)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

if os.environ.get("ICAP_LIB"):  # a variant library (tools/build_variant.py)
    from image_caption_amd import _lib  # noqa: E402

    _lib.load(os.environ["ICAP_LIB"])

from image_caption_amd import weights as W  # noqa: E402
from image_caption_amd.engine import Engine  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
kind = sys.argv[3] if len(sys.argv) > 3 else "grid"
dev = torch.device("cuda", 0)
sd = W.vit_state_dict(0) if kind == "vit" else W.grid_state_dict(0)
eng = Engine(W.to_torch(sd), kind, {}, device=dev)
imgs = torch.from_numpy(W.synthetic_images(B, seed=1)).to(dev)
for _ in range(iters):
    mem = eng.encode(imgs)
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record()
for _ in range(iters):
    mem = eng.encode(imgs)
ev[1].record()
torch.cuda.synchronize()
print(f"encode B={B}: {ev[0].elapsed_time(ev[1]) / iters:.3f} ms  checksum {mem.double().sum().item():.6e}")
