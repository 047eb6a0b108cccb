"""Round 6: the ViT encode's GPU time (events around engine.encode, best / median of 7) with the engine's launch timing
off and on (layers 0 and 6), for the library given (argv[1]).  Measurement tool.
usage: python tools/r6_enc_time.py LIB.so"""
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
imgs = torch.from_numpy(W.synthetic_images(256, seed=1)).to(dev)
eng.encode(imgs)
torch.cuda.synchronize()
for every in (0, 6, 0, 6):
    eng.profile(every > 0, every=max(every, 1))
    ts = []
    for _ in range(7):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        eng.encode(imgs)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    eng.profile(False)
    print(f"{os.path.basename(sys.argv[1]):22s} profile {every}: best {min(ts):.3f} median {sorted(ts)[3]:.3f} ms",
          flush=True)
# sustained: 20 encodes back to back (no host sync between them), and 10 encode + greedy decode steps as bench.py runs
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
a.record()
for _ in range(20):
    eng.encode(imgs)
b.record()
torch.cuda.synchronize()
print(f"{os.path.basename(sys.argv[1]):22s} 20 back-to-back encodes: {a.elapsed_time(b) / 20:.3f} ms each", flush=True)
mem = eng.encode(imgs)
eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, 30)
eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, 30)
ev = []
torch.cuda.synchronize()
for _ in range(10):
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    m = eng.encode(imgs)
    e1.record()
    ids, _ = eng.greedy_raw(m, W.START_TOKEN, W.END_TOKEN, 30)
    e2.record()
    ev.append((e0, e1, e2))
    ids.cpu()
torch.cuda.synchronize()
enc = sum(x.elapsed_time(y) for x, y, _ in ev) / 10
dec = sum(y.elapsed_time(z) for _, y, z in ev) / 10
print(f"{os.path.basename(sys.argv[1]):22s} bench-like steps: encode {enc:.3f} ms, decode {dec:.3f} ms", flush=True)
import time
hs = []
for _ in range(5):  # host time of one encode call (enqueue only) after a sync
    torch.cuda.synchronize()
    t = time.perf_counter()
    eng.encode(imgs)
    hs.append((time.perf_counter() - t) * 1e3)
torch.cuda.synchronize()
print(f"{os.path.basename(sys.argv[1]):22s} host enqueue of one encode: {sorted(hs)[2]:.3f} ms (median of 5)", flush=True)
