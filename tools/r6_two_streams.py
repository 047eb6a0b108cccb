"""Round 6: would the ViT encoder gain from running two half batches concurrently on two streams (the kernel tails and
launch gaps of one stream filled by the other's workgroups)?  Two engines (separate workspaces) encode B/2 images each
on their own stream, against one engine encoding B; GPU time by events, best of a few repetitions.  Measurement tool.
usage: python tools/r6_two_streams.py [B]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import weights as W
from image_caption_amd.engine import Engine

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda", 0)
sd = W.to_torch(W.vit_state_dict(0))
e1 = Engine(sd, "vit", {}, device=dev)
e2 = Engine(sd, "vit", {}, device=dev)
imgs = torch.from_numpy(W.synthetic_images(B, seed=1)).to(dev)
h = B // 2
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
ref = e1.encode(imgs)
for eng in (e1, e2):
    eng.encode(imgs[:h])
torch.cuda.synchronize()


def one():
    return e1.encode(imgs)


def two():
    cur = torch.cuda.current_stream()
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        m1 = e1.encode(imgs[:h])
    with torch.cuda.stream(s2):
        m2 = e2.encode(imgs[h:])
    cur.wait_stream(s1)
    cur.wait_stream(s2)
    return torch.cat([m1, m2])


for name, fn in (("one stream, B", one), ("two streams, B/2 each", two), ("one stream, B", one),
                 ("two streams, B/2 each", two)):
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    print(f"{name:24s} best {min(ts):.3f} ms  median {sorted(ts)[2]:.3f} ms  max|diff| vs one-stream memory "
          f"{(out - ref).abs().max().item():.2e}", flush=True)
