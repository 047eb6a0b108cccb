"""Round 6: host launch latency at the head of a bench step - the ViT encode's GPU time (events around the call) when
the host enters it right after a synchronize (as every bench step does after the previous step's stop rule) against
back-to-back calls (the host already ahead), with the engine's live profiling on and off; the same for the decode.
Measurement tool.  usage: python tools/r6_gap.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import weights as W
from image_caption_amd.engine import Engine

dev = torch.device("cuda", 0)
eng = Engine(W.to_torch(W.vit_state_dict(0)), "vit", {}, device=dev)
imgs = torch.from_numpy(W.synthetic_images(256, seed=1)).to(dev)
mem = eng.encode(imgs)
eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, 30)
eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, 30)
torch.cuda.synchronize()


def timed(fn, sync_each, n=10):
    evs = []
    for _ in range(n):
        if sync_each:
            torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        evs.append((a, b))
    torch.cuda.synchronize()
    return sum(a.elapsed_time(b) for a, b in evs) / n


for prof in (0, 1, 6):  # off, every launch, layers 0 and 6 (bench.py)
    eng.profile(prof > 0, every=max(prof, 1))
    for name, fn in (("encode", lambda: eng.encode(imgs)),
                     ("decode", lambda: eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, 30))):
        t_sync = timed(fn, True)
        t_b2b = timed(fn, False)
        print(f"profile {prof} {name}: after sync {t_sync:.3f} ms, back-to-back {t_b2b:.3f} ms, "
              f"exposed host latency {1e3 * (t_sync - t_b2b):.0f} us", flush=True)
    eng.profile(False)
