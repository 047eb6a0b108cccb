"""Round 6: where the pipelined step loses time against max(encode, decode) - per batch of one 10-batch run
(bench shape: B = 256, stop rule in the post step), each phase's span and the idle time of each stream before its
next phase (encoder stream: end of encode i to start of encode i + 1; decode stream: end of decode i to start of
decode i + 1).  Measurement tool.  usage: python tools/r6_pipe_gaps.py [N_BATCHES]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import weights as W
from image_caption_amd.engine import Engine, apply_stop_rule
from image_caption_amd.pipeline import CaptionPipeline

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
eng = Engine(W.to_torch(W.vit_state_dict(0)), "vit", {}, device=dev)
imgs = torch.from_numpy(W.synthetic_images(256, seed=1)).to(dev)
pipe = CaptionPipeline(eng, W.START_TOKEN, W.END_TOKEN, 30)
post = lambda ids: apply_stop_rule(ids.long(), W.END_TOKEN)
pipe.run([imgs] * 3, post)
torch.cuda.synchronize()
ev = []
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
pipe.run([imgs] * n, post, timing=ev)
b.record()
torch.cuda.synchronize()
total = a.elapsed_time(b)
print(f"{n} batches: {total:.2f} ms, {total / n:.3f} ms per batch")
t0 = ev[0][0]
for i, (e0, e1, d0, d1) in enumerate(ev):
    line = (f"batch {i}: encode {t0.elapsed_time(e0):8.2f} -> {t0.elapsed_time(e1):8.2f} ({e0.elapsed_time(e1):6.2f}) "
            f"decode {t0.elapsed_time(d0):8.2f} -> {t0.elapsed_time(d1):8.2f} ({d0.elapsed_time(d1):6.2f})")
    if i + 1 < n:
        f0, _, g0, _ = ev[i + 1]
        line += f"  idle: encoder {e1.elapsed_time(f0):6.3f}  decode {d1.elapsed_time(g0):6.3f}"
    print(line, flush=True)
