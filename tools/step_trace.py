"""Timeline of the persistent decode step (tools build, ICAP_DEC_STEP_TRACE=1): per-task stamps of one greedy decode
at B = 256 -> per-phase summary (task counts, wait / body durations, when each phase's tasks start and end within a
step).  usage: ICAP_DEC_STEP_TRACE=1 python tools/step_trace.py [B]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from image_caption_amd import weights as W  # noqa: E402
from image_caption_amd.engine import Engine  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda", 0)
eng = Engine(W.to_torch(W.vit_state_dict(0)), "vit", {}, device=dev)
eng.set_graphs(False)
eng.set_decode_step(True)
mem = torch.randn(B, 196, 512, generator=torch.Generator().manual_seed(0)).to(dev)
for _ in range(2):
    eng.greedy_raw(mem, 107, 108, 30)
torch.cuda.synchronize()
L, NT, steps = 6, (B + 15) // 16, 29
ntasks = L * 59 * NT
buf = np.zeros(steps * ntasks * 4, dtype=np.uint64)
fn = eng.lib.icap_dec_step_trace_read
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
assert fn(eng.handle, buf.ctypes.data, buf.nbytes) == 0, eng.lib.icap_last_error()
tr = buf.reshape(steps, ntasks, 4).astype(np.int64)
names = ["SA", "LN1", "C1", "XA", "C2", "LN2", "FF", "LN3"]
cnt = [8, 1, 8, 16, 8, 1, 16, 1]
off = np.cumsum([0] + cnt) * NT
for s in (5, 20):
    t = tr[s]
    valid = t[:, 2] > 0
    t0 = t[valid, 0].min()
    print(f"--- step {s}: span {(t[valid, 2].max() - t0) / 100:.1f} us, tasks {valid.sum()}")
    for l in (0, 1, 5):
        for p, nm in enumerate(names):
            a, b = l * 59 * NT + off[p], l * 59 * NT + off[p + 1]
            x = t[a:b]
            x = x[x[:, 2] > 0]
            if len(x) == 0:
                continue
            wait = (x[:, 1] - x[:, 0]) / 100
            body = (x[:, 2] - x[:, 1]) / 100
            print(f"L{l} {nm:4s} n={len(x):4d} deq {(x[:, 0].min() - t0) / 100:7.1f}..{(x[:, 0].max() - t0) / 100:7.1f}"
                  f"  ready {(x[:, 1].min() - t0) / 100:7.1f}..{(x[:, 1].max() - t0) / 100:7.1f}"
                  f"  done {(x[:, 2].min() - t0) / 100:7.1f}..{(x[:, 2].max() - t0) / 100:7.1f}"
                  f"  wait {wait.mean():6.1f} body {body.mean():6.1f} (max {body.max():6.1f}) us")
