"""Timeline of the group-persistent decode step (tools build, ICAP_DEC_STEP=2 ICAP_XDEC_TRACE=1): per-workgroup
barrier stamps of one greedy decode at B = 256 -> per phase: body time (release of the previous barrier -> arrival),
barrier time (last arrival of the group -> release), averaged over workgroups, layers and steps.
usage: ICAP_DEC_STEP=2 ICAP_XDEC_TRACE=1 python tools/xdec_trace.py [vit|grid]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from image_caption_amd import weights as W  # noqa: E402
from image_caption_amd.engine import Engine  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "vit"
B, S, L, steps, NB = 256, 196 if kind == "vit" else 49, 6, 29, 12 * 8
dev = torch.device("cuda", 0)
sd = W.to_torch(W.vit_state_dict(0) if kind == "vit" else W.grid_state_dict(0))
eng = Engine(sd, kind, {}, device=dev)
eng.set_graphs(False)
mem = torch.randn(B, S, 512, generator=torch.Generator().manual_seed(0)).to(dev)
for _ in range(2):
    eng.greedy_raw(mem, 107, 108, 30)
torch.cuda.synchronize()
buf = np.zeros(steps * 256 * NB * 2, dtype=np.uint64)
fn = eng.lib.icap_dec_step_trace_read
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
assert fn(eng.handle, buf.ctypes.data, buf.nbytes) == 0, eng.lib.icap_last_error()
t = buf.reshape(steps, 256, NB, 2).astype(np.int64)  # [step][wg][barrier][arrive, release], 10 ns ticks
names = ["P1 qkv", "P2 attn", "P3 out", "P456 LN1,q,q~", "P7 xattn", "P8 v", "P9 cout", "P11 LN2,ffn", "P12 LN3"]
NP = len(names)
nbar = NP * L - 1
body = np.zeros((NP,)); bar = np.zeros((NP,)); bmax = np.zeros((NP,)); cnt = np.zeros((NP,))
for st in range(2, steps):
    for k in range(1, nbar):
        arr = t[st, :, k, 0]; rel = t[st, :, k, 1]; prev = t[st, :, k - 1, 1]
        ph = k % NP
        for g in range(8):
            wg = np.arange(g, 256, 8)
            last = arr[wg].max()
            body[ph] += (arr[wg] - prev[wg]).mean() * 10 / 1000
            bmax[ph] += (arr[wg] - prev[wg]).max() * 10 / 1000
            bar[ph] += (rel[wg] - last).mean() * 10 / 1000
            cnt[ph] += 1
print(f"{'phase':14s} {'body avg':>9s} {'body max':>9s} {'barrier':>8s}  (us, steps 2..28, all layers / groups)")
for ph in range(NP):
    print(f"{names[ph]:14s} {body[ph] / cnt[ph]:9.2f} {bmax[ph] / cnt[ph]:9.2f} {bar[ph] / cnt[ph]:8.2f}")
span = (t[2:, :, nbar - 1, 0].max(axis=1) - t[2:, :, 0, 1].min(axis=1)).mean() * 10 / 1000 * L / (L - 1 / NP)
print(f"step span (first release .. last arrival) {span:.1f} us, {span / L:.1f} us per layer")
