"""Repeat-launch check of the f16 head-major encoder attention with the tools build (knobs from the environment):
how many outputs differ between two launches on the same input, and where.  usage: python tools/attn_repeat.py B N H"""
import sys

import torch

from image_caption_amd import _lib as L

lib = L.load("tools/libicap_tools.so")
B, N, H = (int(v) for v in sys.argv[1:4])
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(B * N + H + 7)
qkv = (torch.randn(B, 3, H, N, 64, generator=g) * 1.5).to(torch.float16).to(dev)
outs = []
for _ in range(4):
    o = torch.zeros(B * N, H * 64, device=dev, dtype=torch.float16)
    L.check(lib.icap_op_enc_attention_hm(qkv.data_ptr(), B, N, H, o.data_ptr(), L.stream_ptr()), "attn")
    torch.cuda.synchronize()
    outs.append(o.cpu())
for i in range(1, 4):
    d = (outs[i] != outs[0]).nonzero()
    print(f"launch {i}: {d.shape[0]} differing of {outs[0].numel()}", end="")
    if d.shape[0]:
        rows, cols = d[:, 0], d[:, 1]
        print(f"; tokens {sorted(set((rows % N).tolist()))[:12]} heads {sorted(set((cols // 64).tolist()))[:12]} "
              f"dims {sorted(set((cols % 64).tolist()))[:16]} images {sorted(set((rows // N).tolist()))[:8]}", end="")
    print()
