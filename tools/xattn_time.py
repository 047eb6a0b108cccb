"""Time the decoder cross-attention kernel alone (icap_op_cross_attn) with HIP events: rows x S at
1 row per image (greedy decode shape).  Measurement tool, not product.  usage: python tools/xattn_time.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib as L

lib = L.load(os.environ.get("XATTN_LIB") or None)  # XATTN_LIB=tools/libicap_tools.so: with the tools knobs
dev = torch.device("cuda", 0)
for rows, S in ((128, 196), (256, 196), (128, 64), (128, 32), (128, 1)):
    mem = torch.randn(rows, S, 512, device=dev).to(torch.float16)
    qt = torch.randn(2, rows, 8, 512, device=dev).to(torch.bfloat16)
    out = torch.empty(2, rows, 8, 512, device=dev, dtype=torch.bfloat16)
    run = lambda: L.check(lib.icap_op_cross_attn(qt.data_ptr(), rows * 4096, mem.data_ptr(), rows, 1, S,
                                                 out.data_ptr(), rows * 4096, L.stream_ptr()), "xattn")
    for _ in range(20):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    e0.record()
    for _ in range(n):
        run()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    print(f"rows {rows:4d} S {S:4d}: {us:7.2f} us/launch  {rows * S * 1024 / us / 1e3:7.1f} GB/s", flush=True)
