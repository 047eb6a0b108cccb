"""Per-block fixed cost vs per-stage cost of the 256x256 encoder GEMM: fixed grid (M=4096, N=768,
48 blocks on 48 CUs), K swept; time = fixed + stages * per_stage.  bf16x2, split-plane output."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_caption_amd import _lib

lib = _lib.load()
dev = torch.device("cuda", 0)
a = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
for _ in range(100):
    a @ a
torch.cuda.synchronize()
M, n, ns = 4096, 768, 2
for out in (2, 0):
    res = []
    for k in (256, 768, 1536, 3072):
        A = torch.randn(ns, M, k, device=dev).to(torch.bfloat16)
        W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
        C = torch.zeros(2, M, n, device=dev)
        call = lambda: lib.icap_op_gemm(A.data_ptr(), k, M * k, ns, W.data_ptr(), None, C.data_ptr(), n, M * n,
                                        M, n, k, 0, out, _lib.stream_ptr())
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            call()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 50 * 1e3
        res.append((k // 32, us))
        print(f"out={out} K={k:5d} stages={k // 32:3d}: {us:8.1f} us", flush=True)
    (s0, t0), (s1, t1) = res[0], res[-1]
    per = (t1 - t0) / (s1 - s0)
    print(f"out={out}: per-stage {per:.3f} us, fixed {t0 - s0 * per:.1f} us", flush=True)
