"""Encoder GEMM throughput vs M (A working set): is the 256x256 kernel bound by A's HBM stream
or by its own pipeline?  QKV / MLP-out shapes, bf16x2, no bias, split-plane output."""
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
for (name, n, k) in [("qkv", 2304, 768), ("mlp3", 768, 3072)]:
    for M in (4096, 8192, 16384, 50432):
        for ns in (2,):
            A = torch.randn(ns, M, k, device=dev).to(torch.bfloat16)
            W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
            C = torch.zeros(2, M, n, device=dev, dtype=torch.bfloat16)
            call = lambda: lib.icap_op_gemm(A.data_ptr(), k, M * k, ns, W.data_ptr(), None, C.data_ptr(), n, M * n,
                                            M, n, k, 0, 2, _lib.stream_ptr())
            for _ in range(3):
                call()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            it = max(10, int(2e5 // M))
            e0.record()
            for _ in range(it):
                call()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / it * 1e3
            blocks = (M + 255) // 256 * (n // 256)
            print(f"{name} M={M:6d} ns={ns} blocks={blocks:5d}: {us:8.1f} us  {2*M*n*k*ns/us/1e6:7.1f} MFMA-TF/s  "
                  f"A={ns*M*k*2/1e6:6.1f} MB", flush=True)
