"""Per-block time of the 256x256 encoder GEMM vs the number of concurrently running blocks (one
round, N=2048, K=768, bf16x2): does a block slow down as more CUs stream at once?"""
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
n, k, ns = 2048, int(os.environ.get("GK", 768)), 2
for M in (256, 512, 1024, 2048, 4096, 8192):
    A = torch.randn(ns, M, k, device=dev).to(torch.bfloat16)
    W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    C = torch.zeros(2, M, n, device=dev)
    call = lambda: lib.icap_op_gemm(A.data_ptr(), k, M * k, ns, W.data_ptr(), None, C.data_ptr(), n, M * n,
                                    M, n, k, 0, 0, _lib.stream_ptr())
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
    blocks = M // 256 * (n // 256)
    print(f"blocks={blocks:4d} M={M:5d}: {us:7.1f} us per launch, {2*M*n*k*ns/us/1e6:7.1f} MFMA-TF/s", flush=True)
