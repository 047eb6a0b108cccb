"""Time icap_op_gemm on the encoder GEMM shapes (B=256 ViT) in isolation.
usage: python tools/gemm_bench.py [iters]"""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_caption_amd import _lib

lib = _lib.load()
dev = torch.device("cuda", 0)


def warm(seconds=2.0):
    """Run the GPU at full load first: the first timed shape otherwise pays the clock ramp."""
    import time
    a = torch.randn(8192, 8192, device=dev).to(torch.bfloat16)
    t0 = time.time()
    while time.time() - t0 < seconds:
        for _ in range(20):
            a @ a
        torch.cuda.synchronize()


warm()
M = 256 * 197
shapes = [("qkv", M, 2304, 768, 0, 2), ("out", M, 768, 768, 0, 3), ("mlp0", M, 3072, 768, 1, 2), ("mlp3", M, 768, 3072, 0, 3)]
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
for ns in (2, 1):
    for name, m, n, k, epi, out in shapes:
        A = torch.randn(ns, m, k, device=dev).to(torch.bfloat16)
        W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
        b = torch.randn(n, device=dev)
        C = torch.zeros(2, m, n, device=dev, dtype=torch.float32 if out != 2 else torch.bfloat16)
        call = lambda: lib.icap_op_gemm(A.data_ptr(), k, m * k, ns, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, m * n,
                                        m, n, k, epi, out, _lib.stream_ptr())
        for _ in range(2):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(iters):
            call()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        tf = 2 * m * n * k / ms / 1e9
        print(f"nsplit={ns} {name:5s} M={m} N={n} K={k}: {ms*1e3:8.1f} us  {tf:7.1f} TFLOP/s alg  {tf*ns:7.1f} MFMA-TF/s", flush=True)

# vendor reference point (hipBLASLt via torch.matmul, bf16 in/out, no fused epilogue)
for name, m, n, k, epi, out in shapes:
    a = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(k, n, device=dev) / k ** 0.5).to(torch.bfloat16)
    for _ in range(3):
        c = a @ w
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        c = a @ w
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(f"torch.matmul bf16 {name:5s}: {ms*1e3:8.1f} us  {2*m*n*k/ms/1e9:7.1f} TFLOP/s", flush=True)
