"""Epilogue sensitivity of the encoder GEMM: same main loop, different output modes."""
import sys, os
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
for (name, n, k) in [("qkv", 2304, 768), ("mlp3", 768, 3072)]:
    for ns in (1, 2):
        A = torch.randn(ns, M, k, device=dev).to(torch.bfloat16)
        W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
        C = torch.zeros(2, M, n, device=dev)
        for out, label in [(1, "bf16"), (0, "f32"), (2, "split"), (3, "f32+resid")]:
            for epi in ((0, 1) if out == 2 else (0,)):
                call = lambda: lib.icap_op_gemm(A.data_ptr(), k, M * k, ns, W.data_ptr(), None, C.data_ptr(), n,
                                                M * n, M, n, k, epi, out, _lib.stream_ptr())
                for _ in range(2):
                    call()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    call()
                e1.record()
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / 10 * 1e3
                print(f"{name} ns={ns} out={label:9s} epi={epi}: {us:7.1f} us  {2*M*n*k*ns/us/1e6:7.1f} MFMA-TF/s")
