"""Round-6 study of the vendor GEMM on the four ViT encoder shapes (M = 50432 = 256 images x 197 tokens, fp16 in,
fp16 out, W row-major [N][K] as the product stores it): runs torch.matmul(A, W^T) a few times per shape so that a
`rocprofv3 --kernel-trace --stats` over this script names the hipBLASLt kernels chosen and their durations, and a
`--pmc FETCH_SIZE` pass gives their fetched bytes.  Measurement tool, not part of the product.
usage: python tools/r6_blaslt_trace.py [ITERS]"""
import sys

import torch

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
try:
    torch.backends.cuda.preferred_blas_library("hipblaslt")
except Exception as e:  # older torch: the default is already hipBLASLt on gfx950
    print("preferred_blas_library:", e)
m = 256 * 197
for name, (n, k) in {"qkv": (2304, 768), "out": (768, 768), "mlp0": (3072, 768), "mlp3": (768, 3072)}.items():
    A = torch.rand(m, k, device=dev).sub(0.5).to(torch.float16)
    W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.float16)
    C = torch.empty(m, n, device=dev, dtype=torch.float16)
    for _ in range(2):
        torch.matmul(A, W.t(), out=C)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        torch.matmul(A, W.t(), out=C)
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) * 1e3 / iters
    print(f"{name:5s} M={m} N={n} K={k}: {t:8.1f} us {2.0 * m * n * k / t / 1e6:7.1f} TF/s", flush=True)
