"""Run one encoder GEMM shape N times (for rocprofv3 counter passes)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_caption_amd import _lib
lib = _lib.load()
dev = torch.device("cuda", 0)
m, n, k, ns, epi, out, iters = 256 * 197, 768, 3072, 2, 0, 3, int(sys.argv[1]) if len(sys.argv) > 1 else 5
A = torch.randn(ns, m, k, device=dev).to(torch.bfloat16)
W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
b = torch.randn(n, device=dev)
C = torch.zeros(m, n, device=dev)
for _ in range(iters):
    lib.icap_op_gemm(A.data_ptr(), k, m * k, ns, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, 0, m, n, k, epi, out,
                     _lib.stream_ptr())
torch.cuda.synchronize()
print("done")
