"""Run one encoder GEMM shape N times (for rocprofv3 counter passes).
usage: python tools/gemm_one.py ITERS [qkv|out|mlp0|mlp3] [NSPLIT]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_caption_amd import _lib
lib = _lib.load()
dev = torch.device("cuda", 0)
SHAPES = {"qkv": (2304, 768, 0, 2), "out": (768, 768, 0, 3), "mlp0": (3072, 768, 1, 2), "mlp3": (768, 3072, 0, 3)}
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 5
name = sys.argv[2] if len(sys.argv) > 2 else "mlp3"
ns = int(sys.argv[3]) if len(sys.argv) > 3 else 2
n, k, epi, out = SHAPES[name]
m = int(os.environ.get("GEMM_M", 256 * 197))
A = torch.randn(ns, m, k, device=dev).to(torch.bfloat16)
W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
b = torch.randn(n, device=dev)
C = torch.zeros(2, m, n, device=dev)
for _ in range(iters):
    lib.icap_op_gemm(A.data_ptr(), k, m * k, ns, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, m * n, m, n, k, epi, out,
                     _lib.stream_ptr())
torch.cuda.synchronize()
print("done", name, ns)
