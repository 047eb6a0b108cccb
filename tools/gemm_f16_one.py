"""Run one ViT fp16 GEMM shape ITERS times through icap_op_gemm and through torch.matmul (hipBLASLt), for
rocprofv3 counter passes.  usage: python tools/gemm_f16_one.py ITERS [qkv|out|mlp0|mlp3]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib

lib = _lib.load()
dev = torch.device("cuda", 0)
SHAPES = {"qkv": (2304, 768, 0, 2), "out": (768, 768, 0, 3), "mlp0": (3072, 768, 1, 2), "mlp3": (768, 3072, 0, 3)}
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n, k, epi, out = SHAPES[sys.argv[2] if len(sys.argv) > 2 else "qkv"]
m = int(os.environ.get("GEMM_M", 256 * 197))
A = torch.rand(m, k, device=dev).sub(0.5).to(torch.float16)
W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.float16)
b = torch.randn(n, device=dev)
C = torch.zeros(m, n, device=dev)
C2 = torch.empty(m, n, device=dev, dtype=torch.float16)
for _ in range(iters):
    _lib.check(lib.icap_op_gemm(A.data_ptr(), k, 0, -1, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, 0, m, n, k, epi, out,
                                _lib.stream_ptr()), "gemm f16")
    torch.matmul(A, W.t(), out=C2)
torch.cuda.synchronize()
print("done")
