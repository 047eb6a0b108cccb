"""Time the four ViT encoder GEMM shapes (B=256: M = 50432) through icap_op_gemm, next to the
vendor library (torch.matmul -> hipBLASLt, bf16, no epilogue) on the same bf16x2 work written as
one GEMM with K doubled ([A_hi | A_lo] @ [W; W]).  Measurement tool, not part of the product.
usage: python tools/gemm_shapes.py [ITERS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib

lib = _lib.load()
dev = torch.device("cuda", 0)
SHAPES = {"qkv": (2304, 768, 0, 2), "out": (768, 768, 0, 3), "mlp0": (3072, 768, 1, 2), "mlp3": (768, 3072, 0, 3)}
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
m = int(os.environ.get("GEMM_M", 256 * 197))
ns = 2


def timed(fn):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


tot_ours = tot_lib = 0.0
for name, (n, k, epi, out) in SHAPES.items():
    A = torch.randn(ns, m, k, device=dev).to(torch.bfloat16)
    W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    b = torch.randn(n, device=dev)
    C = torch.zeros(2, m, n, device=dev)

    def ours():
        lib.icap_op_gemm(A.data_ptr(), k, m * k, ns, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, m * n, m, n, k, epi,
                         out, _lib.stream_ptr())

    A2 = torch.cat([A[0], A[1]], 1)
    W2 = torch.cat([W, W], 1).t()
    C2 = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

    def vendor():
        torch.matmul(A2, W2, out=C2)

    t0, t1 = timed(ours), timed(vendor)
    t2 = None
    if name in ("qkv", "mlp0"):
        af = torch.randn(m, k, device=dev)
        wf = torch.randn(n, k, device=dev) / k ** 0.5
        qa = torch.empty(m, 2 * k, device=dev, dtype=torch.int8)
        qw = torch.empty(n, 2 * k, device=dev, dtype=torch.int8)
        sa, sw = torch.empty(m, device=dev), torch.empty(n, device=dev)
        lib.icap_op_pack_i8(af.data_ptr(), m, k, qa.data_ptr(), sa.data_ptr(), _lib.stream_ptr())
        lib.icap_op_pack_i8(wf.data_ptr(), n, k, qw.data_ptr(), sw.data_ptr(), _lib.stream_ptr())
        def i8():  # production form: split planes (QKV head-major)
            lib.icap_op_gemm_i8(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), b.data_ptr(),
                                C.data_ptr(), m, n, k, epi, 2, 197 if name == "qkv" else 0, _lib.stream_ptr())

        t2 = timed(i8)
    fl = 2.0 * m * n * k
    tot_ours += t0
    tot_lib += t1
    print(f"{name:5s} M={m} N={n} K={k}: icap {t0:8.1f} us  {fl / t0 / 1e6:7.1f} alg-TF/s  {2 * fl / t0 / 1e6:7.1f} "
          f"MFMA-TF/s | hipBLASLt K=2x{k} {t1:8.1f} us {2 * fl / t1 / 1e6:7.1f} TF/s"
          + (f" | i8x2 {t2:8.1f} us {fl / t2 / 1e6:7.1f} alg-TF/s" if t2 else ""), flush=True)
print(f"per layer: icap {tot_ours:.1f} us, hipBLASLt {tot_lib:.1f} us")
