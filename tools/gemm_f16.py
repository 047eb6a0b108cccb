"""Time the four ViT encoder GEMM shapes (B=256: M = 50432) in the ICAP_PREC_F16 form (one fp16 plane,
production outputs: QKV / MLP-1 an fp16 plane, out-proj / MLP-2 the fp32 residual +=) through icap_op_gemm,
next to the vendor library (torch.matmul -> hipBLASLt, fp16 in / fp16 out, no epilogue) on the same
shapes.  Measurement tool, not part of the product (the tools build reads ICAP_F16_GEMM).
usage: python tools/gemm_f16.py [ITERS]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib

TOOLS_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libicap_tools.so")  # tools build (ICAP_* knobs read)
lib = _lib.load(os.environ.get("GEMM_LIB") or (TOOLS_LIB if os.path.exists(TOOLS_LIB) else None))  # GEMM_LIB: A/B of two builds
dev = torch.device("cuda", 0)
SHAPES = {"qkv": (2304, 768, 0, 2), "out": (768, 768, 0, 3), "mlp0": (3072, 768, 1, 2), "mlp3": (768, 3072, 0, 3)}
if os.environ.get("SHAPE_NK"):  # SHAPE_NK=2304,768: one plain GEMM of M = GEMM_M rows (fp16 out, bias, no epilogue op)
    _n, _k = map(int, os.environ["SHAPE_NK"].split(","))
    SHAPES = {f"n{_n}k{_k}": (_n, _k, 0, 2)}
if os.environ.get("SQUARE"):  # SQUARE=4096: one plain M = N = K GEMM (fp16 out, no epilogue), e.g. against the guide's template
    _n = int(os.environ["SQUARE"])
    SHAPES = {f"sq{_n}": (_n, _n, 0, 2)}
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
m = int(os.environ.get("GEMM_M", 256 * 197))


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
    A = torch.rand(m, k, device=dev).sub(0.5).to(torch.float16)
    W = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.float16)
    b = torch.randn(n, device=dev)
    C = torch.zeros(m, n, device=dev)

    def ours():
        _lib.check(lib.icap_op_gemm(A.data_ptr(), k, 0, -1, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, 0, m, n, k, epi,
                                    out, _lib.stream_ptr()), "gemm f16")

    Wt = W.t()
    C2 = torch.empty(m, n, device=dev, dtype=torch.float16)

    def vendor():
        torch.matmul(A, Wt, out=C2)

    t0, t1 = timed(ours), timed(vendor)
    fl = 2.0 * m * n * k
    tot_ours += t0
    tot_lib += t1
    print(f"{name:5s} M={m} N={n} K={k}: icap f16 {t0:8.1f} us {fl / t0 / 1e6:7.1f} TF/s | hipBLASLt f16 {t1:8.1f} us "
          f"{fl / t1 / 1e6:7.1f} TF/s", flush=True)
print(f"per layer: icap {tot_ours:.1f} us, hipBLASLt {tot_lib:.1f} us")
