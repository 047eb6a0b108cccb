"""Round 6: check and time the ViT encoder's fp16 GEMM forms of a library (icap_op_gemm, fp16 A / W, fp16 plane out
with bias (+ GELU) or the fp32 residual C += A W^T + b) against torch fp32 on the same fp16 operands, at the ViT
shapes (M = 50432) and edge shapes (ragged M, fewer tiles than CUs, K = 128), then time them next to hipBLASLt
(torch.matmul, fp16 out, no epilogue).  Measurement tool, not part of the product.
usage: python tools/r6_gemm_check.py [LIB.so]   (default: the tree's library; one library per process)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib

dev = torch.device("cuda", 0)
VIT = {"qkv": (50432, 2304, 768, 0, 2), "out": (50432, 768, 768, 0, 3), "mlp0": (50432, 3072, 768, 1, 2),
       "mlp3": (50432, 768, 3072, 0, 3)}
EDGE = {"rag_so": (1000, 512, 256, 0, 2), "rag_gelu": (777, 1024, 384, 1, 2), "rag_res": (1111, 768, 640, 0, 3),
        "k128": (5000, 768, 128, 0, 2), "k128res": (3000, 512, 128, 0, 3), "few": (300, 256, 768, 0, 3)}


def timed(fn, iters=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def run(lib, name, m, n, k, epi, out, do_time):
    g = torch.Generator(device=dev).manual_seed(hash(name) & 0xffff)
    A = (torch.rand(m, k, device=dev, generator=g) - 0.5).to(torch.float16)
    W = (torch.randn(n, k, device=dev, generator=g) / k ** 0.5).to(torch.float16)
    b = torch.randn(n, device=dev, generator=g) * 0.1
    if out == 3:
        C0 = torch.randn(m, n, device=dev, generator=g)
        C = C0.clone()
    else:
        C = torch.full((m, n), float("nan"), device=dev, dtype=torch.float16)

    def ours():
        _lib.check(lib.icap_op_gemm(A.data_ptr(), k, 0, -1, W.data_ptr(), b.data_ptr(), C.data_ptr(), n, 0, m, n, k, epi,
                                    out, _lib.stream_ptr()), name)

    ours()
    torch.cuda.synchronize()
    ref = A.float() @ W.float().t() + b
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    if out == 3:
        ref = ref + C0
    err = (C.float() - ref).abs().max().item() / max(ref.abs().max().item(), 1e-6)
    ok = err < (2e-3 if out == 2 else 1e-5) and torch.isfinite(C.float()).all().item()
    line = f"{name:8s} M={m} N={n} K={k}: rel err {err:.2e} {'ok' if ok else 'FAIL'}"
    if do_time:
        t0 = timed(ours)
        Wt, C2 = W.t(), torch.empty(m, n, device=dev, dtype=torch.float16)
        t1 = timed(lambda: torch.matmul(A, Wt, out=C2))
        fl = 2.0 * m * n * k
        line += f" | icap {t0:7.1f} us {fl / t0 / 1e6:6.1f} TF/s | hipBLASLt {t1:7.1f} us {fl / t1 / 1e6:6.1f} TF/s"
    print(line, flush=True)
    return ok, (t0 if do_time else 0.0)


def main():
    bad = 0
    for path in sys.argv[1:2] or [None]:
        lib = _lib.load(path)
        print("==", path or "tree library", flush=True)
        only = os.environ.get("R6_SHAPES")  # e.g. R6_SHAPES=mlp3,out: those ViT shapes only, no edge checks (profiling)
        for name, sh in ({} if only else EDGE).items():
            bad += not run(lib, name, *sh, False)[0]
        tot = 0.0
        for name, sh in VIT.items():
            if only and name not in only.split(","):
                continue
            ok, t = run(lib, name, *sh, True)
            bad += not ok
            tot += t
        print(f"per ViT layer: {tot:.1f} us", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
