"""Localise GEMM errors: small shapes through icap_op_gemm, error map per 16x16 output tile."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from image_caption_amd import _lib

lib = _lib.load()
dev = torch.device("cuda", 0)
for (M, N, K, ns) in [(16384, 1024, 64, 1), (16384, 1024, 128, 1), (16384, 1024, 192, 1), (16384, 1024, 512, 1),
                      (16484, 1024, 512, 1), (16384, 1024, 64, 2)]:
    g = torch.Generator().manual_seed(1)
    a = torch.randn(ns, M, K, generator=g).to(torch.bfloat16).to(dev)
    w = torch.randn(N, K, generator=g).to(torch.bfloat16).to(dev)
    ref = sum(a[p].double() @ w.double().t() for p in range(ns))
    C = torch.zeros(M, N, device=dev)
    _lib.check(lib.icap_op_gemm(a.data_ptr(), K, M * K, ns, w.data_ptr(), None, C.data_ptr(), N, 0, M, N, K, 0, 0,
                                _lib.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    err = (C.double() - ref).abs()
    Mb = M // 256 * 256
    e = err[:Mb].reshape(Mb // 256, 16, 16, N // 256, 16, 16)
    pos = (e.amax(dim=(2, 5)) > 1e-2)            # [bm, tr, bn, tc]
    blocks = pos.any(dim=(1, 3))
    inblk = pos.any(dim=0).any(dim=1)             # [tr, tc]
    print(f"M={M} N={N} K={K} ns={ns}: max err {err.max().item():.3g}, bad blocks {int(blocks.sum())}/{blocks.numel()}, "
          f"tail rows err {err[Mb:].max().item() if M > Mb else 0:.3g}")
    if inblk.any():
        for r in range(16):
            print("   ", "".join("X" if inblk[r, c] else "." for c in range(16)))
        bb = blocks.nonzero()[:12].tolist()
        print("    first bad blocks (bm, bn):", bb)
