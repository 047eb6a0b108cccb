"""Kernel-level parity of the HIP ops against fp64 torch references of the same op.

Inputs are hi/lo bf16 planes (the engine's activation format), so the exact value the kernel
sees is hi+lo; tolerances are written per test."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _lib():
    from image_caption_amd import _lib

    return _lib, _lib.load()


def planes(x: torch.Tensor, nsplit: int) -> torch.Tensor:
    hi = x.to(torch.bfloat16)
    if nsplit == 1:
        return hi.contiguous()
    lo = (x - hi.float()).to(torch.bfloat16)
    return torch.stack([hi, lo]).contiguous()


def value(p: torch.Tensor, nsplit: int) -> torch.Tensor:
    return p.double() if nsplit == 1 else p[0].double() + p[1].double()


@pytest.mark.parametrize("M,N,K", [(300, 256, 512), (64, 64, 64), (8192, 1024, 768), (50, 512, 2048), (16484, 1024, 512)])
@pytest.mark.parametrize("nsplit", [1, 2])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm(cuda, M, N, K, nsplit, epi):
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(M * 7 + N + K + epi)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    A = planes(a, nsplit)
    ref = value(A, nsplit) @ w.double().t() + bias.double()
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    elif epi == 2:
        ref = torch.relu(ref)
    # fp32 output
    C = torch.empty(M, N, device=cuda)
    L.check(lib.icap_op_gemm(A.data_ptr(), K, M * K, nsplit, w.data_ptr(), bias.data_ptr(), C.data_ptr(), N, 0,
                             M, N, K, epi, 0, L.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    err = (C.double() - ref).abs().max().item()
    assert err < 2e-4 * max(1.0, ref.abs().max().item()), err
    # split-plane output, residual accumulate
    Cs = torch.empty(2, M, N, device=cuda, dtype=torch.bfloat16)
    L.check(lib.icap_op_gemm(A.data_ptr(), K, M * K, nsplit, w.data_ptr(), bias.data_ptr(), Cs.data_ptr(), N, M * N,
                             M, N, K, epi, 2, L.stream_ptr()), "gemm split")
    R = torch.randn(M, N, generator=g).to(cuda)
    R0 = R.clone()
    L.check(lib.icap_op_gemm(A.data_ptr(), K, M * K, nsplit, w.data_ptr(), bias.data_ptr(), R.data_ptr(), N, 0,
                             M, N, K, epi, 3, L.stream_ptr()), "gemm resid")
    torch.cuda.synchronize()
    assert (value(Cs, 2) - C.double()).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item())
    assert (R.double() - R0.double() - C.double()).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item())


def test_gemm_identity_asymmetric(cuda):
    """A = I, asymmetric W: catches a transposed C write (cdna_hip_programming.md §3)."""
    L, lib = _lib()
    n = 128
    A = torch.eye(n, device=cuda).to(torch.bfloat16).contiguous()
    w = (torch.arange(n * n, device=cuda, dtype=torch.float32).reshape(n, n) % 251).to(torch.bfloat16)
    C = torch.empty(n, n, device=cuda)
    L.check(lib.icap_op_gemm(A.data_ptr(), n, 0, 1, w.data_ptr(), None, C.data_ptr(), n, 0, n, n, n, 0, 0,
                             L.stream_ptr()), "gemm")
    torch.cuda.synchronize()
    assert torch.equal(C, w.float().t())


@pytest.mark.parametrize("D", [512, 768])
@pytest.mark.parametrize("nsplit", [1, 2])
def test_layernorm(cuda, D, nsplit):
    L, lib = _lib()
    rows = 333
    x = (torch.randn(rows, D, device=cuda) * 3 + 1).contiguous()
    w = torch.randn(D, device=cuda)
    b = torch.randn(D, device=cuda)
    ref = torch.nn.functional.layer_norm(x.double(), (D,), w.double(), b.double(), 1e-6)
    y = torch.empty_like(x)
    yb = torch.empty(nsplit, rows, D, device=cuda, dtype=torch.bfloat16)
    L.check(lib.icap_op_layernorm(x.data_ptr(), rows, D, w.data_ptr(), b.data_ptr(), 1e-6, y.data_ptr(),
                                  yb.data_ptr(), rows * D, nsplit, L.stream_ptr()), "ln")
    torch.cuda.synchronize()
    assert (y.double() - ref).abs().max().item() < 1e-5
    # bf16 hi plane: |err| <= 2^-9 |y|; hi+lo: ~2^-17 |y|
    rel = 2.0 ** -8 if nsplit == 1 else 2.0 ** -15
    got = value(yb if nsplit == 2 else yb[0], nsplit)
    assert ((got - ref).abs() <= rel * ref.abs() + 1e-6).all()


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (3, 49, 8), (1, 7, 2)])
@pytest.mark.parametrize("nsplit", [1, 2])
def test_enc_attention(cuda, B, N, H, nsplit):
    L, lib = _lib()
    D = H * 64
    g = torch.Generator(device="cpu").manual_seed(B * N + H)
    qkv = (torch.randn(B * N, 3 * D, generator=g) * 1.5).to(cuda)
    P = planes(qkv, nsplit)
    v = value(P, nsplit).view(B, N, 3, H, 64)
    q, k, vv = v[:, :, 0].transpose(1, 2), v[:, :, 1].transpose(1, 2), v[:, :, 2].transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ vv
    ref = ref.transpose(1, 2).reshape(B * N, D)
    out = torch.zeros(nsplit, B * N, D, device=cuda, dtype=torch.bfloat16)
    L.check(lib.icap_op_enc_attention(P.data_ptr(), B * N * 3 * D, B, N, H, out.data_ptr(), B * N * D, nsplit,
                                      L.stream_ptr()), "attn")
    torch.cuda.synchronize()
    got = value(out if nsplit == 2 else out[0], nsplit)
    tol = 3e-2 if nsplit == 1 else 2e-4
    assert (got - ref).abs().max().item() < tol


@pytest.mark.parametrize("rows,rpi,S", [(256, 1, 196), (40, 5, 196), (24, 3, 49), (6, 2, 1), (8, 1, 70),
                                        (37, 1, 49), (5, 1, 1), (16, 1, 17), (9, 1, 256), (3, 1, 33), (85, 1, 196)])
def test_cross_attn_f16(cuda, rows, rpi, S):
    """Key-absorbed decoder cross-attention over one fp16 memory plane (decode loops, beam slots and
    teacher-forced rows of an image share a block): against fp64 softmax(q~ mem^T / 8) mem on the same
    rounded operands, ragged last chunks (S = 196, 70, 49, 1) and odd rows per image.  The product build runs the
    32-key chunk loop (cross_attn_f16_kernel<1, 32>) for every case: S = 1 and 17 are one partial chunk, S = 256
    eight full ones, odd row counts leave the last block with one row.  (The key-split forms are tools-only:
    tools/r4_tools_pytest.sh runs this test with ICAP_XATTN16_S=1 on the tools build.)"""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(rows * 7 + S)
    B = rows // rpi
    mem = (torch.randn(B, S, 512, generator=g)).to(torch.float16)
    qt = torch.randn(rows, 8, 512, generator=g) * 0.3
    Q = planes(qt.to(cuda), 2)
    qv = value(Q, 2).double().cpu()
    m = mem.double()[torch.arange(rows) // rpi]                       # (rows, S, 512)
    p = torch.softmax(torch.einsum("rhd,rsd->rhs", qv, m) / 8.0, -1)
    ref = torch.einsum("rhs,rsd->rhd", p, m)
    out = torch.zeros(2, rows, 8, 512, device=cuda, dtype=torch.bfloat16)
    L.check(lib.icap_op_cross_attn(Q.data_ptr(), rows * 8 * 512, mem.to(cuda).data_ptr(), rows, rpi, S,
                                   out.data_ptr(), rows * 8 * 512, L.stream_ptr()), "cross_attn")
    torch.cuda.synchronize()
    got = value(out, 2).double().cpu()
    assert (got - ref).abs().max().item() < 2e-4
    if rpi == 1:  # repeated launches are bitwise equal (the tools build's key-split merge too)
        for _ in range(3):
            again = torch.zeros_like(out)
            L.check(lib.icap_op_cross_attn(Q.data_ptr(), rows * 8 * 512, mem.to(cuda).data_ptr(), rows, rpi, S,
                                           again.data_ptr(), rows * 8 * 512, L.stream_ptr()), "cross_attn")
            torch.cuda.synchronize()
            assert torch.equal(again, out)


@pytest.mark.parametrize("p", [0.0, 0.1, 0.5])
def test_residual_layernorm_dropout(cuda, p):
    """The decode loops' residual LayerNorm with the train-mode dropout of the sub-layer output
    (x + drop(sum of slabs + bias)): against torch with the oracle's masks (oracle/dropout.py)."""
    from oracle import dropout as D

    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(int(p * 10) + 1)
    rows, nparts, site, layer, pos, seed = 40, 8, 4, 1, 3, 4242
    x = torch.randn(rows, 512, generator=g)
    parts = torch.randn(nparts, rows, 512, generator=g) * 0.3
    bias, w, b = (torch.randn(512, generator=g) for _ in range(3))
    m = D._mask(p, seed, site, layer, np.arange(rows)[:, None], pos, np.arange(512)[None, :]) if p else 1.0
    ref = torch.nn.functional.layer_norm(x + (parts.sum(0) + bias) * m, (512,), w, b, 1e-5)
    xd, pd, bd, wd, bbd = (t.to(cuda) for t in (x, parts, bias, w, b))  # (kept alive across the call)
    out = torch.empty(2, rows, 512, device=cuda, dtype=torch.bfloat16)
    sd = torch.tensor([seed], dtype=torch.int32, device=cuda)
    L.check(lib.icap_op_residual_layernorm(xd.data_ptr(), rows, pd.data_ptr(), nparts, rows * 512, bd.data_ptr(),
                                           wd.data_ptr(), bbd.data_ptr(), out.data_ptr(), rows * 512, p,
                                           sd.data_ptr(), layer, pos, site, L.stream_ptr()), "rln")
    torch.cuda.synchronize()
    assert (xd.cpu() - ref).abs().max().item() < 1e-4


def test_full_chip_kernels_repeat_bitwise(cuda):
    """Races between a wave's LDS reads and another wave's LDS-DMA refill of the same ring slot show
    up as run-to-run differences: the 128x256 two-blocks-per-CU GEMM (full chip, M = 50432, K = 768
    and 3072) and the pipelined encoder attention (B = 256, N = 197) are run repeatedly in one
    process and must reproduce bit for bit, and match the fp64 reference."""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(11)
    for M, N, K in ((50432, 768, 768), (50432, 768, 3072)):
        a = torch.randn(M, K, generator=g).to(cuda)
        w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.bfloat16).to(cuda)
        bias = torch.randn(N, generator=g).to(cuda)
        A = planes(a, 2)
        outs = []
        for _ in range(8):
            C = torch.empty(M, N, device=cuda)
            L.check(lib.icap_op_gemm(A.data_ptr(), K, M * K, 2, w.data_ptr(), bias.data_ptr(), C.data_ptr(), N, 0,
                                     M, N, K, 0, 0, L.stream_ptr()), "gemm")
            outs.append(C)
        torch.cuda.synchronize()
        assert all(torch.equal(o, outs[0]) for o in outs[1:])
        rows = torch.arange(0, M, 997, device=cuda)
        ref = (A[0].double() + A[1].double())[rows] @ w.double().t()
        ref = ref + bias.double()
        assert (outs[0][rows].double() - ref).abs().max().item() < 2e-4 * max(1.0, ref.abs().max().item())
    B, Nt, H = 256, 197, 12
    D = H * 64
    qkv = (torch.randn(B * Nt, 3 * D, generator=g) * 1.5).to(cuda)
    P = planes(qkv, 2)
    outs = []
    for _ in range(6):
        out = torch.zeros(2, B * Nt, D, device=cuda, dtype=torch.bfloat16)
        L.check(lib.icap_op_enc_attention(P.data_ptr(), B * Nt * 3 * D, B, Nt, H, out.data_ptr(), B * Nt * D, 2,
                                          L.stream_ptr()), "attn")
        outs.append(out)
    torch.cuda.synchronize()
    assert all(torch.equal(o, outs[0]) for o in outs[1:])


# ------------------------------------------------------------------ int8 two-slice operands (i8x2)
def _slices(q: torch.Tensor):
    """row images [rows][K/64][2][64] -> (x1, x2) as [rows][K]"""
    rows = q.shape[0]
    v = q.view(rows, -1, 2, 64)
    return v[:, :, 0].reshape(rows, -1), v[:, :, 1].reshape(rows, -1)


def _dequant(q: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    x1, x2 = _slices(q)
    return (256.0 * x1.double() + x2.double()) * s.double()[:, None]


def _pack_i8(L, lib, x: torch.Tensor):
    rows, K = x.shape
    q = torch.empty(rows, 2 * K, device=x.device, dtype=torch.int8)
    s = torch.empty(rows, device=x.device)
    L.check(lib.icap_op_pack_i8(x.data_ptr(), rows, K, q.data_ptr(), s.data_ptr(), L.stream_ptr()), "pack")
    return q, s


@pytest.mark.parametrize("rows,K", [(1000, 768), (7, 3072), (64, 512)])
def test_pack_i8_roundtrip(cuda, rows, K):
    """16-bit fixed point per row: |x - s (256 x1 + x2)| <= s / 2 (+ the fp32 rounding of x / s near
    2^15, < 2^-7 s), x1 in [-127, 127]; zero rows stay zero."""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(rows + K)
    x = (torch.randn(rows, K, generator=g) * torch.logspace(-3, 2, rows)[:, None]).to(cuda)
    x[3] = 0.0
    q, s = _pack_i8(L, lib, x)
    torch.cuda.synchronize()
    assert _slices(q)[0].abs().max().item() <= 127
    err = (_dequant(q, s) - x.double()).abs()
    assert (err <= s.double()[:, None] * (0.5 + 2 ** -7) + 1e-30).all(), err.max().item()
    assert s[3].item() == 0.0 and (q[3] == 0).all()
    amax = x.abs().amax(1).double()
    assert torch.allclose(s.double() * 32639, amax, rtol=1e-6)


def test_layernorm_i8(cuda):
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(5)
    rows, D = 777, 768
    x = (torch.randn(rows, D, generator=g) * 3 + 1).to(cuda)
    w = torch.randn(D, generator=g).to(cuda)
    b = torch.randn(D, generator=g).to(cuda)
    q = torch.empty(rows, 2 * D, device=cuda, dtype=torch.int8)
    s = torch.empty(rows, device=cuda)
    L.check(lib.icap_op_layernorm_i8(x.data_ptr(), rows, D, w.data_ptr(), b.data_ptr(), 1e-6, q.data_ptr(),
                                     s.data_ptr(), L.stream_ptr()), "ln i8")
    torch.cuda.synchronize()
    ref = torch.nn.functional.layer_norm(x.double(), (D,), w.double(), b.double(), 1e-6)
    err = (_dequant(q, s) - ref).abs()
    assert (err <= s.double()[:, None] * (0.5 + 2 ** -7) + 1e-5 * ref.abs().amax(1, keepdim=True)).all(), err.max().item()


@pytest.mark.parametrize("M,N,K", [(1000, 768, 768), (50432, 2304, 768), (129, 512, 1024), (1970, 2304, 768)])
@pytest.mark.parametrize("epi", [0, 1])
def test_gemm_i8(cuda, M, N, K, epi):
    """The int8 two-slice GEMM equals its defining formula exactly up to fp32 rounding
    (65536 A1.W1 + 256 (A1.W2 + A2.W1), scales, bias), and the fp64 product of the original fp32
    operands within the representation's 16-bit bound."""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = torch.randn(M, K, generator=g).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    qa, sa = _pack_i8(L, lib, a)
    qw, sw = _pack_i8(L, lib, w)
    C = torch.empty(M, N, device=cuda)
    L.check(lib.icap_op_gemm_i8(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                C.data_ptr(), M, N, K, epi, 0, 0, L.stream_ptr()), "gemm i8")
    # split-plane output (LDS-staged epilogue), row-major and head-major
    Cs = torch.empty(2, M, N, device=cuda, dtype=torch.bfloat16)
    L.check(lib.icap_op_gemm_i8(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                Cs.data_ptr(), M, N, K, epi, 2, 0, L.stream_ptr()), "gemm i8 split")
    hm = 197 if M % 197 == 0 else (M if M <= 256 else 0)
    Ch = torch.empty(2, M, N, device=cuda, dtype=torch.bfloat16)
    if hm:
        L.check(lib.icap_op_gemm_i8(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                    Ch.data_ptr(), M, N, K, epi, 2, hm, L.stream_ptr()), "gemm i8 head-major")
    torch.cuda.synchronize()
    tol = 1e-5 * max(1.0, C.abs().max().item())
    assert (value(Cs, 2) - C.double()).abs().max().item() < tol
    if hm:  # [image][N/64][token][64] -> [image*token][N]
        Chm = Ch.view(2, M // hm, N // 64, hm, 64).permute(0, 1, 3, 2, 4).reshape(2, M, N)
        assert torch.equal(Chm, Cs)
    rows = slice(0, M) if M <= 4096 else torch.randperm(M, generator=g)[:2048].to(cuda)
    a1, a2 = (t[rows].double() for t in _slices(qa))
    w1, w2 = (t.double() for t in _slices(qw))
    acc = 65536.0 * (a1 @ w1.t()) + 256.0 * (a1 @ w2.t() + a2 @ w1.t())
    form = acc * sa.double()[rows][:, None] * sw.double()[None, :] + bias.double()
    exact = a[rows].double() @ w.double().t() + bias.double()
    if epi == 1:
        form = torch.nn.functional.gelu(form)
        exact = torch.nn.functional.gelu(exact)
    Cr = C[rows].double()
    scale = max(1.0, exact.abs().max().item())
    assert (Cr - form).abs().max().item() < 2e-6 * scale
    assert (Cr - exact).abs().max().item() < 2e-4 * scale


def test_gemm_i8_split_repeat_bitwise(cuda):
    """The int8 GEMM's split-plane path (LDS-staged epilogue through the ring, in row halves for the
    128 x 128 tiles) at full chip: repeated launches reproduce bit for bit (an early ring-slot refill
    shows up as run-to-run differences), and equal the fp32-output path to the bf16x2 plane rounding."""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(12)
    for M, N, K, epi, hm in ((50432, 3072, 768, 1, 0), (50432, 2304, 768, 0, 197), (1001, 512, 256, 1, 0), (1001, 512, 128, 1, 0)):
        a = torch.randn(M, K, generator=g).to(cuda)
        w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda)
        bias = torch.randn(N, generator=g).to(cuda)
        qa, sa = _pack_i8(L, lib, a)
        qw, sw = _pack_i8(L, lib, w)
        outs = []
        for _ in range(6):
            Cs = torch.empty(2, M, N, device=cuda, dtype=torch.bfloat16)
            L.check(lib.icap_op_gemm_i8(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                        Cs.data_ptr(), M, N, K, epi, 2, hm, L.stream_ptr()), "gemm i8 split")
            outs.append(Cs)
        C = torch.empty(M, N, device=cuda)
        L.check(lib.icap_op_gemm_i8(qa.data_ptr(), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), bias.data_ptr(),
                                    C.data_ptr(), M, N, K, epi, 0, 0, L.stream_ptr()), "gemm i8")
        torch.cuda.synchronize()
        assert all(torch.equal(o, outs[0]) for o in outs[1:])
        got = outs[0]
        if hm:
            got = got.view(2, M // hm, N // 64, hm, 64).permute(0, 1, 3, 2, 4).reshape(2, M, N)
        assert (value(got, 2) - C.double()).abs().max().item() < 1e-5 * max(1.0, C.abs().max().item())


def _blocks_dequant(q: torch.Tensor, ks: torch.Tensor) -> torch.Tensor:
    """[M][N/64][2][64] int8 row images with one scale per (row, 128-column block) -> fp64 [M][N]."""
    M = q.shape[0]
    v = q.view(M, -1, 2, 64).double()
    return ((256.0 * v[:, :, 0] + v[:, :, 1]) * ks.double().repeat_interleave(2, 1)[:, :, None]).reshape(M, -1)


@pytest.mark.parametrize("M,K1,N1,N2", [(1000, 768, 3072, 768), (129, 256, 512, 128), (50432, 768, 3072, 768)])
def test_gemm_i8_block_scaled_pair(cuda, M, K1, N1, N2):
    """The i8x2 ViT MLP pair: MLP-1 (+ GELU) written as block-scaled int8 row images (OUT_I8K, one scale
    per row and 128 columns), read by MLP-2 as A with a_kscale, residual-added into fp32.  Checks: the
    block output is the fp32-output GEMM quantised to 16 bits of its block maximum; MLP-2 equals its
    defining formula (per 64-deep step 65536 A1.W1 + 256 (A1.W2 + A2.W1), block and column scales, bias) to fp32
    rounding and the fp64 product of the dequantised operands; full-chip launches repeat bit for bit."""
    L, lib = _lib()
    if not lib.icap_tools_build():
        pytest.skip("measured-and-rejected variant: compiled only into the tools build (-DICAP_TOOLS)")
    g = torch.Generator(device="cpu").manual_seed(M + K1 + N1)
    a = torch.randn(M, K1, generator=g).to(cuda)
    w1 = (torch.randn(N1, K1, generator=g) / K1 ** 0.5).to(cuda)
    b1 = torch.randn(N1, generator=g).to(cuda)
    w2 = (torch.randn(N2, N1, generator=g) / N1 ** 0.5).to(cuda)
    b2 = torch.randn(N2, generator=g).to(cuda)
    res = torch.randn(M, N2, generator=g).to(cuda)
    qa, sa = _pack_i8(L, lib, a)
    qw1, sw1 = _pack_i8(L, lib, w1)
    qw2, sw2 = _pack_i8(L, lib, w2)
    nkb = N1 // 128
    C1 = torch.empty(M, N1, device=cuda)
    L.check(lib.icap_op_gemm_i8_blocks(qa.data_ptr(), sa.data_ptr(), None, qw1.data_ptr(), sw1.data_ptr(),
                                       b1.data_ptr(), C1.data_ptr(), None, M, N1, K1, 1, 0, L.stream_ptr()), "mlp1 f32")
    outs = []
    for _ in range(3 if M > 10000 else 1):
        h = torch.empty(M, 2 * N1, device=cuda, dtype=torch.int8)
        hs = torch.empty(M, nkb, device=cuda)
        L.check(lib.icap_op_gemm_i8_blocks(qa.data_ptr(), sa.data_ptr(), None, qw1.data_ptr(), sw1.data_ptr(),
                                           b1.data_ptr(), h.data_ptr(), hs.data_ptr(), M, N1, K1, 1, 5,
                                           L.stream_ptr()), "mlp1 i8k")
        C2 = res.clone()
        L.check(lib.icap_op_gemm_i8_blocks(h.data_ptr(), None, hs.data_ptr(), qw2.data_ptr(), sw2.data_ptr(),
                                           b2.data_ptr(), C2.data_ptr(), None, M, N2, N1, 0, 3, L.stream_ptr()),
                "mlp2 blocks")
        outs.append((h, hs, C2))
    torch.cuda.synchronize()
    h, hs, C2 = outs[0]
    for o in outs[1:]:
        assert torch.equal(o[0], h) and torch.equal(o[1], hs) and torch.equal(o[2], C2)
    rows = slice(0, M) if M <= 4096 else torch.randperm(M, generator=g)[:2048].to(cuda)
    # block output = quantised fp32 output
    c1 = C1[rows].double()
    blk = c1.view(c1.shape[0], nkb, 128)
    assert torch.allclose(hs[rows].double() * 32639, blk.abs().amax(2), rtol=1e-6, atol=0)
    deq = _blocks_dequant(h[rows], hs[rows])
    bound = (hs[rows].double() * (0.5 + 2 ** -7)).repeat_interleave(128, 1) + 1e-30
    assert ((deq - c1).abs() <= bound).all(), (deq - c1).abs().max().item()
    # MLP-2 against its defining formula and the fp64 product
    v = h[rows].view(-1, 2 * nkb, 2, 64).double()
    x1, x2 = v[:, :, 0], v[:, :, 1]
    y = qw2.view(N2, 2 * nkb, 2, 64).double()
    y1, y2 = y[:, :, 0], y[:, :, 1]
    per = 65536.0 * torch.einsum("mbk,nbk->mbn", x1, y1) + 256.0 * (
        torch.einsum("mbk,nbk->mbn", x1, y2) + torch.einsum("mbk,nbk->mbn", x2, y1))
    form = (per * hs[rows].double().repeat_interleave(2, 1)[:, :, None]).sum(1) * sw2.double()[None, :] + b2.double() + res[rows].double()
    got = C2[rows].double()
    scale = max(1.0, form.abs().max().item())
    assert (got - form).abs().max().item() < 2e-6 * scale
    exact = deq @ w2.double().t() + b2.double() + res[rows].double()
    assert (got - exact).abs().max().item() < 2e-4 * scale


@pytest.mark.parametrize("M,N,K,slots", [(50432, 768, 3072, 64), (50432, 768, 768, 64), (50432, 768, 768, 16),
                                         (12544, 512, 2048, 8)])
def test_gemm_tail_split(cuda, M, N, K, slots):
    """The residual encoder GEMM with its last partial round split in K over two blocks per tile (merged by
    the second finisher through agent-scope stores and a ticket): equal to the unsplit launch up to the
    fp32 rounding of the two half sums, bit-identical over repeated launches, tickets back at zero."""
    L, lib = _lib()
    if not lib.icap_tools_build():
        pytest.skip("measured-and-rejected variant: compiled only into the tools build (-DICAP_TOOLS)")
    g = torch.Generator(device="cpu").manual_seed(M + N + K + slots)
    A = torch.randn(2, M, K, generator=g).to(cuda).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(cuda).to(torch.bfloat16)
    bias = torch.randn(N, generator=g).to(cuda)
    R = torch.randn(M, N, generator=g).to(cuda)
    ref = R.clone()
    L.check(lib.icap_op_gemm(A.data_ptr(), K, M * K, 2, w.data_ptr(), bias.data_ptr(), ref.data_ptr(), N, 0,
                             M, N, K, 0, 3, L.stream_ptr()), "gemm resid")
    ws = torch.empty(8 * slots * 2 * 128 * 256, device=cuda)
    cnt = torch.zeros(8 * slots, device=cuda, dtype=torch.int32)
    outs = []
    for _ in range(4):
        C = R.clone()
        L.check(lib.icap_op_gemm_tail_split(A.data_ptr(), K, M * K, 2, w.data_ptr(), bias.data_ptr(), C.data_ptr(), N,
                                            M, N, K, slots, ws.data_ptr(), cnt.data_ptr(), L.stream_ptr()), "split")
        outs.append(C)
    torch.cuda.synchronize()
    assert all(torch.equal(o, outs[0]) for o in outs[1:])
    assert int(cnt.abs().sum().item()) == 0
    assert (outs[0] - ref).abs().max().item() < 1e-5 * max(1.0, ref.abs().max().item())
    # and the split really ran: a few tail tiles differ from the unsplit sums in their last bits
    tiles = (N // 256) * ((M + 127) // 128)
    if (tiles // 8 + 1) > slots:
        assert not torch.equal(outs[0], ref)


# ---------------------------------------------------------------- fp16 single-plane encoder (ICAP_PREC_F16)
@pytest.mark.parametrize("M,N,K", [(300, 256, 512), (50432, 768, 768), (1000, 3072, 768), (777, 768, 3072),
                                   (8192, 2304, 128), (8192, 1024, 192)])
@pytest.mark.parametrize("epi", [0, 1])
def test_gemm_f16(cuda, M, N, K, epi):
    """fp16 A / W (nsplit = -1), fp32 accumulate: against fp64 on the same fp16 values; fp32, one fp16
    plane (rounding of the output: 2^-11 relative) and residual outputs.  M % 256 == 0 with more tiles than
    CUs runs the persistent plane form across tile seams (2 and 3 k-steps per tile at K = 128 / 192)."""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K + epi)
    a = torch.randn(M, K, generator=g).to(torch.float16).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.float16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    ref = a.double() @ w.double().t() + bias.double()
    if epi == 1:
        ref = torch.nn.functional.gelu(ref)
    C = torch.empty(M, N, device=cuda)
    L.check(lib.icap_op_gemm(a.data_ptr(), K, 0, -1, w.data_ptr(), bias.data_ptr(), C.data_ptr(), N, 0,
                             M, N, K, epi, 0, L.stream_ptr()), "gemm f16")
    Ch = torch.empty(M, N, device=cuda, dtype=torch.float16)
    L.check(lib.icap_op_gemm(a.data_ptr(), K, 0, -1, w.data_ptr(), bias.data_ptr(), Ch.data_ptr(), N, 0,
                             M, N, K, epi, 2, L.stream_ptr()), "gemm f16 plane")
    R = torch.randn(M, N, generator=g).to(cuda)
    R0 = R.clone()
    L.check(lib.icap_op_gemm(a.data_ptr(), K, 0, -1, w.data_ptr(), bias.data_ptr(), R.data_ptr(), N, 0,
                             M, N, K, epi, 3, L.stream_ptr()), "gemm f16 resid")
    torch.cuda.synchronize()
    scale = max(1.0, ref.abs().max().item())
    assert (C.double() - ref).abs().max().item() < 2e-5 * scale
    assert torch.equal(Ch, C.to(torch.float16))  # the plane is the fp32 result rounded once
    assert (R.double() - R0.double() - C.double()).abs().max().item() < 1e-5 * scale


@pytest.mark.parametrize("M,N,K", [(50432, 2304, 768), (25216, 768, 3072), (50000, 3072, 768)])
def test_gemm_f16_persistent_repeat_bitwise(cuda, M, N, K):
    """The persistent fp16 GEMM at full-chip shapes (ViT B = 256 QKV, B = 128 MLP-2, a ragged 50000-row
    MLP-1): its tile seams wait with counted vmcnt that leave the previous tile's stores in flight, so a
    miscounted wait would read a stage before it landed - run to run differences.  Plane (+ GELU) and residual
    outputs, 6 runs each in one process: bitwise equal, and against fp64 on sampled rows."""
    L, lib = _lib()
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g).to(torch.float16).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.float16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    rows = torch.arange(0, M, 991, device=cuda)
    ref = a[rows].double() @ w.double().t() + bias.double()
    R0 = torch.randn(M, N, generator=g).to(cuda)
    for epi, out in ((0, 2), (1, 2), (0, 3)):
        outs = []
        for _ in range(6):
            C = R0.clone() if out == 3 else torch.empty(M, N, device=cuda, dtype=torch.float16)
            L.check(lib.icap_op_gemm(a.data_ptr(), K, 0, -1, w.data_ptr(), bias.data_ptr(), C.data_ptr(), N, 0,
                                     M, N, K, epi, out, L.stream_ptr()), "gemm f16")
            outs.append(C)
        torch.cuda.synchronize()
        assert all(torch.equal(o, outs[0]) for o in outs[1:]), (epi, out)
        want = torch.nn.functional.gelu(ref) if epi == 1 else ref
        got = outs[0][rows].double() - (R0[rows].double() if out == 3 else 0)
        tol = (2e-5 if out == 3 else 2 ** -10) * max(1.0, want.abs().max().item())
        assert (got - want).abs().max().item() < tol, (epi, out)


def test_gemm_f16_plane_past_2gib(cuda):
    """The store-only fp16 plane of the persistent GEMM beyond a 2 GiB byte offset (a buffer resource of
    2^31 - 1 bytes silently dropped those stores - the ViT MLP-1 output from B ~ 1775): a 2.2 GB output whose last
    rows are checked against fp64 (the plane is prefilled with NaN, so a dropped store cannot pass)."""
    L, lib = _lib()
    M, N, K = 360448, 3072, 128  # M N 2 bytes = 2.21e9 > 2^31
    g = torch.Generator(device="cpu").manual_seed(7)
    a = torch.randn(M, K, generator=g).to(torch.float16).to(cuda)
    w = (torch.randn(N, K, generator=g) / K ** 0.5).to(torch.float16).to(cuda)
    bias = torch.randn(N, generator=g).to(cuda)
    C = torch.full((M, N), float("nan"), device=cuda, dtype=torch.float16)
    L.check(lib.icap_op_gemm(a.data_ptr(), K, 0, -1, w.data_ptr(), bias.data_ptr(), C.data_ptr(), N, 0,
                             M, N, K, 0, 2, L.stream_ptr()), "gemm f16 plane > 2 GiB")
    torch.cuda.synchronize()
    first_past = (1 << 31) // (2 * N)  # the first row with bytes past 2 GiB
    rows = torch.cat([torch.arange(0, 64), torch.arange(first_past - 8, first_past + 8), torch.arange(M - 300, M)])
    rows = rows.to(cuda)
    ref = a[rows].double() @ w.double().t() + bias.double()
    got = C[rows].double()
    assert not torch.isnan(got).any()
    assert (got - ref).abs().max().item() < 2 ** -10 * max(1.0, ref.abs().max().item())
    del C


def test_gemm_f16_head_major_via_engine_layout(cuda):
    """Identity A through the fp16 kernel: exact, and not transposed."""
    L, lib = _lib()
    n = 256
    A = torch.eye(n, device=cuda).to(torch.float16).contiguous()
    w = (torch.arange(n * n, device=cuda, dtype=torch.float32).reshape(n, n) % 251).to(torch.float16)
    C = torch.empty(n, n, device=cuda)
    L.check(lib.icap_op_gemm(A.data_ptr(), n, 0, -1, w.data_ptr(), None, C.data_ptr(), n, 0, n, n, n, 0, 0,
                             L.stream_ptr()), "gemm f16")
    torch.cuda.synchronize()
    assert torch.equal(C, w.float().t())


def test_layernorm_f16(cuda):
    L, lib = _lib()
    rows, D = 333, 768
    x = (torch.randn(rows, D, device=cuda) * 3 + 1).contiguous()
    w = torch.randn(D, device=cuda)
    b = torch.randn(D, device=cuda)
    y = torch.empty_like(x)
    yh = torch.empty(rows, D, device=cuda, dtype=torch.float16)
    L.check(lib.icap_op_layernorm(x.data_ptr(), rows, D, w.data_ptr(), b.data_ptr(), 1e-6, y.data_ptr(),
                                  yh.data_ptr(), 0, -1, L.stream_ptr()), "ln f16")
    torch.cuda.synchronize()
    assert torch.equal(yh, y.to(torch.float16))


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (3, 100, 8)])
def test_enc_attention_f16(cuda, B, N, H):
    """One fp16 plane in and out; the probabilities enter the P.V product as fp16 (2^-11 relative)."""
    L, lib = _lib()
    D = H * 64
    g = torch.Generator(device="cpu").manual_seed(B * N + H + 1)
    qkv = (torch.randn(B * N, 3 * D, generator=g) * 1.5).to(torch.float16).to(cuda)
    v = qkv.double().view(B, N, 3, H, 64)
    q, k, vv = v[:, :, 0].transpose(1, 2), v[:, :, 1].transpose(1, 2), v[:, :, 2].transpose(1, 2)
    ref = torch.softmax(q @ k.transpose(-1, -2) / 8.0, -1) @ vv
    ref = ref.transpose(1, 2).reshape(B * N, D)
    out = torch.zeros(B * N, D, device=cuda, dtype=torch.float16)
    L.check(lib.icap_op_enc_attention(qkv.data_ptr(), 0, B, N, H, out.data_ptr(), 0, -1, L.stream_ptr()), "attn f16")
    torch.cuda.synchronize()
    assert (out.double() - ref).abs().max().item() < 4e-3


@pytest.mark.parametrize("B,N,H", [(2, 197, 12), (3, 100, 8), (1, 65, 2), (2, 256, 4), (5, 208, 3), (64, 197, 12),
                                   (45, 197, 12), (97, 120, 8)])
def test_enc_attention_f16_head_major(cuda, B, N, H):
    """The f16 ViT encoder's attention on the head-major qkv its QKV GEMM writes ([B][q|k|v][H][N][64]) against fp64:
    the persistent form (enc_attention_pers_kernel, N <= 240) and the whole-sequence form (N = 256), ragged last key
    tiles (N = 197, 100, 65, 120) and full ones (256, 208); B x H above the CU count (768, 540, 776 items) walks the
    two-item K / V ring of the persistent form (several items per workgroup, an uneven last round); repeated launches
    bitwise equal."""
    L, lib = _lib()
    D = H * 64
    g = torch.Generator(device="cpu").manual_seed(B * N + H + 7)
    hm = (torch.randn(B, 3, H, N, 64, generator=g) * 1.5).to(torch.float16)
    v = hm.double()
    ref = torch.softmax(v[:, 0] @ v[:, 1].transpose(-1, -2) / 8.0, -1) @ v[:, 2]  # (B, H, N, 64)
    ref = ref.transpose(1, 2).reshape(B * N, D)
    qkv = hm.to(cuda).contiguous()
    out = torch.zeros(B * N, D, device=cuda, dtype=torch.float16)
    L.check(lib.icap_op_enc_attention_hm(qkv.data_ptr(), B, N, H, out.data_ptr(), L.stream_ptr()), "attn f16 hm")
    torch.cuda.synchronize()
    assert (out.double().cpu() - ref).abs().max().item() < 4e-3
    again = torch.zeros_like(out)
    L.check(lib.icap_op_enc_attention_hm(qkv.data_ptr(), B, N, H, again.data_ptr(), L.stream_ptr()), "attn f16 hm")
    torch.cuda.synchronize()
    assert torch.equal(again, out)
