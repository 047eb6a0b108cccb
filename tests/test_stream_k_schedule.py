"""The stream-K schedule of the persistent fp16 encoder GEMM (csrc/gemm_kern.h gemm_f16p_kernel; variant builds
-DICAP_F16P_SK=1, measured slower - DESIGN.md section 8), restated on the host and checked for every shape class the ViT encoder and the tests launch: each (tile, k-step) of an XCD's
tiles is computed exactly once, a tile is cut at most once (two units meeting in one workspace slot, the cut tile's
head ending one lane's range and its tail opening the next), every unit spans >= 2 k-steps (the late-barrier k-loop
issues a unit's first two stages at its opening), the slots of one launch are distinct, and the work per lane is
balanced to within one tile - whatever the number of blocks per XCD (the schedule is per virtual lane, so CU-masked
grids compute the same sums).  Host logic only (no GPU)."""
import pytest

VB = 32  # kernels.h F16P_SK_VB


def xcd_tiles(nwg, xcd):
    q, r = nwg >> 3, nwg & 7
    xbase = xcd * (q + 1) if xcd < r else r * (q + 1) + (xcd - r) * q
    return xbase, q + (xcd < r)


def schedule(xcnt, nk, nbx, xbase=0):
    """The units each real block lb < nbx of one XCD runs, in order: (tile, k0, k1, lane); and RP (-1: no stream-K)."""
    xq, xr = divmod(xcnt, VB)
    RP = -1
    if xr and nbx <= VB and nk % 2 == 0 and nk >= 2:
        if xq >= 1 and xr * nk >= 2 * VB:
            RP = xq - 1
        elif xq >= 2:
            RP = xq - 2
    sk = RP >= 0
    sk_t0 = xbase + (RP if sk else 0) * VB
    w2h = (xcnt - RP * VB) * nk // 2 if sk else 0

    def bnd(v):
        return 2 * (v * w2h // VB)

    def sk_unit(v, pos):
        u, k0 = divmod(pos, nk)
        return (sk_t0 + u, k0, min(nk, bnd(v + 1) - u * nk), v, RP)

    def first(v):
        return (xbase + v, 0, nk, v, 0) if RP > 0 else sk_unit(v, bnd(v))

    def nxt(c):
        t, k0, k1, v, r = c
        if not sk:
            return (t + nbx, 0, nk, 0, 0) if t + nbx < xbase + xcnt else None
        if r + 1 < RP:
            return (xbase + v + (r + 1) * VB, 0, nk, v, r + 1)
        if r + 1 == RP:
            return sk_unit(v, bnd(v))
        pos = (t + 1 - sk_t0) * nk
        if k1 == nk and pos < bnd(v + 1):
            return (t + 1, 0, min(nk, bnd(v + 1) - pos), v, RP)
        return first(v + nbx) if v + nbx < VB else None

    out = {}
    for lb in range(min(nbx, xcnt)):
        c = first(lb) if sk else (xbase + lb, 0, nk, 0, 0)
        units = []
        while c is not None:
            units.append(c)
            c = nxt(c)
        out[lb] = units
    return out, RP


# (M rows, N, K, BM): the ViT-B/16 GEMMs at B = 256 and smaller batches, the residual 224-row tiles, ragged M
SHAPES = [(m, n, k, bm) for m in (50432, 256 * 197, 37 * 197, 5 * 197, 8 * 197, 1 * 197, 129 * 197)
          for (n, k, bm) in ((2304, 768, 256), (3072, 768, 256), (768, 768, 224), (768, 3072, 224))]


@pytest.mark.parametrize("M,N,K,BM", SHAPES)
@pytest.mark.parametrize("nbx", [32, 26, 16, 7])
def test_stream_k_covers_every_kstep_once(M, N, K, BM, nbx):
    nk = K // 64
    nwg = (N // 256) * ((M + BM - 1) // BM)
    for xcd in range(8):
        xbase, xcnt = xcd_tiles(nwg, xcd)
        if xcnt == 0:
            continue
        units, RP = schedule(xcnt, nk, nbx, xbase)
        cover = {}
        parts = {}
        for lb, us in units.items():
            for (t, k0, k1, v, r) in us:
                assert xbase <= t < xbase + xcnt and 0 <= k0 < k1 <= nk
                assert k1 - k0 >= 2
                for k in range(k0, k1):
                    assert (t, k) not in cover, (t, k)
                    cover[(t, k)] = lb
                if (k0, k1) != (0, nk):
                    parts.setdefault(t, []).append((k0, k1, v))
        assert len(cover) == xcnt * nk
        slots = set()
        for t, ps in parts.items():  # a cut tile: head [0, k) of lane v, tail [k, nk) of lane v + 1, one slot
            assert len(ps) == 2, (t, ps)
            (a0, a1, va), (b0, b1, vb) = sorted(ps)
            assert a0 == 0 and a1 == b0 and b1 == nk and vb == va + 1
            slot = va + 1
            assert slot not in slots and 1 <= slot < VB
            slots.add(slot)
        if RP >= 0:  # balance: per virtual lane, within one tile of the mean
            per_lane = {}
            for us in units.values():
                for (t, k0, k1, v, r) in us:
                    per_lane[v] = per_lane.get(v, 0) + k1 - k0
            mean = xcnt * nk / VB
            assert max(per_lane.values()) <= mean + nk and min(per_lane.values()) >= mean - nk


def test_stream_k_is_grid_independent():
    """The units (and so the partial sums and their meeting) do not depend on the blocks per XCD."""
    nk = 12
    for xcnt in (296, 295, 85, 84, 222, 221, 40, 33):
        ref, _ = schedule(xcnt, nk, 32)
        lanes = sorted(u for us in ref.values() for u in us)
        for nbx in (31, 16, 9, 1):
            got, _ = schedule(xcnt, nk, nbx)
            assert sorted(u for us in got.values() for u in us) == lanes


def test_stream_k_engages_on_the_vit_shapes():
    """At B = 256 every ViT GEMM runs stream-K on the full chip (no XCD's tile count is a multiple of the lanes)."""
    for (n, k, bm) in ((2304, 768, 256), (3072, 768, 256), (768, 768, 224), (768, 3072, 224)):
        nwg = (n // 256) * ((50432 + bm - 1) // bm)
        for xcd in range(8):
            _, xcnt = xcd_tiles(nwg, xcd)
            _, RP = schedule(xcnt, k // 64, 32)
            assert RP >= 0, (n, k, xcd, xcnt)
