"""End-to-end parity of the HIP engine against the CPU oracle (oracle/captioner.py)."""
import numpy as np
import pytest
import torch

from image_caption_amd import weights as W
from oracle import captioner as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vit_sd():
    return W.to_torch(W.vit_state_dict(0))


@pytest.mark.parametrize("precision", ["f16", "i8x2", "bf16x2", "bf16"])
def test_vit_encode_and_greedy(cuda, vit_sd, precision):
    from image_caption_amd.engine import Engine

    eng = Engine(vit_sd, "vit", {}, precision=precision, device=cuda)
    imgs = torch.from_numpy(W.synthetic_images(4, seed=3))
    mem_ref = O.vit_encode(vit_sd, imgs)
    mem = eng.encode(imgs.to(cuda)).cpu()
    err = (mem - mem_ref).abs().max().item()
    tol = {"bf16": 5e-2, "f16": 4e-3}.get(precision, 1e-3)
    assert err < tol, err
    ids, logits = eng.greedy_raw(mem_ref.to(cuda), 107, 108, 30, want_logits=True)
    ids = ids.cpu().long()
    ref_ids, ref_tr = O.greedy_from_memory(vit_sd, mem_ref, 107, 108, 30, return_trace=True)
    # teacher-forced logits on the reference prefix
    tf = O.teacher_forced_logits(vit_sd, mem_ref, ref_ids)
    tf_hip = eng.decoder_forward(ref_ids[:, :-1].to(cuda), mem_ref.to(cuda), causal=True).cpu()
    lerr = (tf_hip - tf).abs().max().item()
    if precision != "bf16":
        assert lerr < 1e-3, lerr
        assert torch.equal(ids[:, : ref_ids.shape[1]], ref_ids)
        assert (logits.cpu()[: ref_tr.shape[0]] - ref_tr).abs().max().item() < 1e-3
    else:
        assert lerr < 1e-1, lerr


def test_two_chain_decode_matches_one_chain(cuda, vit_sd):
    """The batch decoded as two or three independent graph branches (icap_set_decode_chains; one chain is the
    default since round 4) gives the same greedy ids, step logits and sampled ids / log-probs as one chain,
    for an odd batch (uneven parts 128 + 129, 85 + 86 + 86), eagerly and on graph replay."""
    from image_caption_amd.engine import Engine

    B, L = 257, 12
    mem = torch.from_numpy(np.random.Generator(np.random.PCG64(21)).standard_normal((B, 49, 512)).astype(np.float32))
    mem = mem.to(cuda)
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(3)).to(cuda)
    out = {}
    for nb in ("1", "2", "3"):
        eng = Engine(vit_sd, "vit", {}, device=cuda)
        eng.set_decode_chains(int(nb))
        runs = []
        for _ in range(3):  # eager, capture, replay
            ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
            sid, lp = eng.sample(mem, uni, W.START_TOKEN, W.END_TOKEN, L)
            runs.append((ids.cpu(), lg.cpu(), sid.cpu(), lp.cpu()))
        for r in runs[1:]:
            assert all(torch.equal(a, b) for a, b in zip(r, runs[0]))
        out[nb] = runs[0]
    for nb in ("2", "3"):
        for a, b in zip(out["1"], out[nb]):
            assert torch.equal(a, b)


@pytest.mark.parametrize("B", [8, 256])
def test_pipeline_matches_sequential(cuda, vit_sd, B):
    """CaptionPipeline (encode of batch i+1 on one stream while batch i decodes on a high-priority
    stream) returns exactly the ids of encode + greedy run batch by batch, through the eager, capture
    and replay calls of the decode graph."""
    from image_caption_amd.engine import Engine
    from image_caption_amd.pipeline import CaptionPipeline

    eng = Engine(vit_sd, "vit", {}, device=cuda)
    batches = [torch.from_numpy(W.synthetic_images(B, seed=s)).to(cuda) for s in (11, 12, 13, 14)]
    seq = [eng.greedy_raw(eng.encode(b), 107, 108, 30)[0].cpu() for b in batches]
    got = CaptionPipeline(eng, 107, 108, 30).run(batches)
    torch.cuda.synchronize()
    assert len(got) == len(seq)
    for a, b in zip(got, seq):
        assert torch.equal(a.cpu(), b)
    # with a host-syncing post step (the stop rule), as the bench runs it
    from image_caption_amd.engine import apply_stop_rule

    got2 = CaptionPipeline(eng, 107, 108, 30).run(batches, lambda ids: apply_stop_rule(ids.long(), 108))
    for a, b in zip(got2, seq):
        assert torch.equal(a.cpu(), apply_stop_rule(b.long(), 108))
    # the overlapped encodes run under an encoder CU budget (default OVERLAP_CU_SHARE of the CUs, round 6) that the
    # run restores; the ids do not depend on it (each tile's k-loop is the same whichever block takes the tile)
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    assert eng.encoder_cus == 0
    assert CaptionPipeline(eng, 107, 108, 30).overlap_cus == int(cus * CaptionPipeline.OVERLAP_CU_SHARE) // 8 * 8
    p = CaptionPipeline(eng, 107, 108, 30)
    assert p.overlap_attn_cus == int(cus * CaptionPipeline.OVERLAP_ATTN_CU_SHARE) // 8 * 8
    for budget, attn in ((0, None), (96, None), (160, 40)):
        got3 = CaptionPipeline(eng, 107, 108, 30, encoder_cus=budget, attention_cus=attn).run(batches)
        assert (eng.encoder_cus, eng.encoder_attention_cus) == (0, 0)
        for a, b in zip(got3, seq):
            assert torch.equal(a.cpu(), b)


def test_profile_sampled_layers(cuda, vit_sd):
    """Live launch timing (icap_profile_enable, bench.py's roofline): every = 6 brackets ViT encoder layers 0 and 6 only
    - 8 of the 48 persistent-GEMM launches and 2 of the 12 attentions of an f16 encode at B = 64 - every = 1 all of
    them, with positive device times; the patch / projection GEMMs (another class) are bracketed either way."""
    from image_caption_amd import _lib
    from image_caption_amd.engine import Engine

    eng = Engine(vit_sd, "vit", {}, device=cuda)
    imgs = torch.from_numpy(W.synthetic_images(64, seed=3)).to(cuda)
    eng.encode(imgs)
    for every, gemms, attns in ((1, 48, 12), (6, 8, 2)):
        eng.profile(True, every=every)
        eng.encode(imgs)
        torch.cuda.synchronize()
        g = eng.profile_read(_lib.PROF_GEMM_F16P)
        a = eng.profile_read(_lib.PROF_ENC_ATTN)
        p = eng.profile_read(_lib.PROF_GEMM_256)
        eng.profile(False)
        assert (g["launches"], a["launches"], p["launches"]) == (gemms, attns, 2), (every, g, a, p)
        assert g["ms"] > 0 and a["ms"] > 0


def test_cu_masked_pipelines_budget_stack(cuda, vit_sd):
    """CU-masked pipelines (decode_cus) size the engine's encoder grids (GEMMs and, round 6, the persistent encoder
    attention) to the encoder stream's CUs; two overlapping pipelines deleted in either order leave the newest live
    budget, then the base - and a base the caller changed between pipelines is the one restored.  The
    masked pipeline's ids equal the sequential encode + greedy."""
    import gc

    from image_caption_amd.engine import Engine
    from image_caption_amd.pipeline import CaptionPipeline

    eng = Engine(vit_sd, "vit", {}, device=cuda)
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    for first_deleted in (0, 1):
        assert eng.encoder_cus == 0
        ps = [CaptionPipeline(eng, 107, 108, 30, decode_cus=32), CaptionPipeline(eng, 107, 108, 30, decode_cus=64)]
        assert eng.encoder_cus == cus - 64
        del ps[first_deleted]
        gc.collect()
        assert eng.encoder_cus == (cus - 64 if first_deleted == 0 else cus - 32)
        del ps[0]
        gc.collect()
        assert eng.encoder_cus == 0
    eng.set_encoder_cus(cus - 8)  # the caller's own budget, set while no masked pipeline is alive
    p = CaptionPipeline(eng, 107, 108, 30, decode_cus=48)
    assert eng.encoder_cus == cus - 48
    batches = [torch.from_numpy(W.synthetic_images(8, seed=s)).to(cuda) for s in (21, 22)]
    got = p.run(batches)
    torch.cuda.synchronize()
    del p
    gc.collect()
    assert eng.encoder_cus == cus - 8
    eng.set_encoder_cus(0)
    for a, b in zip(got, batches):
        assert torch.equal(a.cpu(), eng.greedy_raw(eng.encode(b), 107, 108, 30)[0].cpu())


def _tools_only():
    from image_caption_amd import _lib

    if not _lib.load().icap_tools_build():
        pytest.skip("measured-and-rejected decode steps (decstep.hip / xdec.hip): tools build only (-DICAP_TOOLS)")


@pytest.mark.parametrize("kind,B,S", [("vit", 256, 196), ("vit", 37, 196), ("grid", 64, 49)])
def test_persistent_decode_step_matches_launch_loop(cuda, vit_sd, kind, B, S):
    """The persistent decode step (one launch per step running every layer as dependency-ordered tasks,
    csrc/decstep.hip) against the launch-per-block loop on the same memory: greedy ids identical and step logits
    within 1e-4, sampled ids / log-probs with train-mode dropout
    likewise (measured 2.4e-5: 64- instead of 32-key cross-attention chunks and the LayerNorm sums' order; the
    oracle bar is 1e-3); graph capture and replay included (three calls each), a partial last 16-row tile (B = 37)."""
    _tools_only()
    from image_caption_amd.engine import Engine

    sd = vit_sd if kind == "vit" else W.to_torch(W.grid_state_dict(0))
    eng = Engine(sd, kind, {}, device=cuda)
    g = torch.Generator().manual_seed(B)
    mem = torch.randn(B, S, 512, generator=g).to(cuda)
    uni = torch.rand(29, B, generator=g).to(cuda)
    out = {}
    for step in (False, True):
        eng.set_decode_step(step)
        for _ in range(3):  # eager, capture, replay
            ids, lg = eng.greedy_raw(mem, 107, 108, 30, want_logits=True)
            sid, slp = eng.sample(mem, uni, 107, 108, 30, dropout=(0.1, 1234))
        torch.cuda.synchronize()
        assert not eng.range_overflowed()  # also: no persistent step gave up (raises)
        out[step] = (ids.clone(), lg.clone(), sid.clone(), slp.clone())
    a, b = out[False], out[True]
    lerr = (a[1] - b[1]).abs().max().item()
    perr = (a[3] - b[3]).abs().max().item()
    assert torch.equal(a[0], b[0]) and lerr < 1e-4, lerr
    assert torch.equal(a[2], b[2]) and perr < 1e-4, perr


@pytest.mark.parametrize("kind,B,S", [("vit", 256, 196), ("vit", 37, 196), ("grid", 256, 49), ("vit", 128, 196)])
def test_group_decode_step_matches_launch_loop(cuda, vit_sd, kind, B, S):
    """The group-persistent decode step (csrc/xdec.hip: one launch per step, 8 row groups x 32 workgroups, products
    split by output columns, write-through hand-offs between phases) against the launch-per-block loop on the same
    memory: greedy ids identical and step logits within 1e-4 (the residual sums run in another order), sampled ids
    identical and log-probs within 1e-4; graph capture and replay included (three calls each), partial groups
    (B = 37: 5 rows per group, the last group 2), the Grid memory length, the SCST per-rank batch (B = 128)."""
    _tools_only()
    from image_caption_amd.engine import Engine

    sd = vit_sd if kind == "vit" else W.to_torch(W.grid_state_dict(0))
    eng = Engine(sd, kind, {}, device=cuda)
    g = torch.Generator().manual_seed(B + 1)
    mem = torch.randn(B, S, 512, generator=g).to(cuda)
    uni = torch.rand(29, B, generator=g).to(cuda)
    out = {}
    for mode in (0, 2):
        eng.set_decode_step(mode)
        for _ in range(3):  # eager, capture, replay
            ids, lg = eng.greedy_raw(mem, 107, 108, 30, want_logits=True)
            sid, slp = eng.sample(mem, uni, 107, 108, 30)
        torch.cuda.synchronize()
        assert not eng.range_overflowed()  # also: no group gave up waiting (raises)
        out[mode] = (ids.clone(), lg.clone(), sid.clone(), slp.clone())
    a, b = out[0], out[2]
    # greedy: ids identical up to the first step where the launch loop's top-2 logit margin is below 1e-4 (a tie the
    # 1e-5-level reordering may flip); logits within 1e-4 on every row up to that step
    top = a[1].topk(2, dim=-1).values                        # (L-1, B, 2)
    close = (top[..., 0] - top[..., 1]) < 1e-4               # (L-1, B)
    for r in range(B):
        near = torch.nonzero(close[:, r]).flatten()
        upto = int(near[0]) + 1 if len(near) else close.shape[0]  # logit steps computed from identical prefixes
        assert torch.equal(a[0][r, :upto], b[0][r, :upto]) and (len(near) or torch.equal(a[0][r], b[0][r])), r
        lerr = (a[1][:upto, r] - b[1][:upto, r]).abs().max().item()
        assert lerr < 1e-4, (r, lerr)
    # sampled: inverse-CDF draws flip where a uniform lies within ~1e-5 of a CDF boundary (~0.1 expected flips per
    # 256 x 29 draws); rows that agree have log-probs within 1e-4, and at most 2 rows may differ
    same = (a[2] == b[2]).all(dim=1)
    assert int((~same).sum()) <= 2, int((~same).sum())
    perr = (a[3][same] - b[3][same]).abs().max().item()
    assert perr < 1e-4, perr
