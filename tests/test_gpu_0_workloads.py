"""HIP path vs the oracle at the per-GPU workloads of the BASELINE configs, EVERY row checked.

  config 2  ViT-B/16 + decoder, B = 256, greedy max_len 30 (also config 4's per-rank shard: 256 rows of
            the 2048-image batch; the gather + batch-global stop rule is the gloo test in test_host.py)
  config 3  Grid (ResNet-101) + decoder, B = 256, greedy; the trunk features compared directly
  config 5  ViT SCST reward step per rank: 128 rows, sampled decode + greedy baseline (the two decode
            graphs replayed concurrently, as bench --mode scst) + CIDEr-D on the GPU vs the host

The oracle (oracle/captioner.py, fp32) runs on the GPU here - the same device-agnostic torch code; gfx950
has no TF32, so torch fp32 is fp32 - and is tied to its CPU run on a few rows of each workload.

Checks and tolerances (north star: logits within 1e-3, token ids identical):
  * memory (B, S, 512): max |HIP - oracle| < 4e-3 over all rows (the default precision f16: ViT encoder and Grid
    trunk on fp16 operands, |memory| <= ~3); Grid trunk features relative 1e-3,
    and every image's error is < 1/10 of its distance to the nearest other image (an image mix-up
    cannot pass);
  * greedy: the oracle's teacher-forced logits on the HIP ids (every row, every step) within 1e-3 of
    the HIP step logits; each HIP token = the oracle argmax wherever the oracle's top-2 margin exceeds
    2x the measured logit error; and the oracle's own greedy decode on all rows: every row id-identical
    to it, except at most 3 rows whose first differing token comes from a near-tie step (counts printed);
  * sampled: each HIP token = the oracle's inverse-CDF draw on the same uniform wherever the draw is
    further than 2x the measured probability error from a CDF boundary; log-probs within 1e-3 (zero
    after <end>, the reference's masked_fill);
  * CIDEr-D: the GPU pass equals the host restatement to 1e-9 on the decoded ids.
"""
import numpy as np
import pytest
import torch

from image_caption_amd import weights as W
from oracle import captioner as O

pytestmark = pytest.mark.gpu
L = 30
# ViT memory vs the oracle in the default precision (f16: fp16 encoder operands, 2^-11 relative rounding;
# |memory| <= ~3); the logits stay within 1e-3
VIT_MEM_TOL = 4e-3
# Grid memory in the default precision (f16: the ResNet trunk on fp16 planes - the residual stream as fp16 hi/lo, the
# bottleneck branch as one fp16 plane; CPU emulation: trunk features 2.3e-4 relative, memory 8.9e-4, logits 8e-5)
GRID_MEM_TOL = 4e-3
# Grid trunk features (relative to the batch maximum), per image
GRID_FEAT_TOL = 1e-3


def _dev_sd(sd, dev):
    return {k: v.to(dev) for k, v in sd.items()}


@pytest.fixture(scope="module")
def vit_sd():
    return W.to_torch(W.vit_state_dict(0))


@pytest.fixture(scope="module")
def grid_sd():
    return W.to_torch(W.grid_state_dict(0))


def _oracle_memory(fn, sd_dev, imgs, chunk=64):
    with torch.no_grad():
        return torch.cat([fn(sd_dev, imgs[i:i + chunk]) for i in range(0, imgs.shape[0], chunk)])


DIVERGED_ROWS_MAX = 3  # rows whose ids may leave the oracle's greedy ids (at a near-tie step only; verdict r3 item 5)


def _check_greedy(ids, step_logits, sd_dev, mem_o, end, tag=""):
    """ids (B, L) int32 HIP greedy output; step_logits (L-1, B, V) its per-step logits.

    1. The oracle's teacher-forced logits on the HIP ids: within 1e-3 of the HIP step logits on every row and step.
    2. The oracle's OWN greedy decode (O.greedy_from_memory, the reference's _greedy_search loop, vit:296-325) on the
       oracle memory, compared on every row: the rows are id-identical to it, except rows whose FIRST differing token
       comes from a near-tie step - a step whose oracle top-2 margin is within twice that row-step's measured
       HIP-vs-oracle logit error, where either token is a correct reading of the reference (after it the two decodes
       feed different tokens).  Those rows are counted, printed with the near-tie step count, and pinned to
       DIVERGED_ROWS_MAX; a difference at a confident step fails."""
    ids = ids.long()
    tf = O.teacher_forced_logits(sd_dev, mem_o, ids)                      # (B, L-1, V)
    hip = step_logits.permute(1, 0, 2)
    err_rs = (hip - tf).abs().amax(-1)                                    # (B, L-1) per row-step
    err = err_rs.max().item()
    assert err < 1e-3, f"step logits vs oracle {err}"
    top = tf.topk(2, dim=-1)
    margin = top.values[..., 0] - top.values[..., 1]
    sure = margin > 2 * err_rs + 1e-6
    agree = ids[:, 1:] == top.indices[..., 0]
    assert bool(agree[sure].all()), f"{int((~agree & sure).sum())} confident steps disagree"
    with torch.no_grad():
        o_ids = O.greedy_from_memory(sd_dev, mem_o, W.START_TOKEN, end, ids.shape[1])
    assert o_ids.shape == ids.shape  # random-init weights: no batch-global stop before max_len
    diverged = 0
    for r in range(ids.shape[0]):
        diff = torch.nonzero(ids[r] != o_ids[r]).flatten()
        if len(diff) == 0:
            continue
        c = int(diff[0])                    # >= 1 (both start with START); token c comes from step c - 1
        assert not bool(sure[r, c - 1]), (r, c, "first difference at a confident step")
        diverged += 1
    near_rows = int((~sure).any(-1).sum())
    print(f"\n[{tag}] greedy vs oracle greedy: {ids.shape[0]} rows, max logit err {err:.2e}, "
          f"near-tie steps {int((~sure).sum())} (in {near_rows} rows), rows id-identical to the oracle "
          f"{ids.shape[0] - diverged}, rows diverging at a near-tie {diverged}")
    assert diverged <= DIVERGED_ROWS_MAX, f"{diverged} rows diverge from the oracle greedy at a near-tie"
    return err, diverged


def test_config2_vit_b256_every_row(cuda, vit_sd):
    from image_caption_amd.engine import Engine

    B = 256
    eng = Engine(vit_sd, "vit", {}, device=cuda)
    sdd = _dev_sd(vit_sd, cuda)
    for seed in (1, 2):  # bench rank 0 / rank 1 shards (config 2, config 4 per rank)
        imgs = torch.from_numpy(W.synthetic_images(B, seed=seed)).to(cuda)
        mem = eng.encode(imgs)
        ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
        mem_o = _oracle_memory(O.vit_encode, sdd, imgs)
        assert (mem - mem_o).abs().max().item() < VIT_MEM_TOL
        if seed == 1:  # the GPU-run oracle is the CPU oracle
            rows = [0, 255]
            cpu = O.vit_encode(vit_sd, imgs[rows].cpu())
            assert (cpu - mem_o[rows].cpu()).abs().max().item() < 1e-4
        _check_greedy(ids, lg, sdd, mem_o, W.END_TOKEN, f"config2 seed {seed}")
        # the teacher-forced HIP decoder (icap_decoder_forward) on the same ids
        tf = eng.decoder_forward(ids[:, :-1], mem, causal=True)
        assert (tf - O.teacher_forced_logits(sdd, mem_o, ids.long())).abs().max().item() < 1e-3


def test_config2_vit_b256_fp32_weights_every_row(cuda):
    """Config 2 on weights that are NOT bf16-exact (what the reference's trainers write, train_vit_transformer.py:413-423,
    loaded by scripts/inference_vit_transformer.py:20-62): the engine picks hi/lo decoder weights and, since round 5,
    decodes with the fused blocks' hi/lo forms (W_lo fragment images, W_hi . (X_hi + X_lo) + W_lo . X_hi).  HIP encoder
    -> hi/lo decoder on all 256 rows against the fp32 oracle on the same weights: memory, every step's logits within
    1e-3, the oracle's own greedy ids (the same near-tie rule as config 2); and the fused greedy decode equals the
    unfused teacher-forced hi/lo decoder (icap_decoder_forward) on the same ids within 1e-3."""
    from image_caption_amd.engine import Engine

    B = 256
    sd = W.to_torch(W.vit_state_dict(3, bf16_exact=False))
    eng = Engine(sd, "vit", {}, device=cuda)
    assert eng.dec_weight_planes == 2
    sdd = _dev_sd(sd, cuda)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=7)).to(cuda)
    mem = eng.encode(imgs)
    ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
    mem_o = _oracle_memory(O.vit_encode, sdd, imgs)
    assert (mem - mem_o).abs().max().item() < VIT_MEM_TOL
    _check_greedy(ids, lg, sdd, mem_o, W.END_TOKEN, "config2 fp32 weights")
    tf = eng.decoder_forward(ids[:, :-1], mem, causal=True)
    assert (tf - lg.permute(1, 0, 2)).abs().max().item() < 1e-3


def test_config2_fp32_weights_outlier_channels(cuda):
    """Real ViT-B/16 checkpoints carry residual channels far above the rest; the synthetic draws do not.  Config 2 on
    fp32 (not bf16-exact) weights whose MLP-2 rows and biases of 4 residual channels are scaled x20 in layers 2-11: the
    default f16 encoder must keep every step's logits within 1e-3 of the fp32 oracle, and the error is the encoder's
    (HIP memory -> oracle decoder carries it; oracle memory -> HIP decoder stays ~1e-4).  Measured (round 6,
    tools/r6_precision.py): memory error 7.1e-3 against 2.4e-3 without outliers, logits 8.2e-4 (7.9e-4), decoder share
    7.9e-5; the bf16x2 encoder is NOT the more precise choice for such weights (its bf16 weights: logits 6.2e-3), so the
    drop-in keeps f16 (its fp16 range guard re-encodes only on overflow, which these weights do not reach)."""
    from image_caption_amd.engine import Engine

    B, CH = 256, [7, 200, 411, 650]
    sd = W.to_torch(W.vit_state_dict(3, bf16_exact=False))
    for i in range(2, 12):
        p = f"encoder.vit.encoder.layers.encoder_layer_{i}.mlp.3"
        sd[p + ".weight"][CH] *= 20.0
        sd[p + ".bias"][CH] *= 20.0
    eng = Engine(sd, "vit", {}, device=cuda)
    sdd = _dev_sd(sd, cuda)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=7)).to(cuda)
    mem = eng.encode(imgs)
    assert not eng.range_overflowed()
    ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
    ids = ids.long()
    mem_o = _oracle_memory(O.vit_encode, sdd, imgs)
    with torch.no_grad():
        ref = torch.cat([O.teacher_forced_logits(sdd, mem_o[i:i + 64], ids[i:i + 64]) for i in range(0, B, 64)])
        enc = torch.cat([O.teacher_forced_logits(sdd, mem[i:i + 64], ids[i:i + 64]) for i in range(0, B, 64)])
    full = (lg.permute(1, 0, 2) - ref).abs().max().item()
    dec = (eng.decoder_forward(ids[:, :-1], mem_o, causal=True) - ref).abs().max().item()
    enc_share = (enc - ref).abs().max().item()
    merr = (mem - mem_o).abs().max().item()
    print(f"\n[config2 fp32 + outliers] memory err {merr:.2e}, logits {full:.2e} (encoder share {enc_share:.2e}, "
          f"decoder share {dec:.2e})")
    assert full < 1e-3 and dec < 2e-4 and merr < 1.5e-2


def test_config3_grid_b256_trunk_and_every_row(cuda, grid_sd):
    from image_caption_amd.engine import Engine

    B = 256
    eng = Engine(grid_sd, "grid", {}, device=cuda)
    sdd = _dev_sd(grid_sd, cuda)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=3)).to(cuda)
    mem, feats = eng.encode_grid_features(imgs)
    feats_o = _oracle_memory(O.resnet101_trunk, sdd, imgs, chunk=32)
    scale = feats_o.abs().max().item()
    per_img = (feats - feats_o).abs().flatten(1).amax(1)
    print(f"\n[config3] trunk features max err {per_img.max().item() / scale:.2e} of the batch maximum")
    assert per_img.max().item() < GRID_FEAT_TOL * scale, per_img.max().item() / scale
    # discriminative: every image's error is far below its distance to the closest other image
    fo = feats_o.flatten(1)
    d = torch.cdist(fo[None], fo[None], p=float("inf"))[0] + torch.eye(B, device=cuda) * 1e30
    assert bool((per_img * 10 < d.amin(1)).all())
    with torch.no_grad():
        mem_o = O.grid_encode_tail(sdd, feats_o)
    print(f"[config3] memory max err {(mem - mem_o).abs().max().item():.2e}")
    assert (mem - mem_o).abs().max().item() < GRID_MEM_TOL
    rows = [0, 255]
    with torch.no_grad():
        cpu = O.grid_encode(grid_sd, imgs[rows].cpu())
    assert (cpu - mem_o[rows].cpu()).abs().max().item() < 1e-4
    ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
    _check_greedy(ids, lg, sdd, mem_o, W.END_TOKEN, "config3")
    distinct = len({tuple(r) for r in ids.cpu().tolist()})
    assert distinct >= 4, distinct  # the rows really differ (the decoder, not the memory, limits variety)


def test_config5_scst_reward_step_128_rows(cuda, vit_sd):
    from image_caption_amd import cider
    from image_caption_amd.engine import Engine, apply_stop_rule
    from image_caption_amd.scst import sample_and_greedy

    B = 128
    eng = Engine(vit_sd, "vit", {}, device=cuda)
    sdd = _dev_sd(vit_sd, cuda)
    gen = torch.Generator().manual_seed(5)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=9)).to(cuda)
    uni = torch.rand(L - 1, B, generator=gen).to(cuda)
    mem = eng.encode(imgs)
    for _ in range(3):  # eager, capture, replay of both decode graphs
        sid, slp, gid = sample_and_greedy(eng, mem, uni, W.START_TOKEN, W.END_TOKEN, L)
    torch.cuda.synchronize()
    mem_o = _oracle_memory(O.vit_encode, sdd, imgs)
    assert (mem - mem_o).abs().max().item() < VIT_MEM_TOL
    # sampled rows: the oracle's inverse-CDF draw on the same uniform, gated by the boundary distance
    s = sid.long()
    tf = O.teacher_forced_logits(sdd, mem_o, s)                            # (B, L-1, V)
    probs = torch.softmax(tf, -1)
    cdf = probs.cumsum(-1)
    thr = uni.t().unsqueeze(-1) * cdf[..., -1:]
    draw = (cdf <= thr).sum(-1).clamp_max(W.VOCAB_SIZE - 1)
    dist = (cdf - thr).abs().amin(-1)
    lp_o = torch.log_softmax(tf, -1).gather(2, s[:, 1:, None]).squeeze(2)
    ended = (s[:, 1:] == W.END_TOKEN).long().cumsum(1)
    before = torch.cat([torch.zeros_like(ended[:, :1]), ended[:, :-1]], 1) > 0
    lp_o = lp_o.masked_fill(before, 0.0)
    perr = (slp - lp_o).abs().max().item()
    assert perr < 1e-3, perr
    # per step, the draw is decided wherever the threshold is further from every CDF boundary than twice
    # that step's HIP-vs-oracle CDF difference (HIP teacher-forced logits on the same prefix)
    hip_lg = eng.decoder_forward(sid[:, :-1], mem, causal=True)
    assert (hip_lg - tf).abs().max().item() < 1e-3
    cdf_err = (torch.softmax(hip_lg, -1).cumsum(-1) - cdf).abs().amax(-1)
    sure = dist > 2 * cdf_err + 1e-7
    assert bool((draw == s[:, 1:])[sure].all())
    # the gate is a sanity bound, not the check: a draw lands within 2x the CDF error of a boundary with probability
    # ~4x that error (f16 encoder: CDF errors up to ~1e-3, 16 of 3840 draws gated when measured)
    assert int((~sure).sum()) <= max(2, s.numel() // 100), int((~sure).sum())
    assert bool((slp[before] == 0).all())
    # greedy rows (no step logits from the concurrent pair: teacher-forced HIP decoder logits instead)
    g = gid.long()
    hip_tf = eng.decoder_forward(gid[:, :-1], mem, causal=True)
    _check_greedy(gid, hip_tf.permute(1, 0, 2), sdd, mem_o, W.END_TOKEN, "config5 greedy")
    # CIDEr-D of both sets (one reference caption per image), GPU pass vs the host restatement
    refs = [[torch.randint(1, 100, (int(torch.randint(5, 13, (1,), generator=gen)),), generator=gen).tolist()]
            for _ in range(B)]
    g = apply_stop_rule(g, W.END_TOKEN)
    hyp = torch.full((2 * B, L), W.PAD_TOKEN, dtype=torch.int32, device=cuda)
    hyp[:B, : s.shape[1]] = sid
    hyp[B:, : g.shape[1]] = g.int()
    rows, off = cider.pack_references(refs, W.PAD_TOKEN, W.END_TOKEN, W.VOCAB_SIZE)
    r = cider.cider_d_device(hyp, rows.to(cuda), off.to(cuda), W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN)
    host = [cider.caption_ids(x, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN) for x in hyp.cpu().tolist()]
    want = cider.cider_d(host[:B], refs)[1] + cider.cider_d(host[B:], refs)[1]
    assert np.abs(r.cpu().numpy() - np.array(want)).max() < 1e-9
    assert float(np.abs(want).sum()) > 0
