"""Drop-in limits of the HIP path beyond the synthetic benchmark model:
* vocabularies above 128 (the reference builds its vocabulary from the captions, utils/deepfashion_dataset.py
  :76-81): greedy ids, step logits, sampled ids / log-probs and teacher-forced logits against the oracle;
* fp32 weights that are NOT bf16-exact (real checkpoints): the packed bf16 weights' rounding measured against
  the fp32 oracle (tolerance stated in DESIGN.md §3)."""
import numpy as np
import pytest
import torch

from image_caption_amd import weights as W
from oracle import captioner as O

pytestmark = pytest.mark.gpu


def _mem(B, S, seed):
    return torch.from_numpy(np.random.Generator(np.random.PCG64(seed)).standard_normal((B, S, 512)).astype(np.float32))


@pytest.mark.parametrize("vocab", [1000, 4099])
def test_large_vocabulary(cuda, vocab):
    from image_caption_amd.engine import Engine

    sd = W.to_torch(W.vit_state_dict(0, vocab_size=vocab))
    eng = Engine(sd, "vit", {}, device=cuda)
    B, L, S = 6, 12, 196
    mem = _mem(B, S, vocab)
    ids, lg = eng.greedy_raw(mem.to(cuda), W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
    ref_ids, ref_tr = O.greedy_from_memory(sd, mem, W.START_TOKEN, W.END_TOKEN, L, return_trace=True)
    n = ref_ids.shape[1]
    assert torch.equal(ids.cpu().long()[:, :n], ref_ids)
    assert (lg.cpu()[: ref_tr.shape[0]] - ref_tr).abs().max().item() < 1e-3
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(vocab))
    sid, slp = eng.sample(mem.to(cuda), uni.to(cuda), W.START_TOKEN, W.END_TOKEN, L)
    r_sid, r_slp = O.sample_with_log_probs(sd, mem, uni, W.START_TOKEN, W.END_TOKEN, L)
    sid = sid.cpu().long()
    # with V in the thousands the draws sit close to CDF boundaries more often: ids are compared up to
    # the first step whose draw lies within 1e-5 (relative) of one (the logits agree to ~1e-5)
    probs = torch.softmax(O.teacher_forced_logits(sd, mem, r_sid), -1)  # (B, n-1, V)
    cdf = probs.cumsum(-1)
    gap = (cdf - uni.t()[:, : cdf.shape[1], None] * cdf[..., -1:]).abs().min(-1).values
    compared = 0
    for r in range(B):
        close = torch.nonzero(gap[r] < 1e-5)
        upto = int(close[0, 0]) + 1 if len(close) else r_sid.shape[1]
        assert torch.equal(sid[r, :upto], r_sid[r, :upto]), r
        compared += upto
        lp_upto = min(upto - 1, r_sid.shape[1] - 1)  # the draw at the close step may differ
        assert (slp.cpu()[r, :lp_upto] - r_slp[r, :lp_upto]).abs().max().item() < 1e-3
    assert compared >= B * r_sid.shape[1] // 2
    tf = eng.decoder_forward(ref_ids[:, :-1].to(cuda), mem.to(cuda), causal=True).cpu()
    assert (tf - O.teacher_forced_logits(sd, mem, ref_ids)).abs().max().item() < 1e-3


def test_fp32_weights_not_bf16_exact(cuda):
    """The engine packs decoder / encoder GEMM weights to bf16 once: with fp32 weights that are not
    bf16-exact (a real checkpoint) the logits carry that rounding (2^-9 relative per weight).  Measured
    against the fp32 oracle on the same weights: see DESIGN.md §3 for the bound asserted here."""
    from image_caption_amd.engine import Engine

    sd = W.to_torch(W.vit_state_dict(1, bf16_exact=False))
    imgs = torch.from_numpy(W.synthetic_images(4, seed=6))
    eng = Engine(sd, "vit", {}, device=cuda)
    mem = eng.encode(imgs.to(cuda)).cpu()
    ref_mem = O.vit_encode(sd, imgs)
    ids = eng.greedy(ref_mem.to(cuda), W.START_TOKEN, W.END_TOKEN, 30).cpu()
    ref_ids, tr = O.greedy_from_memory(sd, ref_mem, W.START_TOKEN, W.END_TOKEN, 30, return_trace=True)
    tf = eng.decoder_forward(ref_ids[:, :-1].to(cuda), ref_mem.to(cuda), causal=True).cpu()
    lerr = (tf - O.teacher_forced_logits(sd, ref_mem, ref_ids)).abs().max().item()
    merr = (mem - ref_mem).abs().max().item()
    L = min(ids.shape[1], ref_ids.shape[1])
    agree = (ids[:, :L].long() == ref_ids[:, :L]).float().mean().item()
    margin = O.top2_margin(tr).min().item()
    print(f"fp32 weights: memory err {merr:.2e}, decoder logit err {lerr:.2e}, token agreement {agree:.3f}, "
          f"min reference margin {margin:.2e}")
    assert merr < 5e-2 and lerr < 5e-2
    # ids identical up to the first step whose reference top-2 margin is within the error band
    for r in range(ids.shape[0]):
        close = np.nonzero(O.top2_margin(tr[:, r]).numpy() < 4 * lerr)[0]
        upto = (close[0] if len(close) else tr.shape[0]) + 1
        assert torch.equal(ids[r, :upto].long(), ref_ids[r, :upto]), r
