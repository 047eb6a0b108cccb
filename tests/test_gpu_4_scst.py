"""The drop-in SCST training path on the GPU (utils/scst_loss.py, reference utils/scst_loss.py:136-254)
and the in-place weight refresh it relies on (icap_update_weights).

* grad-enabled SCSTLoss.forward: the HIP sampler (injected uniforms, inverse CDF) against the PyTorch
  restatement of the reference loop (`SCSTLoss._sample_torch`) fed the same uniforms, dropout 0: same ids
  and stop length, log-probs within 1e-3, equal rewards, decoder gradients within 1e-3 relative;
* Grid in train mode: the ResNet trunk's BatchNorm running statistics take exactly ONE update per
  SCSTLoss.forward, as in the reference (its sampler encodes once in train mode, `generate` in eval); the
  HIP train-mode trunk (icap_encode_grid_train) against PyTorch's train-mode trunk;
* after an optimizer-style in-place change of decoder (or encoder) weights, `model.hip_engine` re-packs
  the changed part into the same handle and its outputs equal a freshly packed engine's.
"""
import copy

import pytest
import torch

from image_caption_amd import weights as W

pytestmark = pytest.mark.gpu

VOCAB = {f"w{i}": i for i in range(W.VOCAB_SIZE)}
VOCAB.update({"<pad>": 0, "<unk>": 106, "<start>": 107, "<end>": 108})
REFS = [["w1 w2 w3"], ["w4 w5"], ["w6"], ["w7 w8 w9 w10"], ["w3 w3 w9"], ["w11 w2"], ["w5 w6 w7"], ["w8"]]


def _vit_model(cuda, backend="auto", dropout=0.0, precision="f16"):
    from models.vit_transformer_model import build_model

    m = build_model(W.VOCAB_SIZE, {"pretrained_vit": False, "dropout": dropout, "backend": backend,
                                   "hip_precision": precision})
    m.load_state_dict(W.to_torch(W.vit_state_dict(0)))
    return m.to(cuda)


@pytest.mark.parametrize("precision", ["f16", "bf16x2"])
def test_scst_grad_step_matches_torch_sampler(cuda, precision):
    """Gradients of every trainable parameter (decoder: HIP training pass; projection: autograd on the HIP
    trunk's output) against the PyTorch model.  The HIP memory carries the trunk's rounding - fp16
    operands (f16, the default: 4e-3 on the memory) or 16-bit ones (bf16x2: 1e-5) - which the gradients
    inherit: held to 2e-2 of each tensor's norm with the f16 trunk (whose memory flips a few ReLU / softmax
    decisions), to 1e-3 of each tensor's maximum with the bf16x2 trunk.  (The
    backward itself matches fp64 autograd as closely as fp32 autograd does: tests/test_gpu_5_train.py.)"""
    from utils.scst_loss import SCSTLoss

    B, L = 8, 30
    imgs = torch.from_numpy(W.synthetic_images(B, seed=5)).to(cuda)
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(17)).to(cuda)
    hip_m = _vit_model(cuda, precision=precision)
    ref_m = _vit_model(cuda, backend="torch")
    hip_m.train()
    ref_m.train()
    # sampler outputs
    ids_h, lp_h = SCSTLoss()._sample_with_log_probs(hip_m, imgs, 107, 108, L, cuda, uni)
    ids_r, lp_r = SCSTLoss()._sample_with_log_probs(ref_m, imgs, 107, 108, L, cuda, uni)
    assert ids_h.shape == ids_r.shape and torch.equal(ids_h, ids_r)
    assert lp_h.requires_grad and lp_r.requires_grad
    assert (lp_h - lp_r).abs().max().item() < 1e-3
    # the whole step: loss, rewards, decoder gradients
    hip_m.zero_grad()
    ref_m.zero_grad()
    loss_h, info_h = SCSTLoss()(hip_m, imgs, REFS, VOCAB, cuda, max_len=L, uniforms=uni)
    loss_r, info_r = SCSTLoss()(ref_m, imgs, REFS, VOCAB, cuda, max_len=L, uniforms=uni)
    for k in ("sample_reward", "greedy_reward", "advantage"):
        assert abs(info_h[k] - info_r[k]) < 1e-6, (k, info_h[k], info_r[k])
    assert abs(loss_h.item() - loss_r.item()) <= 1e-3 * max(1.0, abs(loss_r.item()))
    loss_h.backward()
    loss_r.backward()
    # the decoder's gradients come from the HIP training pass (image_caption_amd/train.py), the
    # projection's from PyTorch autograd on the HIP trunk's output
    gh = dict(hip_m.named_parameters())
    n = 0
    for name, p in ref_m.named_parameters():
        if p.grad is None:
            continue
        n += 1
        a, b = gh[name].grad, p.grad
        assert a is not None, name
        if precision == "f16":  # a different memory (fp16 trunk): ReLU / softmax flips, so a norm-wise bound
            assert (a - b).norm().item() <= 2e-2 * max(b.norm().item(), 1e-9), name
        else:
            assert (a - b).abs().max().item() <= 1e-3 * max(b.abs().max().item(), 1e-6), name
    assert n > 10 and gh["encoder.projection.weight"].grad is not None


def test_scst_grid_batchnorm_updated_once(cuda):
    """Train-mode Grid SCST: one BatchNorm running-statistics update per step, as the reference."""
    from models.grid_transformer_model import build_model
    from utils.scst_loss import SCSTLoss

    B, L = 4, 12
    m = build_model(W.VOCAB_SIZE, {"pretrained_cnn": False, "dropout": 0.0})
    m.load_state_dict(W.to_torch(W.grid_state_dict(0)))
    m = m.to(cuda)
    twin = copy.deepcopy(m)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=2)).to(cuda)
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(4)).to(cuda)
    loss, _ = SCSTLoss()(m, imgs, REFS[:B], VOCAB, cuda, max_len=L, uniforms=uni)
    loss.backward()
    twin.train()
    with torch.no_grad():
        twin.encoder.cnn(imgs)  # exactly one train-mode pass
    # the step's trunk is the HIP train-mode trunk (icap_encode_grid_train): its batch statistics carry the
    # 16-bit activation planes' rounding (test_grid_train_trunk_matches_torch measures it), hence 2e-3
    for (name, a), (_, b) in zip(m.encoder.cnn.named_buffers(), twin.encoder.cnn.named_buffers()):
        if name.endswith("num_batches_tracked"):
            assert torch.equal(a, b), name
        else:
            assert torch.allclose(a, b, rtol=2e-3, atol=1e-4), name


def test_grid_train_trunk_matches_torch(cuda):
    """icap_encode_grid_train (the HIP ResNet-101 trunk with train-mode BatchNorm: batch statistics, running
    statistics updated in place) against the PyTorch trunk in train mode (fp32) on the same weights: trunk
    features, memory, every BatchNorm's running_mean / running_var / num_batches_tracked, and afterwards the
    eval-mode HIP trunk of the same engine (its folded BatchNorm must follow the updated statistics)."""
    from models.grid_transformer_model import build_model

    B = 8
    m = build_model(W.VOCAB_SIZE, {"pretrained_cnn": False, "dropout": 0.0})
    m.load_state_dict(W.to_torch(W.grid_state_dict(0)))
    m = m.to(cuda)
    twin = build_model(W.VOCAB_SIZE, {"pretrained_cnn": False, "dropout": 0.0, "backend": "torch"})
    twin.load_state_dict(m.state_dict())
    twin = twin.to(cuda)
    imgs = torch.from_numpy(W.synthetic_images(B, seed=5)).to(cuda)
    eng = m.hip_engine(cuda)
    m.encoder.cnn.train()
    twin.encoder.cnn.train()
    with torch.no_grad():
        mem, feats = eng.encode_grid_train(imgs, m.encoder.cnn)
        ref = twin.encoder.cnn(imgs)
        ref_mem = twin.encoder.tail(ref)
    ferr = ((feats - ref).abs().max() / ref.abs().max()).item()
    merr = (mem - ref_mem).abs().max().item()
    print(f"train trunk: feature error {ferr:.2e} (of max), memory error {merr:.2e}")
    assert ferr < 2e-3, ferr
    assert merr < 4e-3, merr
    worst = 0.0
    for (name, a), (_, b) in zip(m.encoder.cnn.named_buffers(), twin.encoder.cnn.named_buffers()):
        if name.endswith("num_batches_tracked"):
            assert torch.equal(a, b), name
        else:
            worst = max(worst, ((a - b).abs() / (b.abs() + 1e-3)).max().item())
    print(f"running statistics: worst relative error {worst:.2e}")
    assert worst < 2e-3, worst
    # eval mode afterwards: the same engine (no re-pack), BatchNorm folded from the updated statistics
    m.eval()
    twin.eval()
    assert m.hip_engine(cuda) is eng
    with torch.no_grad():
        got = eng.encode(imgs)
        want = twin.encoder(imgs)
    eerr = (got - want).abs().max().item()
    print(f"eval trunk after the update: memory error {eerr:.2e}")
    assert eerr < 4e-3, eerr


def test_scst_grid_train_mode_sampler_and_recompute_share_memory(cuda):
    """Grid in train mode with dropout 0.1 everywhere: the tokens are sampled from the same memory the
    log-probs are differentiated on (one train-mode tail per step, its dropout masks torch's), so with the
    same torch seed and the same sampler seed the grad-enabled call returns the no-grad call's ids and its
    recomputed log-probs match the sampler's within the decoder parity tolerance."""
    from models.grid_transformer_model import build_model
    from utils.scst_loss import SCSTLoss

    B, L = 4, 12
    m = build_model(W.VOCAB_SIZE, {"pretrained_cnn": False, "dropout": 0.1})
    m.load_state_dict(W.to_torch(W.grid_state_dict(0)))
    m = m.to(cuda).train()
    imgs = torch.from_numpy(W.synthetic_images(B, seed=2)).to(cuda)
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(4)).to(cuda)
    loss_fn = SCSTLoss()
    out = []
    for grad in (False, True):
        torch.manual_seed(123)
        with torch.set_grad_enabled(grad):
            ids, logp = loss_fn._sample_with_log_probs(m, imgs, W.START_TOKEN, W.END_TOKEN, L, cuda, uniforms=uni,
                                                       dropout_seed=77)
        out.append((ids, logp.detach()))
    assert torch.equal(out[0][0], out[1][0])
    err = (out[0][1] - out[1][1]).abs().max().item()
    print(f"sampler vs recompute log-probs: {err:.2e}")
    assert err < 1e-3, err


@pytest.mark.parametrize("part", ["decoder", "encoder"])
def test_engine_refresh_in_place(cuda, part):
    """model.hip_engine after an in-place weight change re-packs that part into the SAME handle
    (icap_update_weights), and decodes exactly as an engine packed from scratch."""
    from image_caption_amd.engine import Engine

    m = _vit_model(cuda)
    m.eval()
    imgs = torch.from_numpy(W.synthetic_images(4, seed=8)).to(cuda)
    with torch.no_grad():
        eng = m.hip_engine(cuda)
        for _ in range(3):  # eager, capture, replay: the decode graph exists before the update
            m.generate(imgs, 107, 108, 30)
        g = torch.Generator().manual_seed(1)
        with torch.no_grad():
            for name, p in m.named_parameters():
                if name.startswith("decoder.") == (part == "decoder") and p.dim() == 2:
                    p.add_(0.01 * torch.randn(p.shape, generator=g).to(cuda))
        eng2 = m.hip_engine(cuda)
        assert eng2 is eng
        got = m.generate(imgs, 107, 108, 30)
        mem = eng.encode(imgs)
        # the refreshed handle keeps the weight layout it was created with (bf16 decoder weights): compare with a
        # fresh engine of the same layout (left to itself it would pick hi/lo planes for these non-bf16 weights)
        fresh = Engine(m.state_dict(), "vit", {}, device=cuda, decoder_weight_planes=eng.dec_weight_planes)
        mem_f = fresh.encode(imgs)
        assert torch.equal(mem, mem_f)
        want = fresh.greedy(mem_f, 107, 108, 30)
        assert torch.equal(got, want)
        lg = eng.decoder_forward(want[:, :-1], mem, causal=True)
        lg_f = fresh.decoder_forward(want[:, :-1], mem_f, causal=True)
        assert torch.equal(lg, lg_f)


def test_scst_dropout_outside_fused_blocks_uses_reference_loop(cuda):
    """train-mode dropout sampling needs the fused one-token decode blocks (max_len <= 65, d 512,
    8 heads, dim_ff 2048, a parity precision).  Outside them SCSTLoss samples with the reference's own
    PyTorch loop (torch dropout) instead of failing mid-decode; backend='hip' says so up front."""
    from utils.scst_loss import SCSTLoss

    B, L = 2, 70
    imgs = torch.from_numpy(W.synthetic_images(B, seed=2)).to(cuda)
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(3)).to(cuda)
    m = _vit_model(cuda, dropout=0.1)
    m.train()
    assert not m.hip_engine(cuda).dropout_sampling_ok(L) and m.hip_engine(cuda).dropout_sampling_ok(30)
    ids, lp = SCSTLoss()._sample_with_log_probs(m, imgs, 107, 108, L, cuda, uni)
    assert ids.shape[0] == B and lp.shape == (B, ids.shape[1] - 1) and lp.requires_grad
    assert torch.isfinite(lp).all()
    mh = _vit_model(cuda, backend="hip", dropout=0.1)
    mh.train()
    with pytest.raises(ValueError):
        SCSTLoss()._sample_with_log_probs(mh, imgs, 107, 108, L, cuda, uni)
