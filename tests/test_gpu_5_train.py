"""HIP decoder training pass (icap_decoder_train_forward / _backward, image_caption_amd/train.py) against
PyTorch autograd through the same TransformerDecoder (eval mode: dropout off on both sides), at the
SCST per-rank shape of config 5 (128 rows, 29 teacher-forced positions, 196 memory tokens).  Reference:
the autograd graph of SCSTLoss._sample_with_log_probs (utils/scst_loss.py:210-254) and its backward."""
import numpy as np
import pytest
import torch

from models._common import TransformerDecoder
from utils.scst_loss import masked_token_logp

pytestmark = pytest.mark.gpu

END = 108


def _ids(B, L, V, seed):
    g = np.random.Generator(np.random.PCG64(seed))
    ids = g.integers(0, V - 2, size=(B, L))
    ids[:, 0] = 107
    for b in range(0, B, 3):  # an <end> inside some rows: the steps after it are masked
        ids[b, g.integers(2, L - 1)] = END
    ids[1, 1] = END
    return torch.from_numpy(ids)


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _autograd(dec, mem0, ids, adv, names):
    """log-probs, parameter and memory gradients of the SCST loss by PyTorch autograd (dtype of dec)."""
    params = dict(dec.named_parameters())
    mem = mem0.to(next(dec.parameters()).dtype).clone().requires_grad_(True)
    mask = dec.generate_square_subsequent_mask(ids.shape[1] - 1, mem.device).to(mem.dtype)
    lp = masked_token_logp(dec(ids[:, :-1], mem, tgt_mask=mask), ids, END)
    (-(adv.to(mem.dtype) * lp.sum(1)).mean()).backward()
    out = lp.detach(), {k: params[k].grad.clone() for k in names}, mem.grad.clone()
    dec.zero_grad(set_to_none=True)
    return out


@pytest.mark.parametrize("B,L,S", [(128, 30, 196), (5, 7, 49)])
def test_decoder_train_pass_matches_autograd(cuda, B, L, S):
    """Log-probs within 1e-4 and every parameter gradient (and the memory gradient) within 1e-3 relative
    (Frobenius) of fp64 autograd; PyTorch's own fp32 autograd is held to the same bar for comparison."""
    import copy

    from image_caption_amd.train import decoder_param_names, decoder_token_logp

    torch.manual_seed(0)
    dec = TransformerDecoder(109, max_len=100).to(cuda).eval()
    with torch.no_grad():  # non-zero biases / LN affine so every gradient path is exercised
        for n, p in dec.named_parameters():
            if n.endswith("bias") or "norm" in n:
                p.add_(0.05 * torch.randn_like(p))
    ids = _ids(B, L, 109, S).to(cuda)
    mem0 = torch.randn(B, S, 512, generator=torch.Generator().manual_seed(B)).to(cuda)
    adv = torch.randn(B, generator=torch.Generator().manual_seed(7)).to(cuda)
    names = decoder_param_names(6)
    params = dict(dec.named_parameters())

    lp64, g64, dm64 = _autograd(copy.deepcopy(dec).double(), mem0, ids, adv, names)
    lp32, g32, dm32 = _autograd(dec, mem0, ids, adv, names)

    mem2 = mem0.clone().requires_grad_(True)
    lp = decoder_token_logp(dec, mem2, ids, END)
    (-(adv * lp.sum(1)).mean()).backward()
    torch.cuda.synchronize()

    assert (lp.double() - lp64).abs().max().item() < 1e-4
    assert torch.equal(lp == 0, lp64 == 0)  # the same masked steps
    hip = max((_rel(params[k].grad.double(), g64[k]), k) for k in names)
    ref = max((_rel(g32[k].double(), g64[k]), k) for k in names)
    print(f"worst relative gradient error vs fp64: HIP {hip}, torch fp32 {ref}")
    assert hip[0] < 1e-3, (hip, ref)
    assert _rel(mem2.grad.double(), dm64) < 1e-3


def test_decoder_train_pass_repeats_bitwise(cuda):
    """No atomics in the training pass: two backward passes give identical gradients."""
    from image_caption_amd.train import decoder_token_logp

    torch.manual_seed(1)
    dec = TransformerDecoder(109).to(cuda).eval()
    ids = _ids(16, 12, 109, 3).to(cuda)
    mem = torch.randn(16, 49, 512, device=cuda)
    out = []
    for _ in range(2):
        dec.zero_grad(set_to_none=True)
        decoder_token_logp(dec, mem, ids, END).sum().backward()
        out.append([p.grad.clone() for p in dec.parameters()])
    assert all(torch.equal(a, b) for a, b in zip(*out))


def test_train_pass_dropout_matches_oracle_autograd(cuda):
    """Train mode: the HIP training pass with the counter-based dropout masks (p, seed) against PyTorch
    autograd through the oracle's explicit-op decoder given the same masks (oracle/dropout.py): log-probs
    within 1e-4, every gradient within 1e-3 relative (norm)."""
    from image_caption_amd.train import decoder_param_names, decoder_token_logp
    from oracle import captioner as O
    from oracle import dropout as D

    B, L, S, p, seed = 6, 14, 49, 0.1, 987654321
    torch.manual_seed(3)
    dec = TransformerDecoder(109).to(cuda).train()
    ids = _ids(B, L, 109, 11).to(cuda)
    mem0 = torch.randn(B, S, 512, generator=torch.Generator().manual_seed(2)).to(cuda)
    adv = torch.randn(B, generator=torch.Generator().manual_seed(5)).to(cuda)
    names = decoder_param_names(6)
    params = dict(dec.named_parameters())
    masks = {k: v.to(cuda) for k, v in D.decoder_masks(p, seed, B, L - 1, S).items()}
    sd = {"decoder." + k: v for k, v in params.items()}
    sd["decoder.pos_encoder.pe"] = dec.pos_encoder.pe
    mem = mem0.clone().requires_grad_(True)
    lp_ref = masked_token_logp(O.decoder_forward(sd, ids[:, :-1], mem, True, masks=masks), ids, END)
    (-(adv * lp_ref.sum(1)).mean()).backward()
    g_ref = {k: params[k].grad.clone() for k in names}
    dmem_ref = mem.grad.clone()
    dec.zero_grad(set_to_none=True)

    mem2 = mem0.clone().requires_grad_(True)
    lp = decoder_token_logp(dec, mem2, ids, END, dropout=(p, seed))
    (-(adv * lp.sum(1)).mean()).backward()
    torch.cuda.synchronize()
    assert (lp - lp_ref.detach()).abs().max().item() < 1e-4
    worst = max((_rel(params[k].grad, g_ref[k]), k) for k in names)
    assert worst[0] < 1e-3, worst
    assert _rel(mem2.grad, dmem_ref) < 1e-3
    # the masks are active: another seed gives other log-probs
    lp_other = decoder_token_logp(dec, mem0, ids, END, dropout=(p, seed + 1)).detach()
    assert (lp_other - lp.detach()).abs().max().item() > 1e-2


def test_sampler_dropout_matches_oracle_and_training_pass(cuda):
    """Train-mode sampling (icap_decode_sample_dropout) against the oracle's full-prefix sampler given the
    same masks: identical ids, log-probs within 1e-3; and the HIP training pass with the same (p, seed)
    reproduces the sampler's log-probs - the distribution sampled from is the one differentiated."""
    from image_caption_amd.engine import Engine
    from image_caption_amd.train import decoder_token_logp
    from models.vit_transformer_model import ViTTransformerCaptioning
    from oracle import captioner as O
    from oracle import dropout as D
    from image_caption_amd import weights as W

    B, L, S, p, seed = 8, 20, 196, 0.1, 4242
    sd = W.to_torch(W.vit_state_dict(0))
    eng = Engine(sd, "vit", {}, device=cuda)
    mem = torch.from_numpy(np.random.Generator(np.random.PCG64(9)).standard_normal((B, S, 512)).astype(np.float32))
    uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(12))
    runs = [eng.sample(mem.to(cuda), uni.to(cuda), W.START_TOKEN, W.END_TOKEN, L, dropout=(p, seed)) for _ in range(3)]
    ids, lp = runs[0][0].cpu().long(), runs[0][1].cpu()
    for i2, l2 in runs[1:]:  # eager, capture, replay
        assert torch.equal(i2.cpu().long(), ids) and torch.equal(l2.cpu(), lp)
    masks = D.decoder_masks(p, seed, B, L - 1, S)
    ref_ids, ref_lp = O.sample_with_log_probs(sd, mem, uni, W.START_TOKEN, W.END_TOKEN, L, masks=masks)
    n = ref_ids.shape[1]
    assert torch.equal(ids[:, :n], ref_ids)
    assert (lp[:, : n - 1] - ref_lp).abs().max().item() < 1e-3
    plain, _ = eng.sample(mem.to(cuda), uni.to(cuda), W.START_TOKEN, W.END_TOKEN, L)
    assert not torch.equal(plain.cpu().long(), ids)  # dropout changed the draws
    # the training pass on the sampled ids, same masks
    m = ViTTransformerCaptioning(W.VOCAB_SIZE, pretrained_vit=False)
    m.load_state_dict(sd)
    dec = m.decoder.to(cuda).train()
    with torch.no_grad():
        tp = decoder_token_logp(dec, mem.to(cuda), ids.to(cuda), W.END_TOKEN, dropout=(p, seed)).cpu()
    assert (tp - lp).abs().max().item() < 1e-3

