"""Drop-in `utils/scst_loss.py` (reference: utils/scst_loss.py): self-critical sequence training.

SCSTLoss.forward = sample captions with their log-probs, greedy baseline via model.generate,
CIDEr-D rewards, advantage = r(sample) - r(greedy), loss = -mean(advantage * sum(log p)).

Changes on the hot path:
  * sampling runs as one batched HIP decode (icap_decode_sample[_dropout]): fp32 fc_out + softmax and an
    inverse-CDF draw on uniforms that are INJECTED (default torch.rand on the images' device),
    replacing torch.multinomial, so CPU and GPU consume identical randomness; in train mode the
    decoder's dropout (0.1 in the reference, :161) is active with counter-based masks of (seed, site,
    layer, image, position, index) (oracle/dropout.py) instead of torch's RNG stream;
  * when autograd is on, the sampled sequence's log-probs are recomputed teacher-forced with their
    backward on HIP (icap_decoder_train_forward / _backward through a torch.autograd.Function, eval-mode
    like the sampler) after the encoder's trainable part in PyTorch (the ViT projection on the HIP
    trunk's output; the Grid tail), so the REINFORCE loss has a gradient;
  * CIDEr-D is image_caption_amd.cider on token ids (pycocoevalcap is absent; parity unpinned); on
    the HIP path both reward sets are scored in one GPU pass (icap_cider_d, cider.hip).
BLEU / combined rewards and MixedLoss are training-only and not provided.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

from image_caption_amd import cider as _cider
from image_caption_amd.train import decoder_dropout, decoder_token_logp, vit_trunk_frozen


def _split(s: str, word2idx: Optional[dict]) -> List:
    words = s.split()
    return [word2idx.get(w, w) for w in words] if word2idx else words


class CiderRewardCalculator:
    """compute_reward(predictions: list[str], references: list[list[str]]) -> list[float]
    (scst_loss:20-54).  Strings are split on whitespace; with `vocab` given, words map to ids."""

    def __init__(self, vocab: Optional[dict] = None):
        self.word2idx = vocab

    def compute_reward(self, predictions, references):
        hyps = [_split(p, self.word2idx) for p in predictions]
        refs = [[_split(r, self.word2idx) for r in (rs if isinstance(rs, list) else [rs])] for rs in references]
        try:
            return list(_cider.cider_d(hyps, refs)[1])
        except Exception as e:  # the reference returns zero rewards on scorer failure (:52-54)
            print(f"CIDEr failed: {e}")
            return [0.0] * len(predictions)

    def compute_reward_ids(self, hyp_ids: Sequence[Sequence[int]], ref_ids: Sequence[Sequence[Sequence[int]]]):
        return list(_cider.cider_d(hyp_ids, ref_ids)[1])


def sample_stop_length(ids: torch.Tensor, end_token: int) -> int:
    """Columns the reference keeps: it breaks right after the step at which every sequence has
    emitted <end> at least once (scst_loss:246-249)."""
    fin = (ids[:, 1:] == end_token).cummax(dim=1).values.all(dim=0)
    if bool(fin.any()):
        return int(torch.nonzero(fin)[0, 0]) + 2
    return ids.shape[1]


def masked_token_logp(logits: torch.Tensor, ids: torch.Tensor, end_token: int) -> torch.Tensor:
    """log p(ids[:, t+1] | prefix) with steps after a sequence's first <end> zeroed (:236-239)."""
    lp = F.log_softmax(logits, dim=-1).gather(2, ids[:, 1:].unsqueeze(2)).squeeze(2)
    ended = (ids[:, 1:] == end_token).long().cumsum(dim=1)
    finished_before = torch.cat([torch.zeros_like(ended[:, :1]), ended[:, :-1]], dim=1) > 0
    return lp.masked_fill(finished_before, 0.0)


class SCSTLoss(nn.Module):
    def __init__(self, reward_type="cider", cider_weight=1.0, bleu_weight=0.0):
        super().__init__()
        if reward_type != "cider":
            raise NotImplementedError("only the CIDEr reward is on the hot path")
        self.reward_calculator = CiderRewardCalculator()

    def forward(self, model, images, references, vocab, device, sample_method="sample", max_len=50,
                uniforms: Optional[torch.Tensor] = None, dropout_seed: Optional[int] = None):
        start, end, pad = vocab["<start>"], vocab["<end>"], vocab["<pad>"]
        self.reward_calculator.word2idx = vocab
        model.train()
        sample_ids, sample_log_probs = self._sample_with_log_probs(model, images, start, end, max_len, device,
                                                                   uniforms, dropout_seed)
        with torch.no_grad():
            greedy_ids = model.generate(images, start, end, max_len, method="greedy")
        refs = [[_split(r, vocab) for r in (rs if isinstance(rs, list) else [rs])] for rs in references]
        if sample_ids.is_cuda and getattr(model, "hip_backend", "torch") != "torch":
            # both reward sets in one GPU CIDEr-D pass over token ids (icap_cider_d)
            B = sample_ids.shape[0]
            rows, off = _cider.pack_references(refs, pad, end, max(vocab.values()) + 1)
            hyp = torch.full((2 * B, max(sample_ids.shape[1], greedy_ids.shape[1])), pad, dtype=torch.int32,
                             device=sample_ids.device)
            hyp[:B, : sample_ids.shape[1]] = sample_ids
            hyp[B:, : greedy_ids.shape[1]] = greedy_ids
            r = _cider.cider_d_device(hyp, rows, off, start, end, pad).to(device=device, dtype=torch.float)
            s_r, g_r = r[:B], r[B:]
        else:
            s_r = self.reward_calculator.compute_reward_ids(
                [_cider.caption_ids(r, start, end, pad) for r in sample_ids.tolist()], refs)
            g_r = self.reward_calculator.compute_reward_ids(
                [_cider.caption_ids(r, start, end, pad) for r in greedy_ids.tolist()], refs)
            s_r = torch.tensor(s_r, device=device, dtype=torch.float)
            g_r = torch.tensor(g_r, device=device, dtype=torch.float)
        adv = s_r - g_r
        loss = -(adv * sample_log_probs.sum(dim=1)).mean()
        return loss, {"sample_reward": s_r.mean().item(), "greedy_reward": g_r.mean().item(),
                      "advantage": adv.mean().item()}

    def _sample_with_log_probs(self, model, images, start_token, end_token, max_len, device,
                               uniforms: Optional[torch.Tensor] = None, dropout_seed: Optional[int] = None):
        """-> (ids (B, L) int64, log_probs (B, L-1)), L per the reference stop rule.  In train mode the HIP
        sampler and the recompute apply the decoder's dropout with the same counter-based masks (seed drawn
        from torch's generator unless given)."""
        B = images.size(0)
        if uniforms is None:
            uniforms = torch.rand(max_len - 1, B, device=images.device)
        if images.is_cuda and getattr(model, "hip_backend", "torch") != "torch":
            eng = model.hip_engine(images.device)
            p = decoder_dropout(model.decoder)
            if p > 0 and not eng.dropout_sampling_ok(max_len):
                # train-mode dropout outside what the fused HIP decode blocks serve (other decoder widths,
                # precision "bf16", max_len > 65): the reference's own PyTorch loop with torch's dropout
                if getattr(model, "hip_backend", "auto") == "hip":
                    raise ValueError("backend='hip': train-mode dropout sampling needs d_model 512, 8 heads, "
                                     "dim_feedforward 2048, a parity precision and max_len <= 65")
                return self._sample_torch(model, images, start_token, end_token, max_len, uniforms)
            if p > 0 and dropout_seed is None:
                dropout_seed = int(torch.randint(0, 2**31 - 1, (1,)).item())
            drop = (p, int(dropout_seed or 0))
            feats = None
            mem = None
            memory_t = None
            want_grad = torch.is_grad_enabled()
            if getattr(model, "_hip_kind", "") == "grid" and model.encoder.cnn.training:
                # the reference encodes once per step, in train mode (scst_loss:161, :213): the trunk's
                # BatchNorm normalises with batch statistics and updates its running statistics ONCE, and the
                # sampled tokens and the differentiated log-probs see the SAME memory (one forward graph).
                # A frozen trunk on 224x224 images runs as the HIP train-mode trunk (icap_encode_grid_train:
                # batch statistics, running statistics updated in place); a trainable one (or other sizes)
                # runs here in PyTorch, once, grad as enabled.  The tail (projection, PE, encoder layers) then
                # runs once in PyTorch in the module's mode - with train-mode dropout its masks are torch's -
                # and its output is both the sampler's memory (detached) and the recompute's (with grad).
                cnn = model.encoder.cnn
                if (tuple(images.shape[1:]) == (3, 224, 224) and 2 <= images.size(0) <= 256
                        and not any(p.requires_grad for p in cnn.parameters())):
                    with torch.no_grad():
                        _, feats = eng.encode_grid_train(images, cnn)
                else:
                    feats = model.encoder.cnn(images.float())
                memory_t = model.encoder.tail(feats)
                mem = memory_t.detach().float().contiguous()
            vfeats = None
            with torch.no_grad():
                if mem is not None:
                    pass  # the train-mode Grid encoder above
                elif getattr(model, "_hip_kind", "") == "grid" and tuple(images.shape[1:]) != (3, 224, 224):
                    mem = model.encoder(images)  # eval trunk, other sizes: torch trunk (+ HIP tail on 7x7)
                elif want_grad and vit_trunk_frozen(model):
                    # the frozen ViT's output too: the recompute below applies only the trainable projection
                    mem, vfeats = eng.encode_vit_features(images)
                    if eng.range_overflowed():  # f16 range guard: bf16x2 re-encode
                        eng = model.hip_engine(images.device, precision="bf16x2")
                        mem, vfeats = eng.encode_vit_features(images)
                else:  # ViT, or a Grid model whose trunk is in eval mode: the whole encoder on HIP
                    eng, mem = model.checked_encode(images)  # f16 range guard: bf16x2 re-encode on overflow
                # stop_early: the decode ends once every row has emitted <end>, as the reference's loop breaks
                # (:246-249) - a trained model's samples end long before max_len
                ids32, logp = eng.sample(mem, uniforms, start_token, end_token, max_len, dropout=drop, stop_early=True)
            ids = ids32.long()
            L = sample_stop_length(ids, end_token)
            ids, logp = ids[:, :L], logp[:, : L - 1]
            if want_grad:
                # the log-probs with a gradient: encoder's trainable part in PyTorch, then the decoder's
                # forward and backward on HIP (icap_decoder_train_*, image_caption_amd/train.py) with the
                # sampler's dropout masks, so the distribution sampled from is the one differentiated
                if vfeats is not None:
                    memory = model.encoder.projection(vfeats)
                elif memory_t is not None:
                    memory = memory_t  # the memory the tokens were sampled from
                else:
                    memory = model.encoder(images)
                logp = decoder_token_logp(model.decoder, memory, ids, end_token, dropout=drop)
            return ids, logp
        return self._sample_torch(model, images, start_token, end_token, max_len, uniforms)

    @staticmethod
    def _sample_torch(model, images, start_token, end_token, max_len, uniforms):
        """PyTorch loop of the reference (:210-254) with the same inverse-CDF draw."""
        B = images.size(0)
        memory = model.encoder(images)
        generated = torch.full((B, 1), start_token, dtype=torch.long, device=images.device)
        finished = torch.zeros(B, dtype=torch.bool, device=images.device)
        out = []
        for step in range(max_len - 1):
            mask = model.decoder.generate_square_subsequent_mask(generated.size(1), images.device)
            logits = model.decoder(generated, memory, tgt_mask=mask)[:, -1, :]
            probs = F.softmax(logits, dim=-1)
            cdf = probs.cumsum(-1)
            nxt = (cdf <= uniforms[step].unsqueeze(-1) * cdf[:, -1:]).sum(-1).clamp_max(logits.shape[-1] - 1)
            lp = F.log_softmax(logits, dim=-1).gather(1, nxt.unsqueeze(1)).squeeze(1)
            out.append(lp.masked_fill(finished, 0.0))
            generated = torch.cat([generated, nxt.unsqueeze(1)], dim=1)
            finished = finished | (nxt == end_token)
            if bool(finished.all()):
                break
        return generated, torch.stack(out, dim=1)

    def _decode_captions(self, caption_ids, idx2word, end_token, pad_token, start_token):
        from models._common import decode_ids

        return decode_ids(caption_ids.cpu(), idx2word, end_token, pad_token, start_token)


def get_reference_captions(caption_ids, vocab):
    """Reference id rows -> [[caption string]] per image (scst_loss:328-354)."""
    from models._common import decode_ids

    idx2word = {i: w for w, i in vocab.items()}
    caps = decode_ids(caption_ids, idx2word, vocab["<end>"], vocab["<pad>"], vocab["<start>"])
    return [[c] for c in caps]
