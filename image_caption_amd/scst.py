"""Data-parallel SCST training step: HIP sampling + greedy baseline, GPU CIDEr-D
over the GLOBAL batch, teacher-forced log-prob recompute with autograd, DDP gradient all-reduce.

Per rank r of R (one process per GPU, torch.distributed over RCCL; gloo in the CPU tests):
  1. sample ids with log-probs and greedy ids for the local shard (icap_decode_sample /
     icap_decode_greedy on the HIP path, any `sampler` callable otherwise);
  2. all-gather both id sets and the local reference rows (one reference caption per image, as
     get_reference_captions builds them, utils/scst_loss.py:328-354) - the reference computes
     CIDEr's document frequency over the whole batch it scores (scst_loss.py:179-180);
  3. CIDEr-D rewards of both sets over the global batch (icap_cider_d on a GPU, the ids
     restatement on a CPU), advantage = r(sample) - r(greedy), local slice;
  4. teacher-forced recompute of the local samples' token log-probs (on a GPU: the HIP decoder training
     pass, image_caption_amd/train.py; on a CPU: the PyTorch modules) inside a DistributedDataParallel wrapper, loss = -mean(adv * sum_t log p)
     (scst_loss.py:190-191) over the local shard: DDP's gradient average over ranks equals the
     gradient of the global-batch mean.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist
import torch.nn as nn

from . import cider as C
from .parallel import gather_rows


class TeacherForcedLogProbs(nn.Module):
    """forward(images, ids) -> (B, L-1) log p(ids[:, t+1] | ids[:, :t+1], image), zeroed after a
    row's first <end> (the masked_fill of the reference sampler, scst_loss.py:236-239).

    Dropout: `dropout_seed` set and the model in train mode -> the HIP recompute applies the decoder's dropout with
    the counter-based masks of (p, dropout_seed) - the masks `sample_and_greedy(..., dropout=(p, seed))` sampled
    with, as SCSTLoss does on one GPU; `dropout_seed` None -> eval-mode semantics on the HIP path (no dropout,
    matching a sampler without dropout)."""

    def __init__(self, model: nn.Module, end_token: int, dropout_seed: Optional[int] = None):
        super().__init__()
        self.model = model
        self.end_token = end_token
        self.dropout_seed = dropout_seed

    def dropout(self) -> Tuple[float, int]:
        """(p, seed) of the train-mode masks shared with the sampler, or (0, 0)."""
        from .train import decoder_dropout

        if self.dropout_seed is None or not self.model.training:
            return (0.0, 0)
        return (decoder_dropout(self.model.decoder), int(self.dropout_seed))

    def forward(self, images: torch.Tensor, ids: torch.Tensor) -> torch.Tensor:
        from utils.scst_loss import masked_token_logp

        if images.is_cuda and getattr(self.model, "hip_backend", "torch") != "torch":
            # HIP decoder forward + backward (train.py); the encoder's trainable part in PyTorch
            from .train import decoder_token_logp, hip_memory_with_grad

            return decoder_token_logp(self.model.decoder, hip_memory_with_grad(self.model, images), ids,
                                      self.end_token, dropout=self.dropout())
        memory = self.model.encoder(images)
        L = ids.shape[1]
        mask = self.model.decoder.generate_square_subsequent_mask(L - 1, images.device)
        logits = self.model.decoder(ids[:, :-1], memory, tgt_mask=mask)
        return masked_token_logp(logits, ids, self.end_token)


_STREAMS = {}


def sample_and_greedy(eng, memory: torch.Tensor, uniforms: torch.Tensor, start: int, end: int, max_len: int,
                      dropout: Optional[Tuple[float, int]] = None):
    """The SCST step's two decodes of one memory, the sampled one (icap_decode_sample, or with dropout = (p, seed)
    icap_decode_sample_dropout: the train-mode masks TeacherForcedLogProbs(dropout_seed=seed) recomputes with) and the
    greedy baseline (icap_decode_greedy, eval mode as the reference's generate), replayed CONCURRENTLY on two streams:
    each decode mode owns its workspace and captured graph, and both are latency-bound chains of small kernels that
    leave most CUs idle.  Returns (sample_ids, sample_logp, greedy_ids) ready on the current stream."""
    dev = memory.device
    cur = torch.cuda.current_stream(dev)
    if dev not in _STREAMS:
        _STREAMS[dev] = (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
    s1, s2 = _STREAMS[dev]
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        sid, lp = eng.sample(memory, uniforms, start, end, max_len, dropout=dropout)
    with torch.cuda.stream(s2):
        gid, _ = eng.greedy_raw(memory, start, end, max_len)
    for t, st in ((memory, s1), (memory, s2), (uniforms, s1)):
        t.record_stream(st)
    cur.wait_stream(s1)
    cur.wait_stream(s2)
    for t in (sid, lp, gid):
        t.record_stream(cur)
    return sid, lp, gid


def _pad_cols(x: torch.Tensor, L: int, value: int) -> torch.Tensor:
    if x.shape[1] >= L:
        return x
    return torch.cat([x, torch.full((x.shape[0], L - x.shape[1]), value, dtype=x.dtype, device=x.device)], 1)


def _gather_padded(x: torch.Tensor, total: int, value: int) -> torch.Tensor:
    """all-gather rows of possibly different widths per rank (pads to the global max width)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return x
    w = torch.tensor([x.shape[1]], device=x.device)
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    return gather_rows(_pad_cols(x, int(w.item()), value).contiguous(), total)


def rewards(sample_ids: torch.Tensor, greedy_ids: torch.Tensor, ref_rows: torch.Tensor, start: int, end: int,
            pad: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """CIDEr-D of both id sets (global batch, one reference row per image) -> float32 (B,), (B,)."""
    B = sample_ids.shape[0]
    L = max(sample_ids.shape[1], greedy_ids.shape[1])
    hyp = torch.cat([_pad_cols(sample_ids, L, pad), _pad_cols(greedy_ids, L, pad)], 0)
    off = torch.arange(B + 1, dtype=torch.int32)
    if hyp.is_cuda:
        r = C.cider_d_device(hyp, ref_rows, off, start, end, pad).float()
    else:
        refs = [[C.caption_ids(row, start, end, pad)] for row in ref_rows.tolist()]
        hs = [C.caption_ids(row, start, end, pad) for row in hyp.tolist()]
        r = torch.tensor(C.cider_d(hs[:B], refs)[1] + C.cider_d(hs[B:], refs)[1], dtype=torch.float32)
    return r[:B].to(sample_ids.device), r[B:].to(sample_ids.device)


def scst_step(lp_module: nn.Module, images: torch.Tensor, ref_rows: torch.Tensor,
              sampler: Callable[[torch.Tensor], Tuple[torch.Tensor, torch.Tensor]], start: int, end: int, pad: int,
              global_batch: Optional[int] = None, dropout_seed: Optional[int] = None) -> Tuple[torch.Tensor, dict]:
    """One SCST loss on the local shard.  lp_module: TeacherForcedLogProbs, DDP-wrapped when R > 1;
    ref_rows (B_local, Lr) raw id rows; sampler(images) -> (sample_ids, greedy_ids) for the shard.
    dropout_seed: the seed the sampler drew its train-mode dropout masks with (sample_and_greedy(...,
    dropout=(p, seed))); the teacher-forced recompute then applies the same masks (scst_loss.py:114-184 on one
    GPU).  The seed applies to THIS call only (the module's own setting is restored on return); None keeps the
    module's own setting for the call.
    Returns (loss, info); the caller runs loss.backward() (DDP all-reduces) and the optimizer."""
    inner = getattr(lp_module, "module", lp_module)
    saved = getattr(inner, "dropout_seed", None)
    if dropout_seed is not None:
        inner.dropout_seed = int(dropout_seed)
    try:
        return _scst_step(lp_module, images, ref_rows, sampler, start, end, pad, global_batch)
    finally:
        inner.dropout_seed = saved


def _scst_step(lp_module, images, ref_rows, sampler, start, end, pad, global_batch):
    B = images.shape[0]
    total = global_batch or B
    with torch.no_grad():
        sid, gid = sampler(images)
    g_sid = _gather_padded(sid, total, pad)
    g_gid = _gather_padded(gid, total, pad)
    g_ref = _gather_padded(ref_rows.to(sid.device), total, pad)
    s_r, g_r = rewards(g_sid, g_gid, g_ref, start, end, pad)
    adv = s_r - g_r
    rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    lo = sum(_shard_sizes(total)[:rank])
    adv_local = adv[lo: lo + B]
    lp = lp_module(images, sid)
    loss = -(adv_local.to(lp.device) * lp.sum(dim=1)).mean()
    return loss, {"sample_reward": s_r.mean().item(), "greedy_reward": g_r.mean().item(),
                  "advantage": adv.mean().item()}


def _shard_sizes(total: int):
    from .parallel import shard_bounds

    R = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    return [shard_bounds(total, R, r)[1] - shard_bounds(total, R, r)[0] for r in range(R)]
