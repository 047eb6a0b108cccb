"""Data parallelism over images: one process per GPU, contiguous shards of the batch, weights
replicated, no collective inside the decode loop, and ONE all-gather of the int32 token ids
(RCCL over xGMI when the process group is "nccl") after it.  SURVEY.md §8(e).

The reference has no distributed code; what must be preserved is `_greedy_search`'s
batch-global stop rule (vit:321-323): the output length is 1 + the first step at which EVERY
image of the whole batch emitted <end>.  Every rank runs the fixed max_len-1 steps on its shard,
the gathered ids give every rank the global batch, and `apply_stop_rule` on them reproduces the
single-process result exactly (images are independent in the decode).
"""
from __future__ import annotations

import os
from typing import Tuple

import torch
import torch.distributed as dist


def world() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment (1 process = defaults)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def init(backend: str | None = None) -> Tuple[int, int, int]:
    rank, ws, local = world()
    if ws > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=ws, **kw)
    return rank, ws, local


def shard_bounds(total: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous shard [start, end) of `total` images for `rank` (sizes differ by at most 1)."""
    base, rem = divmod(total, world_size)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_rows(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """All-gather the row shards of every rank (contiguous `shard_bounds` layout) into the full
    (total, ...) tensor on every rank.  Shards are padded to equal size for the collective."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return local
    ws = dist.get_world_size(group)
    per = -(-total // ws)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = [torch.empty_like(pad) for _ in range(ws)]
    dist.all_gather(out, pad, group=group)
    rows = []
    for r in range(ws):
        s, e = shard_bounds(total, ws, r)
        rows.append(out[r][: e - s])
    return torch.cat(rows, 0)
