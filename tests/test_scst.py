"""SCST training step (image_caption_amd.scst) across ranks: world_size 2 over
gloo (the RCCL path's CPU stand-in) must give the same loss terms and DDP-averaged gradients as
one process on the whole batch - global-batch CIDEr-D (ids and references all-gathered) and the
local-mean loss under DDP's gradient average."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from image_caption_amd import weights as W

TOTAL, L = 4, 8
CHECK = ["encoder.projection.weight", "decoder.fc_out.weight", "decoder.embedding.weight",
         "decoder.transformer_decoder.layers.5.linear2.weight"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from models.vit_transformer_model import build_model

    torch.manual_seed(0)
    m = build_model(W.VOCAB_SIZE, {"pretrained_vit": False, "backend": "torch"})
    m.load_state_dict(W.to_torch(W.vit_state_dict(0)))
    m.eval()  # dropout off: the two runs must see the same function
    imgs = torch.from_numpy(W.synthetic_images(TOTAL, seed=4))
    g = torch.Generator().manual_seed(9)
    refs = torch.full((TOTAL, 10), W.PAD_TOKEN, dtype=torch.int32)
    for i in range(TOTAL):
        n = int(torch.randint(3, 8, (1,), generator=g))
        refs[i, 0] = W.START_TOKEN
        refs[i, 1: n + 1] = torch.randint(3, 100, (n,), generator=g, dtype=torch.int32)
        refs[i, n + 1] = W.END_TOKEN
    uni = torch.rand(L - 1, TOTAL, generator=g)
    return m, imgs, refs, uni


def _run(model, imgs, refs, uni, lo, hi, wrap):
    from image_caption_amd.scst import TeacherForcedLogProbs, scst_step
    from models._common import greedy_torch
    from utils.scst_loss import SCSTLoss

    lp = wrap(TeacherForcedLogProbs(model, W.END_TOKEN))

    def sampler(im):
        sid, _ = SCSTLoss._sample_torch(model, im, W.START_TOKEN, W.END_TOKEN, L, uni[:, lo:hi])
        return sid, greedy_torch(model, im, W.START_TOKEN, W.END_TOKEN, L)

    loss, info = scst_step(lp, imgs[lo:hi], refs[lo:hi], sampler, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN,
                           global_batch=TOTAL)
    loss.backward()
    grads = {n: p.grad.detach().clone().numpy() for n, p in model.named_parameters() if n in CHECK}
    return grads, info


def _worker(rank, ws, port, q):
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP

    from image_caption_amd.parallel import shard_bounds

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    model, imgs, refs, uni = _setup()
    lo, hi = shard_bounds(TOTAL, ws, rank)
    grads, info = _run(model, imgs, refs, uni, lo, hi, lambda m: DDP(m))
    if rank == 0:
        q.put((grads, info))
    dist.barrier()
    dist.destroy_process_group()


def test_scst_step_ddp_world2_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, info = q.get(timeout=600)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    torch.set_num_threads(4)
    model, imgs, refs, uni = _setup()
    want, info1 = _run(model, imgs, refs, uni, 0, TOTAL, lambda m: m)
    for k in ("sample_reward", "greedy_reward", "advantage"):
        assert abs(info[k] - info1[k]) < 1e-5, k
    for n in CHECK:
        scale = max(np.abs(want[n]).max(), 1e-12)
        assert np.abs(got[n] - want[n]).max() <= 1e-4 * scale + 1e-7, n
    assert any(np.abs(want[n]).max() > 0 for n in CHECK)  # a non-trivial gradient was compared


@pytest.mark.gpu
def test_scst_rewards_gpu_equal_cpu(cuda):
    """scst.rewards on GPU tensors (icap_cider_d, one pass for both sets) == the CPU ids path."""
    from image_caption_amd.scst import rewards

    g = torch.Generator().manual_seed(1)
    B = 96
    sid = torch.randint(0, 60, (B, 12), generator=g, dtype=torch.int32)
    gid = torch.randint(0, 60, (B, 9), generator=g, dtype=torch.int32)
    sid[:, 0] = gid[:, 0] = W.START_TOKEN
    refs = torch.randint(0, 60, (B, 11), generator=g, dtype=torch.int32)
    refs[:, 0] = W.START_TOKEN
    s_cpu, g_cpu = rewards(sid, gid, refs, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN)
    s_gpu, g_gpu = rewards(sid.to(cuda), gid.to(cuda), refs.to(cuda), W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN)
    assert torch.allclose(s_gpu.cpu(), s_cpu, atol=1e-6) and torch.allclose(g_gpu.cpu(), g_cpu, atol=1e-6)
    assert s_cpu.abs().sum() > 0


@pytest.mark.gpu
def test_concurrent_sample_and_greedy_equal_sequential(cuda):
    """scst.sample_and_greedy (both decode graphs replayed concurrently on two streams, one workspace
    per decode mode) returns exactly what the two sequential calls return, on every replay."""
    from image_caption_amd.engine import Engine
    from image_caption_amd.scst import sample_and_greedy

    eng = Engine(W.to_torch(W.vit_state_dict(0)), "vit", {}, device=cuda)
    g = torch.Generator().manual_seed(2)
    mem = torch.randn(96, 49, 512, generator=g).to(cuda)
    uni = torch.rand(11, 96, generator=g).to(cuda)
    ref_s, ref_lp = eng.sample(mem, uni, W.START_TOKEN, W.END_TOKEN, 12)
    ref_g, _ = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, 12)
    for _ in range(4):  # eager, capture, replays
        sid, lp, gid = sample_and_greedy(eng, mem, uni, W.START_TOKEN, W.END_TOKEN, 12)
        torch.cuda.synchronize()
        assert torch.equal(sid, ref_s) and torch.equal(lp, ref_lp) and torch.equal(gid, ref_g)


def test_teacher_forced_dropout_follows_sampler_seed():
    """The DDP SCST recompute takes the sampler's dropout seed (scst_step(dropout_seed=...)) through a DDP-style
    wrapper and applies (p, seed) only in train mode - the masks sample_and_greedy(dropout=(p, seed)) drew - for THAT
    call only: the module's own setting is back afterwards (a later call without a seed never reuses a stale one)."""
    from image_caption_amd.scst import TeacherForcedLogProbs, scst_step

    model, imgs, refs, _ = _setup()
    lp = TeacherForcedLogProbs(model, W.END_TOKEN)
    assert lp.dropout() == (0.0, 0)

    class Wrap(torch.nn.Module):
        def __init__(self, m):
            super().__init__()
            self.module = m

        def forward(self, *a):
            seen.append(self.module.dropout())
            return self.module(*a)

    def sampler(im):
        ids = torch.full((im.shape[0], 3), W.END_TOKEN, dtype=torch.int64)
        ids[:, 0] = W.START_TOKEN
        return ids, ids

    seen = []
    scst_step(Wrap(lp), imgs[:2], refs[:2], sampler, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN, dropout_seed=77)
    assert seen[-1] == (0.0, 0)  # eval mode: no masks
    assert lp.dropout_seed is None  # restored
    model.train()
    try:
        scst_step(Wrap(lp), imgs[:2], refs[:2], sampler, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN, dropout_seed=77)
        p, seed = seen[-1]
        assert seed == 77 and p > 0.0
        assert lp.dropout_seed is None and lp.dropout() == (0.0, 0)
        scst_step(Wrap(lp), imgs[:2], refs[:2], sampler, W.START_TOKEN, W.END_TOKEN, W.PAD_TOKEN)
        assert seen[-1] == (0.0, 0)  # no seed given: no stale masks
    finally:
        model.eval()