"""Round 6: what the decode's residual LayerNorm gains from fewer split-K slabs - the bound on
halving dec_ffn's 16 hidden-slice slabs to 8 (or dec_sa's 8 head slabs to 4).  At B = 256 rows, 200 launches of
icap_op_residual_layernorm per slab count captured in one hipGraph (back-to-back nodes, as in the decode graph) and
replayed; prints the per-node time for nparts = 16, 8, 4.  Measurement tool.
usage: python tools/r6_rln_slabs.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import _lib as L

lib = L.load()
dev = torch.device("cuda", 0)
rows, N = 256, 200
g = torch.Generator(device="cpu").manual_seed(1)
x = torch.randn(rows, 512, generator=g).to(dev)
parts = (torch.randn(16, rows, 512, generator=g) * 0.3).to(dev)
bias, w, b = (torch.randn(512, generator=g).to(dev) for _ in range(3))
out = torch.empty(2, rows, 512, device=dev, dtype=torch.bfloat16)
seed = torch.zeros(1, dtype=torch.int32, device=dev)


def launch(nparts):
    L.check(lib.icap_op_residual_layernorm(x.data_ptr(), rows, parts.data_ptr(), nparts, rows * 512, bias.data_ptr(),
                                           w.data_ptr(), b.data_ptr(), out.data_ptr(), rows * 512, 0.0,
                                           seed.data_ptr(), 0, 0, 0, L.stream_ptr()), "rln")


for nparts in (16, 8, 4, 16, 8, 4):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        launch(nparts)  # warm (attributes, code object)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for _ in range(N):
            launch(nparts)
    graph.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        graph.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"nparts {nparts:2d}: {e0.elapsed_time(e1) * 1e3 / (5 * N):6.2f} us per graph node "
          f"(slab bytes per launch {nparts * rows * 512 * 4 / 1e6:.1f} MB)", flush=True)
