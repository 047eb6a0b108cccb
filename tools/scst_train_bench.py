"""Time the whole SCST training step of the drop-in model (SCSTLoss.forward: HIP sampler + greedy +
GPU CIDEr-D + the teacher-forced recompute; loss.backward(); AdamW step) at config 5's per-rank shape
(B = 128, max_len 30), HIP backend against backend="torch" (the PyTorch modules on the same GPU).
MODEL=grid: the Grid model (train-mode ResNet trunk: icap_encode_grid_train on the HIP backend).
Measurement tool, not product.  usage: [MODEL=vit|grid] python tools/scst_train_bench.py [B] [steps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from image_caption_amd import weights as W
from models import grid_transformer_model, vit_transformer_model
from utils.scst_loss import SCSTLoss

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
vocab = {f"w{i}": i for i in range(W.VOCAB_SIZE)}
vocab.update({"<pad>": 0, "<unk>": 106, "<start>": 107, "<end>": 108})
refs = [[" ".join(f"w{(i * 7 + j) % 100 + 1}" for j in range(3 + i % 9))] for i in range(B)]
imgs = torch.from_numpy(W.synthetic_images(B, seed=5)).to(dev)
for backend in (os.environ.get("BACKENDS", "auto,torch").split(",")):
    if os.environ.get("MODEL", "vit") == "grid":
        m = grid_transformer_model.build_model(W.VOCAB_SIZE, {"pretrained_cnn": False, "backend": backend})
        m.load_state_dict(W.to_torch(W.grid_state_dict(0)))
    else:
        m = vit_transformer_model.build_model(W.VOCAB_SIZE, {"pretrained_vit": False, "backend": backend})
        m.load_state_dict(W.to_torch(W.vit_state_dict(0)))
    m = m.to(dev)
    opt = torch.optim.AdamW([p for p in m.parameters() if p.requires_grad], lr=1e-6)
    loss_fn = SCSTLoss()
    times = []
    for i in range(steps + 2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        loss, info = loss_fn(m, imgs, refs, vocab, dev, max_len=30)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    ms = 1e3 * sum(times[2:]) / steps
    print(f"{os.environ.get('MODEL', 'vit')} backend {backend:5s} B={B}: {ms:8.1f} ms/step  {B / ms * 1e3:8.1f} images/s  loss {loss.item():+.4f}",
          flush=True)
