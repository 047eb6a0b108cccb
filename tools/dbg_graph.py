import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import numpy as np, torch
from image_caption_amd import weights as W
from image_caption_amd.engine import Engine
cuda = torch.device("cuda", 0)
sd = W.to_torch(W.vit_state_dict(0))
B, L = int(sys.argv[1]), 12
mem = torch.from_numpy(np.random.Generator(np.random.PCG64(21)).standard_normal((B, 49, 512)).astype(np.float32)).to(cuda)
uni = torch.rand(L - 1, B, generator=torch.Generator().manual_seed(3)).to(cuda)
os.environ["ICAP_DEC_BRANCHES"] = sys.argv[2]
eng = Engine(sd, "vit", {}, device=cuda)
runs = []
for it in range(3):
    ids, lg = eng.greedy_raw(mem, W.START_TOKEN, W.END_TOKEN, L, want_logits=True)
    sid, lp = eng.sample(mem, uni, W.START_TOKEN, W.END_TOKEN, L)
    torch.cuda.synchronize()
    runs.append((ids.cpu(), lg.cpu(), sid.cpu(), lp.cpu()))
names = ["ids", "logits", "sample_ids", "logp"]
for it in (1, 2):
    for n, a, b in zip(names, runs[it], runs[0]):
        if not torch.equal(a, b):
            d = (a.float() - b.float()).abs()
            idx = torch.nonzero(d)[:5].tolist()
            print(f"B={B} br={sys.argv[2]} run{it} vs run0: {n} differs: max {d.max().item():.3e} at {idx}  count {int((d>0).sum())}")
print("done", B, sys.argv[2])
