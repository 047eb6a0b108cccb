"""Emulate candidate GPU numerics on CPU and count greedy-token divergences vs fp32.

Modes: fp32 (oracle), bf16 (GEMM/attention operands rounded to bf16, fp32 accumulate),
bf16x2 (activation operand split hi+lo bf16, weights bf16-exact; attention 3-term split),
mixed (bf16 encoder, bf16x2 decoder).  Used once to choose the default precision mode
(DESIGN.md §Numerics); not part of the product or the tests.
"""
import sys, math, time
sys.path.insert(0, "/root/repo")
import torch
from image_caption_amd import weights as W
from oracle import captioner as O

torch.set_num_threads(8)
bf = lambda x: x.to(torch.bfloat16).float()

def split_mm(a, b_t, split_b):
    ah = bf(a); al = bf(a - ah)
    if not split_b:
        return ah @ b_t + al @ b_t
    bh = bf(b_t); bl = bf(b_t - bh)
    return ah @ bh + al @ bh + ah @ bl

MODE = {"enc": "fp32", "dec": "fp32"}
CUR = ["enc"]

def mm(a, b_t, act_both=False):
    m = MODE[CUR[0]]
    if m == "fp32":
        return a @ b_t
    if m == "bf16":
        return bf(a) @ bf(b_t)
    return split_mm(a, b_t, act_both)

def linear(x, w, b):
    y = mm(x, w.t())
    return y + b if b is not None else y

def mha(q_in, kv_in, in_w, in_b, out_w, out_b, nhead, causal, key_pad=None):
    B, T, D = q_in.shape; S = kv_in.shape[1]; hd = D // nhead
    q = linear(q_in, in_w[:D], in_b[:D]); k = linear(kv_in, in_w[D:2*D], in_b[D:2*D]); v = linear(kv_in, in_w[2*D:], in_b[2*D:])
    q = q.view(B, T, nhead, hd).transpose(1, 2); k = k.view(B, S, nhead, hd).transpose(1, 2); v = v.view(B, S, nhead, hd).transpose(1, 2)
    s = mm(q, k.transpose(-1, -2), True) / math.sqrt(hd)
    if causal:
        s = s.masked_fill(torch.ones(T, S, dtype=torch.bool).triu(1 + S - T), float("-inf"))
    p = torch.softmax(s, -1)
    o = mm(p, v, True).transpose(1, 2).reshape(B, T, D)
    return linear(o, out_w, out_b)

O.linear = linear; O.mha = mha

def run(sd, img, enc, dec, L=30):
    MODE["enc"], MODE["dec"] = enc, dec
    with torch.no_grad():
        CUR[0] = "enc"; mem = O.vit_encode(sd, img)
        CUR[0] = "dec"; ids, tr = O.greedy_from_memory(sd, mem, 107, 108, L, return_trace=True)
    return mem, ids, tr

if __name__ == "__main__":
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    sd = W.to_torch(W.vit_state_dict(0))
    img = torch.from_numpy(W.synthetic_images(B, seed=1))
    t = time.time(); mem0, ids0, tr0 = run(sd, img, "fp32", "fp32"); print("fp32", time.time() - t)
    marg = O.top2_margin(tr0)
    print("min margin", marg.min().item(), "frac<1e-3", (marg < 1e-3).float().mean().item())
    modes = [tuple(m.split("/")) for m in sys.argv[2].split(",")] if len(sys.argv) > 2 else \
        ([("bf16x2", "bf16x2")] if B > 16 else [("bf16", "bf16"), ("bf16", "bf16x2"), ("bf16x2", "bf16x2")])
    for enc, dec in modes:
        mem, ids, tr = run(sd, img, enc, dec)
        # teacher-forced first-step error
        dl = (tr[0] - tr0[0]).abs().max().item()
        dm = (mem - mem0).abs().max().item()
        nseq = (ids.shape != ids0.shape) or None
        L = min(ids.shape[1], ids0.shape[1])
        diff = (ids[:, :L] != ids0[:, :L])
        print(f"{enc:7s}/{dec:7s} mem err {dm:.2e} step0 logit err {dl:.2e} tokens diff {int(diff.sum())}/{diff.numel()} seqs diff {int(diff.any(1).sum())}/{B}")
