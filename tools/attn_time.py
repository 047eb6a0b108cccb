"""Time the f16 ViT encoder attention op (icap_op_enc_attention_hm, head-major qkv) at B = 256, N = 197, H = 12 with
the tools build; the form / ablation is chosen by the tools knobs in the environment (ICAP_ENC_ATTN16_FULL,
ICAP_EAF_ABL).  usage: python tools/attn_time.py TAG"""
import sys

import torch

from image_caption_amd import _lib as L

lib = L.load("tools/libicap_tools.so")
B, N, H = 256, 197, 12
dev = torch.device("cuda:0")
qkv = (torch.randn(B, 3, H, N, 64, device=dev) * 1.5).to(torch.float16)
out = torch.zeros(B * N, H * 64, device=dev, dtype=torch.float16)
s = L.stream_ptr()
for _ in range(5):
    L.check(lib.icap_op_enc_attention_hm(qkv.data_ptr(), B, N, H, out.data_ptr(), s), "attn")
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
reps = 50
a.record()
for _ in range(reps):
    L.check(lib.icap_op_enc_attention_hm(qkv.data_ptr(), B, N, H, out.data_ptr(), s), "attn")
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) * 1e3 / reps
print(f"{sys.argv[1] if len(sys.argv) > 1 else ''}: {us:.1f} us per launch ({310e6 / (us * 1e-6) / 1e12:.2f} TB/s of "
      f"q|k|v + out)")
