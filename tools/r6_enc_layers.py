"""Round 6: per-layer encoder kernel durations of one encode in each context of tools/r6_enc_ctx2.py (one-stream
library), from a rocprofv3 kernel trace: encode 5 (L1: after a decode + sync) against encode 25 (L3: after a sync,
following an encode) - the four GEMMs + attention + 2 LayerNorms per layer, in us.  Measurement tool.
usage: python tools/r6_enc_layers.py KERNEL_TRACE.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
im = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"]]
print(f"{len(im)} encodes in the trace")
for label, k in (("L1 (after decode)", 3 + 5), ("L2 (after decode, no sync)", 3 + 15), ("L3 (after encode)", 3 + 25)):
    if k >= len(im):
        continue
    seg = []
    for r in rows[im[k]:]:
        n = r["Kernel_Name"]
        if "gemm_f16p" in n or "enc_attention" in n or "layernorm_kernel" in n:
            seg.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if len(seg) == 12 * 7:
            break
    per = [sum(seg[7 * l:7 * l + 7]) for l in range(12)]
    print(f"{label:28s} layers: " + " ".join(f"{p:6.0f}" for p in per) + f"   total {sum(per):.0f} us")
