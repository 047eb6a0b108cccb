"""Round 6: decode kernel durations by decode step (position t0) from a rocprofv3 kernel trace of a bench run: the
last decode of the trace, dec_sa (whose KV history grows with t0) against the others.  Measurement tool.
usage: python tools/r6_dec_by_step.py KERNEL_TRACE.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
sa = [i for i, r in enumerate(rows) if "dec_sa_kernel" in r["Kernel_Name"]]
last = sa[-174:]  # 29 steps x 6 layers
first, end = last[0], last[-1]
per = defaultdict(lambda: defaultdict(list))
k = 0
for r in rows[first:end + 12]:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "dec_sa_kernel" in n:
        t0 = k // 6
        k += 1
    for key in ("dec_sa", "cross_attn", "dec_chain", "dec_ffn", "residual_layernorm", "head_kernel"):
        if key in n:
            per[key][t0].append(d)
for key, d in per.items():
    line = " ".join(f"{sum(v) / len(v):5.1f}" for t, v in sorted(d.items()))
    print(f"{key:20s} {line}")
