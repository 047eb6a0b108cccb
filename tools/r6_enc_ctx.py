"""Round 6: per-kernel durations of the encoder in two contexts, from a rocprofv3 kernel trace of tools/r6_enc_time.py:
the last of the 20 back-to-back encodes against the last bench-like step's encode (after a decode and a host sync).
Measurement tool.  usage: python tools/r6_enc_ctx.py KERNEL_TRACE.csv"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
im = [i for i, r in enumerate(rows) if "im2col" in r["Kernel_Name"]]
dec = [i for i, r in enumerate(rows) if "head_kernel" in r["Kernel_Name"]]


def encode_at(i0):
    """kernels of the encode starting at row i0 up to the next decode kernel or next encode's first im2col pair"""
    out = []
    for r in rows[i0:]:
        n = r["Kernel_Name"]
        if any(k in n for k in ("dec_sa", "cross_attn", "head_kernel")):
            break
        out.append(r)
    return out


# the 20 back-to-back encodes come before the first decode of the bench-like loop's warm-up greedy calls
first_dec = dec[0]
b2b = [i for i in im if i < first_dec]
# the im2col rows of one encode: 1 (one stream) or 2 (two halves); the last back-to-back encode
per = 2 if len(b2b) >= 2 and int(rows[b2b[-1]]["Start_Timestamp"]) - int(rows[b2b[-2]]["Start_Timestamp"]) < 1e6 else 1
ctx = {"back-to-back": b2b[-per], "after decode": [i for i in im if i > dec[-2]][0]}
for name, i0 in ctx.items():
    seg = encode_at(i0)
    agg = defaultdict(float)
    for r in seg:
        agg[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[:40]] += \
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    span = (max(int(r["End_Timestamp"]) for r in seg) - int(seg[0]["Start_Timestamp"])) / 1e3
    print(f"== {name}: {len(seg)} kernels, span {span:.1f} us")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1])[:6]:
        print(f"   {k:42s} {v:9.1f} us")
