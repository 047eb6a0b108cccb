"""Per-convolution time of the last ResNet trunk pass in a rocprofv3 kernel trace (csv or rocpd db):
maps the trunk GEMM launches in order onto stem, [downsample] conv1 conv2 conv3 per block.
usage: python tools/trunk_breakdown.py TRACE(.csv|.db)"""
import csv
import sqlite3
import sys

path = sys.argv[1]
if path.endswith(".db"):
    c = sqlite3.connect(path)
    rows = [(r[0], int(r[1]), int(r[2])) for r in c.execute("select name,start,end from kernels order by start")]
else:
    with open(path) as f:
        rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)),
                      key=lambda r: r[1])
first = [i for i, r in enumerate(rows) if "image_nhwc4" in r[0] or "stem_im2col" in r[0]]
names = ["stem"]
for st, nb in enumerate([3, 4, 23, 3]):
    for j in range(nb):
        names += ([f"l{st + 1}ds"] if j == 0 else []) + [f"l{st + 1}c1", f"l{st + 1}c2", f"l{st + 1}c3"]
agg, gi = {}, 0
for r in rows[first[-1]:]:
    n = r[0].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if "layernorm" in n or "enc_attention" in n:
        break
    d = (r[2] - r[1]) / 1e3
    if "gemm" in n or "conv_rmw" in n:
        key = f"{names[gi] if gi < len(names) else 'tail'} {n[:26]}"
        gi += 1
    else:
        key = n
    a = agg.setdefault(key, [0.0, 0])
    a[0] += d
    a[1] += 1
tot = 0.0
for k, v in agg.items():
    print(f"{k:42s} n={v[1]:3d} us={v[0]:9.1f} avg={v[0] / v[1]:8.1f}")
    tot += v[0]
print(f"trunk total us {tot:.1f}")
