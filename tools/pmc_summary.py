"""Summarise rocprofv3 --pmc passes (counter_collection.csv files under DIR): per kernel, the mean
per-dispatch value of every counter, plus derived ratios."""
import csv, glob, sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    if "copyBuffer" in k or "elementwise" in k or "reduce" in k or "distribution" in k:
        continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(k)
    for n in sorted(m):
        print(f"   {n:28s} {m[n]:16.4g}")
    if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
        wc = m["SQ_WAVE_CYCLES"]
        print(f"   wait_any {m.get('SQ_WAIT_ANY',0)/wc:.3f}  wait_inst {m.get('SQ_WAIT_INST_ANY',0)/wc:.3f}  "
              f"active {m.get('SQ_ACTIVE_INST_ANY',0)/wc:.3f}")
    if "TCC_HIT_sum" in m:
        print(f"   L2 hit rate {m['TCC_HIT_sum'] / max(1, m['TCC_HIT_sum'] + m['TCC_MISS_sum']):.3f}")
    if "FETCH_SIZE" in m:
        print(f"   HBM-side read bytes (FETCH_SIZE x 2, gfx950 correction, KiB units) {2 * m['FETCH_SIZE'] * 1024 / 1e6:.1f} MB")
    if "WRITE_SIZE" in m:
        print(f"   write bytes {m['WRITE_SIZE'] * 1024 / 1e6:.1f} MB")
