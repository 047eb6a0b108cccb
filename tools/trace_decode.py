"""Summarise a rocprofv3 kernel trace of bench.py: per-kernel totals and the per-position
durations of one decoder layer step (13 dispatches) in the last decode loop."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
name = lambda r: r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot = defaultdict(float)
cnt = defaultdict(int)
for r in rows:
    tot[name(r)] += dur(r)
    cnt[name(r)] += 1
for k in sorted(tot, key=lambda k: -tot[k])[:14]:
    print(f"{k:50s} n={cnt[k]:6d} total {tot[k]/1e3:9.2f} ms avg {tot[k]/cnt[k]:8.2f} us")
last = max(i for i, r in enumerate(rows) if "enc_attention" in r["Kernel_Name"])
dec = rows[last + 1:]
start = next(i for i, r in enumerate(dec) if "head_kernel" in r["Kernel_Name"]) + 1
print("--- one decode layer-step (positions) ---")
for i in range(start, start + 14):
    r = dec[i]
    gap = (int(r["Start_Timestamp"]) - int(dec[i - 1]["End_Timestamp"])) / 1e3
    print(f"{name(r):50s} {dur(r):8.2f} us  gap {gap:6.2f} us  grid {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}")
t0 = int(dec[0]["Start_Timestamp"]); t1 = int(dec[-1]["End_Timestamp"])
busy = sum(dur(r) for r in dec)
print(f"decode region: wall {(t1-t0)/1e3:.1f} us, busy {busy:.1f} us, dispatches {len(dec)}")
