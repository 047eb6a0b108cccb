"""Round 6: effective clock of the encoder GEMMs by layer in two contexts (tools/r6_enc_ctx2.py under rocprofv3 --pmc
GRBM_GUI_ACTIVE --kernel-trace): GRBM_GUI_ACTIVE / 8 XCDs / the dispatch's duration, for encode 8 (L1: after a decode)
and encode 28 (L3: after an encode).  Measurement tool.  usage: python tools/r6_enc_clock.py OUTDIR"""
import csv
import glob
import sys

root = sys.argv[1]
cnt = {}
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            cnt[int(r["Dispatch_Id"])] = float(r["Counter_Value"])
tr = []
for f in glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True):
    tr += list(csv.DictReader(open(f)))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
im = [i for i, r in enumerate(tr) if "im2col" in r["Kernel_Name"]]
print(f"{len(im)} encodes, {len(cnt)} counted dispatches")
for label, k in (("L1 (after decode)", 3 + 5), ("L3 (after encode)", 3 + 25)):
    if k >= len(im):
        continue
    clocks, durs = [], []
    for r in tr[im[k]:]:
        if "gemm_f16p" in r["Kernel_Name"]:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
            g = cnt.get(int(r["Dispatch_Id"]))
            clocks.append(g / 8 / d / 1e9 if g else float("nan"))
            durs.append(d * 1e6)
        if len(clocks) == 48:
            break
    per = [sum(clocks[4 * l:4 * l + 4]) / 4 for l in range(12)]
    dl = [sum(durs[4 * l:4 * l + 4]) for l in range(12)]
    print(f"{label:20s} GHz by layer: " + " ".join(f"{c:.2f}" for c in per))
    print(f"{label:20s} GEMM us by layer: " + " ".join(f"{d:5.0f}" for d in dl))
