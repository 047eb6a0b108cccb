"""Per-kernel, per-launch HBM-side traffic from rocprofv3 --pmc passes (FETCH_SIZE / WRITE_SIZE), with
the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE counts 64 B per 128-B request of a wide
coalesced read, so it is doubled; WRITE_SIZE is taken as is.  Units: both counters report KiB.
Prints JSON {kernel: {launches, fetch_bytes, write_bytes, traffic_bytes (per launch means)}}."""
import csv, glob, json, sys
from collections import defaultdict

root = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for k, c in acc.items():
    if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        continue
    fetch = 2 * 1024 * sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
    write = 1024 * sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
    row = {"launches": len(c["FETCH_SIZE"]), "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
        busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / len(c["SQ_VALU_MFMA_BUSY_CYCLES"])
        gui = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"])
        # SQ_VALU_MFMA_BUSY_CYCLES sums over SIMDs (256 CUs x 4); GRBM_GUI_ACTIVE over the 8 XCDs
        row["mfma_busy"] = busy / (gui / 8 * 1024) if gui else None
    out[k] = row
json.dump(out, sys.stdout, indent=1, sort_keys=True)
