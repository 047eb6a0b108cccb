#!/bin/bash
# Round 6: name hipBLASLt's kernels on the four ViT GEMM shapes (kernel trace + stats), then their fetched /
# written bytes (one PMC pass each).  usage: bash tools/r6_blaslt.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6/blaslt; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 tools/r6_blaslt_trace.py 5 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
cat $O/tr.log | grep TF/s
cp $(find $O/tr -name "*kernel_stats.csv" | head -1) $O/kernel_stats.csv
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCP_TOTAL_CACHE_ACCESSES_sum TA_BUSY_avr GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 tools/r6_blaslt_trace.py 2 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 tools/pmc_traffic.py $O > $O/traffic.json
python3 - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/r6/blaslt/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:120]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    print(k, {n: sum(v) / len(v) for n, v in c.items()})
PY
find $O -name "*counter_collection.csv" -delete
