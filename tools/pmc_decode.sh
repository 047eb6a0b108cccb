#!/bin/bash
# PMC passes over the decode kernels (1 decode chain): HBM-side fetch, L2 hit/miss, TA busy.
# usage: bash tools/pmc_decode.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dec}
OUT=gpurun_out/r2/pmcd_$TAG
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --decode-chains 1 > $OUT/p$i.log 2>&1 || exit 1
done
python3 - $OUT <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items()):
    if not any(x in k for x in ("dec_", "chain", "cross", "residual", "head")):
        continue
    s = {n: sum(v) / len(v) for n, v in c.items()}
    hit, miss = s.get("TCC_HIT_sum", 0), s.get("TCC_MISS_sum", 0)
    print(f"{k[:40]:40s} n={len(c.get('FETCH_SIZE', [])):5d} fetchMB={2*s.get('FETCH_SIZE',0)/1024:8.2f} "
          f"L2hit={hit/max(hit+miss,1):.3f} L2req={hit+miss:10.0f} tcp_tcc_rd={s.get('TCP_TCC_READ_REQ_sum',0):10.0f} gui={s.get('GRBM_GUI_ACTIVE',0):8.0f}")
PY
