#!/bin/bash
# LDS bank conflicts of every kernel of the headline bench (one SQ pass).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/bank -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/bank.log 2>&1 || exit 1
cd $R && python3 - <<'PY'
import csv, glob
from collections import defaultdict
v = defaultdict(lambda: defaultdict(float)); n = defaultdict(lambda: defaultdict(int))
for f in glob.glob("gpurun_out/bank/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:56]
        v[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k in sorted(v, key=lambda k: -v[k].get("SQ_LDS_BANK_CONFLICT", 0)):
    m = {c: v[k][c] / n[k][c] for c in v[k]}
    if m.get("SQ_INSTS_LDS", 0) == 0: continue
    print(f"{k:56s} conflict {m.get('SQ_LDS_BANK_CONFLICT',0):10.3g}  lds_active {m.get('SQ_ACTIVE_INST_LDS',0):10.3g}  lds_wait {m.get('SQ_WAIT_INST_LDS',0):10.3g}  wave_cyc {m.get('SQ_WAVE_CYCLES',0):10.3g}")
PY
