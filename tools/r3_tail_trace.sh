#!/bin/bash
# Round 3: kernel trace of one Grid bench pass; prints the launches between the trunk's end and the first decode step
# (the encoder tail) with durations and grid sizes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tt -o run -- python3 bench.py --model grid --steps 1 --warmup 1 --no-cpu-baseline > /dev/null 2>&1 || exit 1
f=$(find $O/tt -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY' > $O/tail_trace.txt
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = [i for i, r in enumerate(rows) if "f16planes_to_bf16" in r["Kernel_Name"]][-1]
for r in rows[last:last + 60]:
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    print(f"{d:8.1f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', '?')):>8}  {n[:90]}")
    if "dec_sa" in n or "head_kernel" in n:
        break
PY
rm -rf $O/tt
cat $O/tail_trace.txt
