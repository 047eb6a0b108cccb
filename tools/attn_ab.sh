#!/bin/bash
# encoder attention A/B: kernel stats of the ViT encoder with each env setting given as an argument
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/at_$i -o run -- python3 $R/tools/encode_grid.py 3 256 vit > $R/gpurun_out/at_$i.log 2>&1 || exit $?
  echo "[$cfg] $(tail -1 $R/gpurun_out/at_$i.log)"
  python3 - "$R/gpurun_out/at_$i/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    if "attention" in n or "gemm_256" in n or "layernorm" in n:
        print(f"   {n[:48]:48s} {r['Calls']:>5s} {float(r['AverageNs']) / 1e3:8.1f} us")
PY
done
