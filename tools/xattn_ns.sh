#!/bin/bash
# cross-attention kernel time with one memory plane (bf16) against two (bf16x2): is it byte-bound?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for P in bf16x2 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/xns_$P -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --precision $P > $R/gpurun_out/xns_$P.log 2>&1 || exit 1
  echo "== $P"; grep -h "cross_attn\|chain_dec\|gemm_dec\|dec_self\|residual_layer\|head_kernel" $R/gpurun_out/xns_$P/*kernel_stats.csv | python3 -c '
import sys,csv
for r in csv.reader(sys.stdin):
    print(f"   {r[0].split(\"(\")[0][-40:]:40s} {float(r[3])/1e3:8.2f} us")'
done
