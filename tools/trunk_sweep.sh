#!/bin/bash
# Trunk tile-class sweep: encode-only kernel traces with the conv GEMM class forced (0 = default rule).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for f in ${CLASSES:-0 256 128 64}; do
  ICAP_CONV_CLASS=$f timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/sw_$f -o run -- python3 $R/tools/encode_grid.py 2 256 > $R/gpurun_out/sw_$f.log 2>&1 || exit $?
  tail -1 $R/gpurun_out/sw_$f.log
  python3 $R/tools/trunk_breakdown.py $R/gpurun_out/sw_$f/run_kernel_trace.csv > $R/gpurun_out/sw_$f.txt
done
