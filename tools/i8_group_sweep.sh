#!/bin/bash
# i8 GEMM raster sweep (ICAP_I8_GROUP) + one PMC pass of L2 hit/miss over the shape timer.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for G in 0 2 4 8 16; do
  echo "== G=$G"; ICAP_I8_GROUP=$G timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" || exit 1
done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_l2 -o run -- python3 tools/gemm_shapes.py 3 > gpurun_out/pmc_l2.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_l2 2>&1 | head -40
