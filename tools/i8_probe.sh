#!/bin/bash
# i8 GEMM: full vs staging-only (ICAP_I8_NOMFMA=1) per raster group, and one L2 hit/miss PMC pass.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for G in 0 16; do for NM in 0 1; do
  echo "== G=$G NOMFMA=$NM"; ICAP_I8_GROUP=$G ICAP_I8_NOMFMA=$NM timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' || exit 1
done; done
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_l2b -o run -- python3 tools/gemm_shapes.py 3 > gpurun_out/pmc_l2b.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_l2b 2>&1 | grep -A4 "gemm_i8\|Cijk\|gemm_256"
