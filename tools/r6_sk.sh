#!/bin/bash
# (Historical: the variant this script measured was removed from the sources after the measurement - see DESIGN.md;
# build it from the commit named there to rerun.)
# Round 6: stream-K scheduling of the persistent fp16 encoder GEMMs - the whole GPU suite on the tree's library, then
# kernel stats and bench lines against whole tiles (tools/ab/libicap_nosk.so, -DICAP_F16P_SK=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -s --timeout 120 --timeout-method thread > $O/sk_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|outliers|Error" $O/sk_tests.log | tail -12
[ $rc -eq 0 ] || { tail -30 $O/sk_tests.log; exit 1; }
bash tools/r6_kstats.sh sk image_caption_amd/libicap.so tools/ab/libicap_nosk.so 2>&1 | grep -E "==|gemm_f16p|layernorm_kernel"
ROUND=r6 bash tools/ab_libs.sh sk 3 image_caption_amd/libicap.so tools/ab/libicap_nosk.so
