#!/bin/bash
# (Historical: the variant this script measured was removed from the sources after the measurement - see DESIGN.md;
# build it from the commit named there to rerun.)
# Round 6: the LayerNorm fold with the residual stream as fp16 hi / lo planes (variant tools/ab/libicap_fold2.so) -
# the encoder / workload parity tests with the variant in place of the tree's library (on the box's copy only), then
# bench lines alternating product / variant.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
cp image_caption_amd/libicap.so tools/ab/libicap_prod.so && cp tools/ab/libicap_fold2.so image_caption_amd/libicap.so || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py -x -q -s --timeout 120 --timeout-method thread > $O/fold2_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|outliers|Error" $O/fold2_tests.log | tail -12
[ $rc -eq 0 ] || { tail -30 $O/fold2_tests.log; exit 1; }
ROUND=r6 bash tools/ab_libs.sh fold2 3 tools/ab/libicap_prod.so tools/ab/libicap_fold2.so || exit 1
timeout -k 10 120 python -u tools/r6_rln_slabs.py > $O/rln_slabs.txt 2>&1; cat $O/rln_slabs.txt
