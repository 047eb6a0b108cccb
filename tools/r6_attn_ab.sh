#!/bin/bash
# Round 6: encoder attention change - the attention / workload tests on the tree's library, kernel stats of both,
# bench lines alternating with the previous build (tools/abx/libicap_base.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py -x -q -s --timeout 120 --timeout-method thread -k "attention or config2 or vit or repeat" > $O/attn_tests.log 2>&1; rc=$?
grep -E "passed|failed|greedy vs oracle|Error" $O/attn_tests.log | tail -8
[ $rc -eq 0 ] || { tail -30 $O/attn_tests.log; exit 1; }
bash tools/r6_kstats.sh at image_caption_amd/libicap.so tools/abx/libicap_base.so 2>&1 | grep -E "==|enc_attention|gemm_f16p"
ROUND=r6 bash tools/ab_libs.sh attn 3 image_caption_amd/libicap.so tools/abx/libicap_base.so
