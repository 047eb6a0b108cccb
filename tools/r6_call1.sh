#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
bash tools/r6_abl.sh s3 image_caption_amd/libicap.so tools/ab/libicap_swz.so tools/ab/libicap_f16h2.so tools/ab/libicap_f16h3.so || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_8_stop.py "tests/test_gpu_2_engine.py::test_cu_masked_pipelines_budget_stack" -x -v -s --timeout 120 --timeout-method thread > $O/stop_tests.log 2>&1; rc=$?
grep -E "PASS|FAIL|SKIP|Error|error|stop after|passed|failed" $O/stop_tests.log | tail -30
exit $rc
