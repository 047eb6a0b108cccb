#!/bin/bash
# Workspace poisoning (every new workspace allocation filled with 0xFF = NaN): the engine tests must
# still pass, i.e. no kernel reads workspace it has not written.
set -o pipefail
cd $GRAFT_REPO_ROOT
ICAP_POISON=1 timeout -k 10 600 python -m pytest tests/test_gpu_2_engine.py tests/test_gpu_1_parity.py tests/test_gpu_6_ops.py -m gpu -q > gpurun_out/poison.log 2>&1
st=$?
grep -E "passed|failed|Error|assert" gpurun_out/poison.log | head -30
exit $st
