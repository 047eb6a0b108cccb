#!/bin/bash
# Round 6: the pipeline's post step deferred one batch on its own stream - pipeline tests, the stream gaps, then
# alternating bench lines against the post step run right after its batch (ICAP_PIPE_DEFER_POST=0).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_2_engine.py -x -q --timeout 200 --timeout-method thread -k "pipeline" > $O/pdefer_tests.log 2>&1 || { tail -20 $O/pdefer_tests.log; exit 1; }
tail -1 $O/pdefer_tests.log
timeout -k 10 200 python tools/r6_pipe_gaps.py > $O/pipe_gaps_deferred.txt 2>&1 || { tail -20 $O/pipe_gaps_deferred.txt; exit 1; }
grep -v amdgpu.ids $O/pipe_gaps_deferred.txt
R6_PV_ROUNDS=3 R6_PV="deferred:X=1:;not_deferred:ICAP_PIPE_DEFER_POST=0:" bash tools/r6_pipe_var.sh
cp $O/pipe_var.txt $O/pipe_defer_ab.txt
