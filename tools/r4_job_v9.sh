#!/bin/bash
# counted opening waits in the FR decode blocks: product (new) vs tools build of the previous tree (old)
cd $GRAFT_REPO_ROOT
bash tools/r4_ab.sh openx "" "tests/test_gpu_2_engine.py tests/test_gpu_0_workloads.py"
