#!/bin/bash
# cross-attention: first chunk's DMA ahead of the q~ loads.  Kernel alone (product vs tools build of HEAD), GPU tests
# that reach the cross-attention, then the bench A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
timeout -k 10 120 python tools/xattn_time.py > $O/xq_new.txt 2>&1 || { tail -20 $O/xq_new.txt; exit 1; }
XATTN_LIB=tools/libicap_tools.so timeout -k 10 120 python tools/xattn_time.py > $O/xq_old.txt 2>&1 || { tail -20 $O/xq_old.txt; exit 1; }
echo new; cat $O/xq_new.txt; echo old; cat $O/xq_old.txt
bash tools/r4_ab.sh xq "" "tests/test_gpu_2_engine.py tests/test_gpu_0_workloads.py tests/test_gpu_4_scst.py tests/test_gpu_6_ops.py tests/test_gpu_1_parity.py"
