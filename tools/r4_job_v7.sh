set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py tests/test_scst.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r4/v7_tests.log 2>&1 || { grep -E "^E |FAILED" gpurun_out/r4/v7_tests.log | head -20; tail -3 gpurun_out/r4/v7_tests.log; exit 1; }
tail -1 gpurun_out/r4/v7_tests.log; grep "greedy vs oracle" gpurun_out/r4/v7_tests.log
echo "== xattn QL"; timeout -k 10 120 python tools/xattn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== xattn tools QL=0"; ICAP_XATTN16_QL=0 XATTN_LIB=tools/libicap_tools.so timeout -k 10 120 python tools/xattn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/r4_sweep.sh v7 'ICAP_XATTN16_QL=1' 'ICAP_XATTN16_QL=0' 'ICAP_XATTN16_QL=1' 'ICAP_XATTN16_QL=0'
