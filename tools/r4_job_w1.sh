set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 500 python -u -m pytest tests/test_gpu_6_ops.py tests/test_gpu_0_workloads.py tests/test_gpu_1_parity.py tests/test_gpu_2_engine.py tests/test_scst.py -m gpu -x -q -s --timeout 120 --timeout-method thread > gpurun_out/r4/w1_tests.log 2>&1
rc=$?
tail -1 gpurun_out/r4/w1_tests.log; grep 'greedy vs oracle' gpurun_out/r4/w1_tests.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/r4/w1_tests.log | head -20; exit 1; }
bash tools/r4_sweep.sh w1 'ICAP_XATTN16_WK=1' 'ICAP_XATTN16_WK=0' 'ICAP_XATTN16_WK=1' || exit 1
bash tools/r4_tools_pytest.sh w1p 'ICAP_ENC_ATTN16_FULL=2' '-k enc_attention' tests/test_gpu_6_ops.py || exit 1
for cfg in "ICAP_ENC_ATTN16_FULL=1" "ICAP_ENC_ATTN16_FULL=2"; do env $cfg PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "$cfg" 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/r4_sweep.sh w1e 'ICAP_ENC_ATTN16_FULL=2' 'ICAP_ENC_ATTN16_FULL=1' || exit 1
bash tools/r4_trace1.sh w1 'ICAP_DEC_BRANCHES=1'
