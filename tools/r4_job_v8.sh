set -o pipefail
bash tools/r4_tools_pytest.sh v8p 'ICAP_RLN_WAVE=1' '-k config2' tests/test_gpu_0_workloads.py || exit 1
bash tools/r4_sweep.sh v8 'ICAP_RLN_WAVE=1' 'ICAP_RLN_WAVE=0' 'ICAP_RLN_WAVE=1' 'ICAP_RLN_WAVE=0'
