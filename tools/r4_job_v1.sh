set -o pipefail
for cfg in "ICAP_EAF_VAR=0" "ICAP_EAF_VAR=1" "ICAP_EAF_VAR=0" "ICAP_EAF_VAR=1"; do env $cfg PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "$cfg" 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/r4_tools_pytest.sh v1p 'ICAP_EAF_VAR=1' '-k enc_attention' tests/test_gpu_6_ops.py || exit 1
