set -o pipefail
mkdir -p gpurun_out/r4
echo "== xattn product (wave-owned key tiles)"; timeout -k 10 120 python tools/xattn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
echo "== xattn tools WK=0 (chunk loop)"; ICAP_XATTN16_WK=0 XATTN_LIB=tools/libicap_tools.so timeout -k 10 120 python tools/xattn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/r4_tools_pytest.sh w2p 'ICAP_ENC_ATTN16_FULL=2' '-k enc_attention' tests/test_gpu_6_ops.py || exit 1
for cfg in "ICAP_ENC_ATTN16_FULL=1" "ICAP_ENC_ATTN16_FULL=2"; do env $cfg PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "$cfg" 2>&1 | grep -v amdgpu.ids || exit 1; done
bash tools/r4_sweep.sh w2e 'ICAP_ENC_ATTN16_FULL=2 ICAP_XATTN16_WK=0' 'ICAP_ENC_ATTN16_FULL=1 ICAP_XATTN16_WK=0' || exit 1
