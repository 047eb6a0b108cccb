set -o pipefail
for cfg in "ICAP_ENC_ATTN16_FULL=1" "ICAP_ENC_ATTN16_FULL=2"; do env $cfg PYTHONPATH=. timeout -k 10 120 python tools/attn_time.py "$cfg" 2>&1 | grep -v amdgpu.ids || exit 1; done
for shape in "2 197 12" "256 197 12"; do ICAP_ENC_ATTN16_FULL=2 PYTHONPATH=. timeout -k 10 120 python tools/attn_repeat.py $shape 2>&1 | grep -v amdgpu.ids || exit 1; done
ICAP_ENC_ATTN16_FULL=1 PYTHONPATH=. timeout -k 10 120 python tools/attn_repeat.py 2 197 12 2>&1 | grep -v amdgpu.ids
