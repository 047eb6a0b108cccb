#!/bin/bash
# Round 4: encoder attention timing ablations (tools build; tools/attn_time.py)
cd $GRAFT_REPO_ROOT
set -o pipefail
for cfg in "ICAP_ENC_ATTN16_FULL=0" "ICAP_ENC_ATTN16_FULL=1" "ICAP_EAF_ABL=1" "ICAP_EAF_ABL=2" "ICAP_EAF_ABL=3"; do
  env $cfg PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 120 python tools/attn_time.py "$cfg" 2>&1 | grep -v amdgpu.ids || exit 1
done
