#!/bin/bash
# Round 4 final checkpoint: tools/r4_check.sh (whole GPU suite, smoke, ViT bench with the CPU baseline, Grid bench,
# rocprofv3 kernel trace + stats), the cross-attention op timing, then the PMC traffic passes (tools/r4_pmc.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r4_check.sh ${1:-ck2} || exit 1
echo "== xattn"; timeout -k 10 120 python tools/xattn_time.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/r4_pmc.sh
