#!/bin/bash
# Persistent decode step timeline (tools build, ICAP_DEC_STEP_TRACE=1).  usage: bash tools/r3_step_trace.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r3
mkdir -p $O
T=${1:-tr}
timeout -k 10 400 python -m image_caption_amd.build --tools > $O/${T}_build.log 2>&1 || { tail -5 $O/${T}_build.log; exit 1; }
ICAP_DEC_STEP_TRACE=1 timeout -k 10 200 python tools/step_trace.py 256 > $O/${T}.txt 2>&1; r=$?
cat $O/${T}.txt | tail -60
exit $r
