#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/lay -o run -- python3 tools/r6_enc_ctx2.py image_caption_amd/libicap.so > $O/lay.log 2>&1 || { tail -5 $O/lay.log; exit 1; }
f=$(find $O/lay -name "*kernel_trace.csv" | head -1)
python3 tools/r6_enc_layers.py $f | tee $O/enc_layers.txt
find $O/lay -name "*.csv" -delete
