#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
for L in image_caption_amd/libicap.so tools/abx/libicap_nosplit.so; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/ctx_$n -o run -- python3 tools/r6_enc_time.py $L > $O/ctx_$n.log 2>&1 || { tail -5 $O/ctx_$n.log; exit 1; }
  f=$(find $O/ctx_$n -name "*kernel_trace.csv" | head -1)
  echo "#### $n"; python3 tools/r6_enc_ctx.py $f
  find $O/ctx_$n -name "*.csv" -delete
done
