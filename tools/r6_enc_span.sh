#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
for L in image_caption_amd/libicap.so tools/abx/libicap_nosplit.so; do
  n=$(basename $L .so)
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/span_$n -o run -- python3 -c "
import sys, runpy
from image_caption_amd import _lib
_lib.load('$L')
sys.argv = ['bench.py', '--no-cpu-baseline', '--steps', '3', '--warmup', '1']
runpy.run_path('bench.py', run_name='__main__')
" > $O/span_$n.log 2>&1 || { tail -5 $O/span_$n.log; exit 1; }
  f=$(find $O/span_$n -name "*kernel_trace.csv" | head -1)
  echo "== $n"; python3 tools/r6_enc_span.py $f
  find $O/span_$n -name "*.csv" -delete
done
