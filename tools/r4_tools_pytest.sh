#!/bin/bash
# Round 4: GPU tests on the tools build with knobs.  usage: bash tools/r4_tools_pytest.sh TAG "K=V ..." "-k expr" FILES...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4; mkdir -p $O
T=$1; KN=$2; K=$3; shift 3
env $KN timeout -k 10 400 python -u -c "
import sys
from image_caption_amd import _lib
_lib.load('tools/libicap_tools.so')
import pytest
sys.exit(pytest.main(sys.argv[1:] + ['-m', 'gpu', '-x', '-q', '-s', '-p', 'no:cacheprovider', '--timeout', '120', '--timeout-method', 'thread']))
" "$@" $K > $O/${T}_tt.log 2>&1 || { tail -30 $O/${T}_tt.log; exit 1; }
tail -1 $O/${T}_tt.log
