#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6; mkdir -p $O
R6_EAGER=1 timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $O/clk -o run -- python3 tools/r6_enc_ctx2.py image_caption_amd/libicap.so > $O/clk.log 2>&1 || { tail -5 $O/clk.log; exit 1; }
python3 tools/r6_enc_clock.py $O/clk | tee $O/enc_clock.txt
find $O/clk -name "*.csv" -delete
