#!/bin/bash
# Round 6: the pipeline's encoder CU budget on by default - pipeline tests, then alternating bench lines: the default
# (overlapped encodes on 160 CUs, the first on all), the budget off (ICAP_PIPE_ENC_CUS=0), 192 and 176 CUs.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_2_engine.py -x -q --timeout 200 --timeout-method thread -k "pipeline" > $O/pcus_tests.log 2>&1 || { tail -20 $O/pcus_tests.log; exit 1; }
tail -1 $O/pcus_tests.log
: > $O/pipe_cus_ab.txt
for r in 1 2 3; do
  for c in "" 0 192 176; do
    ICAP_PIPE_ENC_CUS=$c timeout -k 10 200 python bench.py --no-cpu-baseline > $O/pcus.json 2> $O/pcus.err || { tail -20 $O/pcus.err; exit 1; }
    python -c "import json; d=json.load(open('$O/pcus.json')); p=d['roofline']['phases']; print('enc_cus=${c:-default}', d['config']['encoder_cus_overlapped'], d['value'], d['ms_per_step'], p['encoder']['ms_per_step'], p['decode']['ms_per_step'], d['roofline']['frac'])" | tee -a $O/pipe_cus_ab.txt
  done
done
