#!/bin/bash
# Round 3 (tools build in-tree): decode with one chain and the key-split fp16 cross-attention (ICAP_XATTN16_KS=2)
# against the default three chains.  usage: bash tools/r3_xks.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
run() {
  timeout -k 10 150 env "$@" python bench.py --no-cpu-baseline --steps 10 --warmup 2 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); p=d["roofline"]["phases"]; print(d["value"], d["ms_per_step"], p["encoder"]["ms_per_step"], p["decode"]["ms_per_step"])'
}
for i in 1 2; do
  echo "== 3 chains, KS 1"; run ICAP_DEC_BRANCHES=3 || exit 1
  echo "== 1 chain, KS 2"; run ICAP_DEC_BRANCHES=1 ICAP_XATTN16_KS=2 || exit 1
  echo "== 3 chains, KS 2"; run ICAP_DEC_BRANCHES=3 ICAP_XATTN16_KS=2 || exit 1
  echo "== 2 chains, KS 2"; run ICAP_DEC_BRANCHES=2 ICAP_XATTN16_KS=2 || exit 1
done
