#!/bin/bash
# per-CU weight ingest at the decode kernels' block counts (48 = one chain's dec_sa, 144 = three chains, 256 = all)
cd $GRAFT_REPO_ROOT
for a in "256 48" "256 144" "256 256" "128 144" "64 144" "64 256" "32 256"; do timeout -k 5 60 ./tools/probe_ingest $a || exit 1; done
