#!/bin/bash
cd $GRAFT_REPO_ROOT
for E in "X=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "HIP_FORCE_DEV_KERNARG=0" "HIP_FORCE_DEV_KERNARG=1" "GPU_MAX_HW_QUEUES=1"; do
  echo "== $E"; env $E timeout -k 10 60 ./tools/probe_small | grep -E "alt|ln 256|copy   1024" || exit 1
done
