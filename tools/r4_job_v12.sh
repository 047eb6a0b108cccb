#!/bin/bash
# checkpoint 3: whole GPU suite, smoke, ViT / Grid bench lines, rocprof trace (tools/r4_check.sh); then the decode A/B
# against the product build of the session-start tree 85d6e6a (tools/libicap_prev.so), like against like
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/r4_check.sh ck3 || exit 1
OLD_LIB=tools/libicap_prev.so ARMS="new old new old new old" bash tools/r4_ab.sh ck3ab ""
