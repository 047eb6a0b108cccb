#!/bin/bash
# bias vectors prefetched as each decode block's oldest load: full GPU suite, then product (new) vs tools build of HEAD (old)
cd $GRAFT_REPO_ROOT
bash tools/r4_ab.sh biaspf "" "tests/"
