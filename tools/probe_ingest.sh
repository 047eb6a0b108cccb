#!/bin/bash
cd $GRAFT_REPO_ROOT
for a in "256 256" "128 256" "64 256" "16 256" "256 128"; do timeout -k 5 60 ./tools/probe_ingest $a || exit 1; done
