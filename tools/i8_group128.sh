#!/bin/bash
# raster group sweep of the 128 x 128 int8 GEMM (QKV / MLP-1 us).
set -o pipefail
cd $GRAFT_REPO_ROOT
for G in ${GS:-0 4 8 16 32 64}; do
  echo "== G=$G $(ICAP_I8_GROUP=$G timeout -k 10 120 python tools/gemm_shapes.py 30 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' | tr '\n' ' ')" || exit 1
done
