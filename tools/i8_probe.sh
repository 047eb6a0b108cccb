#!/bin/bash
# i8 GEMM decomposition: full / no MFMA / staging only (no MFMA, no epilogue) per raster group.
set -o pipefail
cd $GRAFT_REPO_ROOT
for G in 0 4 16 64; do for NM in 0 1 2; do
  echo "== G=$G NOMFMA=$NM $(ICAP_I8_GROUP=$G ICAP_I8_NOMFMA=$NM timeout -k 10 120 python tools/gemm_shapes.py 20 2>/dev/null | grep -E "qkv|mlp0" | sed 's/.*| i8x2/i8x2/' | tr '\n' ' ')" || exit 1
done; done
