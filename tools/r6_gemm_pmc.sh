#!/bin/bash
# Round 6: SQ / TA / LDS counters of one library's ViT GEMMs and hipBLASLt's on the same shapes (one pass per group).
# usage: bash tools/r6_gemm_pmc.sh TAG LIB [SHAPES]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; L=$2; export R6_SHAPES=${3:-mlp3,out}
O=gpurun_out/r6/pmc_$T; mkdir -p $O
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $O/p$i -o run -- python3 tools/r6_gemm_check.py $L > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "gemm_f16" in k or "Cijk" in k:
            k = ("icap " if "gemm_f16" in k else "blaslt ") + r.get("Grid_Size", r.get("Grid_Size_X", ""))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in sorted(acc.items()):
    print(k, " ".join(f"{n}={sum(v) / len(v):.4g}" for n, v in sorted(c.items())))
PY
find $O -name "*counter_collection.csv" -delete
