#!/bin/bash
# SCST training-step timing (tools/scst_train_bench.py) for both models, HIP backend vs torch.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r2
for model in vit grid; do
  MODEL=$model timeout -k 10 300 python tools/scst_train_bench.py 128 5 >> gpurun_out/r2/scst_train.txt 2>gpurun_out/r2/scst_train_$model.err || { tail -5 gpurun_out/r2/scst_train_$model.err; exit 1; }
done
cat gpurun_out/r2/scst_train.txt
