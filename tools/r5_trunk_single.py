"""Round 5 (verdict item 5): the Grid config-3 checks on a library whose f16 trunk keeps ONE fp16 residual plane in
layer3-4 (-DICAP_TRUNK_SINGLE=1), with the trunk-feature bar lifted so the north-star checks (memory within 4e-3, every
step's logits within 1e-3, the diverging-row pin) are measured.  usage: python tools/r5_trunk_single.py LIB.so"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch

from image_caption_amd import _lib

_lib.load(sys.argv[1])
sys.path.insert(0, "tests")
import test_gpu_0_workloads as T  # noqa: E402
from image_caption_amd import weights as W  # noqa: E402

T.GRID_FEAT_TOL = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
T.test_config3_grid_b256_trunk_and_every_row(torch.device("cuda", 0), W.to_torch(W.grid_state_dict(0)))
print("config3 checks passed with GRID_FEAT_TOL", T.GRID_FEAT_TOL)
