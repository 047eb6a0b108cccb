"""The drop-in entry scripts end to end on the GPU: the build's own scripts/*.py functions -
load_model on a checkpoint shaped like the reference's training scripts write it (numpy-float scores, optimizer and
scheduler state), generate_caption (greedy and beam_search), batch_generate_captions and scripts/inference.py's
no-mask loop - on PNG files, through the HIP preprocessing, encoder and decoder.  Expected captions and ids: the
reference's OWN script functions on the same PNGs (tests/golden/scripts.json, make_golden.py make_scripts; their
torchvision preprocess_image replaced by the Pillow-pinned oracle restatement).  Exact strings and ids wherever the
oracle's top-2 margin along the reference's output exceeds the gate (every greedy / no-mask case here: >= 2.6e-3
against logits within 1e-3; beam search: 1e-4 on the selection margin, as tests/test_gpu_1_parity.py)."""
import json
import os

import pytest
import torch

from image_caption_amd import weights as W
from tests.test_scripts import VOCAB, reference_checkpoint

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")
GREEDY_GATE = 2e-3
BEAM_GATE = 1e-4


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(GOLD, "scripts.json"), encoding="utf-8") as f:
        return json.load(f)


@pytest.fixture(scope="module")
def pngs(tmp_path_factory):
    from tests.golden.inputs import script_images, write_pngs

    return write_pngs(script_images(), tmp_path_factory.mktemp("pngs"))


def _checkpoint(tmp_path, kind, gold):
    sd = W.to_torch(W.vit_state_dict(0) if kind == "vit" else W.grid_state_dict(0))
    sd["decoder.fc_out.bias"][W.END_TOKEN] += gold["end_bias"][kind]
    p = tmp_path / f"{kind}_best_model.pth"
    p.write_bytes(reference_checkpoint(sd, {"vocab_path": VOCAB, "d_model": 512, "nhead": 8, "num_decoder_layers": 6},
                                       numpy1=kind == "grid"))
    return str(p)


def test_vit_inference_script(cuda, tmp_path, gold, pngs):
    from image_caption_amd import _lib
    from scripts import inference_vit_transformer as S

    model, vocab, _ = S.load_model(_checkpoint(tmp_path, "vit", gold), "cuda")
    assert next(model.parameters()).is_cuda and not model.training
    assert min(gold["vit_greedy_margin"]) > GREEDY_GATE
    for i, p in enumerate(pngs):
        cap, ids = S.generate_caption(model, p, vocab, "cuda")
        assert ids == gold["vit_greedy_ids"][i] and cap == gold["vit_greedy_caps"][i], i
    assert _lib._LIB is not None and model._hip_cache is not None  # the HIP engine served the calls
    assert S.batch_generate_captions(model, pngs, vocab, "cuda") == gold["vit_batch"]
    cap, ids = S.generate_caption(model, pngs[0], vocab, "cuda", method="beam_search")
    if gold["vit_beam_margin"] > BEAM_GATE:
        assert ids == gold["vit_beam_ids"] and cap == gold["vit_beam_cap"]


def test_grid_inference_script(cuda, tmp_path, gold, pngs):
    from scripts import inference_grid_transformer as S

    model, vocab, _ = S.load_model(_checkpoint(tmp_path, "grid", gold), "cuda")  # numpy-1.x-spelled pickle
    assert min(gold["grid_greedy_margin"]) > GREEDY_GATE
    for i, p in enumerate(pngs):
        cap, ids = S.generate_caption(model, p, vocab, "cuda")
        assert ids == gold["grid_greedy_ids"][i] and cap == gold["grid_greedy_caps"][i], i
    assert model.hip_engine(torch.device("cuda", 0)).has_trunk  # the HIP ResNet trunk ran
    cap, ids = S.generate_caption(model, pngs[1], vocab, "cuda", method="beam_search", beam_size=5)
    if gold["grid_beam_margin"] > BEAM_GATE:
        assert ids == gold["grid_beam_ids"] and cap == gold["grid_beam_cap"]


def test_inference_py_script(cuda, tmp_path, gold, pngs):
    """scripts/inference.py's own load_model / preprocess_image / generate_caption (the no-mask loop, max_len 50):
    every model.decoder(inputs, features) call runs the HIP full-prefix decoder without a causal mask."""
    from scripts import inference as S

    model, vocab, _ = S.load_model(_checkpoint(tmp_path, "vit", gold), VOCAB, torch.device("cuda", 0))
    eng = model.hip_engine(torch.device("cuda", 0))
    calls = []
    orig = eng.decoder_forward
    eng.decoder_forward = lambda *a, **k: calls.append(k.get("causal")) or orig(*a, **k)
    assert min(gold["nomask_margin"]) > GREEDY_GATE
    for i, p in enumerate(pngs):
        assert S.generate_caption(model, S.preprocess_image(p), vocab, torch.device("cuda", 0)) == gold["nomask_caps"][i]
    assert calls and all(c is False for c in calls)  # the unmasked HIP decoder served every step
