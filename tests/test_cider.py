"""GPU CIDEr-D (icap_cider_d, SURVEY.md §8(f)2 reward path) against the ids restatement
image_caption_amd.cider.cider_d, itself pinned against the independent string restatement
oracle/cider_ref.py in tests/test_oracle.py (pycocoevalcap is absent: parity with it is unpinned)."""
import numpy as np
import pytest
import torch

from image_caption_amd import cider as C

START, END, PAD = 1, 2, 0


def _rows(seqs, L):
    m = torch.full((len(seqs), L), PAD, dtype=torch.int32)
    for i, s in enumerate(seqs):
        row = [START] + list(s) + [END]
        m[i, : min(len(row), L)] = torch.tensor(row[:L], dtype=torch.int32)
    return m


def _case(seed, B, max_refs=3, vocab=40, maxlen=20):
    rng = np.random.default_rng(seed)
    hyps = [rng.integers(3, vocab, rng.integers(0, maxlen)).tolist() for _ in range(2 * B)]
    refs = [[rng.integers(3, vocab, rng.integers(1, maxlen)).tolist() for _ in range(rng.integers(0, max_refs + 1))]
            for _ in range(B)]
    # edge cases: a hypothesis equal to its reference, repeated tokens, an empty hypothesis
    if B > 2 and refs[1]:
        hyps[1] = list(refs[1][0])
    hyps[0] = [5, 5, 5, 5, 5, 5]
    refs[0] = [[5, 5, 5, 7], [5, 9]]
    hyps[B] = []
    return hyps, refs


def test_pack_references_roundtrip():
    rows, off = C.pack_references([[[3, 4], [5]], [], [["w1", 7, "w1"]]], PAD, END, vocab_size=50)
    assert off.tolist() == [0, 2, 2, 3]
    back = [C.caption_ids(r, START, END, PAD) for r in rows.tolist()]
    assert back[0] == [3, 4] and back[1] == [5] and back[2] == [50, 7, 50]


@pytest.mark.gpu
@pytest.mark.parametrize("seed,B", [(0, 7), (1, 64), (2, 256)])
def test_gpu_cider_matches_restatement(cuda, seed, B):
    hyps, refs = _case(seed, B)
    L = max(len(h) for h in hyps) + 2
    rows, off = C.pack_references(refs, PAD, END, 100)
    got = C.cider_d_device(_rows(hyps, L).to(cuda), rows.to(cuda), off, START, END, PAD).cpu().numpy()
    want = np.array(C.cider_d(hyps[:B], refs)[1] + C.cider_d(hyps[B:], refs)[1])
    assert got.shape == (2 * B,)
    assert np.allclose(got, want, rtol=1e-12, atol=1e-12), np.abs(got - want).max()


@pytest.mark.gpu
def test_gpu_cider_single_image_and_no_refs(cuda):
    """ref_len = log(1) = 0 for a one-image call (every tf-idf weight 0 -> score 0), and images
    without references score 0."""
    rows, off = C.pack_references([[[3, 4, 5]]], PAD, END, 100)
    got = C.cider_d_device(_rows([[3, 4, 5]], 6).to(cuda), rows.to(cuda), off, START, END, PAD).cpu().numpy()
    assert np.allclose(got, C.cider_d([[3, 4, 5]], [[[3, 4, 5]]])[1])
    rows, off = C.pack_references([[], [[3, 4]]], PAD, END, 100)
    got = C.cider_d_device(_rows([[3, 4], [3, 4]], 5).to(cuda), rows.to(cuda), off, START, END, PAD).cpu().numpy()
    assert np.allclose(got, C.cider_d([[3, 4], [3, 4]], [[], [[3, 4]]])[1])
