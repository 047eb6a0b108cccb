"""CIDEr-D reward on token-id sequences (SCST reward, utils/scst_loss.py:20-54).

The reference calls pycocoevalcap's `Cider().compute_score(gts, res)` (third-party, version
unpinned - README.md:175 lists it bare - and absent here).  This restates that published
CiderScorer algorithm: n-grams n = 1..4, tf-idf weights with the document frequency taken over
THIS call's reference sets and ref_len = log(#images), per-n cosine of clipped vectors
(min(hyp, ref) * ref), Gaussian length penalty exp(-delta^2 / (2 * 6^2)) where the "length" is
the term-frequency sum of the n=2 slot (as the scorer computes it), mean over n, mean over refs,
x10.  It operates on ids instead of whitespace-split words: exact, because no vocabulary word
contains whitespace and ids map 1:1 to words.  Parity with pycocoevalcap itself
is unpinned (no fixture in the reference holds a CIDEr value); tests pin it against the
independent string restatement in oracle/cider_ref.py.
"""
from __future__ import annotations

import math
from collections import Counter, defaultdict
from typing import Dict, List, Sequence, Tuple

NGRAM = 4
SIGMA = 6.0

Ngrams = Counter


def ngram_counts(tokens: Sequence[int], n: int = NGRAM) -> Ngrams:
    c: Counter = Counter()
    for k in range(1, n + 1):
        for i in range(len(tokens) - k + 1):
            c[tuple(tokens[i:i + k])] += 1
    return c


def _vec(counts: Ngrams, df: Dict[tuple, float], ref_len: float):
    vec = [dict() for _ in range(NGRAM)]
    norm = [0.0] * NGRAM
    length = 0
    for g, tf in counts.items():
        n = len(g) - 1
        w = float(tf) * (ref_len - math.log(max(1.0, df.get(g, 0.0))))
        vec[n][g] = w
        norm[n] += w * w
        if n == 1:
            length += tf
    return vec, [math.sqrt(x) for x in norm], length


def _sim(vh, nh, lh, vr, nr, lr) -> List[float]:
    delta = float(lh - lr)
    pen = math.exp(-(delta ** 2) / (2 * SIGMA ** 2))
    out = []
    for n in range(NGRAM):
        v = 0.0
        ref_n = vr[n]
        for g, w in vh[n].items():
            r = ref_n.get(g, 0.0)
            v += min(w, r) * r
        if nh[n] != 0 and nr[n] != 0:
            v /= nh[n] * nr[n]
        out.append(v * pen)
    return out


def cider_d(hyps: Sequence[Sequence[int]], refs: Sequence[Sequence[Sequence[int]]]) -> Tuple[float, List[float]]:
    """hyps[i]: token ids of image i's caption; refs[i]: list of reference id sequences.
    Returns (mean score, per-image scores) like Cider.compute_score."""
    assert len(hyps) == len(refs)
    crefs = [[ngram_counts(r) for r in rs] for rs in refs]
    ctest = [ngram_counts(h) for h in hyps]
    df: Dict[tuple, float] = defaultdict(float)
    for rs in crefs:
        for g in set(g for r in rs for g in r):
            df[g] += 1
    ref_len = math.log(float(len(crefs))) if crefs else 0.0
    scores = []
    for test, rs in zip(ctest, crefs):
        vh, nh, lh = _vec(test, df, ref_len)
        acc = [0.0] * NGRAM
        for r in rs:
            vr, nr, lr = _vec(r, df, ref_len)
            acc = [a + b for a, b in zip(acc, _sim(vh, nh, lh, vr, nr, lr))]
        s = sum(acc) / NGRAM
        s /= max(len(rs), 1)
        scores.append(s * 10.0)
    mean = sum(scores) / len(scores) if scores else 0.0
    return mean, scores


def caption_ids(row: Sequence[int], start: int, end: int, pad: int) -> List[int]:
    """Caption token ids as `_decode_captions` keeps them: stop at <end>, drop <start>/<pad>."""
    out = []
    for t in row:
        if t == end:
            break
        if t != start and t != pad:
            out.append(int(t))
    return out


def cider_d_device(hyp, refs, ref_off, start: int, end: int, pad: int):
    """CIDEr-D on the GPU (libicap icap_cider_d): hyp (n_hyp, Lh) raw id rows, hypothesis k scored
    against image k % B; refs (n_ref, Lr) raw id rows with image i's references at rows
    ref_off[i] .. ref_off[i+1] (ref_off: B + 1).  <start>/<pad> are dropped and rows end at <end>
    (caption_ids semantics).  Returns float64 scores (n_hyp,) on the hyp's device, equal to
    cider_d([caption_ids(h)], [[caption_ids(r) ...]]) per image up to double rounding."""
    import torch

    from . import _lib

    lib = _lib.load()
    dev = hyp.device
    if dev.type != "cuda":
        raise _lib.IcapError("icap_cider_d needs GPU tensors")
    h = hyp.to(dtype=torch.int32).contiguous()
    r = refs.to(device=dev, dtype=torch.int32).contiguous()
    off = torch.as_tensor(ref_off, dtype=torch.int32).to(dev).contiguous()
    B = off.numel() - 1
    if r.numel() == 0:  # no reference rows at all: keep a valid pointer
        r = torch.full((1, 1), end, dtype=torch.int32, device=dev)
    n_ref, Lr = r.shape
    ws_bytes = lib.icap_cider_workspace_bytes(n_ref, Lr)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    scores = torch.empty(h.shape[0], dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        _lib.check(lib.icap_cider_d(h.data_ptr(), h.shape[0], h.shape[1], B, r.data_ptr(), n_ref, Lr, off.data_ptr(),
                                    start, end, pad, scores.data_ptr(), ws.data_ptr(), ws_bytes, status.data_ptr(),
                                    _lib.stream_ptr(dev)), "icap_cider_d")
    if int(status.item()):
        raise _lib.IcapError("icap_cider_d: an image's reference set exceeds 4096 distinct n-grams")
    return scores


def pack_references(refs: Sequence[Sequence[Sequence]], pad: int, end: int, vocab_size: int):
    """Per-image reference token lists (ids, or words already mapped) -> (rows (n_ref, Lr) int32 padded
    with <pad> and terminated by <end>, ref_off (B + 1)).  Words that are not ids get fresh ids above
    the vocabulary, consistently within the call, so their n-grams stay distinct."""
    import torch

    extra: Dict = {}
    rows, off = [], [0]
    for rs in refs:
        for ref in rs:
            ids = []
            for t in ref:
                if not isinstance(t, int):
                    t = extra.setdefault(t, vocab_size + len(extra))
                ids.append(int(t))
            rows.append(ids)
        off.append(len(rows))
    Lr = max([len(x) for x in rows] + [0]) + 1
    mat = torch.full((max(len(rows), 1), Lr), pad, dtype=torch.int32)
    for i, ids in enumerate(rows):
        if ids:
            mat[i, : len(ids)] = torch.tensor(ids, dtype=torch.int32)
        mat[i, len(ids)] = end
    return mat, torch.tensor(off, dtype=torch.int32)
