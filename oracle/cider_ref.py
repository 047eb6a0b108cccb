"""ORACLE — test infrastructure only.  String-level restatement of pycocoevalcap's CiderScorer
(third-party dependency of the reference, utils/scst_loss.py:16,27,50; version unpinned, absent
here), written independently of image_caption_amd/cider.py so the two can check each other.
Parity with pycocoevalcap itself is UNPINNED: the reference holds no CIDEr fixture
(utils/scst_loss.py:357-369 only prints)."""
from __future__ import annotations

import math
from collections import defaultdict


def precook(sentence: str, n: int = 4):
    words = sentence.split()
    counts = defaultdict(int)
    for k in range(1, n + 1):
        for i in range(len(words) - k + 1):
            counts[tuple(words[i:i + k])] += 1
    return counts


def compute_score(gts: dict, res: dict, n: int = 4, sigma: float = 6.0):
    """gts: id -> list of reference strings; res: id -> [hypothesis string]."""
    ids = list(gts.keys())
    assert set(ids) == set(res.keys())
    crefs = [[precook(r, n) for r in gts[i]] for i in ids]
    ctest = [precook(res[i][0], n) for i in ids]
    doc_freq = defaultdict(float)
    for refs in crefs:
        for ngram in set(ng for ref in refs for ng in ref):
            doc_freq[ngram] += 1
    ref_len = math.log(float(len(crefs)))

    def counts2vec(cnts):
        vec = [defaultdict(float) for _ in range(n)]
        norm = [0.0] * n
        length = 0
        for ngram, tf in cnts.items():
            k = len(ngram) - 1
            vec[k][ngram] = float(tf) * (ref_len - math.log(max(1.0, doc_freq[ngram])))
            norm[k] += vec[k][ngram] ** 2
            if k == 1:
                length += tf
        return vec, [math.sqrt(x) for x in norm], length

    scores = []
    for test, refs in zip(ctest, crefs):
        vec, norm, length = counts2vec(test)
        total = [0.0] * n
        for ref in refs:
            vr, nr, lr = counts2vec(ref)
            delta = float(length - lr)
            for k in range(n):
                val = 0.0
                for ngram in list(vec[k].keys()):
                    val += min(vec[k][ngram], vr[k][ngram]) * vr[k][ngram]
                if norm[k] != 0 and nr[k] != 0:
                    val /= norm[k] * nr[k]
                total[k] += val * math.e ** (-(delta ** 2) / (2 * sigma ** 2))
        scores.append(sum(total) / n / len(refs) * 10.0)
    return sum(scores) / len(scores), scores
