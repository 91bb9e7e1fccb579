"""utils/eval.py of the reference (utils/eval.py:1-48, marked "Discontinued"
there): sentence-level scores of one tokenized candidate against tokenized
references. score_bleu restates the nltk call it wraps
(nltk.translate.bleu_score.sentence_bleu with SmoothingFunction().method1,
nltk is absent here); score_ROUGEL uses the coco-caption ROUGE-L
(utils/coco_eval.py). The reference leaves SPICE / METEOR / CIDEr-D as
`pass` stubs; they return None here too (corpus CIDEr-D is
utils.coco_eval.Cider, used by dataset.MetricEval).
"""
from __future__ import annotations

import math
from collections import Counter
from fractions import Fraction

from utils.coco_eval import Rouge


def _ngram_counts(words, n):
    return Counter(tuple(words[i:i + n]) for i in range(len(words) - n + 1)) if len(words) >= n else Counter()


def _modified_precision(references, hypothesis, n):
    counts = _ngram_counts(hypothesis, n)
    max_counts = {}
    for ref in references:
        rc = _ngram_counts(ref, n)
        for g in counts:
            max_counts[g] = max(max_counts.get(g, 0), rc[g])
    clipped = {g: min(c, max_counts[g]) for g, c in counts.items()}
    return Fraction(sum(clipped.values()), max(1, sum(counts.values())), _normalize=False)


def sentence_bleu(references, hypothesis, weights=(0.25, 0.25, 0.25, 0.25), epsilon=0.1):
    """nltk sentence_bleu(..., smoothing_function=SmoothingFunction().method1)."""
    p_n = [_modified_precision(references, hypothesis, i) for i, _ in enumerate(weights, start=1)]
    hyp_len = len(hypothesis)
    ref_lens = [len(r) for r in references]
    closest = min(ref_lens, key=lambda rl: (abs(rl - hyp_len), rl))
    if p_n[0].numerator == 0:
        return 0
    if hyp_len > closest:
        bp = 1.0
    elif hyp_len == 0:
        bp = 0.0
    else:
        bp = math.exp(1 - closest / hyp_len)
    p = [(pi.numerator + epsilon) / pi.denominator if pi.numerator == 0 else pi for pi in p_n]
    s = (w * math.log(pi) for w, pi in zip(weights, p))
    return bp * math.exp(math.fsum(s))


def score_bleu(reference, candidate, n=4):
    """utils/eval.py:10-30: BLEU-n with uniform weights, 0 on failure."""
    if n < 1:
        return 0
    weights = [1 / n] * n
    try:
        score = sentence_bleu(reference, candidate, weights=weights)
    except Exception:
        score = 0.0
    return score


def score_ROUGEL(reference, candidate):
    """ROUGE-L (beta 1.2) of one tokenized candidate against tokenized refs."""
    return Rouge().calc_score([" ".join(candidate)], [" ".join(r) for r in reference])


def score_SPICE(reference, candidate):
    return None


def score_METEOR(reference, candidate):
    return None


def score_CIDErD(reference, candidate):
    return None
