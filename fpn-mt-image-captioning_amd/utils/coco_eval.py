"""Caption-quality evaluation: the coco-caption scorers the
reference's MetricEval runs through pycocoevalcap.eval.COCOEvalCap
(dataset.py:260-298), restated because pycocoevalcap is not installed here:

  Bleu(4)   bleu_scorer.py: corpus BLEU-1..4 with the 'closest' reference
            length, tiny / small guards 1e-15 / 1e-9, plus per-image scores
  Rouge     rouge.py: ROUGE-L, beta 1.2, max precision / recall over refs
  Cider     cider_scorer.py (CIDEr-D as coco-caption computes it): n = 4,
            sigma 6, document frequency over the evaluated images' refs,
            log(#images) as ref_len, clipped tf-idf products, the Gaussian
            length penalty on the 2-gram count (`if n == 1` in the original),
            mean over n, / #refs, x 10
  PTBTokenizer  the Stanford PTBTokenizer (Java) run with -preserveLines
            -lowerCase, then the punctuation tokens removed. Java is absent:
            this is a regex approximation that matches it on caption text
            made of words, digits, hyphenated words, clitics ('s, n't, 're,
            've, 'll, 'd, 'm) and the punctuation . , ; : ! ? " ' ( ) ...;
            other inputs are "parity unpinned".
  METEOR / SPICE need their Java jars and are not computed (absent keys).

Host code (string / n-gram work on a few thousand captions): it is not on
the GPU path and runs in a second or two for COCO val.
"""
from __future__ import annotations

import math
import re
from collections import defaultdict

import numpy as np

PUNCTUATIONS = ["''", "'", "``", "`", "-LRB-", "-RRB-", "-LCB-", "-RCB-",
                ".", "?", "!", ",", ":", "-", "--", "...", ";"]

_CLITIC = re.compile(r"(?i)([a-z0-9])('s|'re|'ve|'ll|'d|'m)\b")
_NT = re.compile(r"(?i)([a-z])(n't)\b")
_ELLIPSIS = re.compile(r"\.\.\.")
_DASHES = re.compile(r"--")
_SPLIT_PUNCT = re.compile(r'([?!;:"(){}\[\]`])')
_COMMA = re.compile(r"(?<!\d),|,(?!\d)")
_QUOTE_START = re.compile(r"(^|\s)'(?!(?:s|re|ve|ll|d|m)(?:\s|$))")
_QUOTE_END = re.compile(r"'(\s|$)")
_BRACKETS = {"(": "-LRB-", ")": "-RRB-", "{": "-LCB-", "}": "-RCB-", "[": "-LSB-", "]": "-RSB-"}


def ptb_tokenize_line(s: str) -> list:
    """One caption -> PTB tokens, lower-cased (before punctuation removal)."""
    s = s.replace("\n", " ").lower()
    s = _ELLIPSIS.sub(" ... ", s)
    s = _DASHES.sub(" -- ", s)
    s = _SPLIT_PUNCT.sub(r" \1 ", s)
    s = _COMMA.sub(" , ", s)
    s = _NT.sub(r"\1 \2", s)
    s = _CLITIC.sub(r"\1 \2", s)
    s = _QUOTE_START.sub(r"\1 ' ", s)
    s = _QUOTE_END.sub(r" ' \1", s)
    out = []
    for tok in s.split():
        # a sentence-final / word-final period splits off unless the token is
        # an abbreviation with inner periods (u.s.) or a number (3.5)
        if tok.endswith(".") and tok != "..." and len(tok) > 1 and "." not in tok[:-1]:
            out.extend([tok[:-1], "."])
        elif tok == '"':
            out.append("''")
        else:
            out.append(_BRACKETS.get(tok, tok))
    return out


class PTBTokenizer:
    """pycocoevalcap.tokenizer.ptbtokenizer.PTBTokenizer.tokenize."""

    def tokenize(self, captions_for_image):
        final = {}
        for k, anns in captions_for_image.items():
            final[k] = [" ".join(w for w in ptb_tokenize_line(c["caption"]) if w not in PUNCTUATIONS)
                        for c in anns]
        return final


def _ngrams(words, n):
    counts = defaultdict(int)
    for k in range(1, n + 1):
        for i in range(len(words) - k + 1):
            counts[tuple(words[i:i + k])] += 1
    return counts


class Bleu:
    def __init__(self, n=4):
        self._n = n

    def compute_score(self, gts, res):
        n = self._n
        small, tiny = 1e-9, 1e-15
        bleu_list = [[] for _ in range(n)]
        tot_guess, tot_correct = [0] * n, [0] * n
        tot_test = tot_ref = 0
        for key in gts:
            hypo, refs = res[key], gts[key]
            assert isinstance(hypo, list) and len(hypo) == 1
            assert isinstance(refs, list) and len(refs) >= 1
            reflens, maxcounts = [], {}
            for ref in refs:
                w = ref.split()
                reflens.append(len(w))
                for g, c in _ngrams(w, n).items():
                    maxcounts[g] = max(maxcounts.get(g, 0), c)
            tw = hypo[0].split()
            testlen = len(tw)
            guess = [max(0, testlen - k + 1) for k in range(1, n + 1)]
            correct = [0] * n
            for g, c in _ngrams(tw, n).items():
                correct[len(g) - 1] += min(maxcounts.get(g, 0), c)
            reflen = min((abs(l - testlen), l) for l in reflens)[1]  # 'closest'
            tot_test += testlen
            tot_ref += reflen
            for k in range(n):
                tot_guess[k] += guess[k]
                tot_correct[k] += correct[k]
            b = 1.0
            for k in range(n):
                b *= (float(correct[k]) + tiny) / (float(guess[k]) + small)
                bleu_list[k].append(b ** (1.0 / (k + 1)))
            ratio = (testlen + tiny) / (reflen + small)
            if ratio < 1:
                for k in range(n):
                    bleu_list[k][-1] *= math.exp(1 - 1 / ratio)
        bleus = []
        b = 1.0
        for k in range(n):
            b *= float(tot_correct[k] + tiny) / (tot_guess[k] + small)
            bleus.append(b ** (1.0 / (k + 1)))
        ratio = (tot_test + tiny) / (tot_ref + small)
        if ratio < 1:
            for k in range(n):
                bleus[k] *= math.exp(1 - 1 / ratio)
        return bleus, bleu_list

    def method(self):
        return "Bleu"


def _lcs(a, b):
    if len(a) < len(b):
        a, b = b, a
    prev = [0] * (len(b) + 1)
    for i in range(1, len(a) + 1):
        cur = [0] * (len(b) + 1)
        for j in range(1, len(b) + 1):
            cur[j] = prev[j - 1] + 1 if a[i - 1] == b[j - 1] else max(prev[j], cur[j - 1])
        prev = cur
    return prev[len(b)]


class Rouge:
    def __init__(self):
        self.beta = 1.2

    def calc_score(self, candidate, refs):
        assert len(candidate) == 1 and len(refs) > 0
        prec, rec = [], []
        tc = candidate[0].split(" ")
        for ref in refs:
            tr = ref.split(" ")
            lcs = _lcs(tr, tc)
            prec.append(lcs / float(len(tc)))
            rec.append(lcs / float(len(tr)))
        pm, rm = max(prec), max(rec)
        if pm != 0 and rm != 0:
            return ((1 + self.beta ** 2) * pm * rm) / float(rm + self.beta ** 2 * pm)
        return 0.0

    def compute_score(self, gts, res):
        score = [self.calc_score(res[k], gts[k]) for k in gts]
        return float(np.mean(np.array(score))), np.array(score)

    def method(self):
        return "Rouge"


class Cider:
    def __init__(self, n=4, sigma=6.0):
        self._n, self._sigma = n, sigma

    def compute_score(self, gts, res):
        n, sigma = self._n, self._sigma
        ctest, crefs = [], []
        for k in gts:
            hypo, refs = res[k], gts[k]
            assert isinstance(hypo, list) and len(hypo) == 1
            assert isinstance(refs, list) and len(refs) > 0
            ctest.append(_ngrams(hypo[0].split(), n))
            crefs.append([_ngrams(r.split(), n) for r in refs])
        df = defaultdict(float)
        for refs in crefs:
            for g in {g for r in refs for g in r}:
                df[g] += 1
        assert len(ctest) >= max(df.values())
        ref_len = np.log(float(len(crefs)))

        def counts2vec(cnts):
            vec = [defaultdict(float) for _ in range(n)]
            norm = [0.0] * n
            length = 0
            for g, tf in cnts.items():
                d = np.log(max(1.0, df[g]))
                k = len(g) - 1
                vec[k][g] = float(tf) * (ref_len - d)
                norm[k] += pow(vec[k][g], 2)
                if k == 1:
                    length += tf
            return vec, [np.sqrt(x) for x in norm], length

        def sim(vh, vr, nh, nr, lh, lr):
            delta = float(lh - lr)
            val = np.array([0.0] * n)
            for k in range(n):
                for g in vh[k]:
                    val[k] += min(vh[k][g], vr[k][g]) * vr[k][g]
                if nh[k] != 0 and nr[k] != 0:
                    val[k] /= nh[k] * nr[k]
                assert not math.isnan(val[k])
                val[k] *= np.e ** (-(delta ** 2) / (2 * sigma ** 2))
            return val

        scores = []
        for test, refs in zip(ctest, crefs):
            vec, norm, length = counts2vec(test)
            score = np.array([0.0] * n)
            for ref in refs:
                vr, nr, lr = counts2vec(ref)
                score += sim(vec, vr, norm, nr, length, lr)
            s = np.mean(score) / len(refs) * 10.0
            scores.append(s)
        return float(np.mean(np.array(scores))), np.array(scores)

    def method(self):
        return "CIDEr"


class COCOEvalCap:
    """pycocoevalcap.eval.COCOEvalCap without the Java scorers."""

    def __init__(self, coco, cocoRes):
        self.evalImgs = []
        self.eval = {}
        self.imgToEval = {}
        self.coco = coco
        self.cocoRes = cocoRes
        self.params = {"image_id": coco.getImgIds()}

    def evaluate(self, verbose=False):
        img_ids = self.params["image_id"]
        gts = {i: self.coco.imgToAnns[i] for i in img_ids}
        res = {i: self.cocoRes.imgToAnns[i] for i in img_ids}
        tok = PTBTokenizer()
        gts, res = tok.tokenize(gts), tok.tokenize(res)
        scorers = [(Bleu(4), ["Bleu_1", "Bleu_2", "Bleu_3", "Bleu_4"]), (Rouge(), "ROUGE_L"), (Cider(), "CIDEr")]
        for scorer, method in scorers:
            score, scores = scorer.compute_score(gts, res)
            if isinstance(method, list):
                for sc, scs, m in zip(score, scores, method):
                    self.setEval(sc, m)
                    self.setImgToEvalImgs(scs, list(gts.keys()), m)
                    if verbose:
                        print(f"{m}: {sc:0.3f}")
            else:
                self.setEval(score, method)
                self.setImgToEvalImgs(scores, list(gts.keys()), method)
                if verbose:
                    print(f"{method}: {score:0.3f}")
        self.setEvalImgs()

    def setEval(self, score, method):
        self.eval[method] = score

    def setImgToEvalImgs(self, scores, img_ids, method):
        for img_id, score in zip(img_ids, scores):
            self.imgToEval.setdefault(img_id, {"image_id": img_id})[method] = score

    def setEvalImgs(self):
        self.evalImgs = [e for e in self.imgToEval.values()]
