"""Caption-quality evaluation (reference dataset.py:260-298
MetricEval -> pycocoevalcap COCOEvalCap, utils/eval.py score_bleu -> nltk):
the restated coco-caption scorers and nltk BLEU checked against hand-computed
values of their published formulas (pycocoevalcap / nltk are absent, so these
known answers are the pin)."""
import json
import math

import pytest

from utils import coco_eval as CE
from utils.eval import score_bleu, score_ROUGEL, score_CIDErD


def _two_images():
    gts = {1: ["a b"], 2: ["d e"]}
    res = {1: ["a c"], 2: ["d e"]}
    return gts, res


def test_cider_d_known_answer():
    # df(a)=df(b)=df(ab)=df(d)=df(e)=df(de)=1, ref_len = log 2; image 1 shares
    # only the unigram 'a' with its ref: sim_1 = 1/2, sim_2 = 0 -> mean/4 * 10 = 1.25;
    # image 2 is exact on orders 1, 2 (no 3-/4-grams) -> 5.0
    gts, res = _two_images()
    score, scores = CE.Cider().compute_score(gts, res)
    assert scores.tolist() == pytest.approx([1.25, 5.0], abs=1e-12)
    assert score == pytest.approx(3.125, abs=1e-12)


def test_cider_d_identity_and_length_penalty():
    gts = {1: ["a man riding a horse"], 2: ["two dogs playing in snow"]}
    score, _ = CE.Cider().compute_score(gts, {k: list(v) for k, v in gts.items()})
    assert score == pytest.approx(10.0, abs=1e-12)
    # 3-word captions have no 4-grams: 3 of the 4 orders match
    s2, scores = CE.Cider().compute_score({1: ["a b c"], 2: ["x y z"]}, {1: ["a b c"], 2: ["x y z"]})
    assert s2 == pytest.approx(10.0 * 3 / 4, abs=1e-12)  # no 4-grams in 3-word captions


def test_bleu_corpus_known_answer():
    gts, res = _two_images()
    bleus, per_image = CE.Bleu(4).compute_score(gts, res)
    assert bleus[0] == pytest.approx(0.75, rel=1e-8)
    assert bleus[1] == pytest.approx(math.sqrt(0.375), rel=1e-8)
    assert per_image[0][1] == pytest.approx(1.0, rel=1e-8)  # image 2 exact
    # brevity penalty with the 'closest' reference length
    b, _ = CE.Bleu(4).compute_score({1: ["a b c d", "a b"]}, {1: ["a b c"]})
    # closest of (4, 2) to 3 is (1, 2) -> 2 ... ties broken by the shorter length
    assert b[0] == pytest.approx(1.0, rel=1e-6)


def test_rouge_l_known_answer():
    gts, res = _two_images()
    score, scores = CE.Rouge().compute_score(gts, res)
    assert scores.tolist() == pytest.approx([0.5, 1.0])
    assert score == pytest.approx(0.75)
    # lcs(a b c d, a c d e) = 3 -> P = R = 3/4 -> F = 3/4
    assert CE.Rouge().calc_score(["a b c d"], ["a c d e"]) == pytest.approx(0.75)


def test_ptb_tokenizer_rules():
    t = CE.ptb_tokenize_line
    assert t("A man's dog, running.") == ["a", "man", "'s", "dog", ",", "running", "."]
    assert t("Don't stop") == ["do", "n't", "stop"]
    assert t("a (red) car...") == ["a", "-LRB-", "red", "-RRB-", "car", "..."]
    assert t("the U.S. flag, 3.5 feet") == ["the", "u.s.", "flag", ",", "3.5", "feet"]
    out = CE.PTBTokenizer().tokenize({7: [{"caption": "A dog; running!"}, {"caption": "Two\ncats."}]})
    assert out == {7: ["a dog running", "two cats"]}


def test_nltk_sentence_bleu_restatement():
    # the reference's own example (utils/eval.py:44-48)
    reference = [['this', 'is', 'a', 'test'], ['this', 'is' 'test']]
    candidate = ['this', 'is', 'a', 'test']
    assert score_bleu(reference, candidate) == pytest.approx(1.0)
    # p1 = 2/2, p2 = 1/1, BP = exp(1 - 3/2)
    assert score_bleu([["the", "cat", "sat"]], ["the", "cat"], n=2) == pytest.approx(math.exp(-0.5))
    # method1 smoothing: no bigram match -> (0 + 0.1) / 1
    assert score_bleu([["a", "b"]], ["a", "c"], n=2) == pytest.approx(math.sqrt(0.5 * 0.1))
    assert score_bleu([["a"]], ["z"]) == 0
    assert score_bleu([["a"]], ["a"], n=0) == 0
    assert score_ROUGEL([["a", "c", "d", "e"]], ["a", "b", "c", "d"]) == pytest.approx(0.75)
    assert score_CIDErD([["a"]], ["a"]) is None


def test_metric_eval_end_to_end(tmp_path):
    """dataset.MetricEval over a COCO-format ground truth + a results file:
    loadRes, the PTB pass (case and punctuation dropped), CIDEr returned."""
    import dataset
    (tmp_path / "annotations").mkdir()
    gt = {"images": [{"id": 1, "file_name": "1.jpg"}, {"id": 2, "file_name": "2.jpg"},
                     {"id": 3, "file_name": "3.jpg"}],
          "annotations": [{"id": 10, "image_id": 1, "caption": "A b."},
                          {"id": 11, "image_id": 2, "caption": "D, e"},
                          {"id": 12, "image_id": 3, "caption": "unused"}]}
    with open(tmp_path / "annotations" / "captions_val.json", "w") as f:
        json.dump(gt, f)
    res = [{"image_id": 1, "caption": "a c"}, {"image_id": 2, "caption": "d e"}]
    rf = tmp_path / "res.json"
    with open(rf, "w") as f:
        json.dump(res, f)
    ev = dataset.MetricEval(str(tmp_path), "val")
    cider = ev(str(rf))
    assert cider == pytest.approx(3.125, abs=1e-12)  # only images 1, 2 are evaluated (dataset.py:291)
    assert ev.last_eval["ROUGE_L"] == pytest.approx(0.75)
    assert set(ev.last_eval) == {"Bleu_1", "Bleu_2", "Bleu_3", "Bleu_4", "ROUGE_L", "CIDEr"}
    with pytest.raises(AssertionError):
        ev([{"image_id": 99, "caption": "x"}])
