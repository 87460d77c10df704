"""BLEU restatement (qtx.bleu) pinned against nltk 3.6.5 outputs."""
import json
import os

import pytest

from qtx import bleu

G = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "bleu_golden.json")))


def test_sentence_bleu_matches_nltk():
    for c in G["sentences"]:
        assert bleu.sentence_bleu(c["refs"], c["hyp"]) == pytest.approx(c["bleu"], rel=1e-12, abs=1e-300)
        if c["bleu_m4"] is None:
            with pytest.raises(ValueError):
                bleu.sentence_bleu(c["refs"], c["hyp"], smoothing="method4")
        else:
            assert bleu.sentence_bleu(c["refs"], c["hyp"], smoothing="method4") == pytest.approx(
                c["bleu_m4"], rel=1e-12, abs=1e-300)


def test_corpus_bleu_matches_nltk():
    c = G["corpus"]
    assert bleu.corpus_bleu(c["list_of_references"], c["hypotheses"]) == pytest.approx(c["bleu"], rel=1e-12)


def test_reference_post_processing():
    itos = ["<s>", "</s>", "<blank>", "<unk>", "and", "to@@", "day", "i", "&apos;m"]
    ids = [0, 4, 5, 6, 7, 2, 1, 2, 2]
    assert bleu.hypothesis_tokens(ids, itos) == ["and", "today", "i"]
    assert bleu.target_tokens(["<s>", "and", "to@@", "day", "i", "</s>"]) == ["and", "today", "i"]
    # identical decodes score identically: GPU ids == oracle ids => identical BLEU
    h = bleu.hypothesis_tokens(ids, itos)
    assert bleu.sentence_bleu([h], h) == 1.0 or len(h) < 4
