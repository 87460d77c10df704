"""Golden BLEU values from nltk 3.6.5 (run with /opt/conda/bin/python3.9, the only
interpreter here with nltk): random token sequences over a small vocabulary, sentence
BLEU (method0 / method4) and corpus BLEU.  Writes tests/golden/bleu_golden.json."""
import json
import os
import random
import warnings

from nltk.translate.bleu_score import SmoothingFunction, corpus_bleu, sentence_bleu

warnings.filterwarnings("ignore")
rng = random.Random(20241223)
V = [f"w{i}" for i in range(12)]
cases = []
for t in range(60):
    nref = 1 + (t % 3)
    refs = [[rng.choice(V) for _ in range(rng.randint(1, 14))] for _ in range(nref)]
    hyp = [rng.choice(V) for _ in range(rng.randint(0, 14))] if t % 7 else list(refs[0])
    try:
        m4 = sentence_bleu(refs, hyp, smoothing_function=SmoothingFunction().method4)
    except ValueError:          # nltk: log(0) when a 1-token hypothesis has no matches
        m4 = None
    cases.append({"refs": refs, "hyp": hyp, "bleu": sentence_bleu(refs, hyp), "bleu_m4": m4})
corp = {"list_of_references": [c["refs"] for c in cases[:40]],
        "hypotheses": [c["hyp"] for c in cases[:40]]}
corp["bleu"] = corpus_bleu(corp["list_of_references"], corp["hypotheses"])
out = {"nltk": "3.6.5", "sentences": cases, "corpus": corp}
with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "bleu_golden.json"), "w") as f:
    json.dump(out, f)
print(len(cases), corp["bleu"])
