"""Copies the data files the qtx.data tests read into tests/golden/iwslt14/ (run here,
where /root/reference exists; the GPU box only sees the copies).

* data/vocab/vocab.{de,en}.32000 — the vocabularies (qtx.data.load_vocab rebuilds the
  reference's vocab.pt itos lists from them);
* the first 48 sentence pairs of data/test.{de,en}.bpe plus the longest German test
  sentence (it exceeds max_padding - 2 = 126 tokens: collate_batch crops it).
"""
import os
import shutil

REF = "/root/reference/data"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "iwslt14")

os.makedirs(OUT, exist_ok=True)
for lang in ("de", "en"):
    shutil.copyfile(os.path.join(REF, "vocab", f"vocab.{lang}.32000"),
                    os.path.join(OUT, f"vocab.{lang}.32000"))
with open(os.path.join(REF, "test.de.bpe"), encoding="utf-8") as f:
    de = f.readlines()
with open(os.path.join(REF, "test.en.bpe"), encoding="utf-8") as f:
    en = f.readlines()
longest = max(range(len(de)), key=lambda i: len(de[i].split(" ")))
keep = list(range(48)) + [longest]
for lang, lines in (("de", de), ("en", en)):
    with open(os.path.join(OUT, f"test_sample.{lang}.bpe"), "w", encoding="utf-8") as f:
        f.writelines(lines[i] for i in keep)
print("longest test sentence:", longest, len(de[longest].split(" ")), "tokens")
