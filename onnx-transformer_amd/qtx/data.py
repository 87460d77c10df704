"""The reference's IWSLT14 evaluation pipeline in a fixed order.

What the reference does (reference/onnx_reference_inference.py):

* sentence pairs = the lines of ``data/{valid,test}.{de,en}.bpe`` with the trailing
  newline cut (``create_dataset``, :313-324);
* tokens = ``text.split(" ")`` (``tokenize``, :180-183: the BPE text is pre-tokenized);
* ids = vocabulary lookup, unknown words -> ``<unk>`` (:226-227), ``<s>`` ... ``</s>``
  around them, padded with ``<blank>`` = 2 to ``max_padding`` (``collate_batch``,
  :238-292); ``torch.nn.functional.pad`` with a negative amount CROPS, so a sentence
  longer than ``max_padding - 2`` tokens loses its tail and its ``</s>``;
* greedy decode of 72 steps, then the token post-processing and nltk BLEU of
  :557-591 (restated in :mod:`qtx.bleu`).

The vocabularies are torchtext ``Vocab`` objects pickled in ``data/vocab/vocab.pt``; that
file is never unpickled here.  Their ``itos`` lists are exactly the four specials
``<s> </s> <blank> <unk>`` followed by the words of ``data/vocab/vocab.{de,en}.32000`` in
file order (5 333 + 4 = 5 337 German, 4 440 + 4 = 4 444 English entries; checked once
by disassembling the pickle's string constants with ``pickletools``, which executes
nothing), so :func:`load_vocab` rebuilds them from the text files.

The reference shuffles its validation loader (``shuffle=True``, :364-370); here the
order is the file order, so a run is reproducible.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

from . import bleu
from .weights import BOS, EOS, PAD, UNK

SPECIALS = ("<s>", "</s>", "<blank>", "<unk>")


@dataclass
class Vocab:
    itos: list

    def __post_init__(self):
        self.stoi = {w: i for i, w in enumerate(self.itos)}

    def __len__(self):
        return len(self.itos)

    def __call__(self, tokens):
        """torchtext Vocab.__call__ with default index <unk> (:226-227)."""
        return [self.stoi.get(t, UNK) for t in tokens]


def read_vocab_file(path: str) -> Vocab:
    """``word count`` lines (most frequent first) -> Vocab with the four specials first."""
    words = []
    with open(path, encoding="utf-8") as f:
        for line in f.read().split("\n"):
            if line:
                words.append(line.rsplit(" ", 1)[0])
    return Vocab(list(SPECIALS) + words)


def load_vocab(vocab_dir: str):
    """(vocab_src, vocab_tgt) of the reference: German source, English target."""
    return (read_vocab_file(os.path.join(vocab_dir, "vocab.de.32000")),
            read_vocab_file(os.path.join(vocab_dir, "vocab.en.32000")))


def read_pairs(src_path: str, tgt_path: str, limit: int | None = None):
    """create_dataset (:313-324): zipped lines, last character (the newline) cut."""
    with open(src_path, encoding="utf-8") as fs, open(tgt_path, encoding="utf-8") as ft:
        ls, lt = fs.readlines(), ft.readlines()
    pairs = [(s[:-1], t[:-1]) for s, t in zip(ls, lt)]
    return pairs[:limit] if limit is not None else pairs


def tokenize(text: str):
    return text.split(" ")


def encode_sentence(text: str, vocab: Vocab, max_padding: int) -> np.ndarray:
    """<s> ids </s>, then padded with <blank> (or cropped) to max_padding (:250-285)."""
    ids = [BOS] + vocab(tokenize(text)) + [EOS]
    ids = ids[:max_padding] + [PAD] * max(0, max_padding - len(ids))
    return np.asarray(ids, np.int64)


def collate(pairs, vocab_src: Vocab, vocab_tgt: Vocab, max_padding: int = 128):
    """collate_batch (:238-292) -> (src int64 [B, max_padding], tgt int64 [B, max_padding])."""
    src = np.stack([encode_sentence(s, vocab_src, max_padding) for s, _ in pairs])
    tgt = np.stack([encode_sentence(t, vocab_tgt, max_padding) for _, t in pairs])
    return src, tgt


@dataclass
class EvalResult:
    bleu: float                 # corpus BLEU (nltk corpus_bleu, no smoothing)
    sentence_bleu: list         # per sentence, method4 smoothing (the campaign metric)
    hypotheses: list            # post-processed hypothesis token lists
    references: list            # post-processed reference token lists
    ids: np.ndarray             # int64 [N, max_len] greedy ids


def score(ids, tgt, vocab_tgt: Vocab) -> EvalResult:
    """The post-processing + BLEU of :557-591 over decoded ids and target ids."""
    refs, hyps, sb = [], [], []
    for row, t in zip(np.asarray(ids), np.asarray(tgt)):
        ref = bleu.target_tokens([vocab_tgt.itos[x] for x in t if x != PAD])
        hyp = bleu.hypothesis_tokens(row, vocab_tgt.itos, PAD)
        refs.append([ref])
        hyps.append(hyp)
        try:
            sb.append(bleu.sentence_bleu([ref], hyp, smoothing="method4"))
        except ValueError:      # nltk method4 divides by log(1) for one-token hypotheses
            sb.append(None)
    return EvalResult(bleu.corpus_bleu(refs, hyps), sb, hyps, [r[0] for r in refs],
                      np.asarray(ids))


def evaluate(model, pairs, vocab_src: Vocab, vocab_tgt: Vocab, batch_size: int = 32,
             max_padding: int = 128, max_len: int = 72, decode=None) -> EvalResult:
    """Greedy-decode ``pairs`` in file order, ``batch_size`` sentences per call, and score
    them.  ``decode(src, src_mask, max_len) -> ids`` defaults to the qtx GPU path."""
    if decode is None:
        from .decode import greedy_decode

        def decode(s, m, n):
            return greedy_decode(model, s, m, n, BOS)
    src, tgt = collate(pairs, vocab_src, vocab_tgt, max_padding)
    out = []
    for b0 in range(0, len(pairs), batch_size):
        s = src[b0:b0 + batch_size]
        out.append(np.asarray(decode(s, (s != PAD)[:, None, :], max_len)))
    ids = np.concatenate(out) if out else np.zeros((0, max_len), np.int64)
    return score(ids, tgt, vocab_tgt)
