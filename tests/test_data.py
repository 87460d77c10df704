"""The reference's evaluation tail on the host: vocabularies, the
collate_batch id pipeline, BLEU post-processing, and checkpoint ingestion (weights_only)."""
import os

import numpy as np
import pytest

from qtx import data as D
from qtx import weights as W

FIX = os.path.join(os.path.dirname(__file__), "golden", "iwslt14")


@pytest.fixture(scope="module")
def vocabs():
    return D.load_vocab(FIX)


@pytest.fixture(scope="module")
def pairs():
    return D.read_pairs(os.path.join(FIX, "test_sample.de.bpe"),
                        os.path.join(FIX, "test_sample.en.bpe"))


def test_vocab_sizes_and_specials(vocabs):
    vs, vt = vocabs
    # make_model(len(vocab_src), len(vocab_tgt)) = (5337, 4444)
    assert (len(vs), len(vt)) == (5337, 4444)
    assert vs.itos[:4] == ["<s>", "</s>", "<blank>", "<unk>"] == vt.itos[:4]
    assert vs.itos[4:7] == [",", ".", "und"] and vt.itos[4:7] == [",", ".", "the"]
    assert vs(["und", "no-such-word@@"]) == [6, 3]


def test_collate_matches_collate_batch(vocabs, pairs):
    vs, vt = vocabs
    src, tgt = D.collate(pairs, vs, vt, max_padding=128)
    assert src.shape == tgt.shape == (len(pairs), 128)
    for row, (s, _) in zip(src, pairs):
        toks = s.split(" ")
        n = min(len(toks) + 2, 128)
        assert row[0] == 0
        assert list(row[1:n - 1]) == vs(toks)[:n - 2]
        if len(toks) + 2 <= 128:
            assert row[n - 1] == 1 and (row[n:] == 2).all()
    # the longest test sentence (270 tokens) is cropped by F.pad's negative padding: no
    # </s>, no <blank>
    long = src[-1]
    assert (long != 2).all() and 1 not in long[1:]


def test_score_post_processing(vocabs, pairs):
    _, vt = vocabs
    short = [p for p in pairs if len(p[1].split(" ")) < 60][:3]
    _, tgt = D.collate(short, *vocabs, max_padding=128)
    # "decoded" ids equal to the targets: hypothesis == reference, BLEU 1
    r = D.score(tgt, tgt, vt)
    assert r.hypotheses == r.references
    assert r.bleu == pytest.approx(1.0)
    # pads dropped, cut at the first </s>, BPE joins undone
    ids = np.array([[0, vt.stoi["ple@@"], vt.stoi["as@@"], vt.stoi["ure"], 2, 1, 5, 5]])
    assert D.score(ids, tgt[:1], vt).hypotheses == [["pleasure"]]


def test_evaluate_fixed_order_with_a_decoder(vocabs, pairs):
    """evaluate() batches in file order and hands each batch to the decoder with the
    reference's (src != pad) mask."""
    vs, vt = vocabs
    seen = []

    def fake_decode(s, m, n):
        seen.append(s.copy())
        assert m.shape == (len(s), 1, s.shape[1]) and (m[:, 0] == (s != 2)).all()
        out = np.zeros((len(s), n), np.int64)
        out[:, 1] = 4
        out[:, 2] = 1
        return out

    r = D.evaluate(None, pairs[:10], vs, vt, batch_size=4, max_padding=128, decode=fake_decode)
    assert [len(s) for s in seen] == [4, 4, 2]
    assert np.array_equal(np.concatenate(seen), D.collate(pairs[:10], vs, vt, 128)[0])
    assert r.hypotheses == [[","]] * 10 and 0.0 <= r.bleu <= 1.0


def test_checkpoint_round_trip(tmp_path):
    """torch.save(state_dict) -> load_checkpoint (weights_only) -> identical arrays; the
    reference's pe buffers ride along; a missing tensor is an error."""
    import torch
    sd = W.synthetic_state_dict(7, ln_random=True)
    p = tmp_path / "model.pt"
    torch.save({k: torch.from_numpy(v.copy()) for k, v in sd.items()}, p)
    got = W.load_checkpoint(str(p))
    assert set(got) == set(sd)
    for k in sd:
        np.testing.assert_array_equal(got[k], sd[k])
    del sd["decoder.norm.a_2"]
    torch.save({k: torch.from_numpy(v.copy()) for k, v in sd.items()}, p)
    with pytest.raises(KeyError, match="lacks"):
        W.load_checkpoint(str(p))
