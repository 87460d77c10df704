"""The evaluation tail on the GPU path: checkpoint ingestion feeding the
device model, and the fixed-order IWSLT14 test-set run scored with the reference's BLEU.
Trained-model BLEU stays unpinned (no checkpoint exists here); with synthetic weights the
check is that the GPU ids — and so every BLEU number — equal the oracle's."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "golden", "iwslt14")


@pytest.fixture(scope="module")
def torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_checkpoint_model_decodes_identically(torch, tmp_path, state_dict, gpu_model):
    from qtx.decode import greedy_decode, make_src_mask
    from qtx.model import QtxModel
    from qtx.weights import load_checkpoint
    p = tmp_path / "iwslt14_model_00.pt"
    torch.save({k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in state_dict.items()}, p)
    m2 = QtxModel(load_checkpoint(str(p)))
    rng = np.random.default_rng(12)
    src = np.full((4, 40), 2, np.int64)
    for b, n in enumerate([40, 33, 12, 27]):
        src[b, 0], src[b, n - 1] = 0, 1
        src[b, 1:n - 1] = rng.integers(4, 5337, n - 2)
    m = make_src_mask(src)
    np.testing.assert_array_equal(greedy_decode(m2, src, m, 72, 0),
                                  greedy_decode(gpu_model, src, m, 72, 0))


def test_test_set_bleu_gpu_equals_oracle(torch, gpu_model, oracle_model):
    from qtx import data as D
    vs, vt = D.load_vocab(FIX)
    pairs = D.read_pairs(os.path.join(FIX, "test_sample.de.bpe"),
                         os.path.join(FIX, "test_sample.en.bpe"))
    # the whole sample (49 sentences, src padded to 128, one of them cropped) in file order
    r = D.evaluate(gpu_model, pairs, vs, vt, batch_size=32, max_padding=128)
    assert r.ids.shape == (len(pairs), 72) and (r.ids[:, 0] == 0).all()
    assert 0.0 <= r.bleu <= 1.0
    # two sentences through the oracle: same ids, same hypotheses, same BLEU
    pick = [3, len(pairs) - 1]
    sub = [pairs[i] for i in pick]
    ro = D.evaluate(None, sub, vs, vt, batch_size=2, max_padding=128,
                    decode=lambda s, m, n: oracle_model.greedy_decode(s, m, n))
    np.testing.assert_array_equal(ro.ids, r.ids[pick])
    rg = D.score(r.ids[pick], D.collate(sub, vs, vt, 128)[1], vt)
    assert rg.hypotheses == ro.hypotheses and rg.bleu == ro.bleu
