"""Named intermediates (the reference executor's weight_dict, onnx_optimized_inference.py:57,
300-301) through run_module(expose_intermediates=...) and the op-by-op traced executor."""
import json
import os

import numpy as np
import pytest

from oracle import qtx_oracle as O
from qtx import trace as T

TARGETS = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                      "matmul_targets.json")))


def names_of(t):
    """(input, weight, output) names our map gives a campaign target."""
    from qtx.fault import matmul_target
    mod = "encoder" if t["module"].startswith("Encoder") else "decoder"
    _, L, lin = matmul_target(t["target_layer"], mod)
    nm = T.encoder_names(L) if mod == "encoder" else T.decoder_names(L)
    a, w = nm["act"], nm["weight"]
    mm = nm["matmul"][lin]
    ins = {"QK": ("q", "k"), "PV": ("P", "v"), "CQK": ("c_q", "c_k"), "CPV": ("c_P", "c_v"),
           "FFN1": ("ffn1_in", "FFN1"), "FFN2": ("ffn2_in", "FFN2")}[lin]
    ins = (a[ins[0]], (w if lin.startswith("FFN") else a)[ins[1]])
    return f"Round_{ins[0]}_out0", f"Round_{ins[1]}_out0", f"MatMul_{mm}_out0"


def test_graph_names_match_campaign_target_files():
    """Every reference target file (input/{encoder,decoder}/matmul_*.json) names exactly
    the tensors of our graph-name map."""
    assert len(TARGETS) == 60
    for t in TARGETS:
        assert names_of(t) == (t["input_tensor"], t["weight_tensor"], t["output_tensor"]), t


def _src(B, S, lens, seed=3):
    rng = np.random.default_rng(seed)
    src = np.full((B, S), 2, np.int64)
    for b, n in enumerate(lens):
        src[b, 0], src[b, n - 1] = 0, 1
        src[b, 1:n - 1] = rng.integers(4, 5337, n - 2)
    return src


@pytest.mark.gpu
def test_traced_encoder_equals_fused_and_oracle(gpu_model, oracle_model):
    from qtx.session import run_module
    src = _src(2, 16, [16, 11])
    x = oracle_model.embed(src, oracle_model.src_lut)
    feeds = {"global_in": x, "global_in_1": (src != 2)[:, None, :]}
    fused, _ = run_module("Encoder", feeds, model=gpu_model)
    out, wd = run_module("Encoder", feeds, model=gpu_model, expose_intermediates="weights")
    np.testing.assert_array_equal(out["global_out"], fused["global_out"])
    # layer 0 input codes and Q codes are the oracle's
    lp = oracle_model.enc[0]
    h = O.layer_norm(x, *lp["ln"][0])
    qx, sx = O.quant_rows(h.reshape(-1, 512))
    nm = T.encoder_names(0)
    np.testing.assert_array_equal(wd[f"Round_{nm['act']['in']}_out0"].reshape(-1, 512), qx)
    np.testing.assert_array_equal(wd[f"Round_{nm['act']['in']}_scale"].reshape(-1), sx)
    qq, sq = lp["attn"][0](h, quantize_output=True)
    np.testing.assert_array_equal(wd[f"Round_{nm['act']['q']}_out0"], qq)
    np.testing.assert_array_equal(wd[f"Round_{nm['weight']['Q']}_out0"], lp["attn"][0].q.T)
    # a campaign-style lookup: every encoder FFN target's output is input x weight, exactly
    n = 0
    for t in TARGETS:
        if not t["module"].startswith("Encoder"):
            continue
        if t["module"].endswith("FC"):
            a = wd[t["input_tensor"]]
            w = wd[t["weight_tensor"]]
            acc = np.einsum("bsk,kn->bsn", a.astype(np.float64), w.astype(np.float64))
            np.testing.assert_array_equal(wd[t["output_tensor"]], acc.astype(np.float32))
            n += 1
        elif t["module"].endswith("FirstMatMul"):    # QK^T: q codes x k codes per head
            q4 = O.split_heads(wd[t["input_tensor"]], 8).astype(np.float64)
            k4 = O.split_heads(wd[t["weight_tensor"]], 8).astype(np.float64)
            acc = np.einsum("bhid,bhjd->bhij", q4, k4)
            np.testing.assert_array_equal(wd[t["output_tensor"]], acc.astype(np.float32))
            n += 1
        else:                                         # PV: P codes x v codes -> the context
            L = int(t["target_layer"].split("_")[1]) // 8
            a = T.encoder_names(L)["act"]
            qr, kr, vr = (f"Round_{a[k]}" for k in ("q", "k", "v"))
            q4, k4, v4 = (O.split_heads(wd[f"{r}_out0"].astype(np.int8), 8) for r in (qr, kr, vr))
            sq, sk, sv = (wd[f"{r}_scale"][..., 0] for r in (qr, kr, vr))
            pc = O.softmax_quant(O.attention_scores(q4, sq, k4, sk, (src != 2)[:, None, :]))
            np.testing.assert_array_equal(wd[t["input_tensor"]], pc.astype(np.float32))
            np.testing.assert_array_equal(wd[t["output_tensor"]], O.attention_pv(pc, v4, sv))
            n += 1
    assert n == 24


@pytest.mark.gpu
def test_traced_decoder_equals_fused(gpu_model, oracle_model):
    from qtx.session import run_module
    src = _src(2, 12, [12, 9])
    mem = oracle_model.encode(oracle_model.embed(src, oracle_model.src_lut), (src != 2)[:, None, :])
    ys = np.array([[0, 7, 9, 11, 5], [0, 4, 4, 8, 20]])
    y = oracle_model.embed(ys, oracle_model.tgt_lut)
    feeds = {"global_in": y, "global_in_1": mem, "global_in_2": (src != 2)[:, None, :],
             "global_in_3": O.subsequent_mask(5)}
    fused, _ = run_module("Decoder", feeds, model=gpu_model)
    out, wd = run_module("Decoder", feeds, model=gpu_model, expose_intermediates=True)
    np.testing.assert_array_equal(out["global_out"], fused["global_out"])
    for t in TARGETS:
        if t["module"].startswith("Decoder") and t["module"].endswith("FC"):
            assert wd[t["input_tensor"]].shape[:2] == (2, 5)
            assert t["output_tensor"] in wd
        if t["module"].startswith("Decoder") and "MatMul" in t["module"] and t["target_layer"] in (
                "MatMul_19", "MatMul_31"):           # cross QK^T: q codes x memory K codes
            assert wd[t["input_tensor"]].shape == (2, 5, 512)
            assert wd[t["weight_tensor"]].shape == (2, 12, 512)
            q4 = O.split_heads(wd[t["input_tensor"]], 8).astype(np.float64)
            k4 = O.split_heads(wd[t["weight_tensor"]], 8).astype(np.float64)
            np.testing.assert_array_equal(wd[t["output_tensor"]],
                                          np.einsum("bhid,bhjd->bhij", q4, k4).astype(np.float32))
    # every attention MatMul of every layer is stored by name: self QK^T [B,H,T,T], cross
    # P codes [B,H,T,S], self / cross PV contexts per head
    for L in range(6):
        nm = T.decoder_names(L)
        mm, a = nm["matmul"], nm["act"]
        assert wd[f"MatMul_{mm['QK']}_out0"].shape == (2, 8, 5, 5)
        assert wd[f"Round_{a['c_P']}_out0"].shape == (2, 8, 5, 12)
        assert wd[f"MatMul_{mm['PV']}_out0"].shape == wd[f"MatMul_{mm['CPV']}_out0"].shape == (2, 8, 5, 64)
        # causal mask: P of a future key is 0
        assert (wd[f"Round_{a['P']}_out0"][:, :, 0, 1:] == 0).all()


@pytest.mark.gpu
def test_expose_intermediates_rejects_a_fault(gpu_model):
    from qtx.fault import Fault
    from qtx.session import run_module
    x = np.zeros((1, 4, 512), np.float32)
    with pytest.raises(ValueError):
        run_module("Encoder", {"global_in": x, "global_in_1": np.ones((1, 1, 4), bool)},
                   model=gpu_model, inject_parameters=Fault("INPUT", 0, 0, "Q"),
                   expose_intermediates=True)
