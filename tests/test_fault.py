"""Fault injection: the reference's fault models on the qtx path.

CPU tests: MatMul-name mapping, fault drawing, the oracle's fault semantics (a flipped
int8 operand propagated through the MatMul == the MatMul recomputed on the flipped
operand, windows, RANDOM outputs).  GPU tests: encoder / decoder forward and greedy decode
with a fault == the oracle with the same fault, bit for bit."""
import numpy as np
import pytest

from oracle import qtx_oracle as O
from qtx import fault as F

f32 = np.float32


def test_matmul_names():
    assert F.matmul_target("MatMul_6", "Encoder") == (0, 0, "FFN1")      # matmul_6.json
    assert F.matmul_target("MatMul_47", "Encoder") == (0, 5, "FFN2")
    assert F.matmul_target("MatMul_13", "Encoder") == (0, 1, "O")
    assert F.matmul_target("MatMul_0", "Decoder") == (1, 0, "CK")
    assert F.matmul_target("MatMul_11", "Decoder") == (1, 5, "CV")
    assert F.matmul_target("MatMul_12", "Decoder") == (1, 0, "Q")
    assert F.matmul_target("MatMul_22", "Decoder") == (1, 0, "FFN1")     # matmul_22.json
    assert F.matmul_target("MatMul_23", "Decoder") == (1, 0, "FFN2")     # matmul_23.json
    assert F.matmul_target("MatMul_82", "Decoder") == (1, 5, "FFN1")
    assert F.matmul_target("MatMul_3", "Encoder") == (0, 0, "QK")       # matmul_3.json
    assert F.matmul_target("MatMul_12", "Encoder") == (0, 1, "PV")
    for bad in ("Add_3", "MatMul_48"):
        with pytest.raises(ValueError):
            F.matmul_target(bad, "Encoder")
    assert F.matmul_target("MatMul_15", "Decoder") == (1, 0, "QK")       # matmul_15.json
    assert F.matmul_target("MatMul_16", "Decoder") == (1, 0, "PV")
    assert F.matmul_target("MatMul_19", "Decoder") == (1, 0, "CQK")      # matmul_19.json
    assert F.matmul_target("MatMul_20", "Decoder") == (1, 0, "CPV")


def test_reference_target_files_map():
    """Every target of the reference's campaign files (QK^T, PV, FFN1, FFN2 per layer)
    maps to the matching (module, layer, target)."""
    import glob
    import json
    import os
    d = "/root/reference/input"
    if not os.path.isdir(d):
        pytest.skip("reference not mounted")
    n = 0
    for mod in ("encoder", "decoder"):
        for p in glob.glob(f"{d}/{mod}/matmul_*.json"):
            j = json.load(open(p))
            kind = j["module"].split("/")[1]          # FirstFC / SecondFC / First|SecondMatMul
            _, _, lin = F.matmul_target(j["target_layer"], j["module"])
            want = {"FirstFC": ("FFN1",), "SecondFC": ("FFN2",), "FirstMatMul": ("QK", "CQK"),
                    "SecondMatMul": ("PV", "CPV")}[kind]
            assert lin in want, (p, lin)
            n += 1
    assert n == 24 + 36


def test_random_fault_draws():
    rng = np.random.default_rng(0)
    for kind in ("INPUT", "WEIGHT", "INPUT16", "WEIGHT16", "RANDOM"):
        f = F.random_fault(rng, kind, 0, 2, "FFN1", rows=40, bit=3)
        N, K = F.linear_shape("FFN1")
        if kind.startswith("INPUT"):
            assert 0 <= f.row < 40 and 0 <= f.col < K
        elif kind.startswith("WEIGHT"):
            assert 0 <= f.row < N and 0 <= f.col < K
        if kind == "INPUT16":
            assert f.win_start % 16 == 0 and f.win_len == 16
        if kind == "WEIGHT16":
            assert f.win_start % 16 == 0 and 1 <= f.win_len <= 15
    g = np.ones((40, 2048), f32)
    f = F.random_fault(rng, "RANDOM_BITFLIP", 0, 0, "FFN1", 40, golden_output=g)
    assert f.value != 1.0
    f = F.from_inject_parameters({"inject_type": "WEIGHT", "faulty_operation_name": "MatMul_14",
                                  "targetted_module": "Encoder", "faulty_bit_position": 7}, 16, rng)
    assert (f.module, f.layer, f.linear, f.bit) == (0, 1, "FFN1", 7)


def _lin(rng, N=64, K=128):
    return O.QLinear(rng.standard_normal((N, K)).astype(f32) * 0.1,
                     rng.standard_normal(N).astype(f32) * 0.1)


def test_oracle_input_fault_is_flipped_operand():
    rng = np.random.default_rng(1)
    lin = _lin(rng)
    x = rng.standard_normal((10, 128)).astype(f32)
    qx, sx = O.quant_rows(x)
    flipped = qx.copy()
    flipped[3, 17] = np.int8(np.uint8(flipped[3, 17].view(np.uint8) ^ 64).view(np.int8))
    want = O.linear_epilogue(O.int_gemm(flipped, lin.q), sx, lin.s, lin.b)
    got = lin(x, fault=dict(kind="INPUT", row=3, col=17, bit=6, lo=0, hi=64, value=0))
    np.testing.assert_array_equal(got, want)
    golden = lin(x)
    w16 = lin(x, fault=dict(kind="INPUT16", row=3, col=17, bit=6, lo=16, hi=32, value=0))
    np.testing.assert_array_equal(w16[:, 16:32], want[:, 16:32])
    np.testing.assert_array_equal(w16[:, :16], golden[:, :16])
    np.testing.assert_array_equal(w16[:, 32:], golden[:, 32:])


def test_oracle_weight_and_output_faults():
    rng = np.random.default_rng(2)
    lin = _lin(rng)
    x = rng.standard_normal((12, 128)).astype(f32)
    golden = lin(x)
    wf = lin(x, fault=dict(kind="WEIGHT", row=5, col=9, bit=7, lo=0, hi=12, value=0))
    diff = np.argwhere(wf != golden)
    assert set(diff[:, 1]) <= {5}
    w16 = lin(x, fault=dict(kind="WEIGHT16", row=5, col=9, bit=7, lo=4, hi=8, value=0))
    np.testing.assert_array_equal(w16[4:8], wf[4:8])
    np.testing.assert_array_equal(w16[:4], golden[:4])
    of = lin(x, relu=True, fault=dict(kind="OUTPUT", row=2, col=3, bit=0, lo=0, hi=0, value=-7.0))
    g = lin(x, relu=True)
    assert of[2, 3] == 0.0 and np.sum(of != g) <= 1


# ------------------------------------------------------------------------------ GPU
@pytest.fixture(scope="module")
def torch_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _enc_inputs(oracle_model, B, S, seed):
    rng = np.random.default_rng(seed)
    src = np.full((B, S), 2, np.int64)
    for b, n in enumerate(rng.integers(4, S + 1, B)):
        src[b, 0], src[b, n - 1] = 0, 1
        src[b, 1:n - 1] = rng.integers(4, 5337, max(n - 2, 0))
    m = (src != 2)[:, None, :]
    return src, m, oracle_model.embed(src, oracle_model.src_lut)


ENC_CASES = [("INPUT", "FFN1", 3), ("INPUT16", "FFN2", 5), ("WEIGHT", "Q", 7), ("WEIGHT16", "FFN1", 6),
             ("RANDOM", "O", 0), ("INPUT", "V", 2), ("WEIGHT", "K", 4), ("RANDOM", "FFN1", 0)]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,linear,bit", ENC_CASES)
def test_encoder_fault_matches_oracle(torch_gpu, gpu_model, oracle_model, kind, linear, bit):
    torch = torch_gpu
    B, S = 3, 24
    src, m, x = _enc_inputs(oracle_model, B, S, 11)
    rng = np.random.default_rng(hash((kind, linear)) % 2**32)
    f = F.random_fault(rng, kind, 0, int(rng.integers(6)), linear, B * S, bit=bit)
    if kind == "RANDOM":
        f.value = float(rng.standard_normal() * 50)
    xd = torch.from_numpy(x).cuda()
    md = torch.from_numpy(m.reshape(B, S).astype(np.uint8)).cuda()
    out = gpu_model.encode(xd, md, fault=f).cpu().numpy()
    ref = oracle_model.encode(x, m, fault=f.as_dict())
    np.testing.assert_array_equal(out, ref)
    if kind != "WEIGHT16":          # a golden run differs (WEIGHT16 may hit pad rows only)
        assert not np.array_equal(out, gpu_model.encode(xd, md).cpu().numpy()) or bit < 6


@pytest.mark.gpu
@pytest.mark.parametrize("kind,linear", [("WEIGHT", "CK"), ("INPUT", "CV"), ("INPUT16", "FFN1"),
                                         ("WEIGHT16", "Q"), ("RANDOM", "CO"), ("INPUT", "CQ")])
def test_decoder_fault_matches_oracle(torch_gpu, gpu_model, oracle_model, kind, linear):
    torch = torch_gpu
    B, S, T = 2, 20, 6
    src, m, x = _enc_inputs(oracle_model, B, S, 12)
    rng = np.random.default_rng(7)
    memory = oracle_model.encode(x, m)
    ys = rng.integers(4, 4444, (B, T))
    y = oracle_model.embed(ys, oracle_model.tgt_lut)
    tm = np.tril(np.ones((1, T, T), np.uint8))
    rows = B * S if linear in ("CK", "CV") else B * T
    f = F.random_fault(rng, kind, 1, int(rng.integers(6)), linear, rows, bit=6)
    if kind == "RANDOM":
        f.value = -123.5
    T_ = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = gpu_model.decode(T_(y), T_(memory), T_(m.reshape(B, S).astype(np.uint8)),
                           T_(tm[0]), fault=f).cpu().numpy()
    ref = oracle_model.decode(y, memory, m, tm, fault=f.as_dict())
    np.testing.assert_array_equal(out, ref)


@pytest.mark.gpu
def test_greedy_decode_with_encoder_fault(torch_gpu, gpu_model, oracle_model):
    torch = torch_gpu
    B, S = 2, 16
    src, m, _ = _enc_inputs(oracle_model, B, S, 13)
    f = F.Fault("WEIGHT", 0, 2, "FFN2", row=17, col=100, bit=7)
    ids = gpu_model.greedy(torch.from_numpy(src).cuda(),
                           torch.from_numpy(m.reshape(B, S).astype(np.uint8)).cuda(),
                           max_len=12, fault=f).cpu().numpy()
    ref = oracle_model.greedy_decode(src, m, max_len=12, fault=f.as_dict())
    np.testing.assert_array_equal(ids, ref)


@pytest.mark.gpu
def test_fault_bad_index_rejected(torch_gpu, gpu_model):
    torch = torch_gpu
    from qtx._lib import QtxError
    x = torch.zeros((1, 8, 512), device="cuda")
    md = torch.ones((1, 8), dtype=torch.uint8, device="cuda")
    with pytest.raises(QtxError):
        gpu_model.encode(x, md, fault=F.Fault("INPUT", 0, 0, "FFN1", row=8, col=0))
    with pytest.raises(QtxError):
        gpu_model.encode(x, md, fault=F.Fault("WEIGHT", 0, 0, "CK", row=0, col=0))


@pytest.mark.gpu
def test_run_module_inject_parameters(torch_gpu, gpu_model, oracle_model, golden_model):
    """run_module with the reference's inject_parameters dict (FFN target of a campaign
    file, input/encoder/matmul_6.json) == the oracle with the drawn fault."""
    from qtx.session import run_module
    feeds = {"global_in": golden_model["enc_in"], "global_in_1": golden_model["src_mask"]}
    p = {"inject_type": "INPUT", "faulty_operation_name": "MatMul_6",
         "targetted_module": "Encoder", "faulty_bit_position": 7}
    outs, wd = run_module("Encoder", feeds, None, {}, None, inject_parameters=p,
                          model=gpu_model, rng=np.random.default_rng(3))
    f = wd["qtx_fault"]
    assert (f.module, f.layer, f.linear, f.bit) == (0, 0, "FFN1", 7)
    ref = oracle_model.encode(golden_model["enc_in"], golden_model["src_mask"], fault=f.as_dict())
    np.testing.assert_array_equal(outs["global_out"], ref)


@pytest.mark.gpu
def test_run_module_fault_for_other_module_is_golden(torch_gpu, gpu_model, oracle_model,
                                                     golden_model):
    """An INPUT fault aimed at the decoder leaves an encoder run golden, as the reference's
    `module in inject_parameters["targetted_module"]` test does
    (onnx_optimized_inference.py:74)."""
    from qtx.session import run_module
    feeds = {"global_in": golden_model["enc_in"], "global_in_1": golden_model["src_mask"]}
    p = {"inject_type": "INPUT", "faulty_operation_name": "MatMul_15",
         "targetted_module": "Decoder", "faulty_bit_position": 7}
    outs, wd = run_module("Encoder", feeds, None, {}, None, inject_parameters=p,
                          model=gpu_model, rng=np.random.default_rng(3))
    assert "qtx_fault" not in wd
    ref = oracle_model.encode(golden_model["enc_in"], golden_model["src_mask"])
    np.testing.assert_array_equal(outs["global_out"], ref)


@pytest.mark.gpu
def test_run_module_random_fault_on_foreign_name_is_golden(torch_gpu, gpu_model, oracle_model,
                                                           golden_model):
    """A RANDOM fault names a node alone (onnx_optimized_inference.py:59): on a module whose
    graph has no MatMul of that name (MatMul_60 is a decoder MatMul; the encoder's end at
    MatMul_47) the reference finds nothing to inject and the run is golden."""
    from qtx.session import run_module
    feeds = {"global_in": golden_model["enc_in"], "global_in_1": golden_model["src_mask"]}
    p = {"inject_type": "RANDOM", "faulty_operation_name": "MatMul_60",
         "targetted_module": "Decoder", "faulty_bit_position": 3}
    outs, wd = run_module("Encoder", feeds, None, {}, None, inject_parameters=p,
                          model=gpu_model, rng=np.random.default_rng(3))
    assert "qtx_fault" not in wd
    ref = oracle_model.encode(golden_model["enc_in"], golden_model["src_mask"])
    np.testing.assert_array_equal(outs["global_out"], ref)


ATTN_CASES = [("INPUT", "QK"), ("INPUT16", "QK"), ("WEIGHT", "QK"), ("WEIGHT16", "QK"),
              ("RANDOM", "QK"), ("INPUT", "PV"), ("INPUT16", "PV"), ("WEIGHT", "PV"),
              ("WEIGHT16", "PV"), ("RANDOM", "PV")]


@pytest.mark.gpu
@pytest.mark.parametrize("kind,linear", ATTN_CASES)
def test_encoder_attention_fault_matches_oracle(torch_gpu, gpu_model, oracle_model, kind, linear):
    torch = torch_gpu
    B, S = 3, 24
    src, m, x = _enc_inputs(oracle_model, B, S, 21)
    rng = np.random.default_rng(abs(hash((kind, linear))) % 2**32)
    f = F.random_attn_fault(rng, kind, 0, int(rng.integers(6)), linear, B, S, S, bit=7)
    if kind == "RANDOM":
        f.value = 37.25
    out = gpu_model.encode(torch.from_numpy(x).cuda(),
                           torch.from_numpy(m.reshape(B, S).astype(np.uint8)).cuda(),
                           fault=f).cpu().numpy()
    np.testing.assert_array_equal(out, oracle_model.encode(x, m, fault=f.as_dict()))


@pytest.mark.gpu
@pytest.mark.parametrize("kind,linear", [("INPUT", "CQK"), ("WEIGHT16", "CPV"), ("RANDOM", "CPV"),
                                         ("WEIGHT", "QK"), ("INPUT16", "PV")])
def test_decoder_attention_fault_matches_oracle(torch_gpu, gpu_model, oracle_model, kind, linear):
    torch = torch_gpu
    B, S, T = 2, 20, 6
    src, m, x = _enc_inputs(oracle_model, B, S, 22)
    rng = np.random.default_rng(8)
    memory = oracle_model.encode(x, m)
    y = oracle_model.embed(rng.integers(4, 4444, (B, T)), oracle_model.tgt_lut)
    tm = np.tril(np.ones((1, T, T), np.uint8))
    Sk = S if linear.startswith("C") else T
    f = F.random_attn_fault(rng, kind, 1, int(rng.integers(6)), linear, B, T, Sk, bit=6)
    if kind == "RANDOM":
        f.value = -9.5
    T_ = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()
    out = gpu_model.decode(T_(y), T_(memory), T_(m.reshape(B, S).astype(np.uint8)),
                           T_(tm[0]), fault=f).cpu().numpy()
    np.testing.assert_array_equal(out, oracle_model.decode(y, memory, m, tm, fault=f.as_dict()))


def test_oracle_attention_fault_semantics():
    """Oracle attention with a QK^T INPUT fault over all keys == attention on the flipped q."""
    rng = np.random.default_rng(4)
    B, S = 2, 9
    q, k, v = (rng.integers(-127, 128, (B, S, 512)).astype(np.int8) for _ in range(3))
    sq, sk, sv = (rng.uniform(0.002, 0.03, (B, S)).astype(f32) for _ in range(3))
    mask = np.ones((B, 1, S), np.uint8)
    q2 = q.copy()
    q2[1, 4, 3 * 64 + 10] = O._flip8(q2[1, 4, 3 * 64 + 10], 7)
    want, _ = O.attention(q2, sq, k, sk, v, sv, mask)
    got, _ = O.attention(q, sq, k, sk, v, sv, mask, fault=dict(
        kind="QK_INPUT", b=1, h=3, i=4, j=0, d=10, lo=0, hi=S, bit=7, value=0.0))
    np.testing.assert_array_equal(got, want)
    v2 = v.copy()
    v2[0, 5, 2 * 64 + 7] = O._flip8(v2[0, 5, 2 * 64 + 7], 6)
    want, _ = O.attention(q, sq, k, sk, v2, sv, mask)
    got, _ = O.attention(q, sq, k, sk, v, sv, mask, fault=dict(
        kind="PV_WEIGHT", b=0, h=2, i=0, j=5, d=7, lo=0, hi=S, bit=6, value=0.0))
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,linear,step", [("INPUT", "FFN1", 1), ("WEIGHT", "CPV", 3),
                                              ("RANDOM", "QK", 2)])
def test_greedy_decode_with_decoder_fault(torch_gpu, gpu_model, oracle_model, kind, linear, step):
    """The reference campaign's decode loop with a decoder fault at one step
    (target_inference_number), full-prefix recompute per step, == the oracle."""
    from qtx.decode import greedy_decode_fault
    B, S, L = 2, 14, 8
    src, m, _ = _enc_inputs(oracle_model, B, S, 31)
    rng = np.random.default_rng(9)
    T = step                                       # prefix length of the faulty step
    if linear in F.ATTN:
        f = F.random_attn_fault(rng, kind, 1, 3, linear, B, T, S if linear[0] == "C" else T, bit=7)
    else:
        f = F.random_fault(rng, kind, 1, 3, linear, B * T, bit=7)
    if kind == "RANDOM":
        f.value = 1e4
    ys = greedy_decode_fault(gpu_model, src, m, L, 0, fault=f, target_inference_number=step)
    ref = oracle_model.greedy_decode(src, m, max_len=L, fault=f.as_dict(), fault_step=step - 1)
    np.testing.assert_array_equal(ys, ref)
