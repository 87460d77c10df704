"""The qtx fault model vs the reference's, on one QuantLinear (a toy case restated by hand).

The reference injects an INPUT / WEIGHT bit flip by propagating a separate fp32 delta
(inject_utils/layers.py:87-142 perturb_quantizer: the flipped element alone, dequantized,
minus the golden dequantized value; onnx_optimized_inference.py:111-199: the delta pushed
through the MatMul, windowed for *16, then added to the golden MatMul output).  qtx (and
the oracle, which the GPU matches bit for bit: tests/test_fault.py) instead recomputes
the MatMul on the flipped int8 operand — exact integer accumulators, one epilogue.  Both
are the same real number; this checks they differ only by fp32 rounding of the sum."""
import numpy as np
import pytest

from oracle import qtx_oracle as O

f32 = np.float32


def flip_int8_bit(v, bit):            # inject_utils/layers.py:62-69
    f = int(v) ^ (1 << bit)
    return f - 256 if f > 127 else (f + 256 if f < -128 else f)


def reference_faulty(x, lin, kind, m, k_or_n, bit, lo, hi):
    """The reference's arithmetic restated: golden fake-quant output (quant_linear.py:
    111-119, fp32 F.linear; float64 sums rounded once stand in for MLAS' order) plus the
    fp32 delta of the flipped element propagated through the MatMul."""
    qx, sx = O.quant_rows(x)
    xd = (qx.astype(f32) * sx[:, None]).astype(f32)             # q_x * s_x
    wd = (lin.q.astype(f32) * lin.s[:, None]).astype(f32)       # q_w * s_w
    y = ((xd.astype(np.float64) @ wd.T.astype(np.float64)).astype(f32) + lin.b).astype(f32)
    delta = np.zeros_like(y)
    if kind.startswith("INPUT"):
        k = k_or_n
        fv = flip_int8_bit(qx[m, k], bit)
        d = f32(f32(fv) * sx[m]) - xd[m, k]                       # perturb_quantizer
        delta[m, :] = (d * wd[:, k]).astype(f32)                  # the one-hot delta . W^T
        keep = np.zeros(y.shape[1], bool)
        keep[lo:hi] = True                                        # INPUT16: 16-column window
        delta[m, ~keep] = 0
    else:
        n = k_or_n
        k = m                                                     # weight element (n, k)
        fv = flip_int8_bit(lin.q[n, k], bit)
        d = f32(f32(fv) * lin.s[n]) - wd[n, k]
        delta[:, n] = (xd[:, k] * d).astype(f32)
        keep = np.zeros(y.shape[0], bool)
        keep[lo:hi] = True                                        # WEIGHT16: row window
        delta[~keep, n] = 0
    return (y + delta).astype(f32), y


@pytest.mark.parametrize("kind", ["INPUT", "INPUT16", "WEIGHT", "WEIGHT16"])
@pytest.mark.parametrize("bit", [0, 3, 6, 7])
def test_recompute_equals_delta_propagation(state_dict, kind, bit):
    rng = np.random.default_rng(100 + bit)
    lin = O.QLinear(state_dict["encoder.layers.1.feed_forward.w_1.weight"],
                    state_dict["encoder.layers.1.feed_forward.w_1.bias"])
    x = rng.standard_normal((24, 512)).astype(f32)
    N = lin.q.shape[0]
    if kind.startswith("INPUT"):
        m, c = int(rng.integers(24)), int(rng.integers(512))
        lo, hi = ((16 * int(rng.integers(N // 16)),) * 2) if kind == "INPUT16" else (0, N)
        hi = lo + 16 if kind == "INPUT16" else hi
        fault = dict(kind=kind, row=m, col=c, bit=bit, lo=lo, hi=hi, value=0.0)
        ref, golden = reference_faulty(x, lin, kind, m, c, bit, lo, hi)
    else:
        n, c = int(rng.integers(N)), int(rng.integers(512))
        lo = 16 * int(rng.integers(24 // 16 + 1)) if kind == "WEIGHT16" else 0
        hi = min(24, lo + int(rng.integers(1, 16))) if kind == "WEIGHT16" else 24
        fault = dict(kind=kind, row=n, col=c, bit=bit, lo=lo, hi=hi, value=0.0)
        ref, golden = reference_faulty(x, lin, kind, c, n, bit, lo, hi)
    ours = lin(x, fault=fault)
    clean = lin(x)
    scale = np.abs(golden).max()
    # both fault models move the same elements by the same real amount ...
    moved_ref, moved_ours = ref != golden, np.abs(ours - clean) > 4e-6 * scale
    assert not (moved_ours & ~moved_ref).any()
    # ... and agree to fp32 rounding of the sums (the golden outputs already differ by
    # the reference's summation order: compare the faulty outputs against that floor)
    floor = np.abs(clean - golden).max()
    assert np.abs(ours - ref).max() <= floor + 4e-7 * scale
