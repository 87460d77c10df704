"""Exactness of the arithmetic identities the kernels use in place of divisions (CPU):
div127 (qtx_common.h) — fma(c, RN(1/127), c * RN(1/127 - RN(1/127))) == RN(c / 127) for every
P code c in [0, 127], the quotient of attention.py's P grid — and the biased-rint tie test
of quant_rows512 against quant_pack's floor form."""
from fractions import Fraction

import numpy as np

f32 = np.float32


def rn32(fr: Fraction) -> np.float32:
    """Fraction -> float32, round to nearest even (exact)."""
    x = f32(float(fr))
    best = None
    for v in (np.nextafter(x, f32(-np.inf)), x, np.nextafter(x, f32(np.inf))):
        d = abs(Fraction(float(v)) - fr)
        key = (d, int(np.array(v).view(np.int32)) & 1)
        if best is None or key < best[0]:
            best = (key, v)
    return best[1]


def test_div127_exact_for_every_code():
    hi, lo = f32(float.fromhex("0x1.020408p-7")), f32(float.fromhex("0x1.020408p-35"))
    assert hi == f32(1 / 127) and lo == rn32(Fraction(1, 127) - Fraction(float(hi)))
    for c in range(128):
        t = f32(f32(c) * lo)                                     # c * lo, rounded
        got = rn32(Fraction(c) * Fraction(float(hi)) + Fraction(float(t)))   # fma: one rounding
        assert got == rn32(Fraction(c, 127)), c


def test_biased_rint_tie_window_matches_floor_form():
    rng = np.random.default_rng(0)
    r = np.concatenate([rng.uniform(-127.5, 127.5, 200000).astype(f32),
                        (np.arange(-255, 256) / f32(2)).astype(f32),          # exact ties
                        (np.arange(-255, 256) / f32(2) + f32(2.0 ** -13)).astype(f32),
                        (np.arange(-255, 256) / f32(2) - f32(2.0 ** -13)).astype(f32)])
    B = f32(12582912.0)
    t = (r + B).astype(f32)
    d = (r - (t - B)).astype(f32)
    near_new = np.abs(d) > f32(0.5) - f32(2.0 ** -13)
    fr = (r - np.floor(r)).astype(f32)
    near_old = np.abs(fr - f32(0.5)) < f32(2.0 ** -13)
    # the windows agree wherever r - floor(r) is exact (r >= 0 or |r| >= 1); the test is
    # conservative either way, so the codes never depend on which form ran
    exact = (r >= 0) | (np.abs(r) >= 1)
    assert np.array_equal(near_new[exact], near_old[exact])
    # the biased value carries rint(r) (ties to even) in its low byte
    assert np.array_equal(t.view(np.int32) & 0xff, np.rint(r).astype(np.int32) & 0xff)
