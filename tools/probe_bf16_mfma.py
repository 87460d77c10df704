"""Compare tools/probe_bf16_mfma's v_mfma_f32_16x16x32_bf16 results with rounding models
(exact rational arithmetic): which model reproduces every output bit for bit?
    python tools/probe_bf16_mfma.py bf16_mfma.bin"""
import struct
import sys
from fractions import Fraction

import numpy as np


def rn32(x: Fraction) -> float:
    """Round a rational to the nearest fp32, ties to even (normal range)."""
    if x == 0:
        return 0.0
    s = -1 if x < 0 else 1
    a = abs(x)
    e = a.numerator.bit_length() - a.denominator.bit_length()
    if Fraction(2) ** e > a:
        e -= 1
    n = a * Fraction(2) ** (23 - e)            # in [2^23, 2^24)
    q, r = divmod(n.numerator, n.denominator)
    r2 = 2 * r
    if r2 > n.denominator or (r2 == n.denominator and q & 1):
        q += 1
    return float(np.float32(s * q * 2.0 ** (e - 23)))


def f32(x):
    return float(np.float32(x))


def main():
    fn = sys.argv[1] if len(sys.argv) > 1 else "bf16_mfma.bin"
    raw = open(fn, "rb").read()
    T = struct.unpack_from("i", raw, 0)[0]
    off = 4
    A = np.frombuffer(raw, np.uint16, T * 512, off); off += T * 1024
    B = np.frombuffer(raw, np.uint16, T * 512, off); off += T * 1024
    C = np.frombuffer(raw, np.float32, T * 256, off); off += T * 1024
    D = np.frombuffer(raw, np.float32, T * 256, off)
    bf = lambda u: np.frombuffer((u.astype(np.uint32) << 16).tobytes(), np.float32)
    Af, Bf = bf(A).reshape(T, 64, 8), bf(B).reshape(T, 64, 8)
    def rz32(x: Fraction) -> float:
        """toward zero"""
        if x == 0:
            return 0.0
        sgn = -1 if x < 0 else 1
        a = abs(x)
        e = a.numerator.bit_length() - a.denominator.bit_length()
        if Fraction(2) ** e > a:
            e -= 1
        n = a * Fraction(2) ** (23 - e)
        return float(np.float32(sgn * (n.numerator // n.denominator) * 2.0 ** (e - 23)))

    grp = {}
    for size in (2, 4, 8, 16):
        for order in ("asc", "desc"):
            for rnd in ("rn", "rz"):
                grp[(size, order, rnd)] = 0
    models = {"exact sum + C, rounded once": 0, "products summed exactly, rounded, then + C": 0,
              "sequential fp32 chain from C (k order)": 0, "sequential fp32 chain, C last": 0,
              "fp32 pairwise tree of products, then + C": 0, "per 8-group exact, 4 roundings": 0}
    total = 0
    T = min(T, int(sys.argv[2]) if len(sys.argv) > 2 else T)
    for t in range(T):
        for i in range(16):
            for j in range(16):
                lo = 16 * (i // 4) + j
                d = float(D[t * 256 + lo * 4 + i % 4])
                c = float(C[t * 256 + lo * 4 + i % 4])
                prods = [float(Af[t, 16 * g + i, k]) * float(Bf[t, 16 * g + j, k])
                         for g in range(4) for k in range(8)]        # exact in double
                fp = [Fraction(p) for p in prods]
                total += 1
                models["exact sum + C, rounded once"] += rn32(Fraction(c) + sum(fp)) == d
                models["products summed exactly, rounded, then + C"] += rn32(Fraction(c) + Fraction(rn32(sum(fp)))) == d
                acc = c
                for p in prods:
                    acc = f32(acc + p)
                models["sequential fp32 chain from C (k order)"] += acc == d
                acc = 0.0
                for p in prods:
                    acc = f32(acc + p)
                models["sequential fp32 chain, C last"] += f32(acc + c) == d
                v = [f32(p) for p in prods]
                while len(v) > 1:
                    v = [f32(v[2 * q] + v[2 * q + 1]) for q in range(len(v) // 2)]
                models["fp32 pairwise tree of products, then + C"] += f32(v[0] + c) == d
                acc = Fraction(c)
                for g in range(4):
                    acc = Fraction(rn32(acc + sum(fp[8 * g:8 * g + 8])))
                models["per 8-group exact, 4 roundings"] += float(acc) == d
                for (size, order, rnd), _ in grp.items():
                    idx = list(range(0, 32, size))
                    if order == "desc":
                        idx = idx[::-1]
                    acc = Fraction(c)
                    for b0 in idx:
                        acc = Fraction((rn32 if rnd == "rn" else rz32)(acc + sum(fp[b0:b0 + size])))
                    grp[(size, order, rnd)] += float(acc) == d
    print(f"{total} outputs ({T} trials x 256; half with operand exponents in [-8, 8], half "
          f"in [-2, 2] with mixed signs)")
    for k, v in models.items():
        print(f"  {k:45s}: {v:6d} / {total} bit-exact ({100.0 * v / total:.2f} %)")
    for (size, order, rnd), v in grp.items():
        k = f"groups of {size} (exact), {order} K order, {rnd} per group"
        print(f"  {k:45s}: {v:6d} / {total} bit-exact ({100.0 * v / total:.2f} %)")


if __name__ == "__main__":
    main()
