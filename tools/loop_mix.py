"""Instruction mix of the innermost loops of selected kernels in compiled gfx950 assembly
(diagnostic, not shipped):
    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math \
          --cuda-device-only -S -o t.s onnx-transformer_amd/csrc/qtx_wsgemm.hip
    python tools/loop_mix.py t.s wsq wsy
Prints, per kernel whose mangled name contains one of the patterns: MFMAs, VALU
instructions (v_* without MFMA) and the commonest VALU opcodes inside loop blocks."""
import collections
import re
import sys


def functions(lines):
    name, body = None, []
    for raw in lines:
        m = re.match(r"^(_Z\w+):", raw)
        if m:
            name, body = m.group(1), []
            continue
        if name:
            body.append(raw)
            if raw.startswith(".Lfunc_end"):
                yield name, body
                name = None


def mix(body):
    c, inloop = collections.Counter(), False
    for raw in body:
        if re.match(r"^\.LBB", raw) or raw.startswith("; %bb."):
            inloop = "in Loop" in raw or "Loop Header" in raw
            continue
        op = raw.strip().split(" ")[0]
        if inloop and op and not op.startswith((";", ".")):
            c[op] += 1
    return c


def main(path, pats):
    for name, body in functions(open(path).read().split("\n")):
        if pats and not any(p in name for p in pats):
            continue
        c = mix(body)
        mf = sum(v for k, v in c.items() if "mfma" in k)
        valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
        pk = sum(v for k, v in c.items() if k.startswith("v_pk_"))
        print(f"{name[:70]}\n  loop: mfma {mf}  valu {valu}  (packed {pk})  valu/mfma "
              f"{valu / max(mf, 1):.2f}")
        top = sorted(((v, k) for k, v in c.items() if k.startswith("v_") and "mfma" not in k), reverse=True)
        print("  " + ", ".join(f"{k} {v}" for v, k in top[:16]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
