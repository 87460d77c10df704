"""Static check of the hazards the compiler does not track for MFMAs written as asm
statements (k_gemm_wsq / k_gemm_wss): in a kernel's assembly (hipcc -S), every read or
write of an asm MFMA's result registers by a non-MFMA instruction within PAD wait states of
the MFMA, and every VALU write of a register an asm MFMA reads within 2 wait states before
it.  Wait states are counted as instructions (s_nop N = N + 1); branches end the window
conservatively (a label resets nothing: the check is linear over the text).
    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S -o t.s qtx_wsgemm.hip
    python tools/check_asm_mfma.py t.s k_gemm_wsq k_gemm_wss"""
import re
import sys

PAD = 18          # 16x16x64 (8 passes); the 16-pass 32x32x32 results: PAD32
PAD32 = 20
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def regs(text):
    out = set()
    for m in REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def check(lines, name):
    pending = []          # [dst regs, wait states left]
    recent = []           # [VALU-written regs, wait states since]
    in_asm, bad = False, 0
    for ln, raw in lines:
        s = raw.split(";")[0].strip()
        if raw.strip().startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if raw.strip().startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not s or s.endswith(":") or s.startswith("."):
            continue
        op = s.split()[0]
        ops = s[len(op):]
        ws = int(op == "s_nop" and ops.strip(), 0) + 1 if op == "s_nop" else 1
        if op.startswith("v_mfma"):
            parts = [p.strip() for p in ops.split(",")]
            dst, srcs = regs(parts[0]), set().union(*(regs(p) for p in parts[1:]))
            if in_asm:
                for r, age in recent:
                    if age < 2 and r & srcs:
                        print(f"{name}:{ln}: VALU write {sorted(r & srcs)} {age} wait states before asm MFMA")
                        bad += 1
                pending = [p for p in pending if not (p[0] & dst)]
                pending.append([dst, PAD32 if "32x32" in op else PAD])
        else:
            used = regs(ops)
            for dst, left in pending:
                if dst & used and not op.startswith("s_"):
                    print(f"{name}:{ln}: {op} touches {sorted(dst & used)[:4]} ({left} wait states short) after asm MFMA")
                    bad += 1
            if op.startswith("v_") and not op.startswith("v_mfma"):
                w = regs(ops.split(",")[0])
                recent.append([w, -1])
        for p in pending:
            p[1] -= ws
        pending = [p for p in pending if p[1] > 0]
        for r in recent:
            r[1] += ws
        recent = [r for r in recent if r[1] < 2]
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op == "s_endpgm":
            pending, recent = [], []
    return bad


def main():
    text = open(sys.argv[1]).read().splitlines()
    total = 0
    for k in sys.argv[2:]:
        # every instance (template kernels: one per instantiation)
        starts = [i for i, l in enumerate(text) if re.match(rf"_ZN3qtx\d+{k}[EI]\S*:", l)]
        assert starts, f"kernel {k} not found"
        n = 0
        for start in starts:
            end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
            n += check([(i + 1, text[i]) for i in range(start, end + 1)], text[start].rstrip(":"))
        print(f"{k}: {n} hazards ({len(starts)} instances)")
        total += n
    sys.exit(1 if total else 0)


if __name__ == "__main__":
    main()
