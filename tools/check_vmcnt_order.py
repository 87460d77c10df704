"""Static check of VM_CNT_ORDER (csrc/qtx_common.h) on compiled gfx950 assembly: a hand-counted
`s_waitcnt vmcnt(N)` with N > 0 that waits for an LDS-DMA is exact only when the N youngest
vector-memory operations at the wait are loads (a store, or a compiler load whose own wait is
counted without the asm DMAs, may retire out of order and release the wait early).

Only hand-written waits are checked (inside the ;;#ASMSTART / ;;#ASMEND markers of an asm
statement): the compiler's own counted waits count the compiler's own operations and are
exact for them.  Rule checked, per hand-written counted wait: every vector-memory instruction of the loop that contains it
(the blocks llc annotates "in Loop: Header=<H>" plus the header <H>, innermost loop) is an
LDS-DMA (`global_load_lds_*` / `buffer_load_* ... lds`) — no store, no load to registers, no
scratch access.  A counted wait outside any loop must have only LDS-DMAs between it and the
previous `s_waitcnt vmcnt(0)` of its function.
    hipcc --offload-arch=gfx950 -O3 ... --cuda-device-only -S -o t.s qtx_gemm.hip
    python tools/check_vmcnt_order.py t.s"""
import re
import sys

VM = re.compile(r"^\s*(global_|buffer_|scratch_|flat_)(load|store|atomic)\w*")
WAIT = re.compile(r"s_waitcnt\s+.*vmcnt\((\d+)\)")
LABEL = re.compile(r"^(\.LBB\d+_\d+|[A-Za-z_][\w.$]*):")
INLOOP = re.compile(r"in Loop: Header=(BB\d+_\d+)")
HEADER = re.compile(r"Loop Header: Depth=")


def is_dma(line):
    s = line.split(";")[0]
    return "global_load_lds" in s or (s.strip().startswith("buffer_load") and " lds" in s)


def functions(lines):
    name, body = None, []
    for ln, raw in enumerate(lines, 1):
        m = re.match(r"^(_Z\w+):", raw)
        if m:
            if name:
                yield name, body
            name, body = m.group(1), []
        elif name:
            body.append((ln, raw))
            if raw.startswith(".Lfunc_end"):
                yield name, body
                name, body = None, []


def blocks(body):
    """[(label, loop_header_or_None, is_header, [(ln, text)])] in text order."""
    out, cur = [], ["<entry>", None, False, []]
    for ln, raw in body:
        m = LABEL.match(raw)
        if m or raw.startswith("; %bb."):
            out.append(cur)
            label = m.group(1) if m else raw.split()[1].rstrip(":")
            lp = INLOOP.search(raw)
            cur = [label, lp.group(1) if lp else None, bool(HEADER.search(raw)), []]
            if cur[2]:
                cur[1] = label.lstrip(".L").replace("LBB", "BB") if label.startswith(".LBB") else None
            continue
        cur[3].append((ln, raw))
    out.append(cur)
    return out


def check(path):
    lines = open(path).read().split("\n")
    bad, waits = 0, 0
    for name, body in functions(lines):
        bl = blocks(body)
        for bi, (label, loop, is_hdr, insts) in enumerate(bl):
            in_asm = False
            for k, (ln, raw) in enumerate(insts):
                if raw.strip().startswith(";;#ASMSTART"):
                    in_asm = True
                elif raw.strip().startswith(";;#ASMEND"):
                    in_asm = False
                m = WAIT.search(raw.split(";")[0])
                if not m or int(m.group(1)) == 0 or not in_asm:
                    continue
                waits += 1
                if loop:
                    scope = [b for b in bl if b[1] == loop]
                    where = f"loop {loop}"
                else:               # straight line: back to the previous full drain
                    scope, seen = [], []
                    for b in reversed(bl[:bi + 1]):
                        part = b[3][:k] if b is bl[bi] else b[3]
                        stop = [i for i, (_, r) in enumerate(part) if re.search(r"vmcnt\(0\)", r.split(";")[0])]
                        if stop:
                            seen.append(part[stop[-1] + 1:])
                            break
                        seen.append(part)
                    scope = [[None, None, False, [x for s in seen for x in s]]]
                    where = "straight line"
                for b in scope:
                    for ln2, r2 in b[3]:
                        if VM.match(r2) and not is_dma(r2):
                            print(f"{name}: counted vmcnt({m.group(1)}) at line {ln} ({where}) with "
                                  f"a non-DMA vector-memory op at line {ln2}: {r2.strip()}")
                            bad += 1
    print(f"{path}: {waits} counted vmcnt waits, {bad} violations")
    return bad


if __name__ == "__main__":
    sys.exit(1 if sum(check(p) for p in sys.argv[1:]) else 0)
