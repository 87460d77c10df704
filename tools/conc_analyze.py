"""How two decode chains share the GPU, from rocprofv3 --kernel-trace databases: one
database with two sub-batch chains (QTX_DECODE_GROUPS=2: told apart by HIP stream) or two
databases of two processes (told apart by pid).  Per chain: kernels, HW queue, the span of
its decodes, the fraction of that span with one of its kernels executing (busy), and the
median kernel duration when the other chain has a kernel executing vs not; for the pair:
the fraction of the joint span where both have a kernel executing.
    python tools/conc_analyze.py gpurun_out/conc/g2            (one process, 2 streams)
    python tools/conc_analyze.py gpurun_out/conc/p0 gpurun_out/conc/p1"""
import glob
import os
import sqlite3
import sys

import numpy as np


def load(d):
    db = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))[0]
    c = sqlite3.connect(db)
    return c.execute("select pid, stream_id, queue_id, name, start, end from kernels "
                     "where name not like '%rocclr%' order by start").fetchall()


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(u):
    return sum(e - s for s, e in u)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def covered(u, t):
    """For each time in t: is it inside the union u?"""
    starts = np.array([s for s, _ in u]); ends = np.array([e for _, e in u])
    k = np.searchsorted(starts, t, side="right") - 1
    return (k >= 0) & (t < ends[np.clip(k, 0, None)])


def main():
    dirs = sys.argv[1:]
    rows = [r for d in dirs for r in load(d)]
    key = (lambda r: r[0]) if len(dirs) > 1 else (lambda r: r[1])
    chains = {}
    for r in rows:
        chains.setdefault(key(r), []).append(r)
    chains = {k: v for k, v in chains.items() if len(v) > 1000}   # the decode chains
    ks = sorted(chains)
    print(f"{len(ks)} chains: " + ", ".join(f"{'pid' if len(dirs) > 1 else 'stream'} {k}: {len(chains[k])} kernels, "
                                          f"queues {sorted({r[2] for r in chains[k]})}" for k in ks))
    if len(ks) != 2:
        return
    U = {k: union([(r[4], r[5]) for r in chains[k]]) for k in ks}
    # the window where both chains run: from the later first kernel to the earlier last one
    lo = max(chains[k][0][4] for k in ks)
    hi = min(chains[k][-1][5] for k in ks)
    clip = lambda u: [[max(s, lo), min(e, hi)] for s, e in u if e > lo and s < hi]
    W = hi - lo
    print(f"joint window {W / 1e6:.2f} ms")
    both = length(intersect(clip(U[ks[0]]), clip(U[ks[1]])))
    for a, b in ((ks[0], ks[1]), (ks[1], ks[0])):
        ua = clip(U[a])
        ka = [r for r in chains[a] if r[4] >= lo and r[5] <= hi]
        mid = np.array([(r[4] + r[5]) // 2 for r in ka])
        dur = np.array([r[5] - r[4] for r in ka]) / 1e3
        ov = covered(U[b], mid)
        gaps = np.diff([r[4] for r in ka]) / 1e3
        print(f"chain {a}: busy {length(ua) / W:.3f} of the window, {len(ka)} kernels, "
              f"median kernel {np.median(dur):.2f} us (other chain executing: {np.median(dur[ov]) if ov.any() else 0:.2f} us "
              f"on {ov.mean():.2f} of kernels; not: {np.median(dur[~ov]) if (~ov).any() else 0:.2f} us); "
              f"median start-to-start {np.median(gaps):.2f} us")
    print(f"both chains executing: {both / W:.3f} of the window")


if __name__ == "__main__":
    main()
