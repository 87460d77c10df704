"""Summarize a rocprofv3 run (kernel_stats.csv or results.db) as a markdown table.

    python tools/prof_summary.py gpurun_out/prof > profiles/r01_decode_b32.md
"""
import csv
import glob
import os
import sqlite3
import sys


def from_db(path):
    c = sqlite3.connect(path)
    rows = c.execute("select name, count(*), sum(duration), avg(duration), min(duration), "
                     "max(duration) from kernels group by name").fetchall()
    return [dict(name=r[0], calls=r[1], total_ns=r[2], avg_ns=r[3], min_ns=r[4], max_ns=r[5])
            for r in rows]


def from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append(dict(name=r["Name"], calls=int(r["Calls"]), total_ns=float(r["TotalDurationNs"]),
                            avg_ns=float(r["AverageNs"]), min_ns=float(r["MinNs"]),
                            max_ns=float(r["MaxNs"])))
    return out


def sources_sha16():
    """Digest of the product kernel sources (onnx-transformer_amd/csrc/*.hip, *.h) the
    profiled library was built from; bench.py compares it with the sources it runs."""
    import hashlib
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                        "onnx-transformer_amd", "csrc")
    h = hashlib.sha256()
    for fn in sorted(glob.glob(os.path.join(root, "*.hip")) + glob.glob(os.path.join(root, "*.h"))):
        with open(fn, "rb") as f:
            h.update(os.path.basename(fn).encode() + b"\0" + f.read())
    return h.hexdigest()[:16]


def main(d):
    stats = sorted(glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True))
    if stats:
        rows, src = from_csv(stats[0]), stats[0]
    else:
        dbs = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
        rows, src = from_db(dbs[0]), dbs[0]
    rows.sort(key=lambda r: -r["total_ns"])
    tot = sum(r["total_ns"] for r in rows)
    print(f"source: `{os.path.relpath(src)}`  total kernel time {tot / 1e3:.1f} us\n")
    # the digest of the sources the profiled library was built from: recorded on the GPU box
    # by tools/gpu_round.sh (<tag>/sources_sha16.txt), else of the sources here
    rec = os.path.join(os.path.dirname(os.path.abspath(d)), "sources_sha16.txt")
    sha = open(rec).read().strip() if os.path.exists(rec) else sources_sha16()
    print(f"kernel_sources_sha16: {sha}\n")
    print("| kernel | calls | total us | avg us | min us | max us | % |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for r in rows:
        print(f"| `{r['name'][:90]}` | {r['calls']} | {r['total_ns'] / 1e3:.1f} | "
              f"{r['avg_ns'] / 1e3:.2f} | {r['min_ns'] / 1e3:.2f} | {r['max_ns'] / 1e3:.2f} | "
              f"{100 * r['total_ns'] / tot:.1f} |")


def by_grid(d, top=40):
    """Second table: the same dispatches split by launch grid (one kernel at several
    shapes — e.g. the decode GEMMs at B=32 and B=256 — averaged separately)."""
    dbs = sorted(glob.glob(os.path.join(d, "**", "*.db"), recursive=True))
    if not dbs:
        return
    c = sqlite3.connect(dbs[0])
    rows = c.execute("select name, grid_x, grid_y, workgroup_x, count(*), sum(duration), "
                     "avg(duration), min(duration), max(duration) from kernels "
                     "group by name, grid_x, grid_y, workgroup_x order by sum(duration) desc "
                     f"limit {top}").fetchall()
    print("\n### by launch grid (grid = threads, x * y)\n")
    print("| kernel | grid | calls | total us | avg us | min us | max us |")
    print("|---|---|---:|---:|---:|---:|---:|")
    for n, gx, gy, wx, cnt, tot, avg, mn, mx in rows:
        print(f"| `{n[:90]}` | {gx}x{gy} (wg {wx}) | {cnt} | {tot / 1e3:.1f} | {avg / 1e3:.2f} | "
              f"{mn / 1e3:.2f} | {mx / 1e3:.2f} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
    by_grid(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof")
