"""Per-run kernel durations from a rocprofv3 --kernel-trace database: consecutive
dispatches of one kernel at one grid (>= --min of them with nothing else in between) form
a run — e.g. bench.py's chain of the dominant decode kernel — reported with its average
duration, so the bench's HIP-event figure can be checked against the profiler's.

    python tools/dispatch_runs.py gpurun_out/<tag>/prof [--kernel NAME] [--min 32]
"""
import argparse
import glob
import os
import sqlite3


def runs(db, kernel=None, min_len=32):
    c = sqlite3.connect(db)
    rows = c.execute("select name, grid_x, grid_y, start, end from kernels order by start").fetchall()
    out, cur = [], None
    for name, gx, gy, s, e in rows:
        key = (name, gx, gy)
        if cur and cur["key"] == key:
            cur["d"].append(e - s)
        else:
            if cur and len(cur["d"]) >= min_len:
                out.append(cur)
            cur = {"key": key, "d": [e - s], "t0": s}
    if cur and len(cur["d"]) >= min_len:
        out.append(cur)
    if kernel:
        out = [r for r in out if kernel in r["key"][0]]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel")
    ap.add_argument("--min", type=int, default=32)
    a = ap.parse_args()
    db = sorted(glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True))[0]
    print("| kernel | grid | dispatches | avg us | median us |")
    print("|---|---|---:|---:|---:|")
    for r in runs(db, a.kernel, a.min):
        d = sorted(r["d"])
        n, gx, gy = r["key"]
        print(f"| `{n[:80]}` | {gx}x{gy} | {len(d)} | {sum(d) / len(d) / 1e3:.2f} | {d[len(d) // 2] / 1e3:.2f} |")


if __name__ == "__main__":
    main()
