"""Per-kernel medians of the tools/pmc_encoder.sh passes (the cfg3 encoder as the product
runs it) plus the kernel-trace durations, as JSON.
usage: python tools/pmc_encoder_summary.py gpurun_out/pmc_enc > profiles/<name>.json"""
import collections
import csv
import glob
import json
import sqlite3
import sys

d = sys.argv[1]
short = lambda k: k.split("(")[0].replace("void ", "").replace("qtx::", "")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = {}
for db in glob.glob(d + "/stats/**/*results.db", recursive=True):
    c = sqlite3.connect(db)
    for name, n, avg in c.execute("select name, count(*), avg(duration) from kernels group by name"):
        dur[short(name)] = (n, avg / 1e3)
out = {"note": "cfg3 encoder (B=256, S=128) through QtxModel.encode; medians per dispatch; "
               "FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE x2 for wide reads -> "
               "hbm_read_bytes_corrected); MfmaUtil %; LdsBankConflict % of LDS cycles; "
               "avg_us from the kernel-trace pass"}
for k in sorted(set(vals) | set(dur)):
    if not k.startswith(("k_gemm", "k_attn", "k_rows", "k_embed", "k_skinny")):
        continue
    m = {c: sorted(v)[len(v) // 2] for c, v in vals.get(k, {}).items()}
    if "FETCH_SIZE" in m:
        m["hbm_read_bytes_corrected"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    if k in dur:
        m["dispatches"], m["avg_us"] = dur[k][0], round(dur[k][1], 2)
    out[k] = m
print(json.dumps(out, indent=1))
