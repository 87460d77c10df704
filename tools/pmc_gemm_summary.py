"""Per-kernel medians of the tools/pmc_gemm.sh passes (row GEMM launches) as JSON.
usage: python tools/pmc_gemm_summary.py gpurun_out/pmc_gemm > profiles/<name>.json"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in glob.glob(d + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"]
        if "k_gemm_row" not in k:
            continue
        k = k[k.index("k_gemm_row"):].split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
EPI = {"0": "qkv_quant", "1": "res_ln (O / FFN2)", "2": "ffn1_rowmax", "3": "ffn1_quant"}
out = {"note": "medians per dispatch over tools/rows_bench.py (cfg3 shapes, M=32768); "
               "FETCH_SIZE/WRITE_SIZE in KB (gfx950: FETCH_SIZE x2 for wide reads), "
               "MfmaUtil %, LdsBankConflict % of LDS cycles"}
for k, cs in sorted(vals.items()):
    e = k.split("<")[1].split(",")[0]
    m = {c: sorted(v)[len(v) // 2] for c, v in cs.items()}
    if "FETCH_SIZE" in m:
        m["hbm_read_bytes_corrected"] = 2 * m["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in m:
        m["hbm_write_bytes"] = m["WRITE_SIZE"] * 1024
    out[f"{k} [{EPI.get(e, e)}]"] = m
print(json.dumps(out, indent=1))
