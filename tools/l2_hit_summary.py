"""L2 (TCC) hit rate per kernel from a rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum pass:
    python tools/l2_hit_summary.py gpurun_out/<dir>"""
import collections
import csv
import glob
import sys

short = lambda k: k.split("(")[0].replace("void ", "").replace("qtx::", "")
hit = collections.Counter()
miss = collections.Counter()
disp = collections.defaultdict(set)
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        k = short(r["Kernel_Name"])
        disp[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        if r["Counter_Name"].startswith("TCC_HIT"):
            hit[k] += float(r["Counter_Value"])
        elif r["Counter_Name"].startswith("TCC_MISS"):
            miss[k] += float(r["Counter_Value"])
print(f"{'kernel':58s} {'disp':>6s} {'hit/disp':>10s} {'miss/disp':>10s} {'hit %':>6s}")
tot_h = tot_m = 0
for k in sorted(hit, key=lambda k: -(hit[k] + miss[k])):
    n = max(len(disp[k]), 1)
    h, m = hit[k], miss[k]
    tot_h += h
    tot_m += m
    print(f"{k[:58]:58s} {n:6d} {h / n:10.0f} {m / n:10.0f} {100 * h / max(h + m, 1):6.1f}")
print(f"all: hit {100 * tot_h / max(tot_h + tot_m, 1):.1f} %")
