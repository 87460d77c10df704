"""Average rocprofv3 --pmc counters per kernel (name prefix) from a counter_collection.csv.
usage: python tools/pmc_kernels.py <dir> [substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in files:
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if sub in k:
            agg[k[:40]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in sorted(agg.items()):
    print(k, {c: round(sum(v) / len(v)) for c, v in sorted(cs.items())})
