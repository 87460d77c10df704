"""Summarise tools/ring_probe.sh's rocprofv3 PMC passes over tools/probe_ffn_ring.hip: per
variant (kernel instance), the median over its dispatches of each counter, and derived
ratios (LDS instructions per wave, waiting fraction).  usage: ring_pmc_table.py <dir>"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    for fn in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        with open(fn) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"].split("(")[0].replace("void ", "")
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    cols = ["SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS",
            "SQ_INSTS_LDS", "SQ_INSTS_VALU_MFMA_MOPS_I8", "LdsBankConflict"]
    print("| kernel | " + " | ".join(cols) + " | wait_any / wave_cycles | wait_inst_lds / wave_cycles |")
    print("|---|" + "---:|" * (len(cols) + 2))
    for name, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        row = [f"{med[c]:.4g}" if c in med else "-" for c in cols]
        wc = med.get("SQ_WAVE_CYCLES")
        ra = f"{med['SQ_WAIT_ANY'] / wc:.3f}" if wc and "SQ_WAIT_ANY" in med else "-"
        rl = f"{med['SQ_WAIT_INST_LDS'] / wc:.3f}" if wc and "SQ_WAIT_INST_LDS" in med else "-"
        print(f"| `{name}` | " + " | ".join(row) + f" | {ra} | {rl} |")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ring")
