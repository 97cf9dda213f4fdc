"""Summarise a rocprofv3 --pmc counter_collection.csv: mean counter value per
dispatch for each kernel (the committed profiles/*_pmc_*.csv come from here).

usage: python tools/pmc_summary.py gpurun_out/pmc_sq/run_counter_collection.csv > profiles/r01_pmc_sq.csv
"""
import csv
import sys
from collections import defaultdict


def main(path):
    vals = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in csv.DictReader(open(path)):
        k = row["Kernel_Name"].split("(")[0]
        vals[k][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[k].add(row["Dispatch_Id"])
    counters = sorted({c for v in vals.values() for c in v})
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "dispatches"] + [c + "_per_dispatch" for c in counters])
    for k in sorted(vals, key=lambda k: -len(disp[k])):
        n = len(disp[k])
        w.writerow([k, n] + [f"{vals[k].get(c, 0.0) / n:.1f}" for c in counters])


if __name__ == "__main__":
    main(sys.argv[1])
