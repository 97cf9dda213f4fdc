"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into HBM bytes
per dispatch per kernel (the file bench.py's roofline.traffic reads).

FETCH_SIZE is doubled: on gfx950 it tallies 128-B requests at 64 B
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is taken as is.  Both are KB.
usage: python tools/pmc_traffic.py <fetch pass dir> <write pass dir> [key prefix, e.g. cfg4:] > profiles/<tag>_pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_dispatch(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals, disp = defaultdict(float), defaultdict(set)
    for f in files:
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            k = row["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0].replace("ksg::", "")
            vals[k] += float(row["Counter_Value"])
            disp[k].add(row["Dispatch_Id"])
    return {k: (vals[k] / len(disp[k]), len(disp[k])) for k in vals}


def main(fd, wd, prefix=""):
    f, w = per_dispatch(fd, "FETCH_SIZE"), per_dispatch(wd, "WRITE_SIZE")
    out = {"note": "HBM bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024); gfx950 FETCH_SIZE "
                   "correction per MI355X_MICROARCH.md", "kernels": {}}
    for k in sorted(set(f) | set(w)):
        fk, nf = f.get(k, (0.0, 0))
        wk, nw = w.get(k, (0.0, 0))
        out["kernels"][prefix + k] = {"fetch_kb": fk, "write_kb": wk, "dispatches": [nf, nw],
                             "hbm_bytes_per_dispatch": (2 * fk + wk) * 1024}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
