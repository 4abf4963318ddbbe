"""Aggregate rocprofv3 counter_collection.csv files per kernel: mean counter value per dispatch."""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d):
    out = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
            cn = r.get("Counter_Name") or r.get("Counter-Name")
            val = float(r.get("Counter_Value") or r.get("Counter-Value"))
            disp = r.get("Dispatch_Id") or r.get("Dispatch-Id")
            out[name][cn].append(val)
    return out


def short(n):
    n = n.replace("cgr::", "")
    return n[:90]


def main(root):
    agg = defaultdict(dict)
    for d in sorted(glob.glob(os.path.join(root, "pmc_*"))):
        for k, cs in load(d).items():
            for c, vals in cs.items():
                agg[k][c] = sum(vals) / len(vals)
    for k in sorted(agg, key=lambda k: -agg[k].get("SQ_WAVE_CYCLES", 0)):
        c = agg[k]
        print(short(k))
        print("   " + "  ".join(f"{n}={v:.4g}" for n, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1])
