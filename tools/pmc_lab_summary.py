"""Summarise tools/pmc_lab.sh output: per kernel (name prefix + grid size) mean of each counter."""
import csv, glob, os, sys, collections
root = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
rows = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if filt and filt not in name:
            continue
        key = (name[:90], r.get("Grid_Size", r.get("Grid_Size_X", "")), r.get("Workgroup_Size", ""))
        rows[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in sorted(rows.items()):
    print(key)
    for c, v in sorted(cs.items()):
        print(f"   {c:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
