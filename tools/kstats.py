"""Summarise a rocprofv3 kernel_stats.csv: short kernel name, calls, average / min / max us."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:n]:
    name = re.sub(r"\(.*", "", r["Name"])
    name = re.sub(r"cgr::", "", name)[:90]
    print(f"{name:90s} {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:8.2f} us"
          f"  min {float(r['MinNs'])/1e3:7.2f}  max {float(r['MaxNs'])/1e3:7.2f}  tot% {float(r['Percentage']):5.1f}")
