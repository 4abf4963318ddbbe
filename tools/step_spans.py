"""Per-step spans (k_adam to k_adam) of a rocprofv3 kernel trace of bench.py, and the start of the
first backward kernel (k_head_bwd) inside each step: python tools/step_spans.py run_kernel_trace.csv"""
import csv
import re
import statistics
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
ends = [i for i, r in enumerate(rows) if re.search(r"k_adam\(|k_adam$|cgr::k_adam\b(?!_)", r[2])
        and "step_count" not in r[2]]
spans, fwd = [], []
for a, b in zip(ends, ends[1:]):
    step = rows[a + 1:b + 1]
    t0 = step[0][0]
    spans.append((max(r[1] for r in step) - t0) / 1000)
    hb = [r[0] for r in step if "k_head_bwd" in r[2]]
    if hb:
        fwd.append((hb[0] - t0) / 1000)
print("steps", len(spans), "span median %.1f us" % statistics.median(spans),
      "min %.1f" % min(spans), "| fwd (to k_head_bwd) median %.1f" % statistics.median(fwd))
print("spans", " ".join("%.0f" % s for s in spans))
