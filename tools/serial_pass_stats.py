"""Average duration of a kernel class over the bench's instrumented serial pass, from a rocprofv3
kernel trace of the default bench command (the roofline's HIP-event timing covers exactly these
dispatches: the last `--profile-steps` steps of the training section, before the inference
section, which has no backward kernels).

    python tools/serial_pass_stats.py <run_kernel_trace.csv> <name substring> <dispatches>

prints the average over the last <dispatches> dispatches whose name contains the substring, and
the average over all of them (graph-replayed steps included, which run beside the other stream).
"""
import csv
import sys

path, sub, n = sys.argv[1], sys.argv[2], int(sys.argv[3])
rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
last = dur[-n:]
print(f"{sub}: {len(dur)} dispatches, all {sum(dur) / len(dur):.2f} us; "
      f"last {len(last)} (serial pass) {sum(last) / len(last):.2f} us")
