"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV of bench.py.

usage: python tools/timeline.py gpurun_out/<dir>/run_kernel_trace.csv [step_marker] [k]

Steps are delimited by the fused Adam kernel (k_adam: the last kernel of a training step).  For
the k-th complete step from the end (default 1: the last; a bench run under rocprofv3 ends with its
instrumented serial pass, so pick k past those steps for a graph-replayed one) it prints every kernel (queue, start offset, duration, overlap with other
queues) and per-queue busy time, so the critical chain and the idle gaps can be read off.
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(.*", "", name)
    name = name.replace("void ", "")
    name = re.sub(r"cgr::", "", name)
    return name[:70]


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "k_adam$"
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                     r["Kernel_Name"]))
    rows.sort()
    ends = [i for i, r in enumerate(rows) if re.search(marker + r"\b", short(r[3]))]
    if len(ends) < 2:
        print("fewer than two step markers")
        return
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    a, b = ends[-k - 1] + 1, ends[-k] + 1
    step = rows[a:b]
    t0 = step[0][0]
    t1 = max(r[1] for r in step)
    print(f"step span {(t1 - t0) / 1000:.1f} us, {len(step)} kernels "
          f"(previous step end -> this step start gap {(t0 - rows[a - 1][1]) / 1000:.1f} us)")
    busy = {}
    for s, e, q, n in step:
        busy[q] = busy.get(q, 0) + (e - s)
    print("queue busy (us):", {q: round(v / 1000, 1) for q, v in sorted(busy.items())})
    print(f"{'start':>8} {'dur':>7} {'q':>2}  kernel")
    for s, e, q, n in step:
        print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f} {q:2d}  {short(n)}")
    # union of busy intervals (any queue): idle time of the whole GPU inside the step
    iv = sorted((s, e) for s, e, _, _ in step)
    cover, cs, ce = 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            cover += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    cover += ce - cs
    print(f"GPU busy (any queue) {cover / 1000:.1f} us of {(t1 - t0) / 1000:.1f} us")


if __name__ == "__main__":
    main()
