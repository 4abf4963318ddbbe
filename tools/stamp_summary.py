"""One line per NT launch of a stamp_lab.py JSON: kind, grid, span and median / max per phase."""
import json
import sys

names = {0: "plain", 1: "seg", 2: "tile"}
for path in sys.argv[1:]:
    print("==", path)
    for r in json.load(open(path)):
        ph = " ".join(f"{k}={v['med']:.1f}/{v['max']:.1f}" for k, v in r["phases_us"].items())
        print(f"t={r['t_start_us']:7.1f} {names[r['tag'] & 3]:5s} nf={r['nf']:2d} grid={r['grid']:4d} "
              f"span={r['span_us']:5.1f} clk={r['clock_ghz']:.2f} | {ph}")
