"""PMC HBM traffic of the scatter-add (bench.py scatter_add_roofline) in both cache states.

    python tools/scatter_pmc.py run <warm|cold>          (under rocprofv3 --pmc, by scatter_pmc.sh)
    python tools/scatter_pmc.py collect gpurun_out/<tag> [profiles/traffic.json] [cfg2]

`run` builds the cfg2 bench batch and launches cgr_segment_sum 5 + 50 times per kernel (the dst
scatter, k_segsum_v4m<false, 2>, and its src-gather twin, <true, 2>) in the given cache state.
`collect` reads the FETCH_SIZE / WRITE_SIZE passes, drops each kernel's first 5 dispatches
(warm-up) and writes per-launch HBM bytes, (2 FETCH_SIZE + WRITE_SIZE) x 1024 (gfx950 calibration,
MI355X_MICROARCH.md HBM section), into traffic.json under segsum_dst_fwd (warm),
segsum_dst_fwd_cold and segsum_src_twin_cold.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd")]


def run(state):
    import torch

    import bench
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch

    c = CONFIGS["cfg2"]
    dev = torch.device("cuda:0")
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    ei = torch.from_numpy(b.edge_index).to(dev)
    which = [("segsum_dst_fwd", state), ("segsum_src_bwd", state)]
    res = bench.scatter_add_roofline(ei, b.x.shape[0], c["hidden"], dev, which=which)
    print(json.dumps({f"{k[0]}_{k[1]}": v["avg_launch_us"] for k, v in res.items()}))


def collect(root, out_path=None, cfg="cfg2"):
    res = {}
    for state in ("warm", "cold"):
        vals = {}
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            per = {}
            files = glob.glob(os.path.join(root, f"pmc_{state}_{counter.lower()}", "**",
                                           "*counter_collection.csv"), recursive=True)
            for f in files:
                rows = [r for r in csv.DictReader(open(f)) if r.get("Counter_Name") == counter]
                rows.sort(key=lambda r: int(r.get("Dispatch_Id", 0)))
                for r in rows:
                    per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
            for name, v in per.items():
                kind = "src" if re.search(r"k_segsum\w*<true", name) else "dst"
                v = v[5:]  # warm-up dispatches
                vals.setdefault(kind, {})[counter] = sum(v) / max(1, len(v))
                vals[kind]["n"] = len(v)
        for kind, d in vals.items():
            key = {("dst", "warm"): "segsum_dst_fwd", ("dst", "cold"): "segsum_dst_fwd_cold",
                   ("src", "warm"): "segsum_src_twin_warm",
                   ("src", "cold"): "segsum_src_twin_cold"}[(kind, state)]
            fk, wk = d.get("FETCH_SIZE", 0.0), d.get("WRITE_SIZE", 0.0)
            res[key] = {"dispatches": d["n"], "fetch_size_kib_per_launch": round(fk, 1),
                        "write_size_kib_per_launch": round(wk, 1),
                        "hbm_bytes_per_launch": round((2 * fk + wk) * 1024),
                        "source": "tools/scatter_pmc.py (standalone cgr_segment_sum, " + state +
                                  " cache)"}
    doc = {}
    if out_path and os.path.exists(out_path):
        doc = json.load(open(out_path))
    doc.setdefault(cfg, {}).update(res)
    txt = json.dumps(doc, indent=1, sort_keys=True)
    if out_path:
        open(out_path, "w").write(txt + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        collect(sys.argv[2], *(sys.argv[3:]))
