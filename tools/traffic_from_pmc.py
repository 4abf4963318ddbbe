"""HBM traffic per launch of each native kernel class from rocprofv3 PMC passes.

    python tools/traffic_from_pmc.py gpurun_out/<tag> cfg2 [profiles/traffic.json]

Reads the FETCH_SIZE and WRITE_SIZE passes written by tools/pmc_profile.sh (one counter per
rocprofv3 run, --pmc + --kernel-trace only) and maps each dispatch to the ProfScope class the
bench reports (bench.py algorithmic_work).  MI355X_MICROARCH.md "HBM": both counters are in KiB;
on gfx950 FETCH_SIZE reads exactly half of the bytes of a wide (16 B/lane) coalesced read, so

    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

Infinity-Cache (L3) hits are counted by these memory-side counters, so a table re-read out of L3
still shows up here; traffic well above the algorithmic bytes means re-reads to remove.
"""

from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def classify(name: str, grid: int, grids_by_name: dict) -> str | None:
    n = name
    if "gemm_b3tni_kernel" in n or "gemm_b3tn_kernel" in n:  # split-bf16 TN (gemm_b3.hpp)
        if "LdGatherDiff" in n:
            return "gemm_tn_wgrad_layer"
        if "LdConcat" in n:
            return "gemm_tn_wgrad_readout"
        return "gemm_tn_wgrad_node"
    if "gemm_b3nt_kernel" in n:  # split-bf16 NT
        if "EpLayerBwdSeg" in n:
            return "gemm_nt_layer_bwd_seg"
        if "EpLayerSeg" in n:
            return "gemm_nt_layer_seg_fwd"
        if "EpLayer" in n:
            return "gemm_nt_layer_fwd"
        if "EpSplit2" in n:
            return "gemm_nt_x"
        if "EpReadout" in n:
            return "gemm_nt_readout_fwd"
        if "EpStore" in n:  # the readout backward (ds = dzn W_n[:, F:])
            return "gemm_nt_readout_bwd"
    if "k_b3_eimage" in n:
        return "eimage"
    if "k_b3_pack" in n:
        return "weight_pack"
    if "gemm_tnr_kernel" in n:  # register-direct fp32 TN (shapes the split-bf16 TN does not take)
        if "TnrDiff" in n:
            return "gemm_tn_wgrad_layer"
        if "TnrConcat" in n:
            return "gemm_tn_wgrad_readout"
        return "gemm_tn_wgrad_node"
    if "gemm_tn_kernel" in n:  # fp32 fallback tiles (shapes the split-bf16 TN does not take)
        if "LdGatherDiff" in n:
            return "gemm_tn_wgrad_layer"
        if "LdConcat" in n:
            return "gemm_tn_wgrad_readout"
        # dW0x (B = x, vector width of F) vs dW0e (B = padded edge features, always 4-wide)
        m = re.search(r"LdPlain<\d+>, cgr::LdPlain<(\d+)>", n)
        if m and m.group(1) != "4":
            return "gemm_tn_wgrad_node"
        return "gemm_tn_wgrad_edge"  # ambiguous only when F % 4 == 0; see note in the output
    if "k_segsum" in n:
        return "segsum_src_bwd" if re.search(r"k_segsum\w*<true", n) else "segsum_dst_fwd"
    table = {"k_edge_init_seg": "edge_init_seg_fwd", "k_edge_init": "edge_init_fwd",
             "k_layer_bwd": "layer_act_bwd", "k_pool_head": "pool_head_fwd",
             "k_head_bwd": "head_bwd", "k_readout_bwd": "readout_act_bwd",
             "k_layer_bwd_img": "layer_act_bwd", "k_readout_bwd_img": "readout_act_bwd",
             "k_b3_segsum_eimage": "segsum_src_bwd",
             "k_reduce_slabs": "splitk_reduce"}
    for k, v in table.items():
        if re.search(r"\b" + k + r"[<(]", n):
            return v
    return None


def load(pass_dir: str, counter: str):
    rows = []
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if (r.get("Counter_Name") or "") != counter:
                continue
            rows.append((r["Kernel_Name"], int(r["Grid_Size"]), float(r["Counter_Value"])))
    return rows


def per_class(rows):
    grids = defaultdict(set)
    for n, g, _ in rows:
        grids[n].add(g)
    acc = defaultdict(list)
    for n, g, v in rows:
        c = classify(n, g, grids)
        if c:
            acc[c].append(v)
    return acc


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    out_path = sys.argv[3] if len(sys.argv) > 3 else None
    fetch = per_class(load(os.path.join(root, "pmc_fetch"), "FETCH_SIZE"))
    write = per_class(load(os.path.join(root, "pmc_write"), "WRITE_SIZE"))
    res = {}
    for c in sorted(set(fetch) | set(write)):
        fk = sum(fetch.get(c, [0])) / max(1, len(fetch.get(c, [])))
        wk = sum(write.get(c, [0])) / max(1, len(write.get(c, [])))
        res[c] = {"dispatches": len(fetch.get(c, [])),
                  "fetch_size_kib_per_launch": round(fk, 1),
                  "write_size_kib_per_launch": round(wk, 1),
                  "hbm_bytes_per_launch": round((2 * fk + wk) * 1024)}
    doc = {}
    if out_path and os.path.exists(out_path):
        doc = json.load(open(out_path))
    doc[cfg] = res
    doc["_note"] = ("hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE)*1024 averaged over the "
                    "class's dispatches (gfx950 FETCH_SIZE counts half of 16-B/lane reads; "
                    "MI355X_MICROARCH.md HBM section); eager bench, one counter per rocprofv3 pass")
    txt = json.dumps(doc, indent=1, sort_keys=True)
    if out_path:
        open(out_path, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
