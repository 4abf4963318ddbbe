"""Phase stamps of the split-bf16 NT GEMMs in one training step (diagnostic build, -DCGR_STAMPS).

    tools/build_variant.sh WORKTREE stamps -DCGR_STAMPS
    CGR_MPNN3D_LIB=build/variants/stamps/libcgr_mpnn3d.so python tools/stamp_lab.py [--config cfg2]

Every gemm_b3nt_kernel workgroup writes one record (csrc/stamps.hpp): shader-clock stamps at
entry (0), after the prologue (1), after the main loop (2), after the accumulators reach LDS (3),
after the epilogue's first pass (4: segment walk of the fused backward / apply of the others),
after the fused backward's row pass (5), after its hand-off (6), and at the end (7), plus the
100 MHz realtime clock at entry and end.  Printed per launch: grid, workgroup start spread, kernel
span, and per phase the median / 90th percentile / max over workgroups in microseconds (the
shader clock converted with each workgroup's own cycles-per-realtime ratio).
"""

from __future__ import annotations

import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

PHASES = ["prologue", "mainloop", "acc_to_lds", "epi_pass1", "epi_rows", "handoff", "tail"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--serial", type=int, default=1, help="1: one stream (profile mode)")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.loss import MSELoss
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    dev = torch.device("cuda:0")
    c = CONFIGS[args.config]
    D, H = c["depth"], c["hidden"]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    data = b.to_torch(dev)
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.02] * D,
            use_learnable_skip=c["learnable_skip"]).to(dev).train()
    loss_fn = MSELoss(reduction="sum")
    lib = native.load()

    def step():
        m.zero_grad(set_to_none=True)
        loss_fn(m(data), data.y).backward()

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    cap = 1 << 16
    buf = torch.zeros(2 + 16 * cap, dtype=torch.int64, device=dev)
    if args.serial:
        lib.cgr_profile_enable(1)
    native.check(lib.cgr_debug_stamps(buf.data_ptr(), cap))
    step()
    torch.cuda.synchronize()
    native.check(lib.cgr_debug_stamps(None, 0))
    lib.cgr_profile_enable(0)
    lib.cgr_profile_reset()
    raw = buf.cpu().numpy().view(np.uint64)
    n = int(raw[0] & 0xFFFFFFFF)
    rec = raw[2:2 + 16 * min(n, cap)].reshape(-1, 16).astype(np.int64)
    out = []
    i = 0
    t_first = rec[:, 2].min() if len(rec) else 0
    while i < len(rec):
        tag = int(rec[i, 0] & 0xFFFF)
        grid = int(rec[i, 0] >> 16)
        r = rec[i:i + grid]
        i += grid
        st = r[:, 4:12].astype(np.float64)
        cyc = st[:, 7] - st[:, 0]
        rt = (r[:, 3] - r[:, 2]).astype(np.float64) * 10e-3  # us (100 MHz)
        ghz = np.where(rt > 0, cyc / np.maximum(rt, 1e-9) / 1e3, np.nan)
        per_us = 1.0 / (np.nanmedian(ghz) * 1e3)
        if tag & 0x4000:  # split-bf16 TN (gemm_b3tni_kernel): accumulated cycles, not stamps
            med = lambda v: round(float(np.median(v)) * per_us, 2)
            out.append({"tag": "tn", "tnn": tag & 0xFF, "grid": grid,
                        "t_start_us": round((r[:, 2].min() - t_first) * 1e-2, 2),
                        "span_us": round((r[:, 3].max() - r[:, 2].min()) * 1e-2, 2),
                        "wg_life_us": {"med": round(float(np.median(rt)), 2),
                                       "max": round(float(rt.max()), 2)},
                        "compute_work_us": med(st[:, 1]), "compute_barrier_wait_us": med(st[:, 2]),
                        "staging_work_us": med(st[:, 3]), "staging_barrier_wait_us": med(st[:, 4]),
                        "epilogue_us": med(st[:, 7] - st[:, 5]),
                        "before_loop_us": med(st[:, 5] - st[:, 0] - st[:, 1] - st[:, 2])})
            continue
        row = {"tag": tag, "tile": bool(tag & 2), "seg": bool(tag & 1), "nf": (tag >> 2) & 31,
               "waves": tag >> 7, "grid": grid,
               "t_start_us": round((r[:, 2].min() - t_first) * 1e-2, 2),
               "start_spread_us": round((r[:, 2].max() - r[:, 2].min()) * 1e-2, 2),
               "span_us": round((r[:, 3].max() - r[:, 2].min()) * 1e-2, 2),
               "wg_life_us": {"med": round(float(np.median(rt)), 2), "max": round(float(rt.max()), 2)},
               "clock_ghz": round(float(np.nanmedian(ghz)), 3), "phases_us": {}}
        prev = st[:, 0]
        for k, name in enumerate(PHASES, start=1):
            cur = st[:, k]
            ok = cur > 0
            if ok.any():
                d = (cur[ok] - prev[ok]) * per_us
                row["phases_us"][name] = {"med": round(float(np.median(d)), 2),
                                          "p90": round(float(np.percentile(d, 90)), 2),
                                          "max": round(float(d.max()), 2)}
                prev = np.where(ok, cur, prev)
        out.append(row)
    for row in out:
        print(json.dumps(row))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
