"""Cost of the unpaired-edge fallback of the fused layer backward (ep_bwd.hpp).

The reference's reverse edge is e ^ 1 whatever the edges hold (GNN.py:136-138); when some edge's
partner is not its reverse (status bit 2) the fused backward GEMM stores every dm row and its
grid's last workgroup completes the src sums alone.  This times one eager fwd + bwd of the cfg2
batch as collated (paired) and with the edges of every graph shuffled (unpaired), same weights,
median of 20 after warm-up, and the backward's per-class device times of one instrumented step.

    python tools/unpaired_timing.py [--config cfg2]
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
import warnings
from dataclasses import replace

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()

    from cgr_mpnn_3D._amd import native
    from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    dev = torch.device("cuda:0")
    c = CONFIGS[args.config]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    per = b.edge_index.shape[1] // b.num_graphs
    rng = np.random.default_rng(6)
    order = np.concatenate([g * per + rng.permutation(per) for g in range(b.num_graphs)])
    u = replace(b, edge_index=np.ascontiguousarray(b.edge_index[:, order]),
                edge_attr=np.ascontiguousarray(b.edge_attr[order]))
    lib = native.load()
    out = {"config": args.config}
    for name, batch in (("paired", b), ("unpaired", u)):
        data = batch.to_torch(dev)
        torch.manual_seed(0)
        m = GNN(b.x.shape[1], 14, depth=c["depth"], hidden_sizes=[c["hidden"]] * c["depth"],
                dropout_ps=[0.0] * c["depth"], use_learnable_skip=c["learnable_skip"]).to(dev)

        def step():
            m.zero_grad(set_to_none=True)
            torch.nn.MSELoss(reduction="sum")(m(data), data.y).backward()

        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            for _ in range(5):
                step()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.iters):
            t0 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        lib.cgr_profile_reset()
        lib.cgr_profile_enable(1)
        step()
        torch.cuda.synchronize()
        lib.cgr_profile_enable(0)
        rep = native.profile_report()
        lib.cgr_profile_reset()
        cnt, ms = rep.get("gemm_nt_layer_bwd_seg", (0, float("nan")))
        out[name] = {"fwd_bwd_ms_median": round(1e3 * float(np.median(ts)), 3),
                     "gemm_nt_layer_bwd_seg_us_per_launch": round(1e3 * ms / max(cnt, 1), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
