"""Lab: the standalone scatter-add (bench.py scatter_add_roofline) per k_segsum variant
(CGR_SEGSUM_ITEMS = 1 / 2 / 4 items per thread), warm and cold cache, cfg2 shape.

    python tools/scatter_lab.py [rounds]
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from cgr_mpnn_3D._amd.synth import CONFIGS, make_batch  # noqa: E402

c = CONFIGS["cfg2"]
dev = torch.device("cuda:0")
b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
ei = torch.from_numpy(b.edge_index).to(dev)
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 2
for r in range(rounds):
    for items in ("1", "2", "4"):
        os.environ["CGR_SEGSUM_ITEMS"] = items
        res = bench.scatter_add_roofline(ei, b.x.shape[0], c["hidden"], dev)
        print(json.dumps({"items": int(items), "round": r,
                          **{f"{k[0]}_{k[1]}": [v["avg_launch_us"], v["frac"]]
                             for k, v in res.items()}}), flush=True)
