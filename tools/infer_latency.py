"""Where the single-reaction latency goes.

One cfg2-shaped reaction (30 atoms, 60 directed edges, F = 846, H 400, D 4), eval, no_grad;
median over `--calls` of (call + synchronize) for:
  module_eager       model(data), the forward-only path (GNN.forward + cgr_gnn_predict)
  functional_eager   functional.gnn_predict alone (no GNN.forward Python)
  replay_only        model(data) captured into a HIP graph, its replay alone (the device floor)
  sync_only / tiny_kernel_sync   the floor: a bare synchronize, one tiny kernel + synchronize
plus the host time per call of the first three issued back to back (no sync in between).
"""

import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402


def med(fn, n):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return round(float(np.median(t)) * 1e6, 1)


def host(fn, n=100):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    h = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    return round(h * 1e6, 1)


def main():
    from cgr_mpnn_3D._amd.functional import gnn_predict
    from cgr_mpnn_3D._amd.synth import TorchBatch, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    dev = torch.device("cuda:0")
    b = make_batch(1, 30, 30, 768, seed=4242)
    d = TorchBatch(*(torch.from_numpy(a).to(dev) for a in (b.x, b.edge_index, b.edge_attr)),
                   None)
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=4, hidden_sizes=[400] * 4, dropout_ps=[0.0] * 4).to(dev).eval()
    params = [p.detach() for p in m.native_parameters()]
    cfg = (b.x.shape[1], 14, 400, 4, 0, False, 0, 0)
    out = {}
    with torch.no_grad():
        out["module_eager"] = med(lambda: m(d), n)
        out["module_eager_host"] = host(lambda: m(d))

        def fe():
            return gnn_predict(cfg, d.x, d.edge_index, d.edge_attr, None, None, 1, [0.0] * 4, 0,
                               False, params)
        out["functional_eager"] = med(fe, n)
        out["functional_eager_host"] = host(fe)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            m(d)
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            m(d)
        out["replay_only"] = med(g.replay, n)
        out["replay_only_host"] = host(g.replay)
        z = torch.zeros(16, device=dev)
        out["sync_only"] = med(lambda: None, n)
        out["tiny_kernel_sync"] = med(lambda: z.add_(1.0), n)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
