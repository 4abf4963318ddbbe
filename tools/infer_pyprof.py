"""Where the host time of one single-reaction model(data) call goes (cProfile over many calls,
no synchronisation between them; tools/infer_latency.py times the whole call)."""

import cProfile
import os
import pstats
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cgr-mpnn-3d_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    from cgr_mpnn_3D._amd.synth import TorchBatch, make_batch
    from cgr_mpnn_3D.models.GNN import GNN

    dev = torch.device("cuda:0")
    b = make_batch(1, 30, 30, 768, seed=4242)
    d = TorchBatch(*(torch.from_numpy(a).to(dev) for a in (b.x, b.edge_index, b.edge_attr)),
                   None)
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=4, hidden_sizes=[400] * 4, dropout_ps=[0.0] * 4).to(dev).eval()
    with torch.no_grad():
        for _ in range(50):
            m(d)
        torch.cuda.synchronize()
        pr = cProfile.Profile()
        pr.enable()
        for i in range(2000):
            m(d)
            if i % 50 == 49:
                torch.cuda.synchronize()
        pr.disable()
        torch.cuda.synchronize()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
