"""Per-parameter gradient error of the HIP path vs the fp64 oracle for a few config-space cases
(diagnostic for test_gpu_configs failures): prints max|g - g_ref| / max|g_ref| per tensor and, for
the learnable-skip scalars, the conditioning sum|dpre * h0| / |sum dpre * h0|."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cgr_mpnn_3D._amd.synth import make_batch  # noqa: E402
from cgr_mpnn_3D.models.GNN import GNN  # noqa: E402
from oracle import dmpnn_numpy as on  # noqa: E402

dev = torch.device("cuda:0")
for H, D, skip in [(1000, 4, True), (1000, 4, False), (1000, 3, True), (1000, 5, True),
                   (500, 4, True)]:
    b = make_batch(6, n_atoms=30, n_bonds=30, n_mace=768, seed=H + 10 * D + skip)
    torch.manual_seed(H + D)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.0] * D,
            use_learnable_skip=skip)
    if skip:
        with torch.no_grad():
            for i, w in enumerate(m.skip_weights):
                w.fill_(0.5 + 0.25 * i)
    sd = {k: v.detach().numpy().copy() for k, v in m.state_dict().items()}
    m = m.to(dev).train()
    data = b.to_torch(dev)
    pred = m(data)
    torch.nn.MSELoss(reduction="sum")(pred, data.y).backward()
    _, y_o, g_o = on.loss_and_grads(sd, b.x, b.edge_index, b.edge_attr, b.batch, b.y, D, "relu",
                                    skip, num_graphs=b.num_graphs)
    y = pred.detach().cpu().numpy()
    print(f"H={H} D={D} skip={skip}: y err {np.abs(y - y_o).max() / np.abs(y_o).max():.2e}")
    for k, p in m.named_parameters():
        g = p.grad.cpu().numpy().astype(np.float64)
        r = np.abs(g - g_o[k]).max() / (np.abs(g_o[k]).max() + 1e-30)
        flag = "  <-- over 1e-4" if r > 1e-4 else ""
        print(f"   {k:28s} {r:.2e}  max|g_ref| {np.abs(g_o[k]).max():.3e}{flag}")
