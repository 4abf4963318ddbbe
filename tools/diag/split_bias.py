"""Is the split-bf16 NT GEMM's error biased?  (diagnostic for the learnable-skip precision gap,
DESIGN §2): the H = 1000 / D = 4 / learnable-skip case of tools/diag/cfg_err.py, forward only.
For every layer's pre-activation z (GPU arena, unsorted to the oracle's edge order) against the
fp64 oracle: max relative error, and the bias ratio sum(err * sign(z)) / sum(|err|) (0 for
unbiased rounding, -1 if every error shrinks |z|), beside the same figures for torch fp32 on the
GPU (TF32 off) from the oracle's own fp32-rounded inputs of each layer.  SiLU: the arena keeps
pre-activations only for a smooth activation (ReLU reads its mask from h)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cgr-mpnn-3d_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cgr_mpnn_3D._amd.debug import ArenaRun  # noqa: E402
from cgr_mpnn_3D._amd.synth import make_batch  # noqa: E402
from cgr_mpnn_3D.models.GNN import GNN  # noqa: E402
from oracle import dmpnn_numpy as on  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
dev = torch.device("cuda:0")
H, D, skip = 1000, 4, True
b = make_batch(6, n_atoms=30, n_bonds=30, n_mace=768, seed=H + 10 * D + skip)
torch.manual_seed(H + D)
m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.0] * D,
        use_learnable_skip=skip)
with torch.no_grad():
    for i, w in enumerate(m.skip_weights):
        w.fill_(0.5 + 0.25 * i)
sd = {k: v.detach().numpy().astype(np.float64) for k, v in m.state_dict().items()}
m = m.to(dev)
data = b.to_torch(dev)
F_, Fe = b.x.shape[1], b.edge_attr.shape[1]
run = ArenaRun((F_, Fe, H, D, 1, True, 0, 0), data.x, data.edge_index, data.edge_attr, data.batch,
               data.ptr, b.num_graphs, [p.detach() for p in m.native_parameters()])
torch.cuda.synchronize()
N, E = b.x.shape[0], b.edge_index.shape[1]
perm = run.ints("perm", E).long().cpu().numpy()


def unsort(t):
    out = np.empty_like(t)
    out[perm] = t
    return out


_, cache = on.forward(sd, b.x, b.edge_index, b.edge_attr, b.batch, D, "silu", skip, b.num_graphs)


def stats(z, ref):
    err = z.astype(np.float64) - ref
    rel = np.abs(err).max() / np.abs(ref).max()
    bias = float((err * np.sign(ref)).sum() / (np.abs(err).sum() + 1e-300))
    return f"max rel {rel:.2e}  bias {bias:+.3f}  mean|err|/mean|z| {np.abs(err).mean() / np.abs(ref).mean():.2e}"


for l in range(D):
    z_gpu = unsort(run.floats("pre", E, index=l + 1).cpu().numpy())
    z_ref = cache["zs"][l]
    # torch fp32 from the oracle's fp32-rounded message of this layer
    msg = torch.from_numpy(cache["ms"][l].astype(np.float32)).to(dev)
    W = torch.from_numpy(sd[f"convs.{l}.lin.weight"].astype(np.float32)).to(dev)
    bias_v = torch.from_numpy(sd[f"convs.{l}.lin.bias"].astype(np.float32)).to(dev)
    z_t = (msg @ W.T + bias_v).cpu().numpy()
    z_ref_from_msg = cache["ms"][l].astype(np.float32).astype(np.float64) @ sd[
        f"convs.{l}.lin.weight"].T + sd[f"convs.{l}.lin.bias"]
    print(f"layer {l}: HIP  {stats(z_gpu, z_ref)}")
    print(f"         torch fp32 (same fp32 inputs) {stats(z_t, z_ref_from_msg)}")
