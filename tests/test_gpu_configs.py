"""GPU parity over the reference's own configuration space, and full-size BASELINE cfg4.

The reference trains with `train.py`'s defaults -- depth 3, hidden 300, dropout 0.02
(train.py:156-166; GNN.py:46-47) -- and its hyper-parameter sweep spans hidden in
{100, 300, 500, 1000} x depth {2, 3, 4, 5, 6} with the learnable skip on or off
(hyperparameter_study/sweep_config.json:6-7, expanded at hyperparameter_tuning.py:24-26).  Every
such width must give the oracle's predictions and gradients (tolerances of test_gpu_parity.py).

Which GEMM family a width takes is part of what is tested: widths up to 512 run every weight
gradient on the split-bf16 e-image TN; wider ones fall back to the register-direct fp32 TN
(H % 5 == 0 or H % 4 == 0, e.g. H = 1000: `<class>[tnr]` in the per-class profile) or to the
LDS-staged fp32 TN (`<class>[f32]`, e.g. H = 521).  The test reads the library's per-class
report of one profiled step and asserts the family, so a green run proves the fallback kernels
produced these gradients.
"""

import numpy as np
import pytest
import torch

from test_gpu_parity import AMBIGUOUS_Z, _oracle_compare, assert_g_close, assert_y_close

from cgr_mpnn_3D._amd import native
from cgr_mpnn_3D._amd.synth import make_batch
from cgr_mpnn_3D.models.GNN import GNN

pytestmark = pytest.mark.gpu

TN_CLASSES = ("gemm_tn_wgrad_layer", "gemm_tn_wgrad_node", "gemm_tn_wgrad_readout")


def _expected_family(H):
    if H <= 512:
        return ""  # split-bf16 e-image TN: the plain class name
    if H % 5 == 0 or H % 4 == 0:
        return "[tnr]"
    return "[f32]"


def _profiled_classes(m, data):
    lib = native.load()
    lib.cgr_profile_reset()
    lib.cgr_profile_enable(1)
    try:
        m.zero_grad(set_to_none=True)
        torch.nn.MSELoss(reduction="sum")(m(data), data.y).backward()
        torch.cuda.synchronize()
    finally:
        lib.cgr_profile_enable(0)
    rep = native.profile_report()
    lib.cgr_profile_reset()
    return set(rep)


# every sweep depth (sweep_config.json:6: 2..6) x width x learnable skip
SWEEP = [(H, D, skip) for H in (100, 300, 500, 1000) for D in (2, 3, 4, 5, 6)
         for skip in (False, True)]


@pytest.mark.parametrize("H,D,skip", SWEEP + [(521, 2, False)])
def test_reference_config_space_vs_oracle(H, D, skip, cuda_device):
    b = make_batch(6, n_atoms=30, n_bonds=30, n_mace=768, seed=H + 10 * D + skip)
    _oracle_compare(b, H, D, "relu", skip, cuda_device, seed=H + D)
    # the weight-gradient family that produced those gradients
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[0.0] * D,
            use_learnable_skip=skip).to(cuda_device).train()
    classes = _profiled_classes(m, b.to_torch(cuda_device))
    fam = _expected_family(H)
    for c in TN_CLASSES:
        assert c + fam in classes, (c + fam, sorted(classes))
        for other in ("", "[tnr]", "[f32]"):
            if other != fam:
                assert c + other not in classes, (c + other, sorted(classes))


def test_train_py_default_config_with_dropout_vs_oracle(cuda_device):
    # train.py's defaults: depth 3, hidden 300, dropout 0.02, ReLU, no learnable skip, in train
    # mode.  The dropout mask is ours (counter-based RNG), recovered from the saved
    # activations: with ReLU an element of h_{l+1} is nonzero exactly where z > 0 and the mask
    # keeps it; where it is zero the element contributes nothing forward and gets no gradient,
    # whichever of the two zeroed it.  So the oracle runs with (h != 0) as both the dropout mask
    # and the ReLU decision of every layer (and the GPU's h0 > 0 / hn > 0 for the edge init and
    # the readout), after checking that every GPU decision agrees with fp64 wherever |z| is not
    # within rounding reach of 0 (a kept z > 0 element is nonzero on the GPU; an fp64 z < 0 one
    # is zero).
    from cgr_mpnn_3D._amd.debug import ArenaRun
    from oracle import dmpnn_numpy as on

    from test_gpu_parity import _cfg_tuple

    D, H, p = 3, 300, 0.02
    b = make_batch(32, seed=156)
    torch.manual_seed(3)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[p] * D).to(cuda_device)
    params = [q.detach() for q in m.native_parameters()]
    data = b.to_torch(cuda_device)
    run = ArenaRun(_cfg_tuple(b.x.shape[1], 14, H, D, "relu", False), data.x, data.edge_index,
                   data.edge_attr, data.batch, data.ptr, b.num_graphs, params,
                   dropout_ps=[p] * D, seed=20250227, training=True)
    torch.cuda.synchronize()
    N, E = data.x.shape[0], data.edge_index.shape[1]
    perm = run.ints("perm", E).long().cpu().numpy()

    def unsort(t):
        out = np.empty_like(t)
        out[perm] = t
        return out

    nz = [unsort(run.floats("h", E, index=l + 1).cpu().numpy()) != 0 for l in range(D)]
    rm = {"z0": unsort(run.floats("h", E, index=0).cpu().numpy()) > 0, "zs": nz,
          "zn": run.floats("hn", N).cpu().numpy() > 0}
    masks = [k.astype(np.float64) for k in nz]
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    _, c64 = on.forward(sd, b.x, b.edge_index, b.edge_attr, b.batch, D, "relu",
                        dropout_masks=masks, dropout_ps=[p] * D)

    def clear(z):
        return np.abs(z) > AMBIGUOUS_Z * np.abs(z).max()

    for key, z, g in (("z0", c64["z0"], rm["z0"]), ("zn", c64["zn"], rm["zn"])):
        assert not ((g != (z > 0)) & clear(z)).any(), key
    kept = 0.0
    for l in range(D):
        z = c64["zs"][l]
        assert not (nz[l] & (z < 0) & clear(z)).any(), l  # nonzero only where z > 0
        pos = (z > 0) & clear(z)
        kept += nz[l][pos].mean() / D
    assert abs((1.0 - kept) - p) < 0.01, 1.0 - kept  # the drop rate among clear z > 0
    y_o, cache = on.forward(sd, b.x, b.edge_index, b.edge_attr, b.batch, D, "relu",
                            dropout_masks=masks, dropout_ps=[p] * D, relu_masks=rm)
    assert_y_close(run.y.cpu().numpy(), y_o)
    dy = torch.randn(b.num_graphs, generator=torch.Generator().manual_seed(1)).to(cuda_device)
    grads = run.backward(dy, params)
    g_o = on.backward(sd, cache, dy.cpu().numpy())
    names = [k for k, _ in m.named_parameters()]
    for k, g in zip(names, grads):
        assert_g_close(g.cpu().numpy(), g_o[k], k)


@pytest.mark.timeout(600)
def test_full_cfg4_batch_vs_oracle(cuda_device):
    # BASELINE cfg4 at its bench shape: 256 reactions of 200 atoms / 800 directed edges
    # (N 51,200, E 204,800; the fp32 edge tensors exceed the 256 MB MALL), D 4, H 400
    from cgr_mpnn_3D._amd.synth import CONFIGS

    c = CONFIGS["cfg4"]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    assert b.edge_index.shape[1] == 204800
    _oracle_compare(b, c["hidden"], c["depth"], "relu", c["learnable_skip"], cuda_device,
                    case="cfg4_full_256")
