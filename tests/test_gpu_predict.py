"""GPU: the forward-only inference path (cgr_gnn_predict), SURVEY.md §8(f) rank 3.

GNN.forward takes it whenever no gradient is wanted -- test.py:100-113 and
cli_tool/activation_energy_predictor.py:70-80 call the model under torch.no_grad() in eval mode.
It runs the training forward's kernels in the same order, with h_1 .. h_D on a two-buffer ring,
a_0 .. a_D on a three-buffer ring and weight images packed into its own arena by every call, so its
predictions must equal the training forward's bit for bit (and, through it, the reference goldens
of test_gpu_parity.py, which also run under no_grad).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from cgr_mpnn_3D._amd import native
from cgr_mpnn_3D._amd.functional import make_config
from cgr_mpnn_3D._amd.synth import make_batch
from cgr_mpnn_3D.models.GNN import GNN
from oracle import dmpnn_numpy as on

pytestmark = pytest.mark.gpu


def _model(dev, F_, D, H, act=F.relu, skip=False, p=0.0):
    torch.manual_seed(D * 7 + H)
    m = GNN(F_, 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[p] * D, activation_fn=act,
            use_learnable_skip=skip).to(dev)
    if skip:
        with torch.no_grad():
            for i, w in enumerate(m.skip_weights):
                w.fill_(0.5 + 0.25 * i)
    return m


# depth 1 .. 6: the rings alias h / a buffers from depth 2 / 3 on and the layer epilogue zeroes
# the accumulated entries two layers ahead from depth 4 on
@pytest.mark.parametrize("D,H,act,skip", [(1, 400, "relu", False), (2, 400, "relu", False),
                                          (3, 400, "silu", True), (4, 400, "relu", False),
                                          (6, 512, "relu", True), (5, 37, "gelu", True)])
def test_predict_equals_training_forward_bitwise(D, H, act, skip, cuda_device):
    b = make_batch(48, seed=D + H)
    data = b.to_torch(cuda_device)
    m = _model(cuda_device, b.x.shape[1], D, H, {"relu": F.relu, "silu": F.silu,
                                                   "gelu": F.gelu}[act], skip)
    m.eval()
    y_train = m(data)  # grad enabled, parameters require grad: the training forward
    assert y_train.requires_grad
    with torch.no_grad():
        y_pred = m(data)
    assert not y_pred.requires_grad
    assert torch.equal(y_pred, y_train.detach())


def test_predict_cfg2_batch_vs_oracle_and_arena_size(cuda_device):
    from cgr_mpnn_3D._amd.synth import CONFIGS

    c = CONFIGS["cfg2"]
    b = make_batch(c["num_graphs"], c["n_atoms"], c["n_bonds"], c["n_mace"], seed=1234)
    m = _model(cuda_device, b.x.shape[1], 4, 400).eval()
    sd = {k: v.detach().cpu().numpy().astype(np.float64) for k, v in m.state_dict().items()}
    with torch.no_grad():
        y = m(b.to_torch(cuda_device)).cpu().numpy().astype(np.float64)
    y_o, _ = on.forward(sd, b.x, b.edge_index, b.edge_attr, b.batch, 4, "relu", False,
                        b.num_graphs)
    assert np.all(np.abs(y - y_o) <= 1e-4 * np.abs(y_o) + 1e-6 * np.abs(y_o).max())
    lib = native.load()
    import ctypes

    cfg = make_config(b.x.shape[1], 14, 400, 4, 0, False)
    N, E, B = b.x.shape[0], b.edge_index.shape[1], b.num_graphs
    train = lib.cgr_gnn_arena_bytes(ctypes.byref(cfg), N, E, B)
    pred = lib.cgr_gnn_predict_arena_bytes(ctypes.byref(cfg), N, E, B)
    images = lib.cgr_gnn_image_bytes(ctypes.byref(cfg))  # packed into the predict arena per call
    assert 0 < images < pred
    assert pred - images < 0.7 * train  # (index bookkeeping, x copy and P / Q stay)


def _assert_predict_is_current(m, data):
    m.eval()
    with torch.no_grad():
        y_pred = m(data)
    y_train = m(data)  # grad-enabled forward: packs its images from the current weights
    assert torch.equal(y_pred, y_train.detach())
    m.train()


@pytest.mark.parametrize("opt_kind", ["torch", "fused", "fused_captured"])
def test_predict_follows_every_optimizer_update(opt_kind, cuda_device):
    # a no-grad forward must see the weights after every optimizer step, however the
    # step wrote them: torch.optim.Adam (in-place ops, version counters bump), the native
    # FusedAdam (raw pointers: no version bump) and a captured training step replayed (nothing
    # on the host changes at all) -- the reference trainer validates under no_grad after every
    # epoch (trainer.py:167-170), test.py predicts from the trained weights
    from cgr_mpnn_3D._amd.optim import FusedAdam

    b = make_batch(32, n_mace=32, seed=3)
    data = b.to_torch(cuda_device)
    m = _model(cuda_device, b.x.shape[1], 3, 128)
    opt = (torch.optim.Adam(m.parameters(), lr=1e-2, amsgrad=True) if opt_kind == "torch"
           else FusedAdam(m.parameters(), lr=1e-2, amsgrad=True))
    m.train()

    def step():
        opt.zero_grad(set_to_none=True)
        torch.nn.MSELoss(reduction="sum")(m(data), data.y).backward()
        opt.step()

    _assert_predict_is_current(m, data)
    if opt_kind != "fused_captured":
        for _ in range(3):
            step()
            _assert_predict_is_current(m, data)
        return
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    before = [p.detach().clone() for p in m.parameters()]
    for _ in range(3):
        g.replay()
        torch.cuda.synchronize()
        _assert_predict_is_current(m, data)
    assert not all(torch.equal(a, p) for a, p in zip(before, m.parameters()))


def test_predict_dropout_in_train_mode_under_no_grad(cuda_device):
    # F.dropout(training=self.training) applies under no_grad too (GNN.py:100-102)
    b = make_batch(16, n_mace=16, seed=5)
    data = b.to_torch(cuda_device)
    m = _model(cuda_device, b.x.shape[1], 3, 96, p=0.3)
    m.eval()
    with torch.no_grad():
        y_eval = m(data)
        m.train()
        y1 = m(data)
        y2 = m(data)
    assert not torch.equal(y1, y_eval)
    assert not torch.equal(y1, y2)  # a fresh mask per call (device counter)


def test_captured_batched_inference_replays(cuda_device):
    b = make_batch(64, seed=11)
    data = b.to_torch(cuda_device)
    m = _model(cuda_device, b.x.shape[1], 4, 400).eval()
    with torch.no_grad():
        ref = m(data).clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            m(data)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = m(data)
        g.replay()
        torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_single_reaction_calls_equal_the_batched_path(cuda_device):
    """The reference's inference call pattern -- one reaction per model(data) under no_grad,
    batch=None (cli_tool/activation_energy_predictor.py:72-76) or a one-graph Batch (test.py's
    DataLoader batch_size 1, :85-113): both forms give the same prediction bit for bit, and the
    batched forward of all reactions agrees within fp32 rounding (a dst segment that crosses a
    row tile in the batch is summed as two partials)."""
    from cgr_mpnn_3D._amd.synth import TorchBatch

    b = make_batch(6, n_atoms=30, n_bonds=30, n_mace=768, seed=77, n_atoms_jitter=4)
    m = _model(cuda_device, b.x.shape[1], 4, 400).eval()
    data = b.to_torch(cuda_device)
    with torch.no_grad():
        y_batched = m(data)
        singles = []
        for g in range(b.num_graphs):
            v0, v1 = int(b.ptr[g]), int(b.ptr[g + 1])
            sel = torch.from_numpy((b.edge_index[0] >= v0) & (b.edge_index[0] < v1)).to(cuda_device)
            x = data.x[v0:v1]
            ei = (data.edge_index[:, sel] - v0).contiguous()
            ea = data.edge_attr[sel].contiguous()
            y_none = m(TorchBatch(x, ei, ea, None))
            bt = torch.zeros(x.shape[0], dtype=torch.int64, device=cuda_device)
            ptr = torch.tensor([0, x.shape[0]], dtype=torch.int64, device=cuda_device)
            y_one = m(TorchBatch(x, ei, ea, bt, ptr))
            assert y_none.shape == (1,) and torch.equal(y_none, y_one)
            singles.append(y_none)
    y_single = torch.cat(singles)
    assert torch.allclose(y_single, y_batched, rtol=1e-5, atol=1e-6), (y_single, y_batched)
