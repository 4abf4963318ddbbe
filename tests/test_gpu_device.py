"""Device placement and RNG-stream behaviour of the drop-in GNN."""

import pytest
import torch

from cgr_mpnn_3D._amd.synth import make_batch
from cgr_mpnn_3D.models.GNN import GNN

pytestmark = pytest.mark.gpu


def _model(F, dev, p=0.2, seed=0):
    torch.manual_seed(seed)
    return GNN(F, 14, depth=2, hidden_sizes=[64, 64], dropout_ps=[p, p]).to(dev).train()


def test_training_forward_leaves_cpu_rng_stream(cuda_device):
    """The dropout key comes from the CUDA generator's seed: a training forward consumes no CPU
    random numbers (the reference's F.dropout draws on the device generator only)."""
    b = make_batch(6, n_mace=16, seed=3)
    data = b.to_torch(cuda_device)
    m = _model(b.x.shape[1], cuda_device)
    torch.manual_seed(5)
    ref = torch.rand(4)
    torch.manual_seed(5)
    y = m(data)
    after = torch.rand(4)
    assert torch.equal(ref, after)
    assert torch.isfinite(y).all()


def test_dropout_masks_follow_manual_seed(cuda_device):
    """Same torch.manual_seed, same construction order, same counter -> same masks; a different
    seed -> different masks."""
    b = make_batch(6, n_mace=16, seed=4)
    data = b.to_torch(cuda_device)
    ys = []
    for s in (11, 11, 12):
        GNN._cgr_instances = 0
        m = _model(b.x.shape[1], cuda_device, p=0.4, seed=s)
        ys.append(m(data).detach())
    assert torch.equal(ys[0], ys[1])
    assert not torch.equal(ys[0], ys[2])


def test_input_gradients_under_dropout_and_no_grad(cuda_device):
    """x.grad through cgr_gnn_input_grads in train mode with dropout (the recorded mask applies to
    both backward passes); no_grad still takes the forward-only path."""
    b = make_batch(4, n_mace=16, seed=5)
    data = b.to_torch(cuda_device)
    m = _model(b.x.shape[1], cuda_device, p=0.1)
    m.train()
    data.x.requires_grad_(True)
    y = m(data)
    y.sum().backward()
    assert data.x.grad is not None and torch.isfinite(data.x.grad).all()
    assert data.x.grad.abs().sum() > 0
    with torch.no_grad():
        assert torch.isfinite(m(data)).all()


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two visible GPUs")
def test_model_on_non_current_device():
    """Model and batch on cuda:1 while cuda:0 is current: the native calls switch device and the
    side streams are created on the stream's device; results equal the same run on cuda:0."""
    b = make_batch(6, n_mace=16, seed=6)
    out = []
    for dev in ("cuda:0", "cuda:1"):
        torch.cuda.set_device(0)
        data = b.to_torch(torch.device(dev))
        m = _model(b.x.shape[1], torch.device(dev), p=0.0)
        y = m(data)
        y.sum().backward()
        out.append((y.detach().cpu(), [q.grad.detach().cpu() for q in m.parameters()]))
    assert torch.equal(out[0][0], out[1][0])
    for a, c in zip(out[0][1], out[1][1]):
        assert torch.equal(a, c)
