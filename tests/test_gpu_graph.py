"""Graph-captured dropout: a replayed forward draws a fresh mask each time (device counter in the
GNN module, advanced by the native forward) and each replay equals an eager forward keyed with
the same effective dropout key (seed + 0xD1B54A32D192ED03 * (counter + 1), csrc/kernels.hip
k_rng_key).  Reference dropout: GNN.py:100-102 (F.dropout, training only)."""

import pytest
import torch

from cgr_mpnn_3D._amd.debug import ArenaRun
from cgr_mpnn_3D._amd.synth import make_batch
from cgr_mpnn_3D.models.GNN import GNN

pytestmark = pytest.mark.gpu

MULT = 0xD1B54A32D192ED03


def test_captured_forward_redraws_dropout_mask_per_replay(cuda_device):
    b = make_batch(24, n_mace=32, seed=81)
    data = b.to_torch(cuda_device)
    D, H, p = 3, 64, 0.3
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[p] * D)
    m = m.to(cuda_device).train()
    with torch.no_grad():
        for _ in range(2):  # eager warm-up (lazy native streams, allocator)
            m(data)
    torch.cuda.synchronize()
    counter0 = int(m._cgr_rng_counter.item())
    assert counter0 == 2  # one advance per eager forward

    g = torch.cuda.CUDAGraph()
    torch.manual_seed(1234)
    seed_cap = m._cgr_dropout_seed(torch.device(cuda_device))  # the key base GNN.forward uses
    torch.manual_seed(1234)
    with torch.no_grad(), torch.cuda.graph(g):
        y_cap = m(data)
    ys = []
    for _ in range(3):
        g.replay()
        ys.append(y_cap.clone())
    torch.cuda.synchronize()
    assert int(m._cgr_rng_counter.item()) == counter0 + 3
    assert not torch.equal(ys[0], ys[1]) and not torch.equal(ys[1], ys[2])

    params = [q.detach().contiguous() for q in m.native_parameters()]
    cfg = (b.x.shape[1], 14, H, D, 0, False)
    for k, y in enumerate(ys):
        key = (seed_cap + MULT * (counter0 + k + 1)) % 2**64
        run = ArenaRun(cfg, data.x, data.edge_index, data.edge_attr, data.batch, data.ptr,
                       b.num_graphs, params, dropout_ps=[p] * D, seed=key, training=True)
        assert torch.equal(run.y, y), k


def test_captured_training_step_backward_uses_forward_mask(cuda_device):
    """fwd + bwd captured with dropout: each replay's gradients equal the eager backward of an
    eager forward keyed like that replay."""
    b = make_batch(16, n_mace=32, seed=82)
    data = b.to_torch(cuda_device)
    D, H, p = 2, 64, 0.25
    torch.manual_seed(0)
    m = GNN(b.x.shape[1], 14, depth=D, hidden_sizes=[H] * D, dropout_ps=[p] * D,
            activation_fn=torch.nn.functional.silu).to(cuda_device).train()
    params = list(m.native_parameters())

    def step():
        y = m(data)
        gs = torch.autograd.grad(y.sum(), params)
        return y.detach(), gs

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    counter0 = int(m._cgr_rng_counter.item())
    torch.manual_seed(99)
    seed_cap = m._cgr_dropout_seed(torch.device(cuda_device))
    torch.manual_seed(99)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y_cap, g_cap = step()
    cfg = (b.x.shape[1], 14, H, D, 1, False)
    pd = [q.detach().contiguous() for q in params]
    for k in range(2):
        g.replay()
        torch.cuda.synchronize()
        key = (seed_cap + MULT * (counter0 + k + 1)) % 2**64
        run = ArenaRun(cfg, data.x, data.edge_index, data.edge_attr, data.batch, data.ptr,
                       b.num_graphs, pd, dropout_ps=[p] * D, seed=key, training=True)
        assert torch.equal(run.y, y_cap)
        grads = run.backward(torch.ones_like(run.y), pd)
        for a, c in zip(grads, g_cap):
            assert torch.equal(a, c)
