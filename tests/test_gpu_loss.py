"""Native MSELoss (cgr_mse_loss_forward/_backward) vs torch.nn.MSELoss: the loss train.py:120
builds (reduction="sum") and trainer.py:142-143 applies, plus reduction="mean"."""

import pytest
import torch

from cgr_mpnn_3D._amd.loss import MSELoss

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [1, 7, 256, 1000, 70001])
@pytest.mark.parametrize("reduction", ["sum", "mean"])
def test_mse_matches_torch(n, reduction, cuda_device):
    g = torch.Generator().manual_seed(n)
    y = (torch.randn(n, generator=g) * 3).to(cuda_device).requires_grad_(True)
    t = torch.randn(n, generator=g).to(cuda_device).requires_grad_(True)
    y2 = y.detach().clone().requires_grad_(True)
    t2 = t.detach().clone().requires_grad_(True)
    ours = MSELoss(reduction)(y, t)
    ref = torch.nn.MSELoss(reduction=reduction)(y2, t2)
    assert ours.shape == ref.shape == torch.Size([])
    assert torch.allclose(ours, ref, rtol=2e-6, atol=0)
    (ours * 1.5).backward()
    (ref * 1.5).backward()
    assert torch.allclose(y.grad, y2.grad, rtol=1e-6, atol=1e-7)
    assert torch.allclose(t.grad, t2.grad, rtol=1e-6, atol=1e-7)


def test_mse_deterministic_and_capturable(cuda_device):
    y = torch.randn(256, device=cuda_device, requires_grad=True)
    t = torch.randn(256, device=cuda_device)
    fn = MSELoss("sum")
    a = fn(y, t).item()
    assert all(fn(y, t).item() == a for _ in range(3))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            fn(y, t).backward()
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    y.grad = None
    with torch.cuda.graph(gr):
        loss = fn(y, t)
        loss.backward()
    y.grad.zero_()
    gr.replay()
    torch.cuda.synchronize()
    assert loss.item() == a
    assert torch.allclose(y.grad, 2 * (y - t).detach(), rtol=1e-6, atol=0)


def test_mse_rejects_mismatch(cuda_device):
    fn = MSELoss("sum")
    with pytest.raises(ValueError):
        fn(torch.zeros(4, device=cuda_device), torch.zeros(4, 1, device=cuda_device))
    with pytest.raises(RuntimeError):
        fn(torch.zeros(4), torch.zeros(4))
    with pytest.raises(NotImplementedError):
        MSELoss("none")
