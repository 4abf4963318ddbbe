"""FusedAdam (csrc/optim.hip via cgr_adam_step) against torch.optim.Adam on the same device.

The reference optimiser is ``torch.optim.Adam(..., weight_decay=wd, amsgrad=True)``
(train.py:117-119); the fused kernel must follow the same update (fp32, rtol 1e-5 over several
steps: the only differences are fma contractions inside one element's update).
"""

import copy

import pytest
import torch

from cgr_mpnn_3D._amd.optim import FusedAdam
from cgr_mpnn_3D._amd.synth import make_batch
from cgr_mpnn_3D.models.GNN import GNN

pytestmark = pytest.mark.gpu


def _tensors(dev, shapes, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(s, generator=g).to(dev).requires_grad_() for s in shapes]


SHAPES = [(400, 860), (400,), (400, 400), (1, 400), (1,), (7, 3), (1001,), ()]


@pytest.mark.parametrize("amsgrad,wd,maximize", [(True, 0.0, False), (True, 1e-2, False),
                                                 (False, 0.0, False), (True, 0.0, True)])
def test_fused_adam_matches_torch(amsgrad, wd, maximize, cuda_device):
    ps_ref = _tensors(cuda_device, SHAPES, 0)
    ps = [p.detach().clone().requires_grad_() for p in ps_ref]
    ref = torch.optim.Adam(ps_ref, lr=3e-3, weight_decay=wd, amsgrad=amsgrad, maximize=maximize)
    opt = FusedAdam(ps, lr=3e-3, weight_decay=wd, amsgrad=amsgrad, maximize=maximize)
    g = torch.Generator().manual_seed(1)
    for it in range(6):
        grads = [torch.randn(p.shape, generator=g).to(cuda_device) * (1 + it) for p in ps]
        for p, q, gr in zip(ps, ps_ref, grads):
            p.grad = gr.clone()
            q.grad = gr.clone()
        ps[2].grad = None if it == 3 else ps[2].grad  # p.grad None -> skipped, like torch
        ps_ref[2].grad = None if it == 3 else ps_ref[2].grad
        opt.step()
        ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ps, ps_ref):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)
    for a, b in zip(ps, ps_ref):
        sa, sb = opt.state[a], ref.state[b]
        # ulp-level: |grad| reaches ~6 here (ulp 5e-7)
        torch.testing.assert_close(sa["exp_avg"], sb["exp_avg"], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(sa["exp_avg_sq"], sb["exp_avg_sq"], rtol=1e-5, atol=1e-6)
        if amsgrad:
            torch.testing.assert_close(sa["max_exp_avg_sq"], sb["max_exp_avg_sq"], rtol=1e-5,
                                       atol=1e-6)


def test_fused_adam_loads_torch_adam_state(cuda_device):
    ps_ref = _tensors(cuda_device, [(33, 7), (5,)], 3)
    ps = [p.detach().clone().requires_grad_() for p in ps_ref]
    ref = torch.optim.Adam(ps_ref, lr=1e-2, amsgrad=True)
    for p, q in zip(ps, ps_ref):
        q.grad = torch.randn_like(q)
    ref.step()
    opt = FusedAdam(ps, lr=1e-2, amsgrad=True)
    opt.load_state_dict(copy.deepcopy(ref.state_dict()))  # torch shares the state tensors
    for p, q in zip(ps, ps_ref):
        p.data.copy_(q.data)
        q.grad = torch.randn_like(q)
        p.grad = q.grad.clone()
    ref.step()
    opt.step()
    torch.cuda.synchronize()
    for a, b in zip(ps, ps_ref):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)


def test_fused_adam_table_follows_state_and_parameter_changes(cuda_device):
    """The per-group pointer table is reused across steps (r06 host trim): a reloaded state dict,
    a replaced state tensor, `p.data` moved to new storage and a group that gains a gradient must
    all reach the kernel (checked against torch.optim.Adam after each change)."""
    ps_ref = _tensors(cuda_device, [(40, 9), (9,), (5, 5), ()], 5)
    ps = [p.detach().clone().requires_grad_() for p in ps_ref]
    ref = torch.optim.Adam(ps_ref, lr=2e-2, amsgrad=True)
    opt = FusedAdam(ps, lr=2e-2, amsgrad=True)
    g = torch.Generator().manual_seed(9)

    def both_step(skip=None):
        for i, (p, q) in enumerate(zip(ps, ps_ref)):
            gr = torch.randn(p.shape, generator=g).to(cuda_device)
            p.grad = None if i == skip else gr.clone()
            q.grad = None if i == skip else gr.clone()
        opt.step()
        ref.step()

    def same():
        torch.cuda.synchronize()
        for a, b in zip(ps, ps_ref):
            torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)
            sa, sb = opt.state[a], ref.state[b]
            for k in ("exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
                torch.testing.assert_close(sa[k], sb[k], rtol=1e-5, atol=1e-6)

    both_step()
    both_step()
    same()
    opt.load_state_dict(copy.deepcopy(opt.state_dict()))  # a new state dict
    both_step()
    same()
    st = opt.state[ps[0]]
    st["exp_avg"] = st["exp_avg"].clone()  # a replaced state tensor
    both_step()
    same()
    for p, q in zip(ps, ps_ref):  # new storage under the same parameter objects
        p.data = p.data.clone()
        q.data = q.data.clone()
    both_step()
    same()
    both_step(skip=1)  # one parameter without a gradient this step, then back
    both_step()
    same()


def test_fused_adam_many_tensors_and_misaligned_grads(cuda_device):
    # > CGR_ADAM_GROUP tensors (several launches) and grads that are views at odd offsets of one
    # flat buffer (the native backward's bucket layout): scalar path for those tensors
    shapes = [(3 + i % 5,) for i in range(70)] + [(64, 64)]
    ps_ref = _tensors(cuda_device, shapes, 2)
    ps = [p.detach().clone().requires_grad_() for p in ps_ref]
    ref = torch.optim.Adam(ps_ref, lr=1e-2, amsgrad=True)
    opt = FusedAdam(ps, lr=1e-2, amsgrad=True)
    for it in range(3):
        flat = torch.randn(sum(p.numel() for p in ps), device=cuda_device)
        off = 0
        for p, q in zip(ps, ps_ref):
            n = p.numel()
            p.grad = flat[off:off + n].view(p.shape)
            q.grad = p.grad.clone()
            off += n
        opt.step()
        ref.step()
    torch.cuda.synchronize()
    for a, b in zip(ps, ps_ref):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)


def test_fused_adam_training_step_graph_capture(cuda_device):
    """A whole training step (fwd + MSE + native bwd + FusedAdam) captured once and replayed
    equals the same steps run eagerly (the device step counter advances per replay)."""
    b = make_batch(16, n_mace=32, seed=71)
    data = b.to_torch(cuda_device)

    def build():
        torch.manual_seed(0)
        # dropout 0: the dropout seed is drawn on the host per forward, so a replay would reuse
        # the captured mask (graph capture)
        m = GNN(b.x.shape[1], 14, depth=2, hidden_sizes=[64] * 2, dropout_ps=[0.0] * 2)
        m = m.to(cuda_device).train()
        return m, FusedAdam(m.parameters(), lr=1e-3, amsgrad=True)

    loss_fn = torch.nn.MSELoss(reduction="sum")

    def step(m, opt):
        opt.zero_grad(set_to_none=True)
        loss = loss_fn(m(data), data.y)
        loss.backward()
        opt.step()
        return loss.detach()

    m1, o1 = build()
    eager = [step(m1, o1).item() for _ in range(8)]

    m2, o2 = build()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        warm = [step(m2, o2).item() for _ in range(3)]
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        gl = step(m2, o2)
    replayed = []
    for _ in range(5):
        gr.replay()
        replayed.append(gl.item())
    # capture itself executes nothing: replays continue the eager sequence at step 4
    assert warm == eager[:3]
    torch.testing.assert_close(torch.tensor(replayed), torch.tensor(eager[3:]), rtol=1e-6,
                               atol=0)
    for a, c in zip(m1.parameters(), m2.parameters()):
        torch.testing.assert_close(a, c, rtol=1e-6, atol=1e-7)
