"""Fused Adam / AMSGrad on the MI355X path: ``torch.optim.Adam`` semantics, one native launch.

The reference trains with ``torch.optim.Adam(model.parameters(), lr=lr,
weight_decay=weight_decay, amsgrad=True)`` (train.py:117-119) plus ``ExponentialLR``
(train.py:121).  torch's foreach implementation runs ~11 multi-tensor kernels per step; this class
keeps the same constructor, ``param_groups`` / ``state`` layout (``step``, ``exp_avg``,
``exp_avg_sq``, ``max_exp_avg_sq``) and update rule, and performs the whole update in
``cgr_adam_step`` (csrc/optim.hip): one kernel over every tensor plus a tiny step-counter
kernel.  Each tensor's ``state["step"]`` lives on the device (like ``capturable=True``), so a training step that
includes ``optimizer.step()`` can be captured into a HIP graph and replayed; ``lr`` is read from
``param_groups`` at each call (a graph replays the lr it was captured with, as torch's does).
Parameters must be fp32 CUDA tensors; there is no CPU fallback.
"""

from __future__ import annotations

import ctypes

import torch

from . import native


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 amsgrad=False, *, maximize=False):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=amsgrad,
                        maximize=maximize)
        super().__init__(params, defaults)
        self._lib = native.load()

    def _init_state(self, p):
        st = self.state[p]
        if len(st) == 0:
            if not p.is_cuda or p.dtype != torch.float32:
                raise RuntimeError("FusedAdam: parameters must be float32 tensors on the GPU")
            st["step"] = torch.zeros((), dtype=torch.float32, device=p.device)  # device, like
            # torch's capturable=True: the native kernel advances it
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["max_exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        else:  # e.g. after load_state_dict of a torch.optim.Adam state (CPU step tensors)
            for k in ("step", "exp_avg", "exp_avg_sq", "max_exp_avg_sq"):
                v = st.get(k)
                if v is None:
                    st[k] = (torch.zeros((), dtype=torch.float32, device=p.device) if k == "step"
                             else torch.zeros_like(p, memory_format=torch.preserve_format))
                elif v.device != p.device or v.dtype != torch.float32 or not v.is_contiguous():
                    st[k] = v.to(device=p.device, dtype=torch.float32).contiguous()
        return st

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            beta1, beta2 = group["betas"]
            tab = (native.CgrAdamTensor * len(ps))()
            for i, p in enumerate(ps):
                st = self._init_state(p)
                g = p.grad
                if g.dtype != torch.float32 or not g.is_contiguous() or not p.is_contiguous():
                    raise RuntimeError("FusedAdam: contiguous float32 params/grads required")
                tab[i] = native.CgrAdamTensor(p.data_ptr(), g.data_ptr(),
                                              st["exp_avg"].data_ptr(),
                                              st["exp_avg_sq"].data_ptr(),
                                              st["max_exp_avg_sq"].data_ptr(),
                                              st["step"].data_ptr(), p.numel())
            dev = ps[0].device
            if any(p.device != dev for p in ps):
                raise RuntimeError("FusedAdam: all parameters of a group must be on one device")
            with native.device_guard(dev):
                native.check(self._lib.cgr_adam_step(
                    tab, len(ps), float(group["lr"]), float(beta1), float(beta2),
                    float(group["eps"]), float(group["weight_decay"]),
                    int(bool(group["amsgrad"])), int(bool(group["maximize"])),
                    native.stream_ptr(dev)))
        return loss
