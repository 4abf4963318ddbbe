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
import operator

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

    _STATE_KEYS = ("exp_avg", "exp_avg_sq", "max_exp_avg_sq", "step")

    def _table(self, gi, params, grads):
        """The group's CgrAdamTensor table.  Built once and kept while the group's parameters,
        their state tensors and the state dict itself are the same objects (load_state_dict
        replaces the dict, so it rebuilds); per step only the parameter and gradient pointers are
        rewritten.  Every gradient is still checked (fp32, contiguous) each step."""
        for g in grads:
            if g.dtype != torch.float32 or not g.is_contiguous():
                raise RuntimeError("FusedAdam: contiguous float32 params/grads required")
        cache = self.__dict__.setdefault("_cgr_tables", {})
        hit = cache.get(gi)
        if hit is not None:
            state, ps, sts, tab = hit
            ok = state is self.state and len(ps) == len(params)
            if ok:
                for p, q, s in zip(params, ps, sts):
                    st = state.get(p)
                    if p is not q or st is None or \
                            not all(map(operator.is_, map(st.get, self._STATE_KEYS), s)):
                        ok = False
                        break
            if ok:
                for i, (p, g) in enumerate(zip(params, grads)):
                    e = tab[i]
                    if e.numel != p.numel():  # p.data was replaced by a tensor of another size
                        ok = False
                        break
                    e.param, e.grad = p.data_ptr(), g.data_ptr()
            if ok:
                return tab
        sts = []
        tab = (native.CgrAdamTensor * len(params))()
        for i, (p, g) in enumerate(zip(params, grads)):
            st = self._init_state(p)
            if not p.is_contiguous():
                raise RuntimeError("FusedAdam: contiguous float32 params/grads required")
            s = tuple(st[k] for k in self._STATE_KEYS)
            sts.append(s)
            tab[i] = native.CgrAdamTensor(p.data_ptr(), g.data_ptr(), s[0].data_ptr(),
                                          s[1].data_ptr(), s[2].data_ptr(), s[3].data_ptr(),
                                          p.numel())
        dev = params[0].device
        if any(p.device != dev for p in params):
            raise RuntimeError("FusedAdam: all parameters of a group must be on one device")
        cache[gi] = (self.state, list(params), sts, tab)
        return tab

    def __setstate__(self, state):
        super().__setstate__(state)
        self.__dict__.pop("_cgr_tables", None)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for gi, group in enumerate(self.param_groups):
            ps = group["params"]
            grads = [p.grad for p in ps]
            if any(g is None for g in grads):
                ps = [p for p, g in zip(ps, grads) if g is not None]
                grads = [g for g in grads if g is not None]
            if not ps:
                continue
            beta1, beta2 = group["betas"]
            tab = self._table(gi, ps, grads)
            dev = ps[0].device
            with native.device_guard(dev):
                native.check(self._lib.cgr_adam_step(
                    tab, len(ps), float(group["lr"]), float(beta1), float(beta2),
                    float(group["eps"]), float(group["weight_decay"]),
                    int(bool(group["amsgrad"])), int(bool(group["maximize"])),
                    native.stream_ptr(dev)))
        return loss
