"""``MSELoss`` on the native kernels (``cgr_mse_loss_forward`` / ``_backward``): a drop-in for the
``torch.nn.MSELoss(reduction="sum")`` that train.py:120 hands the trainer (trainer.py:142-143),
``reduction="mean"`` too.  Forward and backward are one launch each (torch: four kernels), so the
captured training step carries two launches for its loss instead of five.  Same values as torch up
to the summation order; deterministic."""

from __future__ import annotations

import torch
from torch import nn

from . import native


class _MSELossFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input, target, mean):
        lib = native.load()
        x = input.contiguous()
        t = target.contiguous()
        out = torch.empty((), dtype=torch.float32, device=x.device)
        with native.device_guard(x.device):
            native.check(lib.cgr_mse_loss_forward(native.ptr(x), native.ptr(t), x.numel(),
                                                  int(mean), native.ptr(out),
                                                  native.stream_ptr(x.device)))
        ctx.save_for_backward(x, t)
        ctx.mean = mean
        return out

    @staticmethod
    def backward(ctx, grad):
        lib = native.load()
        x, t = ctx.saved_tensors
        g = grad.contiguous().float()
        gi = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        gt = torch.empty_like(t) if ctx.needs_input_grad[1] else None
        with native.device_guard(x.device):
            native.check(lib.cgr_mse_loss_backward(
                native.ptr(x), native.ptr(t), native.ptr(g), x.numel(), int(ctx.mean),
                native.ptr(gi) if gi is not None else None,
                native.ptr(gt) if gt is not None else None, native.stream_ptr(x.device)))
        return gi, gt, None


class MSELoss(nn.Module):
    """``torch.nn.MSELoss`` for fp32 CUDA tensors of one shape; reduction "sum" or "mean"."""

    def __init__(self, reduction: str = "mean"):
        super().__init__()
        if reduction not in ("sum", "mean"):
            raise NotImplementedError(
                f"cgr_mpnn_3D MSELoss: reduction={reduction!r} (native: 'sum', 'mean')")
        self.reduction = reduction

    def forward(self, input, target):
        if not (input.is_cuda and target.is_cuda):
            raise RuntimeError("cgr_mpnn_3D MSELoss runs on the GPU only (no CPU fallback)")
        if input.shape != target.shape:
            raise ValueError(f"MSELoss: input {tuple(input.shape)} and target "
                             f"{tuple(target.shape)} must have the same shape (no broadcasting)")
        if input.dtype != torch.float32 or target.dtype != torch.float32:
            raise TypeError("cgr_mpnn_3D MSELoss: fp32 tensors required")
        if input.device != target.device:
            raise RuntimeError("MSELoss: input and target on different devices")
        return _MSELossFunction.apply(input, target, self.reduction == "mean")
